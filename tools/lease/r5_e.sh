#!/bin/bash
# Round 5, lease E: the GPU suite after the native reference-frame path, then the reference-wire
# fan-in rows against the GPU learner.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
    > gpurun_out/r5e_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5e_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u benchmarks/fanin_bench.py --agents 16 64 --transports zmq-ref --seconds 10 \
    --out gpurun_out/r5e_fanin.jsonl > gpurun_out/r5e_fanin.log 2>&1 || exit $?
mkdir -p gpurun_out/prof_flagship_r5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flagship_r5 -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-ttt --host-steps 0 --pong-steps 0 --pong-big-envs 0 --ref-cpu-seconds 0 \
  --convergence off --actor-learner off --phase-steps 0 > gpurun_out/prof_flagship_r5/log.txt 2>&1 || exit $?
exit $rc
