#!/bin/bash
# Round 5, lease K: Pong with the fused render (conv kernels draw the frames from 16-float frame
# histories; no observation tensor) -- bitwise tests, then an ABBA against the observation path.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py -m gpu -q -k "render or fused_conv or pixel" --timeout 240 --timeout-method thread \
    > gpurun_out/r5k_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5k_gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for run in "2048 0" "2048 1" "2048 1" "2048 0" "8192 0" "8192 1" "8192 1" "8192 0"; do
  set -- $run
  echo "{\"fused_render\": $2, \"envs\": $1}" >> gpurun_out/r5k_pong.jsonl
  RRL_PONG_FUSED_RENDER=$2 timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r5k_pong.jsonl 2>> gpurun_out/r5k_pong.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_pong_r5k
RRL_PONG_FUSED_RENDER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong_r5k -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/prof_pong_r5k/log.txt 2>&1 || exit $?
exit 0
