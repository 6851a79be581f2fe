#!/bin/bash
# Round 6, lease F: Pong frame ring (LDS frame-row table, v_perm interleave) (one new frame per env step into a ring of frames; the conv
# kernels interleave 4 frames as they load) -- bitwise tests vs the observation path, then an
# ABBA against the observation path at 2,048 / 8,192 envs and a kernel trace of the ring path.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_frame_ring_gpu.py -x -v --timeout 240 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r6f_ring_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r6f_ring_tests.log
tail -15 gpurun_out/r6f_ring_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for run in "2048 0" "2048 1" "2048 1" "2048 0" "8192 0" "8192 1" "8192 1" "8192 0"; do
  set -- $run
  echo "{\"frame_ring\": $2, \"envs\": $1}" >> gpurun_out/r6f_pong.jsonl
  RRL_PONG_FRAME_RING=$2 timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r6f_pong.jsonl 2>> gpurun_out/r6f_pong.err || exit $?
done
cut -c1-200 gpurun_out/r6f_pong.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_pong_r6f
RRL_PONG_FRAME_RING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong_r6f -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 20 --warmup 3 > gpurun_out/prof_pong_r6f/log.txt 2>&1 || exit $?
exit 0
