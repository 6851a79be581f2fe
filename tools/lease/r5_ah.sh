#!/bin/bash
# Round 5, lease AH: end-of-round kernel tables of the Pong update at 2,048 and 8,192 envs.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_pong_final gpurun_out/prof_pong8192_final
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong_final -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 20 --warmup 3 > gpurun_out/prof_pong_final/log.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong8192_final -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 8192 --steps 12 --warmup 3 > gpurun_out/prof_pong8192_final/log.txt 2>&1 || exit $?
echo PROF_OK
