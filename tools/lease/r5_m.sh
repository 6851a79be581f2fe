#!/bin/bash
# Round 5, lease M: kernel profile of the Pong update at 8,192 envs (the big preset).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_pong8192_r5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong8192_r5 -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 8192 --steps 20 --warmup 3 > gpurun_out/prof_pong8192_r5/log.txt 2>&1 || exit $?
exit 0
