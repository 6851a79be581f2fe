#!/bin/bash
# Round 6, lease J: kernel tables after the round's last kernel change -- the flagship
# and Pong at 8,192 envs on the frame ring; the per-dispatch trace CSVs are dropped (the merge-back
# limit is 64 MiB), the per-kernel stats kept.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
bash tools/prof_flagship.sh || exit 1
rm -f gpurun_out/prof_flagship/run_kernel_trace.csv
bash tools/prof_pong_big.sh || exit 1
rm -f gpurun_out/prof_pong_big/run_kernel_trace.csv
exit 0
