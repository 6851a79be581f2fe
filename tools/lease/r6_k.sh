#!/bin/bash
# Round 6, lease K: the flagship kernel table on its own (headline epochs only).
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
rm -rf gpurun_out/prof_flagship
bash tools/prof_flagship.sh || exit 1
rm -f gpurun_out/prof_flagship/run_kernel_trace.csv
exit 0
