#!/bin/bash
# Round 5, lease AN: Adam with the first float4 loaded before the norm reduction -- the CNN GPU
# tests, then the kernel table of the Pong update at 2,048 envs.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/prof_adam2048
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_gpu.py \
  > gpurun_out/r5an_tests.log 2>&1 || { tail -40 gpurun_out/r5an_tests.log; exit 1; }
tail -2 gpurun_out/r5an_tests.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_adam2048 -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 20 --warmup 3 > gpurun_out/prof_adam2048/log.txt 2>&1 || exit $?
echo PROF_OK
