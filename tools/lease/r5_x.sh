#!/bin/bash
# Round 5, lease X: wave priority (s_setprio) in the 8-wave conv2 / conv3 backward kernels --
# bitwise tests, kernel times (cnn_kbench, rotated rounds), Pong ABBA with the faster forms.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py -k "bitwise_equal" \
  > gpurun_out/r5x_tests.log 2>&1 || { tail -30 gpurun_out/r5x_tests.log; exit 1; }
tail -2 gpurun_out/r5x_tests.log
timeout -k 10 200 python -u tools/cnn_kbench.py --which bwd3,bwd3_sp1,bwd3_sp2,bwd2,bwd2_sp1,bwd2_sp2 --rounds 4 --iters 20 \
  > gpurun_out/r5x_kbench.jsonl 2> gpurun_out/r5x_kbench.err || { tail -20 gpurun_out/r5x_kbench.err; exit 1; }
cat gpurun_out/r5x_kbench.jsonl
