#!/bin/bash
# Round 5, lease Q: the 128 x 128 fc weight-gradient kernel with inline-asm transposed reads (no
# compiler vmcnt(0) before each k-tile's fragment reads) -- numerics, kernel times, Pong ABBA.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py -k "fc_ or pixel_update" \
  > gpurun_out/r5q_tests.log 2>&1 || { tail -30 gpurun_out/r5q_tests.log; exit 1; }
tail -2 gpurun_out/r5q_tests.log
FC_VARIANTS=422,423,b FC_CASES=wgrad_tn_s2,wgrad_tn_s5,wgrad_tn_s8,wgrad40k_tn_s5 timeout -k 10 300 python -u tools/fc_kbench.py \
  > gpurun_out/r5q_fc_kbench.jsonl 2> gpurun_out/r5q_fc_kbench.err || { tail -20 gpurun_out/r5q_fc_kbench.err; exit 1; }
cat gpurun_out/r5q_fc_kbench.jsonl
