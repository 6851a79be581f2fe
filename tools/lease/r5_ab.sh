#!/bin/bash
# Round 5, lease AB: s_setprio around ONE of the two MFMA clusters (wgrad / dgrad) of the conv2 / conv3
# backward -- bitwise tests and kernel times (rotated rounds).
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py -k "bitwise_equal" \
  > gpurun_out/r5ab_tests.log 2>&1 || { tail -30 gpurun_out/r5ab_tests.log; exit 1; }
tail -2 gpurun_out/r5ab_tests.log
timeout -k 10 300 python -u tools/cnn_kbench.py --which bwd3,bwd3_sp0,bwd3_sp_w,bwd3_sp_d,bwd2,bwd2_sp1,bwd2_sp_w,bwd2_sp_d --rounds 6 --iters 20 \
  > gpurun_out/r5ab_kbench.jsonl 2> gpurun_out/r5ab_kbench.err || { tail -20 gpurun_out/r5ab_kbench.err; exit 1; }
cat gpurun_out/r5ab_kbench.jsonl
