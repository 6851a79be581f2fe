#!/bin/bash
# Round 5, lease AG: the 16-wave conv3 backward with s_setprio around its MFMA clusters vs the shipped 8-wave one.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py -k "conv3_bwd_16wave" \
  > gpurun_out/r5ag_tests.log 2>&1 || { tail -30 gpurun_out/r5ag_tests.log; exit 1; }
tail -2 gpurun_out/r5ag_tests.log
timeout -k 10 300 python -u tools/cnn_kbench.py --which bwd3,bwd3_16,bwd3_16_sp --rounds 8 --iters 20 \
  > gpurun_out/r5ag_kbench.jsonl 2> gpurun_out/r5ag_kbench.err || { tail -20 gpurun_out/r5ag_kbench.err; exit 1; }
cat gpurun_out/r5ag_kbench.jsonl
