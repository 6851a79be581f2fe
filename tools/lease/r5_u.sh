#!/bin/bash
# Round 5, lease U: the persistent fc kernels inside a full 20,480-row update vs the 128 x 128 ones.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_cnn_gpu.py -k "persistent_fc or fc_nt_mask or fc_tn" \
  > gpurun_out/r5u_tests.log 2>&1 || { tail -40 gpurun_out/r5u_tests.log; exit 1; }
tail -4 gpurun_out/r5u_tests.log
