#!/bin/bash
# Round 5, lease Z: the s_setprio conv3 backward as the default -- CNN / Pong GPU tests.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py tests/test_capture_robustness_gpu.py tests/test_convergence_gpu.py \
  > gpurun_out/r5z_tests.log 2>&1 || { tail -30 gpurun_out/r5z_tests.log; exit 1; }
tail -2 gpurun_out/r5z_tests.log
