#!/bin/bash
# Round 6, lease X (after the decoder hardening and native encoders): the whole GPU suite, smoke, then the
# 1-GPU bench line (flagship + Pong keys).
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6x_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r6x_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r6x_gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6x_smoke.log 2>&1 && echo SMOKE_OK
timeout -k 10 400 python bench.py > gpurun_out/r6x_bench.json 2> gpurun_out/r6x_bench.err && tail -c 900 gpurun_out/r6x_bench.json
