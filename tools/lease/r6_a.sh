#!/bin/bash
# Round 6, lease A: new GPU tests (preflight child on real RCCL, gloo capture-failure fallback,
# world-2 TTT), the whole GPU suite, smoke, then a 1-GPU bench line.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_bench_gpu.py > gpurun_out/r6a_bench_tests.log 2>&1 || { tail -40 gpurun_out/r6a_bench_tests.log; exit 1; }
tail -3 gpurun_out/r6a_bench_tests.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6a_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r6a_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r6a_gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6a_smoke.log 2>&1 && echo SMOKE_OK
timeout -k 10 400 python bench.py > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err && tail -c 600 gpurun_out/r6a_bench.json
