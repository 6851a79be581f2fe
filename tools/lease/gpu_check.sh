# GPU tests (all, no -x: one run shows every failure), smoke, 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench.log | cut -c1-600
