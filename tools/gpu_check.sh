set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && echo BENCH_OK && tail -3 gpurun_out/bench.log
