# Kernel numerics + micro-benchmarks + the flagship bench (one GPU call).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/q_tests.log 2>&1 && echo TESTS_OK && \
timeout -k 10 120 python tools/kbench.py rslab --iters 50 > gpurun_out/q_kbench.log 2>&1 && \
timeout -k 10 120 python tools/kbench.py adam --iters 50 >> gpurun_out/q_kbench.log 2>&1 && cat gpurun_out/q_kbench.log && \
timeout -k 10 400 python bench.py > gpurun_out/q_bench.log 2>&1 && tail -1 gpurun_out/q_bench.log
