# value-gradient kernel: numerics + timing (both modes) + flagship bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_value_grad_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/vg_tests.log 2>&1 && echo VG_TESTS_OK || { tail -30 gpurun_out/vg_tests.log; exit 1; }
timeout -k 10 120 python tools/kbench.py grad --iters 20 > gpurun_out/vg_kbench.log 2>&1 && cat gpurun_out/vg_kbench.log || exit 1
timeout -k 10 300 python bench.py > gpurun_out/vg_bench.log 2>&1 && tail -1 gpurun_out/vg_bench.log | cut -c1-400
