set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_value_grad_gpu.py tests/test_trainers_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ps_tests.log 2>&1 && echo T_OK && \
bash tools/prof_flagship.sh && \
timeout -k 10 300 python bench.py > gpurun_out/bench_ps.log 2>&1 && echo BENCH_OK && grep metric gpurun_out/bench_ps.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print(r['value'], r['time_to_threshold_s'], r['time_to_threshold_per_seed_s'])"
