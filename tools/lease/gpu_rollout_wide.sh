set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rollout_gpu.py tests/test_trainers_gpu.py tests/test_value_grad_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wide_tests.log 2>&1 && echo T_OK && \
timeout -k 10 200 python tools/ttt_epoch_probe.py > gpurun_out/ttt_probe2.json 2> gpurun_out/ttt_probe2.err && echo P_OK && \
timeout -k 10 300 python bench.py > gpurun_out/bench_wide.log 2>&1 && echo BENCH_OK && grep metric gpurun_out/bench_wide.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print(r['value'], r['time_to_threshold_s'], r['time_to_threshold_per_seed_s'])"
