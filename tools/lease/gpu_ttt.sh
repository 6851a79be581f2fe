set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_trainers_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "average_ep_return or graph_equals" > gpurun_out/ttt_tests.log 2>&1 && echo T_OK && \
timeout -k 10 300 python bench.py > gpurun_out/bench_ttt.log 2>&1 && echo BENCH_OK && grep metric gpurun_out/bench_ttt.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print(r['value'], r['time_to_threshold_s'], r['time_to_threshold_per_seed_s'])"
