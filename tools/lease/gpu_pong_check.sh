# CNN numerics + two Pong A2C benchmark runs (2048 envs).
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py tests/test_pixel.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cnn_tests.log 2>&1 && echo CNN_TESTS_OK || exit 1
for v in 1 2; do
  timeout -k 10 200 python benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 20 --warmup 3 > gpurun_out/pong_$v.log 2>&1 || exit 1
  echo "run$v $(tail -1 gpurun_out/pong_$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],3))')"
done
