set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_actor_learner_gpu.py tests/test_trainers_gpu.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider -k "continuous or chunk" > gpurun_out/al_big_tests.log 2>&1; rc=$?; tail -8 gpurun_out/al_big_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/big_buffer_bench.py > gpurun_out/big_buffer.jsonl 2>&1; rc=$?; tail -3 gpurun_out/big_buffer.jsonl; exit $rc
