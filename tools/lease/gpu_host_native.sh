# Host-env path with the C++ rollout driver: numerics vs the Python loop, then throughput
# with and without the actor / learner CU partition.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_trainers_gpu.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider -k "host or native" > gpurun_out/host_tests.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python benchmarks/configs_bench.py --presets cartpole-reinforce-host halfcheetah-ppo-host --steps 8 --warmup 2 > gpurun_out/host_native.jsonl 2>&1 && grep preset gpurun_out/host_native.jsonl | cut -c 1-60,200-700 && \
timeout -k 10 300 python benchmarks/configs_bench.py --presets cartpole-reinforce-host halfcheetah-ppo-host --steps 8 --warmup 2 --set actor_cus=32 > gpurun_out/host_native_32.jsonl 2>&1 && grep preset gpurun_out/host_native_32.jsonl | cut -c 1-60,200-700
