# host-env presets (C++ rollout driver, lag-1 overlap): throughput + per-step breakdown
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/configs_bench.py --presets cartpole-reinforce-host halfcheetah-ppo-host --steps 8 --warmup 2 > gpurun_out/host_bench.jsonl 2>&1; rc=$?
grep preset gpurun_out/host_bench.jsonl | cut -c 1-45,190-640; exit $rc
