set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u benchmarks/configs_bench.py --presets cartpole-reinforce-baseline lunarlander-reinforce-baseline pong-a2c halfcheetah-ppo halfcheetah-ppo-host --steps 5 --warmup 2 > gpurun_out/configs_v4.jsonl 2> gpurun_out/configs_v4.err && echo CFG_OK && \
timeout -k 10 300 python -u benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 20 --warmup 3 > gpurun_out/pong_v4.jsonl 2> gpurun_out/pong_v4.err && echo PONG_OK
