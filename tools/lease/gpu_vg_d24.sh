set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_value_grad_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/vg_tests.log 2>&1 && echo VG_OK && \
timeout -k 10 300 python -u benchmarks/configs_bench.py --presets lunarlander-reinforce-baseline halfcheetah-ppo cartpole-reinforce-baseline --steps 5 --warmup 2 > gpurun_out/configs_v3.jsonl 2> gpurun_out/configs_v3.err && echo CFG_OK
