# bf16x6 gradient kernel heads: numerics (value, categorical A=2..4, Gaussian), timing, preset benches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_value_grad_gpu.py tests/test_kernels_gpu.py tests/test_trainers_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/vg_heads_tests.log 2>&1; rc=$?; tail -3 gpurun_out/vg_heads_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/kbench.py grad --iters 20 > gpurun_out/vg_heads_kbench.jsonl 2>&1 && \
timeout -k 10 200 python tools/kbench.py pgrad --iters 20 >> gpurun_out/vg_heads_kbench.jsonl 2>&1 && \
timeout -k 10 300 python tools/kbench.py pgauss --iters 10 >> gpurun_out/vg_heads_kbench.jsonl 2>&1 && grep -v amdgpu.ids gpurun_out/vg_heads_kbench.jsonl && \
timeout -k 10 400 python benchmarks/configs_bench.py --presets cartpole-reinforce-baseline lunarlander-reinforce-baseline halfcheetah-ppo --steps 5 --warmup 2 > gpurun_out/vg_heads_configs.jsonl 2>&1; grep preset gpurun_out/vg_heads_configs.jsonl | cut -c1-300
