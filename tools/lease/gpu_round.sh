# Full round check: GPU tests, smoke, headline bench, preset benches, flagship kernel profile.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_flagship
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench.log | cut -c1-400 && \
timeout -k 10 400 python benchmarks/configs_bench.py --presets cartpole-reinforce-baseline lunarlander-reinforce-baseline halfcheetah-ppo pong-a2c cartpole-reinforce-host halfcheetah-ppo-host --steps 5 --warmup 2 > gpurun_out/configs.jsonl 2>&1 && grep preset gpurun_out/configs.jsonl | cut -c1-200 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flagship -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-ttt --ref-cpu-seconds 0 > gpurun_out/prof_flagship/log.txt 2>&1 && \
python tools/prof_summary.py gpurun_out/prof_flagship/run_kernel_stats.csv > gpurun_out/prof_flagship_summary.txt && head -8 gpurun_out/prof_flagship_summary.txt
