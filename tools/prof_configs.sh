# rocprofv3 kernel-time summaries of the LunarLander and HalfCheetah presets.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for p in lunarlander-reinforce-baseline halfcheetah-ppo; do
  mkdir -p gpurun_out/prof_$p
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$p -o run -- \
    python3 benchmarks/configs_bench.py --presets $p --steps 3 --warmup 1 > gpurun_out/prof_$p/log.txt 2>&1 || exit 1
  tail -1 gpurun_out/prof_$p/log.txt | cut -c1-300
done
