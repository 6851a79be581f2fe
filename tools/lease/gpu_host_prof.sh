# rocprofv3 kernel trace of the host-env preset (C++ rollout driver, no overlap)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_host
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_host -o run -- \
  python3 benchmarks/configs_bench.py --presets cartpole-reinforce-host --steps 3 --warmup 1 --set overlap=false > gpurun_out/prof_host/log.txt 2>&1 && \
python tools/prof_summary.py gpurun_out/prof_host/run_kernel_stats.csv > gpurun_out/prof_host_summary.txt && cat gpurun_out/prof_host_summary.txt | head -20 && grep preset gpurun_out/prof_host/log.txt | cut -c 200-700
