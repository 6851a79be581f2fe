# Kernel timeline of the overlapped, CU-partitioned host-env preset (analysed on the host)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_hostov
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_hostov -o run -- \
  python3 benchmarks/configs_bench.py --presets cartpole-reinforce-host --steps 3 --warmup 1 > gpurun_out/prof_hostov/log.txt 2>&1; rc=$?
ls -la gpurun_out/prof_hostov; exit $rc
