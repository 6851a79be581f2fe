# rocprofv3 kernel-time summary of the Pong A2C benchmark (2048 envs).
set -o pipefail
mkdir -p gpurun_out/prof_pong
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 12 --warmup 2 > gpurun_out/prof_pong/log.txt 2>&1 && echo PROF_OK
