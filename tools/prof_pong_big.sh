# rocprofv3 kernel-time summary of the Pong A2C benchmark at 8192 envs.
set -o pipefail
mkdir -p gpurun_out/prof_pong_big
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong_big -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 8192 --steps 8 --warmup 2 > gpurun_out/prof_pong_big/log.txt 2>&1 && echo PROF_OK
