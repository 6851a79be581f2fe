# Pong update timelines (kernel start/end) at 2,048 and 8,192 envs, for the overlap analysis
set -o pipefail
mkdir -p gpurun_out/tl2048 gpurun_out/tl8192
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl2048 -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 12 --warmup 2 > gpurun_out/tl2048/log.txt 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl8192 -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 8192 --steps 8 --warmup 2 > gpurun_out/tl8192/log.txt 2>&1 && echo TL_OK
