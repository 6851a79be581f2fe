# the fused policy head + env step + render launch at 8,192 envs with the frame ring (round 5
# measured it -0.3 % there before the ring): ABBA vs the separate head / step launches
set -o pipefail
mkdir -p gpurun_out/fh8k
o=gpurun_out/r6z_fh8k_ab.jsonl
run() {  # $1 = RRL_PONG_FUSED_HEAD
  RRL_PONG_FUSED_HEAD=$1 timeout -k 10 120 python benchmarks/pong_a2c_bench.py --num-envs 8192 --steps 20 --warmup 3 \
    | sed "s/^{/{\"fused_head\": $1, /" >> $o
}
for f in 0 1 1 0 0 1 1 0; do run $f || exit $?; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RRL_PONG_FUSED_HEAD=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fh8k -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 8192 --steps 8 --warmup 2 > gpurun_out/fh8k/log.txt 2>&1 && echo FH_OK
