# conv3 backward as 2 x CUs workgroups held to ONE per CU (RRL_CNN_BWD3_WGS=2 + RRL_CNN_BWD3_LDS_KB=82):
# the dispatcher places the second round where CUs are free (the side stream's fc GEMM holds some
# at conv3's start); static image sets, same result for any placement. ABBA on one box.
set -o pipefail
mkdir -p gpurun_out/c3pad
o=gpurun_out/r6z_c3pad_ab.jsonl
run() {  # $1 = label, $2 = envs, rest = env assignments
  local lab=$1 envs=$2; shift 2
  env "$@" timeout -k 10 120 python benchmarks/pong_a2c_bench.py --num-envs $envs --steps 20 --warmup 3 \
    | sed "s/^{/{\"v\": \"$lab\", \"envs\": $envs, /" >> $o
}
for envs in 2048 8192; do
  for k in a b b a a b b a; do
    if [ $k = a ]; then run base $envs RRL_X=0 || exit $?; else run pad2 $envs RRL_CNN_BWD3_WGS=2 RRL_CNN_BWD3_LDS_KB=82 || exit $?; fi
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RRL_CNN_BWD3_WGS=2 RRL_CNN_BWD3_LDS_KB=82 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3pad -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 12 --warmup 2 > gpurun_out/c3pad/log.txt 2>&1 && echo C3PAD_OK
