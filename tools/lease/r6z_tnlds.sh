# the fc weight-gradient GEMM (side stream) held to one workgroup per CU (RRL_FC_TN_LDS_KB=84) so
# the conv3 backward's workgroups land beside it at once; at 8,192 envs also the 128 x 128
# kernel instead of the persistent 256 x 128 one (RRL_FC_TN_BIG=0).  ABBA on one box.
set -o pipefail
mkdir -p gpurun_out/tn84
o=gpurun_out/r6z_tnlds_ab.jsonl
run() {  # $1 = label, $2 = envs, rest = env assignments
  local lab=$1 envs=$2; shift 2
  env "$@" timeout -k 10 120 python benchmarks/pong_a2c_bench.py --num-envs $envs --steps 20 --warmup 3 \
    | sed "s/^{/{\"v\": \"$lab\", /" >> $o
}
for k in a b b a a b b a; do
  if [ $k = a ]; then run base 2048 RRL_X=0 || exit $?; else run tn84 2048 RRL_FC_TN_LDS_KB=84 || exit $?; fi
done
for k in a b c c b a; do
  case $k in
    a) run base 8192 RRL_X=0 || exit $? ;;
    b) run tn84_small 8192 RRL_FC_TN_BIG=0 RRL_FC_TN_LDS_KB=84 || exit $? ;;
    c) run small 8192 RRL_FC_TN_BIG=0 || exit $? ;;
  esac
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RRL_FC_TN_LDS_KB=84 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tn84 -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 12 --warmup 2 > gpurun_out/tn84/log.txt 2>&1 && echo TN_OK
