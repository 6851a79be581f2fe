# conv3 backward at 2 resident workgroups per CU (RRL_CNN_BWD3_WGS=2) vs 1: Pong ABBA at 2,048 and
# 8,192 envs, then a kernel trace of each at 2,048
set -o pipefail
mkdir -p gpurun_out/c3w1 gpurun_out/c3w2
o=gpurun_out/r6z_c3wgs_ab.jsonl
run() {  # $1 = wgs, $2 = envs
  RRL_CNN_BWD3_WGS=$1 timeout -k 10 120 python benchmarks/pong_a2c_bench.py --num-envs $2 --steps 20 --warmup 3 \
    | sed "s/^{/{\"wgs\": $1, /" >> $o
}
for envs in 2048 8192; do
  for w in 1 2 2 1 1 2; do run $w $envs || exit $?; done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in 1 2; do
  RRL_CNN_BWD3_WGS=$w timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3w$w -o run -- \
    python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 12 --warmup 2 > gpurun_out/c3w$w/log.txt 2>&1 || exit $?
done
echo C3W_OK
