# Round 4: the side stream at all (RRL_CNN_SIDE 1, A) vs one stream (0, B), Pong ABBA on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for v in A B B A A B B A; do i=$((i+1)); for n in 2048 8192; do
  if [ $v = A ]; then d=1; else d=0; fi
  RRL_CNN_SIDE=$d timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_ak_${n}_$v.$i.json 2>&1 || exit 1
  echo "$n $v(side $d) run$i $(tail -1 gpurun_out/pong_ak_${n}_$v.$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3))')"
done; done
mkdir -p gpurun_out/prof_ak
RRL_CNN_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ak -o run -- python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/prof_ak/log.txt 2>&1 && echo PROF_OK
