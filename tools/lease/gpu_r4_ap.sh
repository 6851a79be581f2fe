# Round 4: side stream vs one stream again after the few-split fc sum (RRL_CNN_SIDE 1 A, 0 B), ABBA
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for v in A B B A A B B A; do i=$((i+1)); for n in 2048 8192; do
  if [ $v = A ]; then d=1; else d=0; fi
  RRL_CNN_SIDE=$d timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_ap_${n}_$v.$i.json 2>&1 || exit 1
  echo "$n $v(side $d) run$i $(tail -1 gpurun_out/pong_ap_${n}_$v.$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3))')"
done; done
