# Round 4: the current tree vs the session-start commit 1b58077 (built in _old/), Pong ABBA on
# one box -- a regression check of the day's kernel / model changes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for v in A B B A A B B A; do i=$((i+1)); for n in 2048 8192; do
  if [ $v = A ]; then d=.; else d=_old; fi
  (cd $d && PYTHONPATH=. timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5) > gpurun_out/pong_ab_${n}_$v.$i.json 2>&1 || exit 1
  echo "$n $v($d) run$i $(tail -1 gpurun_out/pong_ab_${n}_$v.$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3))')"
done; done
