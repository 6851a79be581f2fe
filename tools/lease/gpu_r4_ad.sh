# Round 4: rollout fc split-K cap A/B inside the Pong update (RRL_FC_SPLITS 8 = default, i.e. 4
# splits at 2,048 rows; 2 = two splits, half the partial traffic into the head), ABBA
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for v in A B B A A B B A; do i=$((i+1)); for n in 2048 8192; do
  if [ $v = A ]; then c=8; else c=2; fi
  RRL_FC_SPLITS=$c timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_ad_${n}_$v.$i.json 2>&1 || exit 1
  echo "$n $v(cap $c) run$i $(tail -1 gpurun_out/pong_ad_${n}_$v.$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3))')"
done; done
mkdir -p gpurun_out/prof_ad
RRL_FC_SPLITS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ad -o run -- python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 30 --warmup 3 > gpurun_out/prof_ad/log.txt 2>&1 && echo PROF_OK
