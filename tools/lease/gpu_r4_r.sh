# Round 4: side-stream mode A/B, 4 alternations of early / sums / late at 2048 and 8192 envs, one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3 4; do for mode in early sums late; do for n in 2048 8192; do
  RRL_CNN_SIDE_MODE=$mode timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_r_${n}_$mode.r$r.json 2>&1 || exit 1
  echo "$n $mode r$r $(tail -1 gpurun_out/pong_r_${n}_$mode.r$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), d.get("ms_per_step"))')"
done; done; done
