# NOTE: a record of profiles/r4_head_rows_ab.txt; the RRL_HEAD_ROWS knob it sets was removed after the A/B.
# Round 4: rollout head rows per wave (1 / 2 / 4), alternated twice on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for rows in 1 2 4; do
  RRL_HEAD_ROWS=$rows timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/pong_o_rows$rows.r$r.json 2>&1 || exit 1
  echo "rows=$rows r$r $(tail -1 gpurun_out/pong_o_rows$rows.r$r.json | cut -c60-110)"
done; done
