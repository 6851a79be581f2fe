# Round 4: lagged threshold check A/B (RRL_TTT_LAGGED_CHECK 1 / 0), both TTT measurements of
# bench.py, alternated on one box; the rest of the bench skipped
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_engine_gpu.py tests/test_lagged_threshold_check.py > gpurun_out/s_tests.log 2>&1 || { tail -20 gpurun_out/s_tests.log; exit 1; }
tail -1 gpurun_out/s_tests.log
for r in 1 2; do for lag in 1 0; do
  RRL_TTT_LAGGED_CHECK=$lag timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --ref-cpu-seconds 0 --host-steps 0 --pong-steps 0 --pong-big-envs 0 --phase-steps 0 --ttt-seeds 10 --ttt-ref-seeds 7 > gpurun_out/ttt_s_lag$lag.r$r.json 2> gpurun_out/ttt_s_lag$lag.r$r.err || exit 1
  echo "lag=$lag r$r $(tail -1 gpurun_out/ttt_s_lag$lag.r$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); t=d["time_to_threshold"]; print(d["time_to_threshold_s"], d["time_to_threshold_reference_hparams_s"], t["tuned"].get("per_seed_s"), t["reference_hparams"].get("per_seed_s"), t["reference_hparams"].get("epochs"))')"
done; done
