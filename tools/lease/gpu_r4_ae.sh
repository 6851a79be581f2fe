# Round 4: column_sums + async episode sums tests, then the TTT phases of bench.py twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_episode_sums_gpu.py tests/test_engine_gpu.py > gpurun_out/ae_tests.log 2>&1 || { tail -30 gpurun_out/ae_tests.log; exit 1; }
tail -1 gpurun_out/ae_tests.log
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --ref-cpu-seconds 0 --host-steps 0 --pong-steps 0 --pong-big-envs 0 --phase-steps 0 --ttt-seeds 10 --ttt-ref-seeds 7 > gpurun_out/ttt_ae.r$r.json 2> gpurun_out/ttt_ae.r$r.err || exit 1
  echo "r$r $(tail -1 gpurun_out/ttt_ae.r$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); t=d["time_to_threshold"]; print(d["time_to_threshold_s"], d["time_to_threshold_reference_hparams_s"], t["reference_hparams"].get("per_seed_s"))')"
done
mkdir -p gpurun_out/prof_ae
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ae -o run -- python3 bench.py --steps 2 --warmup 1 --ref-cpu-seconds 0 --host-steps 0 --pong-steps 0 --pong-big-envs 0 --phase-steps 0 --ttt-seeds 2 --ttt-ref-seeds 2 > gpurun_out/prof_ae/log.txt 2>&1 && echo PROF_OK
