# Round 4: deferred policy loss-slab sum + column_sums episode sums: full GPU suite, then the
# TTT phases of bench.py twice and a kernel profile of them
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_af.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_af.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" gpurun_out/gpu_tests_af.log | head -20; exit $rc; }
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --ref-cpu-seconds 0 --host-steps 0 --pong-steps 0 --pong-big-envs 0 --phase-steps 0 --ttt-seeds 10 --ttt-ref-seeds 7 > gpurun_out/ttt_af.r$r.json 2> gpurun_out/ttt_af.r$r.err || exit 1
  echo "r$r $(tail -1 gpurun_out/ttt_af.r$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); t=d["time_to_threshold"]; print(d["time_to_threshold_s"], d["time_to_threshold_reference_hparams_s"], t["reference_hparams"].get("per_seed_s"))')"
done
mkdir -p gpurun_out/prof_af
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_af -o run -- python3 bench.py --steps 2 --warmup 1 --ref-cpu-seconds 0 --host-steps 0 --pong-steps 0 --pong-big-envs 0 --phase-steps 0 --ttt-seeds 2 --ttt-ref-seeds 2 > gpurun_out/prof_af/log.txt 2>&1 && echo PROF_OK
