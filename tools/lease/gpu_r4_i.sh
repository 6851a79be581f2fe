# Round 4: the Adam loop form of the step counter (one arrival ticket per value loop)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_ttt_ref_i
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_value_grad_gpu.py tests/test_forced_collectives_gpu.py tests/test_engine_gpu.py -q -x --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/kern_tests_i.log 2>&1; rc=$?
tail -3 gpurun_out/kern_tests_i.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" gpurun_out/kern_tests_i.log | head -20; exit $rc; }
timeout -k 10 200 python3 -u tools/ttt_levers_probe.py --caps 0 > gpurun_out/ttt_levers_i.jsonl 2> gpurun_out/ttt_levers_i.err || { tail -20 gpurun_out/ttt_levers_i.err; exit 1; }
cat gpurun_out/ttt_levers_i.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ttt_ref_i -o run -- \
  python3 tools/ttt_epoch_probe.py --ref --shape 512 16 > gpurun_out/prof_ttt_ref_i/log.txt 2>&1 && echo PROF_TTT_OK || exit 1
timeout -k 10 600 python3 bench.py --steps 10 --warmup 3 --host-steps 0 --ref-cpu-seconds 0 --pong-steps 0 > gpurun_out/bench_i.json 2> gpurun_out/bench_i.err || { tail -20 gpurun_out/bench_i.err; exit 1; }
cut -c1-300 gpurun_out/bench_i.json
python3 -c "import json; d=json.loads(open('gpurun_out/bench_i.json').read().splitlines()[-1]); print({k: d.get(k) for k in ('time_to_threshold_s', 'time_to_threshold_reference_hparams_s')})"
