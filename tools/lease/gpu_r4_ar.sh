# Round 4: end-of-session state check: full GPU suite,
# smoke, the default bench line (all phases, reference CPU run skipped)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_ar.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_ar.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" gpurun_out/gpu_tests_ar.log | head -20; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke_ar.log 2>&1 && tail -1 gpurun_out/smoke_ar.log || { tail -20 gpurun_out/smoke_ar.log; exit 1; }
timeout -k 10 700 python3 bench.py --ref-cpu-seconds 0 > gpurun_out/bench_ar.json 2> gpurun_out/bench_ar.err || { tail -20 gpurun_out/bench_ar.err; exit 1; }
cut -c1-400 gpurun_out/bench_ar.json
