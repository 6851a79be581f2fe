# Round 4: last full GPU suite + smoke of the session
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_at.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_at.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" gpurun_out/gpu_tests_at.log | head -20; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke_at.log 2>&1 && tail -1 gpurun_out/smoke_at.log
