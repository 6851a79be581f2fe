# Round 4: GPU tests, the forced multi-rank path (captured vs eager, LunarLander epoch kbench), quick bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/forced_collectives_probe.py --check --bench > gpurun_out/forced_probe.json 2> gpurun_out/forced_probe.err || { tail -20 gpurun_out/forced_probe.err; exit 1; }
cat gpurun_out/forced_probe.json
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --host-steps 0 --ref-cpu-seconds 0 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -20 gpurun_out/bench_quick.err; exit 1; }
cut -c1-400 gpurun_out/bench_quick.json
