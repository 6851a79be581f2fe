# end-of-round evidence: the whole GPU suite, smoke(), the bench line, the flagship kernel table
set -o pipefail
mkdir -p gpurun_out/prof_flag
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r6z_final_gpu_tests.txt 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/r6z_final_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6z_final_smoke.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r6z_final_bench.json 2> gpurun_out/r6z_final_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flag -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-ttt --ref-cpu-seconds 0 --convergence off --phase-steps 0 --host-steps 0 --pong-steps 0 > gpurun_out/prof_flag/log.txt 2>&1 && echo FINAL_OK
