# after the conv3 LDS knob (default launch unchanged) (default launch unchanged): the whole GPU suite, smoke and the bench line again
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r6z_final3_gpu_tests.txt 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/r6z_final3_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6z_final3_smoke.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r6z_final3_bench.json 2> gpurun_out/r6z_final3_bench.err && echo FINAL2_OK
