#!/bin/bash
# Round 5, lease AP: the final state after the Adam prefetch and the opt-in head variants -- GPU suite, smoke(), the bench line as the driver runs it.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
    > gpurun_out/r5ap_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5ap_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5ap_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5ap_bench.json 2> gpurun_out/r5ap_bench.err || exit $?
exit $rc
