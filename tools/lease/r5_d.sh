#!/bin/bash
# Round 5, lease D: the persistent-loop skeleton (efficient reduce phase), the new GPU tests,
# the zmq-ref fan-in rows with the native pickle decoder, a sync probe, profiles.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 120 ./tools/value_loop_skeleton 17665 80 > gpurun_out/r5d_skeleton.json 2> gpurun_out/r5d_skeleton.err || exit $?
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_capture_collectives_gpu.py \
    tests/test_capture_robustness_gpu.py tests/test_forced_collectives_gpu.py tests/test_kernels_fuzz_gpu.py \
    tests/test_bench_gpu.py > gpurun_out/r5d_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5d_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 200 python -u tools/forced_collectives_probe.py --syncs \
    > gpurun_out/r5d_syncs.json 2> gpurun_out/r5d_syncs.err || exit $?
timeout -k 10 400 python -u benchmarks/fanin_bench.py --agents 16 64 --transports zmq-ref --seconds 10 \
    --out gpurun_out/r5d_fanin.jsonl > gpurun_out/r5d_fanin.log 2>&1 || exit $?
exit $rc
