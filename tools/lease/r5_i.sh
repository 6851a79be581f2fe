#!/bin/bash
# Round 5, lease I: the GPU suite after the test fix and the decoder changes, the reference-wire
# fan-in rows with the faster decoder, then the full bench line.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
    > gpurun_out/r5i_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5i_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u benchmarks/fanin_bench.py --agents 16 64 --transports zmq-ref --seconds 10 \
    --out gpurun_out/r5i_fanin.jsonl > gpurun_out/r5i_fanin.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r5i_bench.json 2> gpurun_out/r5i_bench.err || exit $?
exit $rc
