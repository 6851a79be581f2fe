#!/bin/bash
# Round 5, lease C: persistent-loop skeleton timing, the GPU suite, the fan-in bench against the
# GPU learner, then the bench line.  rc 1 (failed test) continues; any other failure stops.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 120 ./tools/value_loop_skeleton 17665 80 > gpurun_out/r5c_skeleton.json 2> gpurun_out/r5c_skeleton.err || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
    > gpurun_out/r5c_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5c_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u benchmarks/fanin_bench.py --agents 16 64 --transports zmq zmq-ref grpc --seconds 10 \
    --out gpurun_out/r5c_fanin.jsonl > gpurun_out/r5c_fanin.log 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/fanin_bench.py --agents 16 --transports zmq grpc --seconds 8 --paced 25 50 100 \
    --traj-size 10 --out gpurun_out/r5c_fanin.jsonl >> gpurun_out/r5c_fanin.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5c_bench.json 2> gpurun_out/r5c_bench.err || exit $?
exit $rc
