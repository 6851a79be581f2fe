#!/bin/bash
# Round 5, lease A: the GPU suite after the learner / engine changes, then the convergence sweeps.
# A failing test (rc 1) does not stop the sweeps; a fault / abort / timeout (any other rc) does.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/r5a_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5a_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u benchmarks/convergence_bench.py --presets pong-a2c --seeds 1 2 3 --max-seconds 40 \
    --every 500 --out gpurun_out/r5a_conv.jsonl > gpurun_out/r5a_conv.log 2>&1 || exit $?
timeout -k 10 100 python -u benchmarks/convergence_bench.py --presets pong-a2c --set lr=7e-4 --max-seconds 40 \
    --every 500 --out gpurun_out/r5a_conv.jsonl >> gpurun_out/r5a_conv.log 2>&1 || exit $?
for mb in 4 16 64; do
    timeout -k 10 100 python -u benchmarks/convergence_bench.py --presets halfcheetah-ppo --set num_minibatches=$mb \
        --max-seconds 45 --every 50 --out gpurun_out/r5a_conv.jsonl >> gpurun_out/r5a_conv.log 2>&1 || exit $?
done
exit $rc
