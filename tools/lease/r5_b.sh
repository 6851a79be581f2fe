#!/bin/bash
# Round 5, lease B: the grad-fuzz failure probe, the rest of the GPU suite, longer convergence runs.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 180 python -u tools/grad_fuzz_probe.py --sweep > gpurun_out/r5b_probe.jsonl 2> gpurun_out/r5b_probe.err || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
    --deselect tests/test_kernels_fuzz_gpu.py::test_grad_fuzz > gpurun_out/r5b_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5b_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 100 python -u benchmarks/convergence_bench.py --presets pong-a2c --max-seconds 40 \
    --every 500 --out gpurun_out/r5b_conv.jsonl > gpurun_out/r5b_conv.log 2>&1 || exit $?
timeout -k 10 100 python -u benchmarks/convergence_bench.py --presets halfcheetah-ppo --max-seconds 60 \
    --every 20 --out gpurun_out/r5b_conv.jsonl >> gpurun_out/r5b_conv.log 2>&1 || exit $?
exit $rc
