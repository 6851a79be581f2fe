# value-grad kernel: numerics tests, then timing of the scheduling variants (interleaved, one process).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_value_grad_gpu.py tests/test_kernels_gpu.py tests/test_actor_learner_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/vg_tests.log 2>&1; rc=$?; tail -2 gpurun_out/vg_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do timeout -k 10 120 python tools/kbench.py grad --iters 30 --tunes 0,1,2,0 || exit 1; done > gpurun_out/vg_tune.jsonl 2>&1
cat gpurun_out/vg_tune.jsonl | grep value
