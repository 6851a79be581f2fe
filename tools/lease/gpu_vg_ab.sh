# A/B of value_grad scheduling variants (interleaved in one process) + numerics.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_value_grad_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/vg_ab_tests.log 2>&1; rc=$?; tail -1 gpurun_out/vg_ab_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do timeout -k 10 120 python tools/kbench.py grad --iters 30 --tunes ${VG_TUNES:-0,4,0,4} || exit 1; done 2>&1 | grep value
timeout -k 10 200 python tools/kbench.py pgauss --iters 10 2>&1 | grep gauss
