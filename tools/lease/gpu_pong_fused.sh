# Fused conv-stack forward: numerics tests, then the Pong A2C bench fused vs per-layer, and a kernel profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cnn_tests.log 2>&1; rc=$?
tail -3 gpurun_out/cnn_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 20 --warmup 3 > gpurun_out/pong_fused.json 2>&1 || exit $?
RRL_CNN_FUSED=0 timeout -k 10 120 python benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 20 --warmup 3 > gpurun_out/pong_perlayer.json 2>&1 || exit $?
tail -1 gpurun_out/pong_fused.json | cut -c1-200
tail -1 gpurun_out/pong_perlayer.json | cut -c1-200
bash tools/prof_pong.sh
