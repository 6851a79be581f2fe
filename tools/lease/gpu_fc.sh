# Pixel model: numerics (the CNN GPU tests), Pong A2C A/B on one switch (AB_VAR, default
# RRL_CNN_SIDE), kernel profile.
set -o pipefail
mkdir -p gpurun_out
AB_VAR=${AB_VAR:-RRL_CNN_SIDE}
timeout -k 10 400 python -u -m pytest tests/test_cnn_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/fc_tests.log 2>&1; rc=$?; tail -3 gpurun_out/fc_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for f in 1 0; do
    env $AB_VAR=$f timeout -k 10 200 python benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 30 --warmup 3 \
      > gpurun_out/pong_ab$f.$i.json 2>gpurun_out/pong_ab$f.err || exit $?
    echo "$AB_VAR=$f run $i: $(tail -1 gpurun_out/pong_ab$f.$i.json | cut -c1-200)"
  done
done
bash tools/prof_pong.sh
