#!/bin/bash
# Round 5, lease P: persistent fc GEMMs at the sizes where they measured faster (fc forward at
# >= 4,096 rows, fc weight gradient at >= 20,480 rows) -- numerics, then Pong 8,192 envs ABBA
# against RRL_FC_BIG=0 (the 128 x 128 kernels everywhere), and 2,048 envs (unchanged path) once each.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py -k "fc_ or pixel_update" \
  > gpurun_out/r5p_tests.log 2>&1 || { tail -30 gpurun_out/r5p_tests.log; exit 1; }
tail -2 gpurun_out/r5p_tests.log
for run in "8192 A" "8192 B" "8192 B" "8192 A" "8192 A" "8192 B" "2048 A" "2048 B"; do
  set -- $run
  if [ "$2" = A ]; then big=0; else big=; fi
  echo "{\"cfg\": \"$2\", \"envs\": $1}" >> gpurun_out/r5p_pong.jsonl
  RRL_FC_BIG=$big timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r5p_pong.jsonl 2>> gpurun_out/r5p_pong.err || exit $?
done
cat gpurun_out/r5p_pong.jsonl
