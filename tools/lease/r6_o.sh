#!/bin/bash
# Round 6, lease O: ring forward with the bank-conflict-free unit mapping (half-waves take the two row pairs
# of 32 positions) vs the s2d path -- ring tests (bitwise), kernel micro-bench, ABBA.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_frame_ring_gpu.py -x -q --timeout 240 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r6o_ring_tests.log 2>&1 || { tail -30 gpurun_out/r6o_ring_tests.log; exit 1; }
tail -2 gpurun_out/r6o_ring_tests.log
for fr in 2048 8192; do
  timeout -k 10 200 python -u tools/cnn_kbench.py --which fwd16,fwd16_ring --iters 20 --rounds 6 \
      --frames $fr --bwd-frames $((fr * 5)) >> gpurun_out/r6o_kbench.jsonl 2>> gpurun_out/r6o_kbench.err || exit $?
done
cat gpurun_out/r6o_kbench.jsonl
for run in "2048 0" "2048 1" "2048 1" "2048 0" "8192 0" "8192 1" "8192 1" "8192 0"; do
  set -- $run
  echo "{\"frame_ring\": $2, \"envs\": $1}" >> gpurun_out/r6o_pong.jsonl
  RRL_PONG_FRAME_RING=$2 timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r6o_pong.jsonl 2>> gpurun_out/r6o_pong.err || exit $?
done
cut -c1-160 gpurun_out/r6o_pong.jsonl
