#!/bin/bash
# Round 6, lease G: Pong frame ring, third form (first image rows straight from fidx, the rest from
# the LDS table a stage ahead; v_perm interleave): bitwise tests, kernel micro-bench ring vs s2d at
# 2,048 / 8,192 frames (+ the env-major conv1 weight gradient), ABBA, kernel traces of BOTH paths on one box.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_frame_ring_gpu.py -x -q --timeout 240 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r6g_ring_tests.log 2>&1 || { tail -30 gpurun_out/r6g_ring_tests.log; exit 1; }
tail -2 gpurun_out/r6g_ring_tests.log
for fr in 2048 8192; do
  timeout -k 10 200 python -u tools/cnn_kbench.py --which fwd16,fwd16_ring,wgrad1_8,wgrad1_8_ring,wgrad1_8_ring_em --iters 20 --rounds 4 \
      --frames $fr --bwd-frames $((fr * 5)) >> gpurun_out/r6g_kbench.jsonl 2>> gpurun_out/r6g_kbench.err || exit $?
done
cat gpurun_out/r6g_kbench.jsonl
for run in "2048 0" "2048 1" "2048 1" "2048 0" "8192 0" "8192 1" "8192 1" "8192 0"; do
  set -- $run
  echo "{\"frame_ring\": $2, \"envs\": $1}" >> gpurun_out/r6g_pong.jsonl
  RRL_PONG_FRAME_RING=$2 timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r6g_pong.jsonl 2>> gpurun_out/r6g_pong.err || exit $?
done
cut -c1-160 gpurun_out/r6g_pong.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for ring in 0 1; do
  mkdir -p gpurun_out/prof_pong_r6g_$ring
  RRL_PONG_FRAME_RING=$ring timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong_r6g_$ring -o run -- \
    python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 20 --warmup 3 > gpurun_out/prof_pong_r6g_$ring/log.txt 2>&1 || exit $?
done
exit 0
