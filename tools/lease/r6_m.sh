#!/bin/bash
# Round 6, lease M: ring forward with 16-byte loads on lane pairs + a DPP row swap (probe 192) vs the 8-byte
# row pieces -- ring tests (bitwise), kernel micro-bench.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_frame_ring_gpu.py -x -q --timeout 240 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r6m_ring_tests.log 2>&1 || { tail -30 gpurun_out/r6m_ring_tests.log; exit 1; }
tail -2 gpurun_out/r6m_ring_tests.log
for fr in 2048 8192; do
  timeout -k 10 200 python -u tools/cnn_kbench.py --which fwd16,fwd16_ring,fwd16_ring16 --iters 20 --rounds 4 \
      --frames $fr --bwd-frames $((fr * 5)) >> gpurun_out/r6m_kbench.jsonl 2>> gpurun_out/r6m_kbench.err || exit $?
done
cat gpurun_out/r6m_kbench.jsonl
