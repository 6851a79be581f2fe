#!/bin/bash
# Round 5, lease G: the 16-wave forward with its activations copied out through LDS (16-byte
# stores) -- oracle tests, kernel timing, Pong ABBA.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cnn_gpu.py -m gpu -q --timeout 240 --timeout-method thread \
    -k "fused_conv_stack or pixel_update" > gpurun_out/r5g_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5g_gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/cnn_kbench.py --which fwd8,fwd16,fwd16_staged,fwd16_staged_grid3,bwd2,bwd2_16 --rounds 4 --iters 20 \
    > gpurun_out/r5g_kbench.jsonl 2> gpurun_out/r5g_kbench.err || exit $?
timeout -k 10 120 python -u tools/cnn_kbench.py --which fwd8,fwd16,fwd16_staged,fwd16_staged_grid3 --rounds 4 --iters 10 --frames 8192 \
    >> gpurun_out/r5g_kbench.jsonl 2>> gpurun_out/r5g_kbench.err || exit $?
cfg() {
  case $1 in
    A) echo "RRL_CNN_FWD_LAYOUT=128 RRL_CNN_BWD2_VARIANT=0 RRL_CNN_BWD3_VARIANT=0" ;;
    B) echo "RRL_CNN_FWD_LAYOUT=64 RRL_CNN_BWD2_VARIANT=0 RRL_CNN_BWD3_VARIANT=0" ;;
    S) echo "RRL_CNN_FWD_LAYOUT=65 RRL_CNN_BWD2_VARIANT=0 RRL_CNN_BWD3_VARIANT=0" ;;
    E) echo "RRL_CNN_FWD_LAYOUT=65 RRL_CNN_BWD2_VARIANT=3 RRL_CNN_BWD3_VARIANT=0" ;;
  esac
}
for run in "2048 A" "2048 B" "2048 S" "2048 E" "2048 E" "2048 S" "2048 B" "2048 A" "8192 A" "8192 S" "8192 E" "8192 E" "8192 S" "8192 A"; do
  set -- $run
  echo "{\"cfg\": \"$2\", \"envs\": $1}" >> gpurun_out/r5g_pong.jsonl
  env $(cfg $2) timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r5g_pong.jsonl 2>> gpurun_out/r5g_pong.err || exit $?
done
exit 0
