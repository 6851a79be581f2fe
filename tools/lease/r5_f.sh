#!/bin/bash
# Round 5, lease F: the GPU suite (with the 16-wave conv-stack forward's oracle tests), its kernel
# timing against the 8-wave kernel, a Pong ABBA at 2,048 and 8,192 envs, the reference-wire fan-in
# rows, then the flagship kernel profile.  rc 1 (failed test) continues; any other failure stops.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
    > gpurun_out/r5f_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5f_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/cnn_kbench.py --which fwd8,fwd16,fwd16_phase,fwd16_grid3,fwd16_both,bwd2,bwd2_16,bwd3,bwd3_16 --rounds 4 --iters 20 \
    > gpurun_out/r5f_kbench.jsonl 2> gpurun_out/r5f_kbench.err || exit $?
timeout -k 10 120 python -u tools/cnn_kbench.py --which fwd8,fwd16,fwd16_phase,fwd16_grid3,fwd16_both --rounds 4 --iters 10 --frames 8192 \
    >> gpurun_out/r5f_kbench.jsonl 2>> gpurun_out/r5f_kbench.err || exit $?
# Pong configs: A = 8-wave kernels, B = 16-wave forward, C = + 16-wave conv2 / conv3 backward,
# D = C + conv2_bwd / conv1_wgrad8 in two chunks
cfg() {
  case $1 in
    A) echo "RRL_CNN_FWD_LAYOUT=128 RRL_CNN_BWD2_VARIANT=0 RRL_CNN_BWD3_VARIANT=0 RRL_CNN_BWD21_CHUNKS=1" ;;
    B) echo "RRL_CNN_FWD_LAYOUT=64 RRL_CNN_BWD2_VARIANT=0 RRL_CNN_BWD3_VARIANT=0 RRL_CNN_BWD21_CHUNKS=1" ;;
    C) echo "RRL_CNN_FWD_LAYOUT=64 RRL_CNN_BWD2_VARIANT=3 RRL_CNN_BWD3_VARIANT=1 RRL_CNN_BWD21_CHUNKS=1" ;;
    D) echo "RRL_CNN_FWD_LAYOUT=64 RRL_CNN_BWD2_VARIANT=3 RRL_CNN_BWD3_VARIANT=1 RRL_CNN_BWD21_CHUNKS=2" ;;
  esac
}
for run in "2048 A" "2048 B" "2048 C" "2048 D" "2048 D" "2048 C" "2048 B" "2048 A" "8192 A" "8192 C" "8192 D" "8192 A"; do
  set -- $run
  echo "{\"cfg\": \"$2\", \"envs\": $1}" >> gpurun_out/r5f_pong.jsonl
  env $(cfg $2) timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r5f_pong.jsonl 2>> gpurun_out/r5f_pong.err || exit $?
done
timeout -k 10 400 python -u benchmarks/fanin_bench.py --agents 16 64 --transports zmq-ref --seconds 10 \
    --out gpurun_out/r5f_fanin.jsonl > gpurun_out/r5f_fanin.log 2>&1 || exit $?
mkdir -p gpurun_out/prof_flagship_r5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flagship_r5 -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-ttt --host-steps 0 --pong-steps 0 --pong-big-envs 0 --ref-cpu-seconds 0 \
  --convergence off --actor-learner off --phase-steps 0 > gpurun_out/prof_flagship_r5/log.txt 2>&1 || exit $?
mkdir -p gpurun_out/prof_pong_r5
env $(cfg C) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong_r5 -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/prof_pong_r5/log.txt 2>&1 || exit $?
exit $rc
