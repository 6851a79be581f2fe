#!/bin/bash
# Round 6, lease R: conv3 / conv2 backward dgrad reads with non-negative constant LDS offsets (ds_read
# immediates instead of a v_add per read) -- numerics tests, then A/B of the two builds of the HIP
# extension (abtmp/ops_old.so = before, ops_new.so = after), swapped between processes.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
SO=relayrl_prototype_amd/_hip_ops.cpython-310-x86_64-linux-gnu.so
cp abtmp/ops_new.so $SO
timeout -k 10 400 python -u -m pytest tests/test_cnn_gpu.py -x -q --timeout 240 --timeout-method thread -k "bwd or backward or grad" \
    -p no:cacheprovider > gpurun_out/r6r_tests.log 2>&1 || { tail -30 gpurun_out/r6r_tests.log; exit 1; }
tail -2 gpurun_out/r6r_tests.log
for v in old new new old old new; do
  cp abtmp/ops_$v.so $SO
  echo "{\"build\": \"$v\"}" >> gpurun_out/r6r_kbench.jsonl
  timeout -k 10 200 python -u tools/cnn_kbench.py --which bwd3,bwd2 --iters 20 --rounds 3 \
      --frames 2048 --bwd-frames 10240 >> gpurun_out/r6r_kbench.jsonl 2>> gpurun_out/r6r_kbench.err || exit $?
done
cat gpurun_out/r6r_kbench.jsonl
for run in "2048 old" "2048 new" "2048 new" "2048 old" "8192 old" "8192 new" "8192 new" "8192 old"; do
  set -- $run
  cp abtmp/ops_$2.so $SO
  echo "{\"build\": \"$2\", \"envs\": $1}" >> gpurun_out/r6r_pong.jsonl
  timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r6r_pong.jsonl 2>> gpurun_out/r6r_pong.err || exit $?
done
cp abtmp/ops_new.so $SO
cut -c1-160 gpurun_out/r6r_pong.jsonl
