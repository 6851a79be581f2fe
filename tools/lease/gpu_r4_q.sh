# Round 4: side-stream mode A/B (early = current default, sums = fc GEMMs in sequence on the
# main stream, only the head gradient + split sums forked beside conv3_bwd), alternated on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_gpu.py -k side_stream > gpurun_out/q_side_test.log 2>&1 || { tail -20 gpurun_out/q_side_test.log; exit 1; }
tail -2 gpurun_out/q_side_test.log
for r in 1 2; do for mode in early sums; do
  RRL_CNN_SIDE_MODE=$mode timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/pong_q_2048_$mode.r$r.json 2>&1 || exit 1
  echo "2048 $mode r$r $(tail -1 gpurun_out/pong_q_2048_$mode.r$r.json | cut -c1-140)"
  RRL_CNN_SIDE_MODE=$mode timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 8192 --steps 20 --warmup 3 > gpurun_out/pong_q_8192_$mode.r$r.json 2>&1 || exit 1
  echo "8192 $mode r$r $(tail -1 gpurun_out/pong_q_8192_$mode.r$r.json | cut -c1-140)"
done; done
mkdir -p gpurun_out/prof_pong_q
RRL_CNN_SIDE_MODE=sums timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong_q -o run -- python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/prof_pong_q/log.txt 2>&1 && echo PROF_OK
