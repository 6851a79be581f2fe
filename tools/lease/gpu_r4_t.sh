# Round 4: fused forward with a1 as phase images (48-element rows, 9 x 10 conv2 grid), a 7 x 9
# conv3 grid, and the conv2 backward dgrad on a 10 x 12 grid -- numerics, kernel time, Pong, a PMC pass; then the lagged-check TTT A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_gpu.py > gpurun_out/t_cnn_tests.log 2>&1 || { tail -30 gpurun_out/t_cnn_tests.log; exit 1; }
tail -1 gpurun_out/t_cnn_tests.log
timeout -k 10 200 python3 tools/cnn_kbench.py > gpurun_out/kb_cnn_t.json 2>&1 && tail -1 gpurun_out/kb_cnn_t.json || exit 1
for n in 2048 8192; do
  timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_t_$n.json 2>&1 || exit 1
  echo "$n $(tail -1 gpurun_out/pong_t_$n.json | cut -c1-150)"
done
mkdir -p gpurun_out/pmc_t1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  --kernel-trace --output-format csv -d gpurun_out/pmc_t1 -o run -- python3 tools/cnn_kbench.py --which fwd,bwd2 --iters 2 > gpurun_out/pmc_t1/log.txt 2>&1 && echo PMC_OK || exit 1
bash tools/lease/gpu_r4_s.sh
