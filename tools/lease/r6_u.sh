#!/bin/bash
# Round 6, lease U: the shipped Pong update's kernel table at 2,048 envs (frame ring on), and PMC passes
# over the conv backward kernels (conv3_bwd, conv2_bwd, conv1 weight gradient on the ring, env-major).
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/prof_pong_u gpurun_out/pmc_bwd1 gpurun_out/pmc_bwd2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong_u -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 20 --warmup 3 > gpurun_out/prof_pong_u/log.txt 2>&1 && echo PROF_OK && \
python3 tools/prof_summary.py gpurun_out/prof_pong_u/run_kernel_stats.csv > gpurun_out/r6u_pong_kernels.txt 2>&1; \
rm -f gpurun_out/prof_pong_u/run_kernel_trace.csv
W="bwd3,bwd2,wgrad1_8_ring"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  --kernel-trace --output-format csv -d gpurun_out/pmc_bwd1 -o run -- python3 tools/cnn_kbench.py --which $W --iters 3 > gpurun_out/pmc_bwd1/log.txt 2>&1 && echo PASS1_OK && \
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES \
  --kernel-trace --output-format csv -d gpurun_out/pmc_bwd2 -o run -- python3 tools/cnn_kbench.py --which $W --iters 3 > gpurun_out/pmc_bwd2/log.txt 2>&1 && echo PASS2_OK
rm -f gpurun_out/pmc_bwd*/run_kernel_trace.csv
head -25 gpurun_out/r6u_pong_kernels.txt
exit 0
