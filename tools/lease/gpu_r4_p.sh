# Round 4: PMC of the current conv kernels (after the double buffering / layouts)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_p1 gpurun_out/pmc_p2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  --kernel-trace --output-format csv -d gpurun_out/pmc_p1 -o run -- python3 tools/cnn_kbench.py --which fwd,bwd3,bwd2,wgrad1_8 --iters 2 > gpurun_out/pmc_p1/log.txt 2>&1 && echo PASS1_OK && \
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_WAVES \
  --kernel-trace --output-format csv -d gpurun_out/pmc_p2 -o run -- python3 tools/cnn_kbench.py --which fwd,bwd3,bwd2,wgrad1_8 --iters 2 > gpurun_out/pmc_p2/log.txt 2>&1 && echo PASS2_OK
