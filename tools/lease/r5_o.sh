#!/bin/bash
# Round 5, lease O: PMC of the fc GEMMs, 128 x 128 per workgroup ("422") vs persistent 256 x 128 ("b"):
# wave-state split and L2 hit / miss (two passes, each its own run).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_fcp1 gpurun_out/pmc_fcp2
export FC_CASES=dgrad_mask,wgrad_tn_s5,fwd_part_s8 FC_ROUNDS=1 FC_VARIANTS=422,b
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d gpurun_out/pmc_fcp1 -o run -- python3 tools/fc_kbench.py > gpurun_out/pmc_fcp1/log.txt 2>&1 || exit 1
python3 tools/pmc_show.py gpurun_out/pmc_fcp1 fc
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d gpurun_out/pmc_fcp2 -o run -- python3 tools/fc_kbench.py > gpurun_out/pmc_fcp2/log.txt 2>&1 || exit 2
python3 tools/pmc_show.py gpurun_out/pmc_fcp2 fc
