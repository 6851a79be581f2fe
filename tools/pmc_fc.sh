# PMC pass over tools/fc_kbench.py (fc.hip GEMMs at the Pong shapes): MFMA busy, LDS bank
# conflicts vs LDS activity (the source-side XOR swizzles), wave waits.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_fc1
FC_VARIANTS=422 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS \
  --kernel-trace --output-format csv -d gpurun_out/pmc_fc1 -o run -- python3 tools/fc_kbench.py > gpurun_out/pmc_fc1/log.txt 2>&1 && echo PASS1_OK
