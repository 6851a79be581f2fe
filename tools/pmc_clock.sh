# Effective clock + matrix-pipe occupancy of the value-gradient kernel (one PMC pass).
# Run from the repo root on the GPU box: bash tools/pmc_clock.sh
set -o pipefail
mkdir -p gpurun_out/pmc_clock
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  --kernel-trace --output-format csv -d gpurun_out/pmc_clock -o run -- python3 tools/kbench.py grad --iters 5 \
  > gpurun_out/pmc_clock/log.txt 2>&1 && echo PMC_OK
