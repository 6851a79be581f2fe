#!/bin/bash
# Round 5, lease H: the GPU suite with the 16-wave forward as the default, the full bench line,
# then PMC passes over the 8- and 16-wave forwards.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
    > gpurun_out/r5h_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5h_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/r5h_bench.json 2> gpurun_out/r5h_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_h1 gpurun_out/pmc_h2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  --kernel-trace --output-format csv -d gpurun_out/pmc_h1 -o run -- python3 tools/cnn_kbench.py --which fwd8,fwd16 --iters 2 > gpurun_out/pmc_h1/log.txt 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_WAVES \
  --kernel-trace --output-format csv -d gpurun_out/pmc_h2 -o run -- python3 tools/cnn_kbench.py --which fwd8,fwd16 --iters 2 > gpurun_out/pmc_h2/log.txt 2>&1 || exit $?
exit $rc
