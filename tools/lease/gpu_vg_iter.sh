# value-grad iteration: numerics, timing (3 rounds), stamps, one PMC pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_it
timeout -k 10 300 python -u -m pytest tests/test_value_grad_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/vg_tests.log 2>&1; rc=$?; tail -2 gpurun_out/vg_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do timeout -k 10 120 python tools/kbench.py grad --iters 30 ${VG_TUNES:+--tunes $VG_TUNES} || exit 1; done > gpurun_out/vg_time.jsonl 2>&1
grep value gpurun_out/vg_time.jsonl
timeout -k 10 120 python tools/kbench.py grad --iters 5 --stamps 2>&1 | grep stamps
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  --kernel-trace --output-format csv -d gpurun_out/pmc_it -o run -- python3 tools/kbench.py grad --iters 3 > gpurun_out/pmc_it/log.txt 2>&1 && echo PMC_OK
