# Evidence pass: flagship with the value loop captured vs launched eagerly (the multi-rank path
# launches eagerly), and one PMC pass of the shipped value-grad kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_ship
timeout -k 10 300 python bench.py --no-ttt --ref-cpu-seconds 0 > gpurun_out/bench_graph.log 2>&1 && tail -1 gpurun_out/bench_graph.log | cut -c1-300 && \
timeout -k 10 300 python bench.py --no-ttt --ref-cpu-seconds 0 --no-graphs > gpurun_out/bench_eager.log 2>&1 && tail -1 gpurun_out/bench_eager.log | cut -c1-300 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  --kernel-trace --output-format csv -d gpurun_out/pmc_ship -o run -- python3 tools/kbench.py grad --iters 3 > gpurun_out/pmc_ship/log.txt 2>&1 && \
python tools/pmc_show.py gpurun_out/pmc_ship > gpurun_out/pmc_ship_summary.txt && head -3 gpurun_out/pmc_ship_summary.txt | cut -c1-600
