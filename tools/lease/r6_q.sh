#!/bin/bash
# Round 6, lease Q: the secondary configuration presets re-measured (configs_bench: their README numbers
# are from round 4), then two PMC passes over the 16-wave forward on s2d observations vs the frame ring.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u benchmarks/configs_bench.py --presets cartpole-reinforce-baseline lunarlander-reinforce-baseline \
    halfcheetah-ppo pong-a2c --steps 5 --warmup 2 > gpurun_out/r6q_configs.jsonl 2> gpurun_out/r6q_configs.err || exit $?
cut -c1-300 gpurun_out/r6q_configs.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_ring1 gpurun_out/pmc_ring2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  --kernel-trace --output-format csv -d gpurun_out/pmc_ring1 -o run -- python3 tools/cnn_kbench.py --which fwd16,fwd16_ring --iters 2 \
  > gpurun_out/pmc_ring1/log.txt 2>&1 && echo PASS1_OK && \
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES \
  --kernel-trace --output-format csv -d gpurun_out/pmc_ring2 -o run -- python3 tools/cnn_kbench.py --which fwd16,fwd16_ring --iters 2 \
  > gpurun_out/pmc_ring2/log.txt 2>&1 && echo PASS2_OK
python3 tools/pmc_show.py gpurun_out/pmc_ring1 conv_stack16 && python3 tools/pmc_show.py gpurun_out/pmc_ring2 conv_stack16
rm -f gpurun_out/pmc_ring*/run_kernel_trace.csv
exit 0
