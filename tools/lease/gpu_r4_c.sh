# NOTE: a record of the run behind its profiles/r4_* files; the A/B options it passes (the pair conv split
# fwd_split / fwd_pair, RRL_FC_HEAD, RRL_FH_STAGES, RRL_CONV21, bwd21) were removed after measuring slower.
# Round 4: PMC of the conv stack forward (per-layer vs pair split), flagship kernel profile,
# TTT value-loop levers (slab-count sweep, stamps, epoch profile)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_cs1 gpurun_out/pmc_cs2 gpurun_out/pmc_cs3 gpurun_out/pmc_cs4 gpurun_out/prof_flagship gpurun_out/prof_ttt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  --kernel-trace --output-format csv -d gpurun_out/pmc_cs1 -o run -- python3 tools/cnn_kbench.py --which fwd,fwd_pair,bwd3,bwd2,wgrad1_8 --iters 2 > gpurun_out/pmc_cs1/log.txt 2>&1 && echo PASS1_OK && \
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_WAVES \
  --kernel-trace --output-format csv -d gpurun_out/pmc_cs2 -o run -- python3 tools/cnn_kbench.py --which fwd,fwd_pair,bwd3,bwd2,wgrad1_8 --iters 2 > gpurun_out/pmc_cs2/log.txt 2>&1 && echo PASS2_OK && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d gpurun_out/pmc_cs3 -o run -- python3 tools/cnn_kbench.py --which fwd,fwd_pair,bwd3,bwd2,wgrad1_8 --iters 2 > gpurun_out/pmc_cs3/log.txt 2>&1 && echo PASS3_OK && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE \
  --kernel-trace --output-format csv -d gpurun_out/pmc_cs4 -o run -- python3 tools/cnn_kbench.py --which fwd,fwd_pair,bwd3,bwd2,wgrad1_8 --iters 2 > gpurun_out/pmc_cs4/log.txt 2>&1 && echo PASS4_OK || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flagship -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-ttt --host-steps 0 --pong-steps 0 --ref-cpu-seconds 0 --phase-steps 0 > gpurun_out/prof_flagship/log.txt 2>&1 || exit 1
grep metric gpurun_out/prof_flagship/log.txt | cut -c1-200
timeout -k 10 200 python3 -u tools/ttt_levers_probe.py > gpurun_out/ttt_levers.jsonl 2> gpurun_out/ttt_levers.err || { tail -20 gpurun_out/ttt_levers.err; exit 1; }
cat gpurun_out/ttt_levers.jsonl
timeout -k 10 120 python3 -u tools/kbench.py grad --B 8192 --iters 50 --stamps > gpurun_out/kb_stamps_8192.json 2>&1 || { tail -20 gpurun_out/kb_stamps_8192.json; exit 1; }
tail -2 gpurun_out/kb_stamps_8192.json | cut -c1-1500
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ttt -o run -- \
  python3 tools/ttt_epoch_probe.py > gpurun_out/prof_ttt/log.txt 2>&1 || exit 1
tail -1 gpurun_out/prof_ttt/log.txt | cut -c1-300
