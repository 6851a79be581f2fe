#!/bin/bash
# Round 5, lease N: persistent 256 x 128 fc GEMMs -- numerics (both kernel families) and the
# fc kernel bench (128 x 128 "422" vs persistent "b"), interleaved in one process.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py -k "fc_" \
  > gpurun_out/r5n_fc_tests.log 2>&1 || { tail -30 gpurun_out/r5n_fc_tests.log; exit 1; }
tail -3 gpurun_out/r5n_fc_tests.log
FC_VARIANTS=422,b,bn FC_CASES=fwd_part_s4,fwd_part_s8,fwd8k_part_s2,dgrad_mask,dgrad_mask_direct,dgrad40k_mask,wgrad_tn_s5,wgrad40k_tn_s5 timeout -k 10 300 python -u tools/fc_kbench.py > gpurun_out/r5n_fc_kbench.jsonl 2> gpurun_out/r5n_fc_kbench.err || { tail -20 gpurun_out/r5n_fc_kbench.err; exit 1; }
cat gpurun_out/r5n_fc_kbench.jsonl
