# Round 4: double-buffered conv3 backward (one barrier per image, direct masked da2 stores)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_pong_d gpurun_out/pmc_c3
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cnn_tests.log 2>&1; rc=$?
tail -3 gpurun_out/cnn_tests.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" gpurun_out/cnn_tests.log | head -20; exit $rc; }
timeout -k 10 120 python -u tools/cnn_kbench.py --which fwd,bwd3,bwd2,wgrad1_8 > gpurun_out/kb_cnn_d.json 2>&1 && tail -1 gpurun_out/kb_cnn_d.json || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  --kernel-trace --output-format csv -d gpurun_out/pmc_c3 -o run -- python3 tools/cnn_kbench.py --which bwd3 --iters 2 > gpurun_out/pmc_c3/log.txt 2>&1 && echo PMC_OK || exit 1
timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 30 --warmup 3 > gpurun_out/pong_2048.json 2>&1 && tail -1 gpurun_out/pong_2048.json | cut -c1-400 || exit 1
timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 8192 --steps 20 --warmup 3 > gpurun_out/pong_8192.json 2>&1 && tail -1 gpurun_out/pong_8192.json | cut -c1-400 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong_d -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/prof_pong_d/log.txt 2>&1 && echo PROF_OK
mkdir -p gpurun_out/prof_ttt_ref
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ttt_ref -o run -- \
  python3 tools/ttt_epoch_probe.py --ref --shape 512 16 > gpurun_out/prof_ttt_ref/log.txt 2>&1 && echo PROF_TTT_OK
