# NOTE: a record of the run behind its profiles/r4_* files; the A/B options it passes (the pair conv split
# fwd_split / fwd_pair, RRL_FC_HEAD, RRL_FH_STAGES, RRL_CONV21, bwd21) were removed after measuring slower.
# Round 4: kernel changes (binary factored policy head, value forward split, device row count,
# conv stack co-tile pair split), full GPU suite, quick bench, Pong profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_value_grad_gpu.py tests/test_cnn_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/kern_tests.log 2>&1; rc=$?
tail -3 gpurun_out/kern_tests.log
[ $rc -eq 0 ] || { grep -n "Error\|assert" gpurun_out/kern_tests.log | head -20; exit $rc; }
timeout -k 10 120 python -u tools/kbench.py pgrad --B 2097152 > gpurun_out/kb_pgrad.json 2>&1 && cat gpurun_out/kb_pgrad.json
timeout -k 10 120 python -u tools/kbench.py fwd --B 2129920 > gpurun_out/kb_fwd.json 2>&1 && cat gpurun_out/kb_fwd.json
timeout -k 10 120 python -u tools/cnn_kbench.py --which fwd,fwd_split,bwd3,bwd2,wgrad1_8 > gpurun_out/kb_cnn.json 2>&1 && cat gpurun_out/kb_cnn.json
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" gpurun_out/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --host-steps 0 --ref-cpu-seconds 0 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -20 gpurun_out/bench_quick.err; exit 1; }
cut -c1-300 gpurun_out/bench_quick.json
mkdir -p gpurun_out/prof_pong
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/prof_pong/log.txt 2>&1 && echo PROF_OK
