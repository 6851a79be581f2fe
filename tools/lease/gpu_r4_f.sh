# NOTE: a record of the run behind its profiles/r4_* files; the A/B options it passes (the pair conv split
# fwd_split / fwd_pair, RRL_FC_HEAD, RRL_FH_STAGES, RRL_CONV21, bwd21) were removed after measuring slower.
# Round 4: padding-only LDS layouts of the conv backward kernels, 28-wide frame rows in the fused
# forward, the rollout fc + head in one full-K GEMM launch (A/B against the split-K head), conv2 backward +
# conv1 weight gradient fused (A/B), Pong render with row flags / LDS state
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_pong_f
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cnn_tests.log 2>&1; rc=$?
tail -3 gpurun_out/cnn_tests.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" gpurun_out/cnn_tests.log | head -20; exit $rc; }
timeout -k 10 120 python -u tools/cnn_kbench.py --which fwd,bwd3,bwd2,wgrad1_8,bwd21 > gpurun_out/kb_cnn_f.json 2>&1 && tail -1 gpurun_out/kb_cnn_f.json || exit 1
RRL_CONV21=0 timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 30 --warmup 3 > gpurun_out/pong_2048_c21off.json 2>&1 && echo "conv21=0" && tail -1 gpurun_out/pong_2048_c21off.json | cut -c1-160 || exit 1
for fh in 1 0; do
  RRL_FC_HEAD=$fh timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 30 --warmup 3 > gpurun_out/pong_2048_fh$fh.json 2>&1 && echo "fc_head=$fh" && tail -1 gpurun_out/pong_2048_fh$fh.json | cut -c1-160 || exit 1
done
RRL_FH_STAGES=3 timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 30 --warmup 3 > gpurun_out/pong_2048_fhs3.json 2>&1 && echo "fc_head stages 3" && tail -1 gpurun_out/pong_2048_fhs3.json | cut -c1-160 || exit 1
timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 8192 --steps 20 --warmup 3 > gpurun_out/pong_8192_f.json 2>&1 && tail -1 gpurun_out/pong_8192_f.json | cut -c1-160 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong_f -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/prof_pong_f/log.txt 2>&1 && echo PROF_OK
