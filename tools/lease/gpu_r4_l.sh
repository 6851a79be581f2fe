# Round 4: conv1 weight-gradient LDS layout; Pong with the late side-stream fork default
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cnn_tests_l.log 2>&1; rc=$?
tail -2 gpurun_out/cnn_tests_l.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" gpurun_out/cnn_tests_l.log | head -20; exit $rc; }
timeout -k 10 120 python -u tools/cnn_kbench.py --which fwd,bwd3,bwd2,wgrad1_8 > gpurun_out/kb_cnn_l.json 2>&1 && tail -1 gpurun_out/kb_cnn_l.json || exit 1
for r in 1 2; do
timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/pong_2048_l$r.json 2>&1 && tail -1 gpurun_out/pong_2048_l$r.json | cut -c1-160 || exit 1
done
timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 8192 --steps 20 --warmup 3 > gpurun_out/pong_8192_l.json 2>&1 && tail -1 gpurun_out/pong_8192_l.json | cut -c1-160 || exit 1
