# Round 4: final-state check: Adam loop form, conv1 weight-gradient layout, early side-stream fork: full GPU suite, smoke, Pong 2048 / 8192 with a
# kernel profile, quick bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_pong_n
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_n.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_n.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" gpurun_out/gpu_tests_n.log | head -20; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke_n.log 2>&1 && tail -1 gpurun_out/smoke_n.log || { tail -20 gpurun_out/smoke_n.log; exit 1; }
timeout -k 10 120 python -u tools/cnn_kbench.py --which fwd,bwd3,bwd2,wgrad1_8 > gpurun_out/kb_cnn_n.json 2>&1 && tail -1 gpurun_out/kb_cnn_n.json || exit 1
timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 30 --warmup 3 > gpurun_out/pong_2048_n.json 2>&1 && tail -1 gpurun_out/pong_2048_n.json | cut -c1-200 || exit 1
timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 8192 --steps 20 --warmup 3 > gpurun_out/pong_8192_n.json 2>&1 && tail -1 gpurun_out/pong_8192_n.json | cut -c1-200 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong_n -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/prof_pong_n/log.txt 2>&1 && echo PROF_OK || exit 1
timeout -k 10 600 python3 bench.py --steps 10 --warmup 3 --host-steps 0 --ref-cpu-seconds 0 > gpurun_out/bench_n.json 2> gpurun_out/bench_n.err || { tail -20 gpurun_out/bench_n.err; exit 1; }
cut -c1-300 gpurun_out/bench_n.json
