# Round 4: Pong side-stream fork after the fc data gradient (A/B, twice), every BASELINE preset
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "side_stream or graph_replay or overlapped" > gpurun_out/cnn_side_tests.log 2>&1; rc=$?
tail -2 gpurun_out/cnn_side_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do for late in 0 1; do
  RRL_CNN_SIDE_LATE=$late timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/pong_late$late.r$r.json 2>&1 || exit 1
  echo "late=$late round $r $(tail -1 gpurun_out/pong_late$late.r$r.json | cut -c1-140)"
done; done
timeout -k 10 900 python3 -u benchmarks/configs_bench.py --steps 5 --warmup 2 > gpurun_out/configs_k.jsonl 2> gpurun_out/configs_k.err || { tail -20 gpurun_out/configs_k.err; exit 1; }
cut -c1-300 gpurun_out/configs_k.jsonl
