# Round 4: confirm the shipped forward (conv3 grid) + conv2-backward grid: CNN tests, kernel
# times, Pong at 2,048 / 8,192 envs twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_gpu.py > gpurun_out/v_cnn_tests.log 2>&1 || { tail -30 gpurun_out/v_cnn_tests.log; exit 1; }
tail -1 gpurun_out/v_cnn_tests.log
timeout -k 10 200 python3 tools/cnn_kbench.py --which fwd,fwd_c3_49px,fwd_phase_a1,bwd3,bwd2,wgrad1_8 --iters 50 > gpurun_out/kb_cnn_v.json 2>&1 && tail -1 gpurun_out/kb_cnn_v.json || exit 1
for r in 1 2; do for n in 2048 8192; do
  timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_v_${n}_r$r.json 2>&1 || exit 1
  echo "$n r$r $(tail -1 gpurun_out/pong_v_${n}_r$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), d.get("ms_per_step"))')"
done; done
