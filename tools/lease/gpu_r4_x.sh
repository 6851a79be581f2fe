# Round 4: conv2-backward dgrad grid A/B inside the Pong update (RRL_CNN_BWD2_VARIANT 0 = 10 x 12
# NOTE: ran against a .so whose rebuild had failed: variant 2 launched the staged-epilogue kernel (profiles/r4_bwd2_grid_ab.txt)
# grid, 2 = 7 tiles), alternated 3x on one box; kernel times over 4 alternating-order rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_gpu.py > gpurun_out/x_cnn_tests.log 2>&1 || { tail -30 gpurun_out/x_cnn_tests.log; exit 1; }
tail -1 gpurun_out/x_cnn_tests.log
timeout -k 10 300 python3 tools/cnn_kbench.py --which fwd,fwd_c3_grid,fwd_phase_a1,bwd3,bwd2,bwd2_7tiles,wgrad1_8 --iters 50 --rounds 4 > gpurun_out/kb_x.json 2>&1 && tail -1 gpurun_out/kb_x.json || exit 1
for r in 1 2 3; do for v in 0 2; do for n in 2048 8192; do
  RRL_CNN_BWD2_VARIANT=$v timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_x_${n}_$v.r$r.json 2>&1 || exit 1
  echo "$n bwd2=$v r$r $(tail -1 gpurun_out/pong_x_${n}_$v.r$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), d.get("ms_per_step"))')"
done; done; done
