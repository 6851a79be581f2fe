# Round 4: forward conv3-grid A/B inside the Pong update with per-variant LDS allocations
# NOTE: ran against a .so whose rebuild had failed: there layout 0 was the 7 x 9 conv3 grid and 32 the 49-pixel conv3 (profiles/r4_fwd_layouts.txt)
# (RRL_CNN_FWD_LAYOUT 0 = conv3 over its 49 pixels, 32 = over a 7 x 9 grid), alternated 3x
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 tools/cnn_kbench.py --which fwd,fwd_c3_grid --iters 50 --rounds 6 > gpurun_out/kb_y.json 2>&1 && tail -1 gpurun_out/kb_y.json || exit 1
for r in 1 2 3; do for lay in 0 32; do for n in 2048 8192; do
  RRL_CNN_FWD_LAYOUT=$lay timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_y_${n}_$lay.r$r.json 2>&1 || exit 1
  echo "$n layout=$lay r$r $(tail -1 gpurun_out/pong_y_${n}_$lay.r$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), d.get("ms_per_step"))')"
done; done; done
