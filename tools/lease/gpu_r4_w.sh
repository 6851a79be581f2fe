# Round 4: forward layout A/B inside the Pong update (RRL_CNN_FWD_LAYOUT 0 = conv3 7x9 grid,
# 32 = conv3 over its 49 pixels), alternated 3x on one box, plus kernel times in both orders
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python3 tools/cnn_kbench.py --which fwd,fwd_c3_49px --iters 100 > gpurun_out/kb_w1.json 2>&1 && tail -1 gpurun_out/kb_w1.json || exit 1
timeout -k 10 200 python3 tools/cnn_kbench.py --which fwd_c3_49px,fwd --iters 100 > gpurun_out/kb_w2.json 2>&1 && tail -1 gpurun_out/kb_w2.json || exit 1
for r in 1 2 3; do for lay in 0 32; do for n in 2048 8192; do
  RRL_CNN_FWD_LAYOUT=$lay timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_w_${n}_$lay.r$r.json 2>&1 || exit 1
  echo "$n layout=$lay r$r $(tail -1 gpurun_out/pong_w_${n}_$lay.r$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), d.get("ms_per_step"))')"
done; done; done
