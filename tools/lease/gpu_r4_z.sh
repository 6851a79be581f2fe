# Round 4: forward conv3-grid A/B inside the Pong update, ABBA order (0 = conv3 over its 49
# NOTE: ran against a .so whose rebuild had failed: there layout 0 was the 7 x 9 conv3 grid and 32 the 49-pixel conv3 (profiles/r4_fwd_layouts.txt)
# pixels, 32 = over a 7 x 9 grid), per-variant LDS allocations
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for lay in 32 0 0 32 32 0 0 32; do i=$((i+1)); for n in 2048 8192; do
  RRL_CNN_FWD_LAYOUT=$lay timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_z_${n}_$lay.$i.json 2>&1 || exit 1
  echo "$n layout=$lay run$i $(tail -1 gpurun_out/pong_z_${n}_$lay.$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), d.get("ms_per_step"))')"
done; done
