#!/bin/bash
# Round 5, lease R: the policy head fused into the Pong env-step launch -- bitwise tests
# (fused vs head-then-step, whole pixel updates), then Pong ABBA (RRL_PONG_FUSED_HEAD=0 vs 1).
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py tests/test_capture_robustness_gpu.py \
  -k "fused_head or pixel_update or fused_render or capture or fc_head" > gpurun_out/r5r_tests.log 2>&1 || { tail -40 gpurun_out/r5r_tests.log; exit 1; }
tail -2 gpurun_out/r5r_tests.log
rm -f gpurun_out/r5r_pong.jsonl
for run in "2048 A" "2048 B" "2048 B" "2048 A" "2048 A" "2048 B" "8192 A" "8192 B" "8192 B" "8192 A"; do
  set -- $run
  if [ "$2" = A ]; then fh=0; else fh=1; fi
  echo "{\"cfg\": \"$2\", \"envs\": $1}" >> gpurun_out/r5r_pong.jsonl
  RRL_PONG_FUSED_HEAD=$fh timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r5r_pong.jsonl 2>> gpurun_out/r5r_pong.err || exit $?
done
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open("gpurun_out/r5r_pong.jsonl")]
for c,r in zip(rows[::2],rows[1::2]): print(c["cfg"], c["envs"], round(r["value"]/1e6,3))
PY
