#!/bin/bash
# Round 5, lease V: the a3 ReLU mask as bits (written by the 16-wave forward, read by the fc data
# gradient) -- tests, then Pong ABBA (RRL_FC_MASK_BITS=0 vs 1) at 2,048 and 8,192 envs.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py tests/test_capture_robustness_gpu.py \
  -k "relu_bits or mask_bits or fc_ or pixel_update or fused_render or fused_head or fused_conv or capture or layout" > gpurun_out/r5v_tests.log 2>&1 || { tail -40 gpurun_out/r5v_tests.log; exit 1; }
tail -2 gpurun_out/r5v_tests.log
rm -f gpurun_out/r5v_pong.jsonl
for run in "2048 A" "2048 B" "2048 B" "2048 A" "2048 A" "2048 B" "8192 A" "8192 B" "8192 B" "8192 A" "8192 A" "8192 B"; do
  set -- $run
  if [ "$2" = A ]; then mb=0; else mb=1; fi
  echo "{\"cfg\": \"$2\", \"envs\": $1}" >> gpurun_out/r5v_pong.jsonl
  RRL_FC_MASK_BITS=$mb timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r5v_pong.jsonl 2>> gpurun_out/r5v_pong.err || exit $?
done
python3 - <<'PY'
import json, collections
rows=[json.loads(l) for l in open("gpurun_out/r5v_pong.jsonl")]
agg=collections.defaultdict(list)
for c,r in zip(rows[::2],rows[1::2]): agg[(c["envs"],c["cfg"])].append(round(r["value"]/1e6,3))
for k,v in sorted(agg.items()): print(k, v)
PY
