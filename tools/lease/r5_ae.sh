#!/bin/bash
# Round 5, lease AE: the conv2 backward's da1 leaving as 16-byte stores (lane swaps) -- bitwise test, kernel times, Pong ABBA.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py -k "bitwise_equal" \
  > gpurun_out/r5ae_tests.log 2>&1 || { tail -30 gpurun_out/r5ae_tests.log; exit 1; }
tail -2 gpurun_out/r5ae_tests.log
timeout -k 10 300 python -u tools/cnn_kbench.py --which bwd2,bwd2_st16 --rounds 8 --iters 20 \
  > gpurun_out/r5ae_kbench.jsonl 2> gpurun_out/r5ae_kbench.err || { tail -20 gpurun_out/r5ae_kbench.err; exit 1; }
cat gpurun_out/r5ae_kbench.jsonl
rm -f gpurun_out/r5ae_pong.jsonl
for run in "2048 0" "2048 8" "2048 8" "2048 0" "8192 0" "8192 8" "8192 8" "8192 0"; do
  set -- $run
  echo "{\"cfg\": \"$2\", \"envs\": $1}" >> gpurun_out/r5ae_pong.jsonl
  RRL_CNN_BWD2_VARIANT=$2 timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r5ae_pong.jsonl 2>> gpurun_out/r5ae_pong.err || exit $?
done
python3 - <<'PY'
import json, collections
rows=[json.loads(l) for l in open("gpurun_out/r5ae_pong.jsonl")]
agg=collections.defaultdict(list)
for c,r in zip(rows[::2],rows[1::2]): agg[(c["envs"],c["cfg"])].append(round(r["value"]/1e6,3))
for k,v in sorted(agg.items()): print(k, v)
PY
