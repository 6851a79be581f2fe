#!/bin/bash
# Round 5, lease AC: s_setprio around the k-tile MFMAs of the 128 x 128 fc GEMMs (RRL_FC_SETPRIO) --
# numerics, kernel times ("422" vs "422p"), and if it helps a Pong ABBA.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
RRL_FC_SETPRIO=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py -k "fc_" \
  > gpurun_out/r5ac_tests.log 2>&1 || { tail -30 gpurun_out/r5ac_tests.log; exit 1; }
tail -2 gpurun_out/r5ac_tests.log
FC_VARIANTS=422,422p FC_CASES=fwd_part_s4,dgrad_mask,wgrad_tn_s5,dgrad40k_mask,wgrad40k_tn_s5 timeout -k 10 300 python -u tools/fc_kbench.py \
  > gpurun_out/r5ac_fc_kbench.jsonl 2> gpurun_out/r5ac_fc_kbench.err || { tail -20 gpurun_out/r5ac_fc_kbench.err; exit 1; }
cat gpurun_out/r5ac_fc_kbench.jsonl
rm -f gpurun_out/r5ac_pong.jsonl
for run in "2048 0" "2048 1" "2048 1" "2048 0"; do
  set -- $run
  echo "{\"cfg\": \"$2\", \"envs\": $1}" >> gpurun_out/r5ac_pong.jsonl
  RRL_FC_SETPRIO=$2 timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r5ac_pong.jsonl 2>> gpurun_out/r5ac_pong.err || exit $?
done
python3 - <<'PY'
import json, collections
rows=[json.loads(l) for l in open("gpurun_out/r5ac_pong.jsonl")]
agg=collections.defaultdict(list)
for c,r in zip(rows[::2],rows[1::2]): agg[(c["envs"],c["cfg"])].append(round(r["value"]/1e6,3))
for k,v in sorted(agg.items()): print(k, v)
PY
