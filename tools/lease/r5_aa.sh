#!/bin/bash
# Round 5, lease AA: static wave priority for the 16-wave forward's conv2 / conv3 roles --
# bitwise layout tests, kernel times, Pong ABBA at 2,048 envs (A = default, P2 / P3 / P23).
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py tests/test_capture_robustness_gpu.py \
  > gpurun_out/r5aa_tests.log 2>&1 || { tail -30 gpurun_out/r5aa_tests.log; exit 1; }
tail -2 gpurun_out/r5aa_tests.log
timeout -k 10 200 python -u tools/cnn_kbench.py --which fwd16,fwd16_prio2,fwd16_prio3,fwd16_prio23 --rounds 6 --iters 20 \
  > gpurun_out/r5aa_kbench.jsonl 2> gpurun_out/r5aa_kbench.err || { tail -20 gpurun_out/r5aa_kbench.err; exit 1; }
timeout -k 10 200 python -u tools/cnn_kbench.py --which fwd16,fwd16_prio2,fwd16_prio3,fwd16_prio23 --rounds 4 --iters 10 --frames 8192 \
  >> gpurun_out/r5aa_kbench.jsonl 2>> gpurun_out/r5aa_kbench.err || { tail -20 gpurun_out/r5aa_kbench.err; exit 1; }
cat gpurun_out/r5aa_kbench.jsonl
rm -f gpurun_out/r5aa_pong.jsonl
for run in "2048 64" "2048 65" "2048 72" "2048 73" "2048 73" "2048 72" "2048 65" "2048 64"; do
  set -- $run
  echo "{\"cfg\": \"$2\", \"envs\": $1}" >> gpurun_out/r5aa_pong.jsonl
  RRL_CNN_FWD_LAYOUT=$2 timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r5aa_pong.jsonl 2>> gpurun_out/r5aa_pong.err || exit $?
done
python3 - <<'PY'
import json, collections
rows=[json.loads(l) for l in open("gpurun_out/r5aa_pong.jsonl")]
agg=collections.defaultdict(list)
for c,r in zip(rows[::2],rows[1::2]): agg[(c["envs"],c["cfg"])].append(round(r["value"]/1e6,3))
for k,v in sorted(agg.items()): print(k, v)
PY
