#!/bin/bash
# Round 5, lease Y: s_setprio around the MFMA clusters of the Pong conv kernels -- bitwise /
# oracle tests, kernel times (rotated rounds), then Pong ABBA: A = defaults, P = the setprio
# forms of conv3 / conv2 backward (+ forward, conv1 weight gradient).
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py -k "bitwise_equal or conv1_wgrad8" \
  > gpurun_out/r5y_tests.log 2>&1 || { tail -30 gpurun_out/r5y_tests.log; exit 1; }
tail -2 gpurun_out/r5y_tests.log
timeout -k 10 200 python -u tools/cnn_kbench.py --which fwd16,fwd16_sp,wgrad1_8,wgrad1_8_sp,bwd3,bwd3_sp1,bwd2,bwd2_sp1 --rounds 4 --iters 20 \
  > gpurun_out/r5y_kbench.jsonl 2> gpurun_out/r5y_kbench.err || { tail -20 gpurun_out/r5y_kbench.err; exit 1; }
cat gpurun_out/r5y_kbench.jsonl
rm -f gpurun_out/r5y_pong.jsonl
cfg() {
  case $1 in
    A) echo "RRL_CNN_BWD3_VARIANT=0" ;;
    B) echo "RRL_CNN_BWD3_VARIANT=2" ;;
    C) echo "RRL_CNN_BWD3_VARIANT=2 RRL_CNN_BWD2_VARIANT=4 RRL_CNN_FWD_LAYOUT=68 RRL_CNN_WGRAD1_SETPRIO=1" ;;
  esac
}
for run in "2048 A" "2048 B" "2048 C" "2048 C" "2048 B" "2048 A" "8192 A" "8192 B" "8192 C" "8192 C" "8192 B" "8192 A"; do
  set -- $run
  echo "{\"cfg\": \"$2\", \"envs\": $1}" >> gpurun_out/r5y_pong.jsonl
  env $(cfg $2) timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r5y_pong.jsonl 2>> gpurun_out/r5y_pong.err || exit $?
done
python3 - <<'PY'
import json, collections
rows=[json.loads(l) for l in open("gpurun_out/r5y_pong.jsonl")]
agg=collections.defaultdict(list)
for c,r in zip(rows[::2],rows[1::2]): agg[(c["envs"],c["cfg"])].append(round(r["value"]/1e6,3))
for k,v in sorted(agg.items()): print(k, v)
PY
