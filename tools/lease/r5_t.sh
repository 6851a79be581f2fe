#!/bin/bash
# Round 5, lease T: re-measure the fc / side-stream choices after the fc kernel changes (inline-asm
# transposed reads, persistent tiles): A = defaults, E = staged fc-dgrad epilogue
# (RRL_FC_DIRECT_EPI=0), S = side mode "sums", L = side mode "late"; Pong ABBA-style rotations.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
rm -f gpurun_out/r5t_pong.jsonl
cfg() {
  case $1 in
    A) echo "RRL_CNN_SIDE_MODE=early" ;;
    E) echo "RRL_FC_DIRECT_EPI=0" ;;
    S) echo "RRL_CNN_SIDE_MODE=sums" ;;
    L) echo "RRL_CNN_SIDE_MODE=late" ;;
  esac
}
for run in "2048 A" "2048 E" "2048 S" "2048 L" "2048 L" "2048 S" "2048 E" "2048 A" "8192 A" "8192 E" "8192 S" "8192 L" "8192 L" "8192 S" "8192 E" "8192 A"; do
  set -- $run
  echo "{\"cfg\": \"$2\", \"envs\": $1}" >> gpurun_out/r5t_pong.jsonl
  env $(cfg $2) timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r5t_pong.jsonl 2>> gpurun_out/r5t_pong.err || exit $?
done
python3 - <<'PY'
import json, collections
rows=[json.loads(l) for l in open("gpurun_out/r5t_pong.jsonl")]
agg=collections.defaultdict(list)
for c,r in zip(rows[::2],rows[1::2]): agg[(c["envs"],c["cfg"])].append(round(r["value"]/1e6,3))
for k,v in sorted(agg.items()): print(k, v)
PY
