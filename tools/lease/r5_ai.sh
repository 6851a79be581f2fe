#!/bin/bash
# Round 5, lease AI: side-stream work captured after the fc data gradient ("early_main": same
# graph edges, main branch inserted first) vs "early" -- race-free test, then Pong ABBA.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_gpu.py -k "side_stream_is_race_free" \
  > gpurun_out/r5ai_tests.log 2>&1 || { tail -30 gpurun_out/r5ai_tests.log; exit 1; }
tail -2 gpurun_out/r5ai_tests.log
rm -f gpurun_out/r5ai_pong.jsonl
cfg() {
  case $1 in
    A) echo "RRL_CNN_SIDE_MODE=${A_MODE:-early}" ;;
    M) echo "RRL_CNN_SIDE_MODE=early_main" ;;
    F) echo "RRL_CNN_SIDE_FC_FIRST=1" ;;
    C) echo "RRL_CNN_SIDE_MODE=c3" ;;
    P) echo "RRL_PIXEL_REPLAY_PRIO=1" ;;
  esac
}
RUNS=${RUNS:-"2048 A|2048 M|2048 M|2048 A|2048 A|2048 M|8192 A|8192 M|8192 M|8192 A|8192 A|8192 M"}
IFS="|" read -ra RUNA <<< "$RUNS"
for run in "${RUNA[@]}"; do
  set -- $run
  echo "{\"cfg\": \"$2\", \"envs\": $1}" >> gpurun_out/r5ai_pong.jsonl
  env $(cfg $2) timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r5ai_pong.jsonl 2>> gpurun_out/r5ai_pong.err || exit $?
done
python3 - <<'PY'
import json, collections
rows=[json.loads(l) for l in open("gpurun_out/r5ai_pong.jsonl")]
agg=collections.defaultdict(list)
for c,r in zip(rows[::2],rows[1::2]): agg[(c["envs"],c["cfg"])].append(round(r["value"]/1e6,3))
for k,v in sorted(agg.items()): print(k, v)
PY
[ -n "$SKIP_PROF" ] && exit 0
mkdir -p gpurun_out/prof_early_main
export TMPDIR=/tmp RRL_CNN_SIDE_MODE=${PROF_MODE:-early_main}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_early_main -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 10 --warmup 3 > gpurun_out/prof_early_main/log.txt 2>&1 || exit $?
