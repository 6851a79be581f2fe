#!/bin/bash
# Round 5, lease AO: the fused head-step kernel with the head weights through LDS (RRL_PONG_HEAD_WLDS=1) -- tests, Pong ABBA, kernel tables.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_gpu.py \
  -k "fused_head_step or pixel_update_side_stream" > gpurun_out/r5ao_tests.log 2>&1 || { tail -40 gpurun_out/r5ao_tests.log; exit 1; }
tail -2 gpurun_out/r5ao_tests.log
rm -f gpurun_out/r5ao_pong.jsonl
cfg() {
  case $1 in
    A) echo "RRL_PONG_HEAD_WLDS=0" ;;
    M) echo "RRL_PONG_HEAD_WLDS=1" ;;
  esac
}
RUNS=${RUNS:-"2048 A|2048 M|2048 M|2048 A|2048 A|2048 M|8192 A|8192 M|8192 M|8192 A|8192 A|8192 M"}
IFS="|" read -ra RUNA <<< "$RUNS"
for run in "${RUNA[@]}"; do
  set -- $run
  echo "{\"cfg\": \"$2\", \"envs\": $1}" >> gpurun_out/r5ao_pong.jsonl
  env $(cfg $2) timeout -k 10 200 python -u benchmarks/pong_a2c_bench.py --num-envs $1 --steps 40 --warmup 5 \
      >> gpurun_out/r5ao_pong.jsonl 2>> gpurun_out/r5ao_pong.err || exit $?
done
python3 - <<'PY'
import json, collections
rows=[json.loads(l) for l in open("gpurun_out/r5ao_pong.jsonl")]
agg=collections.defaultdict(list)
for c,r in zip(rows[::2],rows[1::2]): agg[(c["envs"],c["cfg"])].append(round(r["value"]/1e6,3))
for k,v in sorted(agg.items()): print(k, v)
PY
mkdir -p gpurun_out/prof_hw8192 gpurun_out/prof_hw2048
export TMPDIR=/tmp RRL_PONG_HEAD_WLDS=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hw8192 -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 8192 --steps 10 --warmup 3 > gpurun_out/prof_hw8192/log.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hw2048 -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 10 --warmup 3 > gpurun_out/prof_hw2048/log.txt 2>&1 || exit $?
echo PROF_OK
