# Round 4: backward A2C head rows per wave (RRL_HEAD_BWD_ROWS 4 = default, A; 1, B): CNN tests
# under the variant, Pong ABBA, kernel time of the head in both
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RRL_HEAD_BWD_ROWS=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_gpu.py -k "pixel or head or backward" > gpurun_out/aq_tests.log 2>&1 || { tail -30 gpurun_out/aq_tests.log; exit 1; }
tail -1 gpurun_out/aq_tests.log
i=0
for v in A B B A A B B A; do i=$((i+1)); for n in 2048 8192; do
  if [ $v = A ]; then d=4; else d=1; fi
  RRL_HEAD_BWD_ROWS=$d timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_aq_${n}_$v.$i.json 2>&1 || exit 1
  echo "$n $v(rows $d) run$i $(tail -1 gpurun_out/pong_aq_${n}_$v.$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3))')"
done; done
for d in 4 2 1; do
  mkdir -p gpurun_out/prof_aq$d
  RRL_HEAD_BWD_ROWS=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_aq$d -o run -- python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
  echo "rows $d: $(grep 'a2c_head_kernel<true' gpurun_out/prof_aq$d/run_kernel_stats.csv | cut -d, -f1-4)"
done
