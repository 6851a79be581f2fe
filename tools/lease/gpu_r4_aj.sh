# Round 4: conv slab sums forked to the side stream as each conv backward finishes
# (RRL_CNN_SIDE_CONV_SUMS 1, A) vs all three in one launch at the end (0, B): CNN tests, Pong ABBA,
# a kernel trace of the new schedule
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_gpu.py > gpurun_out/aj_tests.log 2>&1 || { tail -30 gpurun_out/aj_tests.log; exit 1; }
tail -1 gpurun_out/aj_tests.log
i=0
for v in A B B A A B B A; do i=$((i+1)); for n in 2048 8192; do
  if [ $v = A ]; then d=1; else d=0; fi
  RRL_CNN_SIDE_CONV_SUMS=$d timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_aj_${n}_$v.$i.json 2>&1 || exit 1
  echo "$n $v(conv sums side $d) run$i $(tail -1 gpurun_out/pong_aj_${n}_$v.$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3))')"
done; done
mkdir -p gpurun_out/prof_aj
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_aj -o run -- python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/prof_aj/log.txt 2>&1 && echo PROF_OK
