# Round 4: conv backward bias partials folded over the 8 waves (64 per workgroup): CNN tests, Pong, kernel profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ls -la --time-style=+%H:%M:%S relayrl_prototype_amd/_hip_ops*.so
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_gpu.py > gpurun_out/as_tests.log 2>&1 || { tail -30 gpurun_out/as_tests.log; exit 1; }
tail -1 gpurun_out/as_tests.log
for r in 1 2; do for n in 2048 8192; do
  timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_as_$n.$r.json 2>&1 || exit 1
  echo "$n r$r $(tail -1 gpurun_out/pong_as_$n.$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), d.get("ms_per_step"))')"
done; done
mkdir -p gpurun_out/prof_as
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_as -o run -- python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/prof_as/log.txt 2>&1 && echo PROF_OK
RRL_CNN_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_as1 -o run -- python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > /dev/null 2>&1 && echo PROF1_OK
