# Round 4: vectorised clip + Adam and sum of squares, the Wfc transpose beside the rollout: CNN GPU tests, Pong, kernel profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ls -la --time-style=+%H:%M:%S relayrl_prototype_amd/_hip_ops*.so
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_gpu.py tests/test_forced_collectives_gpu.py > gpurun_out/ah_tests.log 2>&1 || { tail -30 gpurun_out/ah_tests.log; exit 1; }
tail -1 gpurun_out/ah_tests.log
for n in 2048 8192; do
  timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_ah_$n.json 2>&1 || exit 1
  echo "$n $(tail -1 gpurun_out/pong_ah_$n.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), d.get("ms_per_step"))')"
done
mkdir -p gpurun_out/prof_ah
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ah -o run -- python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/prof_ah/log.txt 2>&1 && echo PROF_OK
