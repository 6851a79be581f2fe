# Pong A2C env-count scan on the current kernels (one MI355X).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/pong_scan.jsonl
for n in 2048 4096 8192 16384; do
  timeout -k 10 200 python benchmarks/pong_a2c_bench.py --num-envs $n --steps 20 --warmup 3 > gpurun_out/pong_scan_$n.json \
    2> gpurun_out/pong_scan_$n.err || exit $?
  tail -1 gpurun_out/pong_scan_$n.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'bench':'pong_a2c','num_envs':$n,'env_steps_per_s':round(d['value']),'ms_per_update':round(d['ms_per_step'],3)}))" | tee -a gpurun_out/pong_scan.jsonl
done
