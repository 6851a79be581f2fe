set -o pipefail
mkdir -p gpurun_out
for w in 0 1 2; do
timeout -k 10 200 python benchmarks/configs_bench.py --presets cartpole-reinforce-host halfcheetah-ppo-host --steps 8 --warmup 2 --set driver_wait=$w > gpurun_out/host_wait$w.jsonl 2>&1 || exit 1
echo "wait $w"; grep preset gpurun_out/host_wait$w.jsonl | cut -c 1-40,200-520
done
timeout -k 10 200 python benchmarks/configs_bench.py --presets cartpole-reinforce-host --steps 8 --warmup 2 --set driver_wait=1 actor_cus=0 > gpurun_out/host_wait1_nosplit.jsonl 2>&1 && echo "wait 1 nosplit" && grep preset gpurun_out/host_wait1_nosplit.jsonl | cut -c 1-40,200-520
