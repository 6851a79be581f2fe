# gloo device-tensor P2P: unfenced vs fenced vs Comm.gather_to, then the affected GPU tests
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
o=gpurun_out/r6z_gloo_p2p.jsonl
for args in "--via dist --fence 0" "--via dist --fence 1" "--via comm --fence 0"; do
  timeout -k 10 90 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
    --master-port=$((29600 + RANDOM % 300)) tools/probes/gloo_device_p2p_probe.py $args --rounds 12 >> $o 2>> gpurun_out/r6z_gloo_p2p.err || exit $?
done
timeout -k 10 400 python -u -m pytest tests/test_gloo_p2p_gpu.py tests/test_bench_gpu.py tests/test_actor_learner_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/r6z_gloo_tests.txt 2>&1
