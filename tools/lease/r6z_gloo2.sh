# gloo collectives (all_reduce, broadcast) on device tensors written just before: ordered or not?
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
o=gpurun_out/r6z_gloo_coll.jsonl
for op in all_reduce broadcast; do
  timeout -k 10 90 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
    --master-port=$((29600 + RANDOM % 300)) tools/probes/gloo_device_p2p_probe.py --op $op --fence 0 --rounds 12 >> $o 2>> gpurun_out/r6z_gloo_coll.err || exit $?
done
echo COLL_OK
