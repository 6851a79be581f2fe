mkdir -p gpurun_out
export RRL_DIST_BACKEND=gloo RRL_FORCE_DEVICE=0
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 2 --steps 2 --warmup 1 --num-envs 1024 --vf-iters 4 --al-num-envs 256 --al-rollout-len 32 --al-vf-iters 8 --multi-ttt-seeds 1 --ttt-max-s 15 > gpurun_out/r6z_2rank.out 2> gpurun_out/r6z_2rank.err
echo "2rank exit=$?" >> gpurun_out/r6z_2rank.out
unset RRL_DIST_BACKEND RRL_FORCE_DEVICE
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r6z_gpu_tests.txt 2>&1
rc=$?
echo "pytest exit=$rc" >> gpurun_out/r6z_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6z_smoke.txt 2>&1 && timeout -k 10 300 python bench.py > gpurun_out/r6z_bench.json 2> gpurun_out/r6z_bench.err
