# Value-grad prologue change: numerics, per-launch timing at small and large batches, TTT epoch probe.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_value_grad_gpu.py tests/test_kernels_gpu.py tests/test_trainers_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pro_tests.log 2>&1; rc=$?; tail -2 gpurun_out/pro_tests.log; [ $rc -eq 0 ] || exit $rc
for B in 8192 65536 2097152; do timeout -k 10 120 python tools/kbench.py grad --B $B --iters 50 --tunes 176 || exit 1; done > gpurun_out/pro_time.jsonl 2>&1
timeout -k 10 120 python tools/kbench.py grad --B 262144 --vd 8 --iters 50 --tunes 144 >> gpurun_out/pro_time.jsonl 2>&1 || exit 1
timeout -k 10 120 python tools/kbench.py pgauss --iters 20 >> gpurun_out/pro_time.jsonl 2>&1 || exit 1
grep -h "_us" gpurun_out/pro_time.jsonl | cut -c1-300
timeout -k 10 120 python tools/kbench.py grad --B 65536 --iters 5 --stamps > gpurun_out/pro_stamps.txt 2>&1 || exit 1
timeout -k 10 120 python tools/ttt_epoch_probe.py --ref --shape 512 16 > gpurun_out/pro_ttt_probe.json 2>&1 && cat gpurun_out/pro_ttt_probe.json | cut -c1-200
