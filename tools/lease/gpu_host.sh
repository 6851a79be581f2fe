# Host-env path on the GPU: tests, overlap on/off benches, kernel+copy timeline of the overlapped preset.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_host
timeout -k 10 300 python -u -m pytest tests/test_trainers_gpu.py tests/test_actor_learner_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/host_tests.log 2>&1; rc=$?; tail -2 gpurun_out/host_tests.log; [ $rc -eq 0 ] || exit $rc
for ov in false true; do
  timeout -k 10 300 python benchmarks/configs_bench.py --presets cartpole-reinforce-host halfcheetah-ppo-host --steps 5 --warmup 2 --set overlap=$ov || exit 1
done > gpurun_out/host_bench.jsonl 2>&1
cat gpurun_out/host_bench.jsonl | grep preset | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_host -o run -- \
  python3 benchmarks/configs_bench.py --presets halfcheetah-ppo-host --steps 3 --warmup 1 > gpurun_out/prof_host/log.txt 2>&1 && \
python tools/overlap_summary.py gpurun_out/prof_host/run
