set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/host_rollout_probe.py > gpurun_out/host_probe.jsonl 2>&1; rc=$?; cat gpurun_out/host_probe.jsonl | tail -30; exit $rc
