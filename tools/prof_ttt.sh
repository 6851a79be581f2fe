# rocprofv3 kernel-time summary of the time-to-threshold configuration (tools/ttt_epoch_probe.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_ttt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ttt -o run -- \
  python3 tools/ttt_epoch_probe.py > gpurun_out/prof_ttt/log.txt 2>&1 || exit 1
tail -1 gpurun_out/prof_ttt/log.txt | cut -c1-200
