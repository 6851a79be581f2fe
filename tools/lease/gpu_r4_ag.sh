# Round 4: fused forward time vs frames per launch (per-launch fill / drain cost)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for f in 256 512 1024 2048 4096 8192; do
  timeout -k 10 120 python3 tools/cnn_kbench.py --which fwd --frames $f --bwd-frames 256 --iters 50 --rounds 3 > gpurun_out/kb_ag_$f.json 2>&1 && echo "$f $(tail -1 gpurun_out/kb_ag_$f.json)" || exit 1
done
