# Round 4: forward LDS layout variants in one build (FwdLayout probe bits), alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  timeout -k 10 200 python3 tools/cnn_kbench.py --which fwd,fwd_l16,fwd_l32,fwd_l48 --iters 50 > gpurun_out/kb_u$r.json 2>&1 && tail -1 gpurun_out/kb_u$r.json || exit 1
done
