# Round 4: per-segment stamps of the value step vs the 2-action policy step at the flagship shape
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python3 -u tools/kbench.py grad --B 2097152 --iters 5 --stamps > gpurun_out/kb_stamps_value.json 2>&1 || { tail -5 gpurun_out/kb_stamps_value.json; exit 1; }
grep '^{' gpurun_out/kb_stamps_value.json | cut -c1-1600
timeout -k 10 200 python3 -u tools/kbench.py pgrad --B 2097152 --iters 5 --stamps > gpurun_out/kb_stamps_policy.json 2>&1 || { tail -5 gpurun_out/kb_stamps_policy.json; exit 1; }
grep '^{' gpurun_out/kb_stamps_policy.json | cut -c1-1600
