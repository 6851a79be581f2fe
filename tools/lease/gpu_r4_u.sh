# Round 4: forward LDS layout variants in one build (FwdLayout probe bits), alternated, after
# the variants' bitwise-equality test
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_cnn_gpu.py -k "layout_variants or fused_conv_stack or conv2" > gpurun_out/u_tests.log 2>&1 || { tail -30 gpurun_out/u_tests.log; exit 1; }
tail -1 gpurun_out/u_tests.log
for r in 1 2 3; do
  timeout -k 10 200 python3 tools/cnn_kbench.py --which fwd,fwd_l16,fwd_l32,fwd_l48,bwd2 --iters 50 > gpurun_out/kb_u$r.json 2>&1 && tail -1 gpurun_out/kb_u$r.json || exit 1
done
