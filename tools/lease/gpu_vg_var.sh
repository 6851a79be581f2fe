# Structural A/B of the factored value head (V variants via tune bit 7), numerics first; then
# the policy (CartPole PG) and HalfCheetah (Gaussian PPO, D = 17 value) steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_value_grad_gpu.py tests/test_ppo_minibatch.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/vg_var_tests.log 2>&1; rc=$?; tail -1 gpurun_out/vg_var_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do timeout -k 10 120 python tools/kbench.py grad --iters 30 --tunes ${VG_TUNES:-128,176,240,128,176,240} || exit 1; done 2>&1 | grep value
timeout -k 10 200 python tools/kbench.py pgrad --iters 10 2>&1 | grep -v "^\s*$" | tail -1 | cut -c1-400
timeout -k 10 200 python tools/kbench.py pgauss --iters 10 2>&1 | grep gauss | cut -c1-400
if [ -n "$VG_STAMP_TUNES" ]; then timeout -k 10 120 python tools/kbench.py grad --iters 3 --stamp-tunes $VG_STAMP_TUNES 2>&1 | grep stamps; fi
