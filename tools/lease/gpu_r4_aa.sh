# Round 4: the shipped forward (conv3 over its 49 pixels) vs the 7 x 9 conv3 grid, and the conv2
# backward dgrad over a 10 x 12 grid vs 7 tiles -- ABBA runs of the Pong update, kernels over
# alternating-order rounds; the .so's build time printed first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ls -la --time-style=+%H:%M:%S relayrl_prototype_amd/_hip_ops*.so
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_gpu.py > gpurun_out/aa_cnn_tests.log 2>&1 || { tail -30 gpurun_out/aa_cnn_tests.log; exit 1; }
tail -1 gpurun_out/aa_cnn_tests.log
timeout -k 10 300 python3 tools/cnn_kbench.py --which fwd,fwd_c3_grid,bwd2,bwd2_7tiles,bwd2_staged --iters 50 --rounds 4 > gpurun_out/kb_aa.json 2>&1 && tail -1 gpurun_out/kb_aa.json || exit 1
i=0
for v in A B B A A B B A; do i=$((i+1)); for n in 2048 8192; do
  if [ $v = A ]; then lay=0; b2=0; else lay=32; b2=2; fi
  RRL_CNN_FWD_LAYOUT=$lay timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_aa_f_${n}_$v.$i.json 2>&1 || exit 1
  RRL_CNN_BWD2_VARIANT=$b2 timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs $n --steps 60 --warmup 5 > gpurun_out/pong_aa_b_${n}_$v.$i.json 2>&1 || exit 1
  echo "$n $v run$i fwd_layout=$lay $(tail -1 gpurun_out/pong_aa_f_${n}_$v.$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3))') bwd2_variant=$b2 $(tail -1 gpurun_out/pong_aa_b_${n}_$v.$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3))')"
done; done
