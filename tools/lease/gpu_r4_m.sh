# Round 4: side-stream fork A/B on one box at 2048 and 8192 envs, alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for late in early late; do
  RRL_CNN_SIDE_MODE=$late timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/pong_m_2048_late$late.r$r.json 2>&1 || exit 1
  echo "2048 late=$late r$r $(tail -1 gpurun_out/pong_m_2048_late$late.r$r.json | cut -c60-110)"
  RRL_CNN_SIDE_MODE=$late timeout -k 10 300 python3 benchmarks/pong_a2c_bench.py --num-envs 8192 --steps 20 --warmup 3 > gpurun_out/pong_m_8192_late$late.r$r.json 2>&1 || exit 1
  echo "8192 late=$late r$r $(tail -1 gpurun_out/pong_m_8192_late$late.r$r.json | cut -c60-110)"
done; done
