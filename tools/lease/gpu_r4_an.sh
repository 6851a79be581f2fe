# Round 4: final kernel profiles -- the flagship bench epoch and the Pong update at 2,048 envs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_flagship_final gpurun_out/prof_pong_final
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flagship_final -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-ttt --host-steps 0 --pong-steps 0 --pong-big-envs 0 --ref-cpu-seconds 0 > gpurun_out/prof_flagship_final/log.txt 2>&1 || exit 1
grep metric gpurun_out/prof_flagship_final/log.txt | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pong_final -o run -- \
  python3 benchmarks/pong_a2c_bench.py --num-envs 2048 --steps 40 --warmup 3 > gpurun_out/prof_pong_final/log.txt 2>&1 && echo PROF_OK
