# rocprofv3 kernel-time summary of the flagship bench (CartPole REINFORCE-with-baseline, 1 GPU) -- the
# headline epochs only: the Pong / host-env / convergence / reference-CPU probes of the bench line are off.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_flagship
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flagship -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-ttt --pong-steps 0 --convergence off --host-steps 0 --ref-cpu-seconds 0 \
  > gpurun_out/prof_flagship/log.txt 2>&1 || exit 1
grep metric gpurun_out/prof_flagship/log.txt | cut -c1-200
