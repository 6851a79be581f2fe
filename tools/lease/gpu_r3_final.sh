# Round-3 final evidence: clean flagship kernel profile (no side probes) and the preset bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_flagship_clean
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flagship_clean -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-ttt --host-steps 0 --pong-steps 0 --ref-cpu-seconds 0 --phase-steps 0 \
  > gpurun_out/prof_flagship_clean/log.txt 2>&1 || exit 1
grep metric gpurun_out/prof_flagship_clean/log.txt | cut -c1-200
timeout -k 10 600 python3 benchmarks/configs_bench.py > gpurun_out/configs_bench_r3.jsonl 2> gpurun_out/configs_bench_r3.err || exit 1
cut -c1-250 gpurun_out/configs_bench_r3.jsonl
