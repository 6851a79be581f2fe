# Round 4: end-state bench line (driver's flags, reference CPU run skipped)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python3 bench.py --gpus 1 --steps 20 --warmup 5 --ref-cpu-seconds 0 > gpurun_out/bench_au.json 2> gpurun_out/bench_au.err || { tail -20 gpurun_out/bench_au.err; exit 1; }
cut -c1-300 gpurun_out/bench_au.json
