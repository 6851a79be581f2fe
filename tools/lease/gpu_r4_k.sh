# Round 4: every BASELINE preset on one GPU after the round-4 changes (Adam loop form, Pong kernels)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u benchmarks/configs_bench.py --steps 5 --warmup 2 > gpurun_out/configs_k.jsonl 2> gpurun_out/configs_k.err || { tail -20 gpurun_out/configs_k.err; exit 1; }
cut -c1-300 gpurun_out/configs_k.jsonl
