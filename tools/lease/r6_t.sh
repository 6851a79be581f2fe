#!/bin/bash
# Round 6, lease T: the agent / transport micro-benchmarks (T1, CPU-side) on the GPU box's host CPU.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u benchmarks/transport_bench.py > gpurun_out/r6t_transport.jsonl 2> gpurun_out/r6t_transport.err || exit $?
lscpu | grep -E "Model name|^CPU\(s\)|MHz" > gpurun_out/r6t_cpu.txt || true
cut -c1-300 gpurun_out/r6t_transport.jsonl
