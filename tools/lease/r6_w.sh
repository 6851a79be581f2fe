#!/bin/bash
# Round 6, lease W: ingest ceiling again with senders that do not run out of pre-encoded episodes.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u benchmarks/ingest_ceiling.py --senders 1 4 8 --seconds 4 --frames-per-sender 400000 > gpurun_out/r6w_ingest_cpu.jsonl 2> gpurun_out/r6w_ingest_cpu.err || exit $?
timeout -k 10 400 python -u benchmarks/ingest_ceiling.py --senders 4 8 --seconds 4 --frames-per-sender 400000 --engine vec > gpurun_out/r6w_ingest_vec.jsonl 2> gpurun_out/r6w_ingest_vec.err || exit $?
cat gpurun_out/r6w_ingest_cpu.jsonl gpurun_out/r6w_ingest_vec.jsonl | cut -c1-260
