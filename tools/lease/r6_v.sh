#!/bin/bash
# Round 6, lease V: the TrainingServer's ingest ceiling with the Python learner service in the loop
# (benchmarks/ingest_ceiling.py: native PUSH senders replaying pre-encoded RRLC episodes), CPU
# trajectory learner and the GPU engine; plus the native gRPC / ZMTP endpoint ceilings on the box CPU.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/ingest_ceiling.py --senders 1 4 8 --seconds 4 > gpurun_out/r6v_ingest_cpu.jsonl 2> gpurun_out/r6v_ingest_cpu.err || exit $?
timeout -k 10 300 python -u benchmarks/ingest_ceiling.py --senders 1 4 8 --seconds 4 --engine vec > gpurun_out/r6v_ingest_vec.jsonl 2> gpurun_out/r6v_ingest_vec.err || exit $?
timeout -k 10 200 bash tools/h2_rate.sh 3 4096 > gpurun_out/r6v_h2_rate.jsonl 2>&1 || exit $?
timeout -k 10 200 bash tools/zmtp_rate.sh 3 4096 > gpurun_out/r6v_zmtp_rate.jsonl 2>&1 || exit $?
cat gpurun_out/r6v_ingest_cpu.jsonl gpurun_out/r6v_ingest_vec.jsonl gpurun_out/r6v_h2_rate.jsonl gpurun_out/r6v_zmtp_rate.jsonl | cut -c1-220
