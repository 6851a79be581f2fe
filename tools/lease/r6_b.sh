#!/bin/bash
# Round 6, lease B: fan-in with the async model publisher (zmq-ref rows) and the grpc.aio server,
# 16 / 64 agent processes against the GPU engine; then the transport GPU tests.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 500 python -u benchmarks/fanin_bench.py --agents 16 64 --transports zmq zmq-ref grpc --seconds 10 \
  --out gpurun_out/r6b_fanin.jsonl > gpurun_out/r6b_fanin.log 2>&1 || { tail -30 gpurun_out/r6b_fanin.log; exit 1; }
cat gpurun_out/r6b_fanin.jsonl | cut -c1-400
