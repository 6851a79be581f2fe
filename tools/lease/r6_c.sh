#!/bin/bash
# Round 6, lease C: fan-in after the GIL-free reference decoder (zmq-ref) and grpc.aio, 16 / 64 agents.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u benchmarks/fanin_bench.py --agents 16 64 --transports zmq-ref grpc zmq --seconds 10 \
  --out gpurun_out/r6c_fanin.jsonl > gpurun_out/r6c_fanin.log 2>&1 || { tail -30 gpurun_out/r6c_fanin.log; exit 1; }
cat gpurun_out/r6c_fanin.jsonl | cut -c1-300
