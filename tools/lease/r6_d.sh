#!/bin/bash
# Round 6, lease D (re-run after the container rebuild): fan-in with the async newest-wins model
# publisher, the GIL-free reference decoder (zmq-ref) and the native C++ gRPC server, 16 / 64 agents.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 500 python -u benchmarks/fanin_bench.py --agents 16 64 --transports zmq-ref grpc zmq --seconds 10 \
  --out gpurun_out/r6d_fanin.jsonl > gpurun_out/r6d_fanin.log 2>&1 || { tail -30 gpurun_out/r6d_fanin.log; exit 1; }
cut -c1-400 gpurun_out/r6d_fanin.jsonl
