#!/bin/bash
# The native gRPC server's ingest ceiling without Python agents (csrc/net/selftest/h2_selftest.cpp
# "rate" mode, -O2): native nghttp2 clients upload frames back to back while one consumer drains.
#   tools/h2_rate.sh [SECONDS BYTES]   -> one JSON line per client count (1, 4, 16, 64)
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${ROOT}/build/h2rate"
mkdir -p "$OUT"
NG="${RRL_NGHTTP2_PREFIX:-/opt/conda}"
${CXX:-g++} -std=c++17 -O2 -pthread -I "$ROOT/csrc/net" -I "$NG/include" "$ROOT/csrc/net/h2grpc.cpp" \
  "$ROOT/csrc/net/selftest/h2_selftest.cpp" "$NG/lib/libnghttp2.so" -o "$OUT/h2_selftest"
for c in 1 4 16 64; do "$OUT/h2_selftest" rate "$c" "${1:-3}" "${2:-4096}"; done
