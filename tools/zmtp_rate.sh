#!/bin/bash
# The C++ ZMTP PULL endpoint's ingest ceiling without Python agents (csrc/host/selftest/host_selftest.cpp
# "zmtp-rate" mode, -O2): PUSH clients send back to back, over one connection each and with a new
# connection per message (the reference agent's pattern), while one thread drains the PULL.
#   tools/zmtp_rate.sh [SECONDS BYTES]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${ROOT}/build/zmtprate"
mkdir -p "$OUT"
${CXX:-g++} -std=c++17 -O2 -pthread -I "$ROOT/csrc/host" "$ROOT/csrc/host/selftest/host_selftest.cpp" \
  "$ROOT/csrc/host/codec.cpp" "$ROOT/csrc/host/zmtp.cpp" "$ROOT/csrc/host/vecenv.cpp" "$ROOT/csrc/host/policy.cpp" \
  -o "$OUT/host_selftest"
for c in 1 4 16 64; do "$OUT/host_selftest" zmtp-rate "$c" "${1:-3}" "${2:-4096}"; done
for c in 4 16; do "$OUT/host_selftest" zmtp-rate "$c" "${1:-3}" "${2:-4096}" reconnect; done
