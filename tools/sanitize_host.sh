#!/bin/bash
# Sanitizer builds of the C++ host runtime (SURVEY §5.2 -- the reference has none).
#   tools/sanitize_host.sh           # ASan+UBSan and TSan builds, then run both (+ the ZMTP fuzz)
#   tools/sanitize_host.sh h2 [THREADS CALLS MUTANTS SEED]
#                                    # the native gRPC server under ASan+UBSan / TSan: concurrent
#                                    # nghttp2 clients, then mutated HTTP/2 client byte streams
#   tools/sanitize_host.sh fuzz N SEED_FILE...
#                                    # ASan+UBSan build of the network-facing parsers (pickle VM,
#                                    # TensorData reader, safetensors decoder) driven by N mutants
# Host code only: GPU sanitizers (xnack+) are not available on the MI355X pool.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${ROOT}/build/sanitize"
mkdir -p "$OUT"
if [ "${1:-}" = "h2" ]; then
  # the native gRPC server (csrc/net/h2grpc.cpp) with an nghttp2 client harness: concurrent traffic
  # under ASan+UBSan and TSan, then mutated client byte streams under ASan+UBSan
  #   tools/sanitize_host.sh h2 [THREADS CALLS MUTANTS SEED]
  shift
  CXX="${CXX:-g++}"
  NG="${RRL_NGHTTP2_PREFIX:-/opt/conda}"
  H2SRC="$ROOT/csrc/net/h2grpc.cpp $ROOT/csrc/net/selftest/h2_selftest.cpp"
  # the library file linked by path (no -L / rpath into the conda tree, whose libstdc++ is older):
  # its soname, libnghttp2.so.14, resolves to the system copy at run time
  $CXX -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
    -pthread -I "$ROOT/csrc/net" -I "$NG/include" $H2SRC "$NG/lib/libnghttp2.so" -o "$OUT/h2_selftest_asan"
  $CXX -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=thread -pthread -I "$ROOT/csrc/net" -I "$NG/include" \
    $H2SRC "$NG/lib/libnghttp2.so" -o "$OUT/h2_selftest_tsan"
  echo "== gRPC server traffic (ASan + UBSan)"
  ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 "$OUT/h2_selftest_asan" traffic "${1:-8}" "${2:-200}"
  echo "== gRPC server traffic (TSan)"
  TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 "$OUT/h2_selftest_tsan" traffic "${1:-8}" "${2:-200}"
  echo "== gRPC server fuzz (ASan + UBSan)"
  ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 "$OUT/h2_selftest_asan" fuzz "${3:-3000}" "${4:-1}"
  exit $?
fi
if [ "${1:-}" = "fuzz" ]; then
  shift
  CXX="${CXX:-g++}"
  $CXX -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
    -I "$ROOT/csrc/host" "$ROOT/csrc/host/selftest/parser_fuzz.cpp" "$ROOT/csrc/host/codec.cpp" -o "$OUT/parser_fuzz_asan"
  echo "== parser fuzz (ASan + UBSan)"
  ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 "$OUT/parser_fuzz_asan" "$@"
  exit $?
fi
SRCS="$ROOT/csrc/host/selftest/host_selftest.cpp $ROOT/csrc/host/codec.cpp $ROOT/csrc/host/zmtp.cpp $ROOT/csrc/host/vecenv.cpp $ROOT/csrc/host/policy.cpp"
CXX="${CXX:-g++}"
$CXX -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  -pthread -I "$ROOT/csrc/host" $SRCS -o "$OUT/host_selftest_asan"
$CXX -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=thread -pthread -I "$ROOT/csrc/host" $SRCS \
  -o "$OUT/host_selftest_tsan"
echo "== ASan + UBSan"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 "$OUT/host_selftest_asan"
echo "== TSan"
TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 "$OUT/host_selftest_tsan"
# the ZMTP PULL endpoint (every reference agent's upload lands here) against mutated peer
# conversations: truncations, flips, huge long-frame sizes, junk, multipart pile-ups, stray commands
echo "== ZMTP fuzz (ASan + UBSan)"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 "$OUT/host_selftest_asan" zmtp-fuzz "${RRL_ZMTP_FUZZ:-5000}" 1
echo "== ZMTP fuzz (TSan)"
TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 "$OUT/host_selftest_tsan" zmtp-fuzz 1000 2
