#!/bin/bash
# Build and run the native runtime self-test plain, with ASan+UBSan and with TSan
# (host code only; no GPU involved).  SURVEY §5.2.
set -euo pipefail
cd "$(dirname "$0")/.."
RT=cake_amd/csrc/runtime
SRC="cake_amd/csrc/tests/runtime_selftest.cpp $RT/json.cpp $RT/topology.cpp $RT/proto.cpp $RT/net.cpp $RT/safetensors.cpp $RT/server.cpp"
OUT=${OUT_DIR:-/tmp/cake_sanitize}
mkdir -p "$OUT"
for v in ${VARIANTS:-plain asan tsan}; do
  case $v in
    plain) F="-O2" ;;
    asan)  F="-O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined" ;;
    tsan)  F="-O1 -g -fsanitize=thread" ;;
  esac
  g++ -std=c++17 $F -pthread $SRC -o "$OUT/selftest_$v"
  echo "== $v"
  ASAN_OPTIONS=detect_leaks=1 TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" "$OUT/selftest_$v"
done
