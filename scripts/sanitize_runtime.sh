#!/bin/bash
# Build and run the native runtime self-tests plain, with ASan+UBSan and with TSan
# (host code only; no GPU involved).  SURVEY §5.2.
#   runtime_selftest: json / topology / wire codec / safetensors / framed TCP / WorkerServer
#   worker_selftest:  the native text + SD workers (native_worker.cpp: multi-master
#                     sessions, the compute lock, request validation, disconnects, stop)
#                     over a host stub of libcake_engine.so (stub_engine.cpp)
set -euo pipefail
cd "$(dirname "$0")/.."
RT=cake_amd/csrc/runtime
T=cake_amd/csrc/tests
SRC="$T/runtime_selftest.cpp $RT/json.cpp $RT/topology.cpp $RT/proto.cpp $RT/net.cpp $RT/safetensors.cpp $RT/server.cpp"
WSRC="$T/worker_selftest.cpp $RT/native_worker.cpp $RT/json.cpp $RT/topology.cpp $RT/proto.cpp $RT/net.cpp $RT/server.cpp"
OUT=${OUT_DIR:-/tmp/cake_sanitize}
mkdir -p "$OUT"
for v in ${VARIANTS:-plain asan tsan}; do
  case $v in
    plain) F="-O2" ;;
    asan)  F="-O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined" ;;
    tsan)  F="-O1 -g -fsanitize=thread" ;;
  esac
  g++ -std=c++17 $F -pthread $SRC -o "$OUT/selftest_$v"
  g++ -std=c++17 $F -shared -fPIC $T/stub_engine.cpp -o "$OUT/libstub_engine_$v.so"
  g++ -std=c++17 $F -pthread $WSRC -ldl -o "$OUT/worker_selftest_$v"
  echo "== $v"
  ASAN_OPTIONS=detect_leaks=1 TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" "$OUT/selftest_$v"
  CAKE_ENGINE_LIB="$OUT/libstub_engine_$v.so" ASAN_OPTIONS=detect_leaks=1 \
    TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" "$OUT/worker_selftest_$v"
done
