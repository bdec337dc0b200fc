// Native text worker: the WorkerServer control plane (server.cpp) over the native engine
// (libcake_engine.so, dlopen'ed): only the node's layers, one KV cache per master
// connection, no interpreter.  Reference: cake-core/src/cake/worker.rs:150-303.  Shared
// by cake-cli --mode worker and the embeddable cake_start_worker (capi.cpp).
#pragma once

#include <string>

#include "topology.h"

namespace cake {

struct NativeWorkerOpts {
  std::string model_dir;
  std::string address = "0.0.0.0:10128";
  int device = 0;
  int max_seq = 4096;
  bool bf16 = false;  // the reference's default dtype is f16
  std::string log_tag = "cake-cli";
};

// Serve `node` until the server stops; the exit code (1 = engine failure, 2 = no layers).
int run_native_worker(const NativeWorkerOpts& o, const TopoNode& node);
// libcake_engine.so next to this library / executable exists and a GPU is present
bool native_engine_available();

}  // namespace cake
