// Native text worker: the WorkerServer control plane (server.cpp) over the native engine
// (libcake_engine.so, dlopen'ed): only the node's layers, one KV cache per master
// connection, no interpreter.  Reference: cake-core/src/cake/worker.rs:150-303.  Shared
// by cake-cli --mode worker and the embeddable cake_start_worker (capi.cpp).
#pragma once

#include <functional>
#include <string>

#include "topology.h"

namespace cake {

class WorkerServer;

struct NativeWorkerOpts {
  std::string model_dir;
  std::string address = "0.0.0.0:10128";
  int device = 0;
  int max_seq = 4096;
  bool bf16 = false;  // the reference's default dtype is f16
  std::string log_tag = "cake-cli";
  // image model (run_native_sd_worker): version ("" = cake_sd.json / v1-5), resolution
  // (0 = the version's), component file overrides (unet, vae, clip, clip2)
  std::string sd_version;
  int sd_width = 0, sd_height = 0;
  std::string sd_paths[4];
  // called once the server listens, before it blocks in serve() (the host self-test
  // takes the server here to stop it: csrc/tests/worker_selftest.cpp)
  std::function<void(WorkerServer&)> on_serving;
};

// Serve `node` until the server stops; the exit code (1 = engine failure, 2 = no layers).
int run_native_worker(const NativeWorkerOpts& o, const TopoNode& node);
// Native SD worker: serves the node's components (unet, clip, clip2, vae encode / decode)
// from the native SD engine (sd_engine.cpp) with the reference's packed-tensor SingleOp
// interface (sd_shardable.rs:29-45, unet.rs:81-100, vae.rs:87-108); the VAE posterior
// sample uses the worker's own seeded normals.
int run_native_sd_worker(const NativeWorkerOpts& o, const TopoNode& node);
// every unit of the node is an SD component the native worker serves
bool native_sd_components(const TopoNode& node);
// libcake_engine.so next to this library / executable exists and a GPU is present
bool native_engine_available();

}  // namespace cake
