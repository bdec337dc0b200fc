// Embeddable worker entry point (C ABI).
//
// Counterpart of the reference's uniffi export
// `start_worker(name, model_path, topology_path, model_type)`
// (cake-ios/src/lib.rs:6-87), which runs a worker on 0.0.0.0:10128 with
// default args inside the calling process.  Same here: the worker runs IN this
// process — native WorkerServer control plane, compute runtime in the embedded
// interpreter (embed.cpp; an interpreter the host process already runs is
// reused) — and the call returns the worker's exit code when it stops.
#include <string>

#include "embed.h"

extern "C" __attribute__((visibility("default"))) int cake_start_worker(
    const char* name, const char* model_path, const char* topology_path, const char* model_type,
    const char* address) {
  using cake::PyArg;
  cake::PyArgs o;
  o["mode"] = PyArg{PyArg::kStr, "worker"};
  o["name"] = PyArg{PyArg::kStr, name ? name : "worker"};
  o["model"] = PyArg{PyArg::kStr, model_path ? model_path : "."};
  o["topology"] = PyArg{PyArg::kStr, topology_path ? topology_path : "topology.yml"};
  o["address"] = PyArg{PyArg::kStr, address && *address ? address : "0.0.0.0:10128"};
  const std::string mt = model_type ? model_type : "text";
  o["model_type"] = PyArg{PyArg::kStr, mt == "image" ? "image-model" : "text-model"};
  return cake::run_embedded(o);
}
