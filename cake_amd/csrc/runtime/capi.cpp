// Embeddable worker entry point (C ABI).
//
// Counterpart of the reference's uniffi export
// `start_worker(name, model_path, topology_path, model_type)`
// (cake-ios/src/lib.rs:6-87), which runs a worker on 0.0.0.0:10128 with
// default args inside the calling process.  Same here: the worker runs IN this
// process and the call returns the worker's exit code when it stops.  Text and image
// workers are the native ones (WorkerServer over the native Llama / SD engines,
// native_worker.cpp; no interpreter); CAKE_NATIVE=0 (and nodes with units the native
// SD worker does not serve) run the compute runtime in the embedded interpreter
// (embed.cpp; an interpreter the host process already runs is reused).
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "embed.h"
#include "native_worker.h"
#include "topology.h"

extern "C" __attribute__((visibility("default"))) int cake_start_worker(
    const char* name, const char* model_path, const char* topology_path, const char* model_type,
    const char* address) {
  using cake::PyArg;
  const std::string mt = model_type ? model_type : "text";
  const std::string nm = name ? name : "worker";
  const std::string addr = address && *address ? address : "0.0.0.0:10128";
  const char* nat = std::getenv("CAKE_NATIVE");
  // text: the native worker in this process (engine over the WorkerServer), as
  // cake-cli --mode worker; the topology decides the layers (first node when the name
  // is not in it, worker.rs:90-104)
  if (!(nat && std::string(nat) == "0") && cake::native_engine_available()) {
    try {
      const cake::Topology topo = cake::Topology::from_path(
          topology_path ? topology_path : "topology.yml", mt != "image");
      if (topo.nodes.empty()) {
        std::fprintf(stderr, "cake_start_worker: topology has no workers\n");
        return 2;
      }
      const cake::TopoNode* nd = topo.find(nm);
      if (!nd)
        std::fprintf(stderr, "cake_start_worker: worker %s not in the topology: serving the "
                     "FIRST node '%s'\n", nm.c_str(), topo.nodes[0].name.c_str());
      cake::NativeWorkerOpts w;
      w.model_dir = model_path ? model_path : ".";
      w.address = addr;
      w.log_tag = "cake_start_worker";
      const cake::TopoNode& node = nd ? *nd : topo.nodes[0];
      if (mt != "image") return cake::run_native_worker(w, node);
      // image: the native SD worker for the components it serves (else the runtime below)
      if (cake::native_sd_components(node)) return cake::run_native_sd_worker(w, node);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "cake_start_worker: %s\n", e.what());
      return 2;
    }
  }
  cake::PyArgs o;
  o["mode"] = PyArg{PyArg::kStr, "worker"};
  o["name"] = PyArg{PyArg::kStr, nm};
  o["model"] = PyArg{PyArg::kStr, model_path ? model_path : "."};
  o["topology"] = PyArg{PyArg::kStr, topology_path ? topology_path : "topology.yml"};
  o["address"] = PyArg{PyArg::kStr, addr};
  o["model_type"] = PyArg{PyArg::kStr, mt == "image" ? "image-model" : "text-model"};
  return cake::run_embedded(o);
}
