// Native text worker (see native_worker.h).
#include "native_worker.h"

#include <dlfcn.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../engine/llama_engine.h"
#include "server.h"

namespace cake {
namespace {

// <root>/cake_amd/lib/libcake_engine.so: next to the library / executable holding this
std::string engine_path() {
  Dl_info info{};
  if (dladdr(reinterpret_cast<void*>(&engine_path), &info) && info.dli_fname) {
    char buf[4096];
    const char* p = realpath(info.dli_fname, buf);
    std::string s = p ? p : info.dli_fname;
    const auto cut = s.find_last_of('/');
    if (cut != std::string::npos) return s.substr(0, cut) + "/libcake_engine.so";
  }
  return "libcake_engine.so";
}

// Native TCP worker (--mode worker, text model): the native WorkerServer's compute is
// the engine (only this node's layers, one KV cache per master connection), no
// interpreter at all.  Reference: cake-core/src/cake/worker.rs:150-303.
float half_to_f32(uint16_t h, bool bf16) {
  uint32_t bits;
  if (bf16) {
    bits = (uint32_t)h << 16;
  } else {
    const uint32_t s = (uint32_t)(h & 0x8000) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff;
    if (e == 0) {
      if (m == 0) bits = s;
      else {  // subnormal
        int ee = -1;
        uint32_t mm = m;
        do { ++ee; mm <<= 1; } while (!(mm & 0x400));
        bits = s | ((uint32_t)(127 - 15 - ee) << 23) | ((mm & 0x3ff) << 13);
      }
    } else if (e == 31) {
      bits = s | 0x7f800000u | (m << 13);
    } else {
      bits = s | ((e + 127 - 15) << 23) | (m << 13);
    }
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

}  // namespace

// the engine library is built and this machine exposes an AMD GPU (the KFD device node:
// checked without initialising the HIP runtime in the host process)
bool native_engine_available() {
  return access(engine_path().c_str(), R_OK) == 0 && access("/dev/kfd", R_OK | W_OK) == 0;
}

int run_native_worker(const NativeWorkerOpts& o, const TopoNode& node) {
  const std::string tag = o.log_tag;
  const std::string lib = engine_path();
  void* h = dlopen(lib.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "%s: %s\n", tag.c_str(), dlerror());
    return 1;
  }
  using OpenLayers = void* (*)(const char*, const CakeEngineOpts*, const int32_t*, int32_t, char*,
                               int32_t);
  using Forward = int32_t (*)(void*, uint64_t, const int32_t*, int32_t, int32_t, float*, int32_t,
                              char*, int32_t);
  using Drop = void (*)(void*, uint64_t);
  auto open_layers = reinterpret_cast<OpenLayers>(dlsym(h, "cake_engine_open_layers"));
  auto forward = reinterpret_cast<Forward>(dlsym(h, "cake_engine_forward"));
  auto drop = reinterpret_cast<Drop>(dlsym(h, "cake_engine_drop_session"));
  if (!open_layers || !forward || !drop) {
    std::fprintf(stderr, "%s: engine symbols missing in %s\n", tag.c_str(), lib.c_str());
    return 1;
  }
  std::vector<int32_t> layers;
  const std::string pre = "model.layers.";
  for (const auto& l : node.layers)
    if (l.rfind(pre, 0) == 0) layers.push_back((int32_t)std::atoi(l.c_str() + pre.size()));
  if (layers.empty()) {
    std::fprintf(stderr, "%s: worker %s owns no model.layers.*\n", tag.c_str(),
                 node.name.c_str());
    return 2;
  }
  const bool bf16 = o.bf16;
  CakeEngineOpts eo{};
  eo.max_seq = o.max_seq;
  eo.dtype = bf16 ? 0 : 1;
  eo.device = o.device;
  eo.steps_per_graph = 1;
  char err[1024] = {0};
  void* eng = open_layers(o.model_dir.c_str(), &eo, layers.data(), (int32_t)layers.size(),
                          err, sizeof(err));
  if (!eng) {
    std::fprintf(stderr, "%s: native worker: %s\n", tag.c_str(), err);
    return 1;
  }
  WorkerInfo info;
  info.version = "0.1.0";
  info.dtype = bf16 ? "bf16" : "f16";
  info.os = "linux";
  info.arch = "x86_64";
  info.device = "rocm";
  info.device_idx = (uint64_t)eo.device;
  std::string host;
  int port = 0;
  {
    const std::string a = o.address;
    const auto c = a.rfind(':');
    host = c == std::string::npos ? a : a.substr(0, c);
    port = c == std::string::npos ? 10128 : std::atoi(a.c_str() + c + 1);
    if (host.empty()) host = "0.0.0.0";
  }
  WorkerServer server(host, port, info, node.name);
  std::mutex mu;  // one compute at a time (the GPU stream is shared)
  server.set_compute([&](uint64_t session, const std::vector<BatchItem>& ops,
                         const RawTensor& x) {
    OpResult r;
    try {
      const uint64_t H = x.shape.empty() ? 0 : x.shape.back();
      uint64_t n = 1;
      for (auto d : x.shape) n *= d;
      std::vector<float> buf(n);
      if (x.dtype == "f32" && x.nbytes == n * 4) {
        std::memcpy(buf.data(), x.data, n * 4);
      } else if ((x.dtype == "f16" || x.dtype == "bf16") && x.nbytes == n * 2) {
        const uint16_t* p = reinterpret_cast<const uint16_t*>(x.data);
        for (uint64_t i = 0; i < n; ++i) buf[i] = half_to_f32(p[i], x.dtype == "bf16");
      } else {
        throw std::runtime_error("unsupported tensor " + x.dtype);
      }
      const int T = H ? (int)(n / H) : 0;
      std::lock_guard<std::mutex> g(mu);
      size_t i = 0;
      while (i < ops.size()) {  // consecutive ops at one position -> one engine call
        const uint64_t pos = ops[i].index_pos;
        std::vector<int32_t> ls;
        for (; i < ops.size() && ops[i].index_pos == pos; ++i) {
          const std::string& nm = ops[i].layer_name;
          if (nm.rfind(pre, 0) != 0) throw std::runtime_error("not a layer: " + nm);
          ls.push_back((int32_t)std::atoi(nm.c_str() + pre.size()));
        }
        char e2[512] = {0};
        if (forward(eng, session, ls.data(), (int32_t)ls.size(), (int32_t)pos, buf.data(), T, e2,
                    sizeof(e2)))
          throw std::runtime_error(e2);
      }
      r.dtype = "f32";
      r.shape = x.shape;
      r.data.assign(reinterpret_cast<const char*>(buf.data()), n * 4);
    } catch (const std::exception& e) {
      r.error = e.what();
    }
    return r;
  });
  server.set_drop([&](uint64_t session) {
    std::lock_guard<std::mutex> g(mu);
    drop(eng, session);
  });
  server.set_reset([](uint64_t) {});  // positions are rewritten; nothing to clear
  server.set_log([tag](const std::string& m) { std::fprintf(stderr, "[%s] %s\n", tag.c_str(), m.c_str()); });
  std::fprintf(stderr, "[%s] native worker %s: %zu layers on device %d, listening on %s:%d\n",
               tag.c_str(), node.name.c_str(), layers.size(), eo.device, host.c_str(), server.port());
  server.serve();
  return 0;
}


}  // namespace cake
