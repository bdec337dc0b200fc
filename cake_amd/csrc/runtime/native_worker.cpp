// Native text worker (see native_worker.h).
#include "native_worker.h"

#include <dlfcn.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../engine/llama_engine.h"
#include "../engine/sd_engine.h"
#include "server.h"

namespace cake {
namespace {

// <root>/cake_amd/lib/libcake_engine.so: next to the library / executable holding this
// (CAKE_ENGINE_LIB overrides: the host self-test's stub engine)
std::string engine_path() {
  if (const char* e = std::getenv("CAKE_ENGINE_LIB"); e && *e) return e;
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
  using InfoFn = int32_t (*)(void*, int32_t*);
  using CloseFn = void (*)(void*);
  auto open_layers = reinterpret_cast<OpenLayers>(dlsym(h, "cake_engine_open_layers"));
  auto forward = reinterpret_cast<Forward>(dlsym(h, "cake_engine_forward"));
  auto drop = reinterpret_cast<Drop>(dlsym(h, "cake_engine_drop_session"));
  auto einfo = reinterpret_cast<InfoFn>(dlsym(h, "cake_engine_info"));
  auto eclose = reinterpret_cast<CloseFn>(dlsym(h, "cake_engine_close"));
  if (!open_layers || !forward || !drop || !einfo || !eclose) {
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
  int32_t einf[8] = {0};
  einfo(eng, einf);
  const uint64_t hidden = (uint64_t)einf[1];  // the model width every Batch row must have
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
  auto srv = std::make_unique<WorkerServer>(host, port, info, node.name);
  WorkerServer& server = *srv;
  std::mutex mu;  // one compute at a time (the GPU stream is shared)
  server.set_compute([&](uint64_t session, const std::vector<BatchItem>& ops,
                         const RawTensor& x) {
    OpResult r;
    try {
      // the engine reads and writes T rows of exactly `hidden` floats: a client tensor of
      // another width (or a byte count that disagrees with its shape) is refused here,
      // before any host buffer is sized from it
      const uint64_t H = x.shape.empty() ? 0 : x.shape.back();
      if (H != hidden)
        throw std::runtime_error("hidden width " + std::to_string(H) + " != the model's " +
                                 std::to_string(hidden));
      uint64_t n = 1;
      for (auto d : x.shape) {
        if (d != 0 && n > (uint64_t)INT32_MAX * hidden / d)
          throw std::runtime_error("tensor too large");
        n *= d;
      }
      if (n == 0 || n % H != 0 || n / H > (uint64_t)INT32_MAX)
        throw std::runtime_error("tensor is not whole rows of the model width");
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
        if (pos > (uint64_t)INT32_MAX) throw std::runtime_error("index_pos out of range");
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
  if (o.on_serving) o.on_serving(server);
  server.serve();
  srv.reset();  // stops and joins every connection thread: no compute left in flight
  eclose(eng);
  return 0;
}

namespace {

// any numeric wire tensor -> f32 values (ids arrive as integers, packs as f32)
std::vector<float> as_f32(const RawTensor& x) {
  uint64_t n = 1;
  for (auto d : x.shape) n *= d;
  std::vector<float> v(n);
  const uint8_t* p = x.data;
  auto need = [&](uint64_t es) {
    if (x.nbytes != n * es) throw std::runtime_error("tensor byte size does not match its shape");
  };
  if (x.dtype == "f32") {
    need(4);
    std::memcpy(v.data(), p, n * 4);
  } else if (x.dtype == "f16" || x.dtype == "bf16") {
    need(2);
    const uint16_t* h = reinterpret_cast<const uint16_t*>(p);
    for (uint64_t i = 0; i < n; ++i) v[i] = half_to_f32(h[i], x.dtype == "bf16");
  } else if (x.dtype == "i64") {
    need(8);
    for (uint64_t i = 0; i < n; ++i) { int64_t t; std::memcpy(&t, p + 8 * i, 8); v[i] = (float)t; }
  } else if (x.dtype == "u32" || x.dtype == "i32") {
    need(4);
    for (uint64_t i = 0; i < n; ++i) {
      uint32_t t;
      std::memcpy(&t, p + 4 * i, 4);
      v[i] = x.dtype == "u32" ? (float)t : (float)(int32_t)t;
    }
  } else if (x.dtype == "u8") {
    need(1);
    for (uint64_t i = 0; i < n; ++i) v[i] = (float)p[i];
  } else {
    throw std::runtime_error("unsupported tensor dtype " + x.dtype);
  }
  return v;
}

struct Packed {  // util.rs pack: [n, ndim, dims..., data..., ndim, ...]
  std::vector<std::vector<uint64_t>> shapes;
  std::vector<const float*> data;
};

// a pack header value: a finite, non-negative integer below 2^31 (anything else is a
// malformed request, and casting it would be undefined behaviour)
size_t pack_dim(float v) {
  if (!(v >= 0.f) || v > 2147483647.f || v != std::floor(v))
    throw std::runtime_error("malformed packed tensor header");
  return (size_t)v;
}

Packed unpack(const std::vector<float>& f) {
  Packed out;
  if (f.empty()) throw std::runtime_error("empty packed tensor");
  const size_t n = pack_dim(f[0]);
  size_t i = 1;
  for (size_t k = 0; k < n; ++k) {
    if (i >= f.size()) throw std::runtime_error("truncated packed tensor");
    const size_t nd = pack_dim(f[i++]);
    std::vector<uint64_t> shp;
    uint64_t numel = 1;
    for (size_t d = 0; d < nd; ++d) {
      if (i >= f.size()) throw std::runtime_error("truncated packed tensor");
      shp.push_back(pack_dim(f[i++]));
      if (shp.back() != 0 && numel > f.size() / shp.back())
        throw std::runtime_error("truncated packed tensor");
      numel *= shp.back();
    }
    if (numel > f.size() - i) throw std::runtime_error("truncated packed tensor");
    out.shapes.push_back(shp);
    out.data.push_back(f.data() + i);
    i += numel;
  }
  return out;
}

// number of elements of one unpacked item
uint64_t numel_of(const std::vector<uint64_t>& s) {
  uint64_t n = 1;
  for (auto d : s) n *= d;
  return n;
}

const char* kSdParts[4] = {"unet", "vae", "clip", "clip2"};

}  // namespace

bool native_sd_components(const TopoNode& node) {
  if (node.layers.empty()) return false;
  for (const auto& l : node.layers)
    if (std::find(std::begin(kSdParts), std::end(kSdParts), l) == std::end(kSdParts)) return false;
  return true;
}

int run_native_sd_worker(const NativeWorkerOpts& o, const TopoNode& node) {
  const std::string tag = o.log_tag;
  const std::string lib = engine_path();
  void* h = dlopen(lib.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "%s: %s\n", tag.c_str(), dlerror());
    return 1;
  }
  using Open = void* (*)(const char*, const CakeSdOpts*, char*, int32_t);
  using Text = int32_t (*)(void*, int32_t, const int32_t*, int32_t, float*, char*, int32_t);
  using Unet = int32_t (*)(void*, const float*, int32_t, float, const float*, float*, char*, int32_t);
  using Vae = int32_t (*)(void*, const float*, float*, char*, int32_t);
  using Info = void (*)(void*, int32_t*);
  using Close = void (*)(void*);
  auto vae_enc = reinterpret_cast<Vae>(dlsym(h, "cake_sd_vae_encode"));
  auto open = reinterpret_cast<Open>(dlsym(h, "cake_sd_open"));
  auto text = reinterpret_cast<Text>(dlsym(h, "cake_sd_text"));
  auto unet = reinterpret_cast<Unet>(dlsym(h, "cake_sd_unet"));
  auto vae = reinterpret_cast<Vae>(dlsym(h, "cake_sd_vae_decode"));
  auto info = reinterpret_cast<Info>(dlsym(h, "cake_sd_info"));
  auto sclose = reinterpret_cast<Close>(dlsym(h, "cake_sd_close"));
  if (!open || !text || !unet || !vae || !vae_enc || !info || !sclose) {
    std::fprintf(stderr, "%s: SD engine symbols missing in %s\n", tag.c_str(), lib.c_str());
    return 1;
  }
  if (!native_sd_components(node)) {
    std::fprintf(stderr, "%s: worker %s serves units the native SD worker does not\n",
                 tag.c_str(), node.name.c_str());
    return 2;
  }
  int parts = 0;
  for (const auto& l : node.layers)
    for (int k = 0; k < 4; ++k)
      if (l == kSdParts[k]) parts |= 1 << k;
  CakeSdOpts so{};
  so.version = o.sd_version.empty() ? nullptr : o.sd_version.c_str();
  so.width = o.sd_width;
  so.height = o.sd_height;
  so.dtype = o.bf16 ? 0 : 1;
  so.device = o.device;
  so.autotune = 1;
  so.parts = parts;
  const char** pp[4] = {&so.unet_path, &so.vae_path, &so.clip_path, &so.clip2_path};
  for (int k = 0; k < 4; ++k) *pp[k] = o.sd_paths[k].empty() ? nullptr : o.sd_paths[k].c_str();
  char err[1024] = {0};
  void* eng = open(o.model_dir.c_str(), &so, err, sizeof(err));
  if (!eng) {
    std::fprintf(stderr, "%s: native SD worker: %s\n", tag.c_str(), err);
    return 1;
  }
  int32_t inf[6];
  info(eng, inf);
  WorkerInfo wi;
  wi.version = "0.1.0";
  wi.dtype = o.bf16 ? "bf16" : "f16";
  wi.os = "linux";
  wi.arch = "x86_64";
  wi.device = "rocm";
  wi.device_idx = (uint64_t)o.device;
  std::string host;
  int port = 0;
  {
    const auto c = o.address.rfind(':');
    host = c == std::string::npos ? o.address : o.address.substr(0, c);
    port = c == std::string::npos ? 10128 : std::atoi(o.address.c_str() + c + 1);
    if (host.empty()) host = "0.0.0.0";
  }
  auto srv = std::make_unique<WorkerServer>(host, port, wi, node.name);
  WorkerServer& server = *srv;
  std::mutex mu;
  std::mt19937 rng(0x5eedu);  // VAE posterior samples (parity with torch's stream unpinned)
  const int W = inf[0], H = inf[1], Dc = inf[2];
  server.set_compute([&](uint64_t, const std::vector<BatchItem>& ops, const RawTensor& x) {
    OpResult r;
    try {
      if (ops.size() != 1) throw std::runtime_error("one SD component per request");
      const std::string& name = ops[0].layer_name;
      const std::vector<float> f = as_f32(x);
      std::lock_guard<std::mutex> g(mu);
      char e2[512] = {0};
      std::vector<float> out;
      if (name == "clip" || name == "clip2") {
        if (f.size() % 77) throw std::runtime_error("token ids must be [B, 77]");
        const int B = (int)(f.size() / 77);
        std::vector<int32_t> ids(f.size());
        for (size_t i = 0; i < f.size(); ++i) ids[i] = (int32_t)f[i];
        const int D = name == "clip" ? inf[4] : inf[5];
        out.resize((size_t)B * 77 * D);
        if (text(eng, name == "clip" ? 0 : 1, ids.data(), B, out.data(), e2, sizeof(e2)))
          throw std::runtime_error(e2);
        r.shape = {(uint64_t)B, 77, (uint64_t)D};
      } else if (name == "unet") {
        const Packed pk = unpack(f);
        if (pk.shapes.size() != 3 || pk.shapes[0].size() != 4 || numel_of(pk.shapes[2]) < 1)
          throw std::runtime_error("unet expects pack([latents, text_embeddings, timestep])");
        const auto& ls = pk.shapes[0];
        const int B = (int)ls[0];
        if ((int)ls[1] != 4 || (int)ls[2] != H / 8 || (int)ls[3] != W / 8)
          throw std::runtime_error("latents " + std::to_string(ls[2]) + "x" +
                                   std::to_string(ls[3]) + " do not match the engine's " +
                                   std::to_string(W) + "x" + std::to_string(H) + " (--sd-width/height)");
        uint64_t ne = 1;
        for (auto d : pk.shapes[1]) ne *= d;
        if (ne != (uint64_t)B * 77 * Dc) throw std::runtime_error("text embedding shape mismatch");
        out.resize((size_t)B * 4 * (H / 8) * (W / 8));
        if (unet(eng, pk.data[0], B, pk.data[2][0], pk.data[1], out.data(), e2, sizeof(e2)))
          throw std::runtime_error(e2);
        r.shape = ls;
      } else if (name == "vae") {
        const Packed pk = unpack(f);
        if (pk.shapes.size() != 2 || numel_of(pk.shapes[0]) < 1)
          throw std::runtime_error("vae expects pack([direction, x])");
        if (pk.data[0][0] == 1.0f) {  // encode: the posterior sample of the image
          const auto& is = pk.shapes[1];
          if (is.size() != 4 || is[0] != 1 || is[1] != 3 || (int)is[2] != H || (int)is[3] != W)
            throw std::runtime_error("vae encode expects [1, 3, H, W] at the engine's resolution");
          const size_t nl = (size_t)4 * (H / 8) * (W / 8);
          std::vector<float> mo(2 * nl);
          if (vae_enc(eng, pk.data[1], mo.data(), e2, sizeof(e2))) throw std::runtime_error(e2);
          // mean + exp(logvar / 2) eps (vae.py encode; the worker's own seeded normals)
          std::normal_distribution<float> nd(0.f, 1.f);
          out.resize(nl);
          for (size_t i = 0; i < nl; ++i) {
            const float lv = std::min(20.f, std::max(-30.f, mo[nl + i]));
            out[i] = mo[i] + std::exp(0.5f * lv) * nd(rng);
          }
          r.shape = {1, 4, (uint64_t)(H / 8), (uint64_t)(W / 8)};
          r.dtype = "f32";
          r.data.assign(reinterpret_cast<const char*>(out.data()), out.size() * 4);
          return r;
        }
        const auto& zs = pk.shapes[1];
        if (zs.size() != 4 || zs[0] != 1 || zs[1] != 4 || (int)zs[2] != H / 8 || (int)zs[3] != W / 8)
          throw std::runtime_error("vae decode expects [1, 4, h, w] at the engine's resolution");
        out.resize((size_t)3 * H * W);
        if (vae(eng, pk.data[1], out.data(), e2, sizeof(e2))) throw std::runtime_error(e2);
        r.shape = {1, 3, (uint64_t)H, (uint64_t)W};
      } else {
        throw std::runtime_error("unknown SD component " + name);
      }
      r.dtype = "f32";
      r.data.assign(reinterpret_cast<const char*>(out.data()), out.size() * 4);
    } catch (const std::exception& e) {
      r.error = e.what();
    }
    return r;
  });
  server.set_drop([](uint64_t) {});
  server.set_reset([](uint64_t) {});
  server.set_log([tag](const std::string& m) { std::fprintf(stderr, "[%s] %s\n", tag.c_str(), m.c_str()); });
  std::string units;
  for (const auto& l : node.layers) units += (units.empty() ? "" : ",") + l;
  std::fprintf(stderr, "[%s] native SD worker %s: %s (%dx%d) on device %d, listening on %s:%d\n",
               tag.c_str(), node.name.c_str(), units.c_str(), W, H, o.device, host.c_str(),
               server.port());
  if (o.on_serving) o.on_serving(server);
  server.serve();
  srv.reset();  // stops and joins every connection thread
  sclose(eng);
  return 0;
}

}  // namespace cake
