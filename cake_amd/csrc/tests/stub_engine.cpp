// Host-only stand-in for libcake_engine.so (no GPU, no HIP): the C ABI the native
// workers dlopen (native_worker.cpp), with deterministic host math, so the worker's
// threaded control plane can run under ASan+UBSan and TSan (worker_selftest.cpp,
// scripts/sanitize_runtime.sh).
//
// Text: layer l at position p adds (l + 1) * 0.5 + p * 0.25 to every element of the
// row; every session keeps the positions it has seen (a KV cache stand-in), checked
// for contiguity.  SD: the components return a fixed function of their inputs.  Both
// count calls that overlap (the worker must serialise compute on its engine) and
// buffer sizes the worker passes (every read / write is bounds-checked by ASan against
// the worker's own std::vector allocations).
#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../engine/llama_engine.h"
#include "../engine/sd_engine.h"

#define STUB_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kH = 64, kL = 8, kS = 256, kV = 128;

struct Busy {  // counts overlapping calls into one engine
  std::atomic<int>& n;
  std::atomic<int>& overlaps;
  Busy(std::atomic<int>& c, std::atomic<int>& o) : n(c), overlaps(o) {
    if (n.fetch_add(1) != 0) overlaps.fetch_add(1);
  }
  ~Busy() { n.fetch_sub(1); }
};

struct TextEngine {
  std::vector<int> owned;
  std::map<uint64_t, int> kv_len;  // session -> positions written
  std::atomic<int> in_flight{0}, overlaps{0};
};

struct SdEngine {
  std::atomic<int> in_flight{0}, overlaps{0};
};

std::atomic<int> g_overlaps{0};  // summed over every closed engine

void put(char* err, int32_t n, const std::string& m) {
  if (err && n > 0) std::snprintf(err, (size_t)n, "%s", m.c_str());
}

}  // namespace

STUB_API void* cake_engine_open_layers(const char*, const CakeEngineOpts* o, const int32_t* layers,
                                       int32_t n, char* err, int32_t errlen) {
  if (!o || !layers || n <= 0) {
    put(err, errlen, "bad arguments");
    return nullptr;
  }
  auto* e = new TextEngine;
  e->owned.assign(layers, layers + n);
  return e;
}

STUB_API int32_t cake_engine_forward(void* h, uint64_t session, const int32_t* layers, int32_t n,
                                     int32_t pos0, float* hidden, int32_t T, char* err,
                                     int32_t errlen) {
  auto* e = static_cast<TextEngine*>(h);
  Busy b(e->in_flight, e->overlaps);
  if (T < 1 || pos0 < 0 || (int64_t)pos0 + T > kS) {
    put(err, errlen, "positions exceed the KV cache");
    return 1;
  }
  for (int i = 0; i < n; ++i) {
    bool mine = false;
    for (int l : e->owned) mine |= l == layers[i];
    if (!mine) {
      put(err, errlen, "layer " + std::to_string(layers[i]) + " is not served here");
      return 1;
    }
  }
  int& len = e->kv_len[session];
  if (pos0 > len) {  // a gap in the cache
    put(err, errlen, "position " + std::to_string(pos0) + " after a gap (cache holds " +
                         std::to_string(len) + ")");
    return 1;
  }
  len = pos0 + T;
  for (int i = 0; i < n; ++i)
    for (int t = 0; t < T; ++t)
      for (int c = 0; c < kH; ++c)  // reads and writes exactly T * H floats
        hidden[(size_t)t * kH + c] += (layers[i] + 1) * 0.5f + (pos0 + t) * 0.25f;
  return 0;
}

STUB_API void cake_engine_drop_session(void* h, uint64_t session) {
  auto* e = static_cast<TextEngine*>(h);
  Busy b(e->in_flight, e->overlaps);
  e->kv_len.erase(session);
}

STUB_API int32_t cake_engine_info(void* h, int32_t* o) {
  if (!h || !o) return 1;
  const int32_t v[8] = {kV, kH, kL, 4, 1, kH / 4, 4 * kH, kS};
  std::memcpy(o, v, sizeof(v));
  return 0;
}

STUB_API void cake_engine_close(void* h) {
  auto* e = static_cast<TextEngine*>(h);
  g_overlaps += e->overlaps.load();
  delete e;
}

// overlapping engine calls seen by every closed engine (the self-test's check that the
// worker serialises compute)
STUB_API int32_t stub_engine_overlaps() { return g_overlaps.load(); }

// ---- SD ------------------------------------------------------------------------------
constexpr int kW = 64, kHt = 64, kDc = 16, kD1 = 8, kD2 = 8;

STUB_API void* cake_sd_open(const char*, const CakeSdOpts*, char*, int32_t) { return new SdEngine; }
STUB_API void cake_sd_close(void* h) {
  auto* e = static_cast<SdEngine*>(h);
  g_overlaps += e->overlaps.load();
  delete e;
}
STUB_API void cake_sd_info(void*, int32_t* out6) {
  const int32_t v[6] = {kW, kHt, kDc, 1, kD1, kD2};
  std::memcpy(out6, v, sizeof(v));
}
STUB_API int32_t cake_sd_text(void* h, int32_t which, const int32_t* ids, int32_t B, float* out,
                              char*, int32_t) {
  auto* e = static_cast<SdEngine*>(h);
  Busy b(e->in_flight, e->overlaps);
  const int D = which == 0 ? kD1 : kD2;
  for (int i = 0; i < B * 77; ++i)
    for (int d = 0; d < D; ++d) out[(size_t)i * D + d] = (float)ids[i] + 0.01f * d;
  return 0;
}
STUB_API int32_t cake_sd_unet(void* h, const float* sample, int32_t B, float t, const float* ctx,
                              float* out, char*, int32_t) {
  auto* e = static_cast<SdEngine*>(h);
  Busy b(e->in_flight, e->overlaps);
  const size_t n = (size_t)B * 4 * (kHt / 8) * (kW / 8);
  float c = 0.f;
  for (size_t i = 0; i < (size_t)B * 77 * kDc; ++i) c += ctx[i];
  for (size_t i = 0; i < n; ++i) out[i] = 0.5f * sample[i] + t + 1e-6f * c;
  return 0;
}
STUB_API int32_t cake_sd_vae_decode(void* h, const float* z, float* img, char*, int32_t) {
  auto* e = static_cast<SdEngine*>(h);
  Busy b(e->in_flight, e->overlaps);
  const size_t nz = (size_t)4 * (kHt / 8) * (kW / 8);
  for (size_t i = 0; i < (size_t)3 * kHt * kW; ++i) img[i] = z[i % nz];
  return 0;
}
STUB_API int32_t cake_sd_vae_encode(void* h, const float* img, float* moments, char*, int32_t) {
  auto* e = static_cast<SdEngine*>(h);
  Busy b(e->in_flight, e->overlaps);
  const size_t nl = (size_t)4 * (kHt / 8) * (kW / 8);
  for (size_t i = 0; i < nl; ++i) {
    moments[i] = img[i];
    moments[nl + i] = -2.f;
  }
  const volatile float last = img[(size_t)3 * kHt * kW - 1];  // the whole image is readable
  (void)last;
  return 0;
}
