// Native Stable Diffusion engine (see sd_engine.h): host orchestration in C++ over the
// gfx950 kernels' C entry points — what models/sd/{pipeline,shardable,unet,vae,clip,ops}.py
// and ops/{gemm,conv}.py do through PyTorch, in the same kernels and launch order (so the
// two agree to rounding; tests/test_sd_engine_gpu.py), with no interpreter, no torch
// allocator and no torch graphs.
//
//   * weights: diffusers safetensors (mmap) uploaded once in the model dtype; every
//     convolution packed NHWC [OC][KH][KW][IC] on the host during the upload, the fused
//     operands (self-attention q|k|v, cross-attention k|v, every resnet's time projection
//     stacked into one matrix, the VAE / CLIP q|k|v with their biases) loaded in place;
//   * activations: region allocators (one per component) that hand out the same
//     addresses for the same call sequence, so the eager first step and the captured
//     step graph share every buffer and a replay needs nothing from the host;
//   * tiles: the GEMM planner of ops/gemm.py (measured table + cost model), the
//     convolution variant picked per shape by timing every candidate on the first step
//     (ops/conv.py autotune) or by the cost model;
//   * schedulers: DDIM (eps / v-prediction) and Euler-ancestral step tables computed in
//     f64 as models/sd/schedulers.py does, applied on the device by sched_step.
// Reference: cake-core/src/models/sd/sd.rs:320-532 (generate_image), unet.rs:43-100,
// vae.rs:55-108, clip.rs:24-75.
#include "sd_engine.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../runtime/json.h"
#include "../runtime/net.h"
#include "../runtime/proto.h"
#include "../runtime/safetensors.h"
#include "engine_util.h"

#define CAKE_API extern "C" __attribute__((visibility("default")))

// gfx950 kernel entry points (libcake_kernels.so)
extern "C" {
int cake_cast16(int src_kind, int dt, const void* src, void* dst, size_t n, hipStream_t st);
int cake_fill_normal(int dt, void* dst, size_t n, float mean, float std, unsigned long long key,
                     hipStream_t st);
long long cake_gemm_ws_floats(int cfg, int splits, int M, int N, int K, int gated);
int cake_gemm(int dt, int epi, int cfg, int splits, const void* a, long long lda, const void* b,
              long long ldb, void* c, long long ldc, const void* bias, void* resid,
              long long ldr, float* ws, const void* zeros, int M, int N, int K, hipStream_t st);
int cake_flash_attn_ws(int dt, const void* q, const void* k, const void* v, void* o, int B, int H,
                       int Hkv, int N, int M, int D, const long long* strides, float scale,
                       int causal, int pos0, void* ws, long long ws_bytes, hipStream_t st);
int cake_attn512(int dt, const void* q, const void* k, const void* v, void* o, int B, int N, int M,
                 long long sq, long long sk, long long sv, long long so, long long bq,
                 long long bk, long long bv, long long bo, float scale, const void* zeros,
                 hipStream_t st);
int cake_groupnorm_nhwc2(int dt, const void* x, const void* x2, int Cx, void* cat,
                         const void* gamma, const void* beta, int N, int HW, int C, int G,
                         float eps, int silu_act, double* part, unsigned int* tickets,
                         float* stats, void* y, hipStream_t st);
int cake_groupnorm_nhwc_splits(int HW);
int cake_layernorm(int dt, const void* x, const void* gamma, const void* beta, long long rows,
                   int C, float eps, void* y, hipStream_t st);
int cake_conv2d_nhwc2(int dt, const void* x, const void* w, const void* bias, const float* bias2,
                      const void* resid, void* out, float* ws, const void* zeros, int N, int H,
                      int W, int IC, int OC, int KH, int KW, int stride, int pad, int up, int cfg,
                      int splits, int th, int tw, int bias2_ld, int layout, hipStream_t st);
int cake_conv1x1_small(int dt, const void* x, const void* w, const void* bias, void* out, int N,
                       int HW, int IC, int OC, int layout, hipStream_t st);
int cake_timestep_embed(int dt, const float* t_table, const int* step, int B, int dim, int flip,
                        float shift, int out16, void* out, hipStream_t st);
int cake_sched_step(int dt, float* x, const void* pred, long long n, int cfg, float guidance,
                    const void* coef, const int* step, const void* seed, void* next_in,
                    hipStream_t st);
int cake_step_advance(int* step, hipStream_t st);
int cake_scale_copy(int dt, const float* x, long long n, float scale, int dup, void* out,
                    hipStream_t st);
int cake_to_rgb8(int dt, const void* img, int B, int H, int W, int nhwc, void* out,
                 hipStream_t st);
int cake_clip_embed(int dt, const void* tok, const void* pos, const int* ids, int rows, int T,
                    int D, int V, void* out, hipStream_t st);
int cake_widen16(int dt, const void* x, long long n, float* y, hipStream_t st);
int cake_hop_alloc(size_t bytes, void** ptr);
int cake_hop_free(void* ptr);
int cake_bulk_send(const void* const* srcs, const unsigned long long* bytes,
                   const unsigned long long* offs, int nseg, void* dst_rx,
                   unsigned long long rx_bytes, unsigned int* seq, unsigned int* count,
                   hipStream_t st);
int cake_bulk_recv(const void* rx, unsigned long long bytes, void* dst, unsigned int* seq,
                   int* err, double timeout_s, hipStream_t st);
}

namespace cake {
namespace {

constexpr int kTok = 77;  // CLIP max_position_embeddings (every SD text encoder)

// ---------------------------------------------------------------------------
// configuration (models/sd/config.py: get_config / tiny_config / mini_config)
// ---------------------------------------------------------------------------
struct ClipCfg {
  int vocab = 49408, D = 768, I = 3072, L = 12, heads = 12;
  bool quick_gelu = true;
  double eps = 1e-5;
};
struct UBlock {
  int ch;
  bool attn;
  int heads, layers;
};
struct UCfg {
  std::vector<UBlock> blocks;
  int in_ch = 4, out_ch = 4, lpb = 2, ctx = 768, groups = 32;
  bool linear_proj = false, flip = true;
  double eps = 1e-5, shift = 0.0;
};
struct VCfg {
  std::vector<int> ch{128, 256, 512, 512};
  int lpb = 2, latent = 4, groups = 32, out_ch = 3;
};
struct SchedCfg {
  bool euler_a = false, vpred = false;
  double b0 = 0.00085, b1 = 0.012;
  int T = 1000, offset = 1;
  std::string spacing = "leading";
};
struct SdCfg {
  std::string version;
  int width = 512, height = 512;
  UCfg unet;
  VCfg vae;
  ClipCfg clip;
  bool xl = false;
  ClipCfg clip2;
  SchedCfg sched;
  double vae_scale = 0.18215;
  int ctx_dim() const { return clip.D + (xl ? clip2.D : 0); }
};

SdCfg make_config(const std::string& v, const std::string& arch) {
  SdCfg c;
  c.version = v;
  ClipCfg bigg;
  bigg.D = 1280; bigg.I = 5120; bigg.L = 32; bigg.heads = 20; bigg.quick_gelu = false;
  if (v == "v1-5") {
    c.unet.blocks = {{320, true, 8, 1}, {640, true, 8, 1}, {1280, true, 8, 1}, {1280, false, 8, 1}};
  } else if (v == "v2-1") {
    c.width = c.height = 768;
    c.unet.blocks = {{320, true, 5, 1}, {640, true, 10, 1}, {1280, true, 20, 1},
                     {1280, false, 20, 1}};
    c.unet.ctx = 1024;
    c.unet.linear_proj = true;
    c.clip.D = 1024; c.clip.I = 4096; c.clip.L = 23; c.clip.heads = 16; c.clip.quick_gelu = false;
    c.sched.vpred = true;
  } else if (v == "xl" || v == "turbo") {
    c.unet.blocks = {{320, false, 5, 1}, {640, true, 10, 2}, {1280, true, 20, 10}};
    c.unet.ctx = 2048;
    c.unet.linear_proj = true;
    c.xl = true;
    c.clip2 = bigg;
    if (v == "xl") {
      c.width = c.height = 1024;
    } else {
      c.sched.euler_a = true;
      c.sched.spacing = "trailing";
      c.vae_scale = 0.13025;
    }
  } else {
    throw Error("unknown sd version '" + v + "' (v1-5, v2-1, xl, turbo)");
  }
  if (arch == "mini" || arch == "tiny") {
    const bool mini = arch == "mini";
    const int a = mini ? 64 : 32, b = mini ? 128 : 64, g = mini ? 16 : 8;
    ClipCfg small;
    small.vocab = 512; small.D = a / (mini ? 1 : 1); small.I = 2 * small.D; small.L = 2;
    small.heads = 2;
    if (!mini) { small.D = 32; small.I = 64; }
    if (c.xl) {
      c.unet.blocks = {{a, false, 2, 1}, {b, true, 2, 2}};
      c.unet.ctx = mini ? 128 : 64;
      c.unet.linear_proj = true;
      c.clip = small;
      c.clip2 = small;
      c.clip2.quick_gelu = false;
    } else {
      c.unet.blocks = mini ? std::vector<UBlock>{{a, true, 2, 1}, {b, true, 2, 1}, {b, false, 2, 1}}
                           : std::vector<UBlock>{{32, true, 4, 1}, {64, true, 4, 1}, {64, false, 4, 1}};
      c.unet.ctx = mini ? 64 : 32;
      c.unet.linear_proj = v == "v2-1";
      c.clip = small;
      c.clip.quick_gelu = true;
    }
    c.unet.groups = g;
    c.vae.ch = mini ? std::vector<int>{64, 64, 128, 128} : std::vector<int>{16, 16, 32, 32};
    c.vae.lpb = 1;
    c.vae.groups = g;
    c.width = c.height = 64;
  }
  return c;
}

// ---------------------------------------------------------------------------
// schedulers (models/sd/schedulers.py; f64 host math, f32 device tables)
// ---------------------------------------------------------------------------
// torch.linspace(start, end, n) in f64: the symmetric two-sided formula
std::vector<double> linspace(double a, double b, int n) {
  std::vector<double> out(n);
  if (n == 1) { out[0] = a; return out; }
  const double step = (b - a) / (double)(n - 1);
  const int half = n / 2;
  for (int i = 0; i < n; ++i) out[i] = i < half ? a + step * i : b - step * (double)(n - 1 - i);
  return out;
}

std::vector<double> alphas_cumprod(const SchedCfg& c) {
  const auto s = linspace(std::sqrt(c.b0), std::sqrt(c.b1), c.T);
  std::vector<double> out(c.T);
  double p = 1.0;
  for (int i = 0; i < c.T; ++i) {
    const double beta = s[i] * s[i];
    p *= 1.0 - beta;
    out[i] = p;
  }
  return out;
}

struct Schedule {
  std::vector<int> ts;
  std::vector<std::array<float, 4>> coef;  // (A, B, N, S_next) per step
  double init_sigma = 1.0;
  double first_scale = 1.0;                // input scale of step 0
  std::vector<double> in_scale;            // input scale of every step (Euler-a; DDIM: 1)
};

Schedule build_schedule(const SchedCfg& c, int steps) {
  if (steps < 1) throw Error("n_steps must be >= 1");
  Schedule s;
  const auto acp = alphas_cumprod(c);
  if (!c.euler_a) {  // DDIM, eta = 0
    const int ratio = c.T / steps;
    for (int i = steps - 1; i >= 0; --i) s.ts.push_back(i * ratio + c.offset);
    for (int i = 0; i < steps; ++i) {
      const int t = s.ts[i] < (int)acp.size() ? s.ts[i] : s.ts[i] - 1;
      const int prev = t - ratio;
      const double a_t = acp[t], a_p = prev >= 0 ? acp[prev] : acp[0];
      double A, B;
      if (!c.vpred) {
        A = std::sqrt(a_p / a_t);
        B = std::sqrt(1.0 - a_p) - std::sqrt(a_p * (1.0 - a_t) / a_t);
      } else {
        A = std::sqrt(a_p * a_t) + std::sqrt((1.0 - a_p) * (1.0 - a_t));
        B = std::sqrt((1.0 - a_p) * a_t) - std::sqrt(a_p * (1.0 - a_t));
      }
      s.coef.push_back({(float)A, (float)B, 0.f, 1.f});
    }
    return s;
  }
  // Euler-ancestral (epsilon prediction)
  std::vector<double> sig(c.T);
  for (int i = 0; i < c.T; ++i) sig[i] = std::sqrt((1.0 - acp[i]) / acp[i]);
  std::vector<double> tsd;
  const double T = c.T;
  if (c.spacing == "trailing") {
    const double step = -T / steps;
    const long n = (long)std::ceil((0.0 - T) / step);
    for (long i = 0; i < n; ++i) tsd.push_back(std::nearbyint(T + step * (double)i) - 1.0);
  } else if (c.spacing == "leading") {
    const int ratio = c.T / steps;
    for (int i = steps - 1; i >= 0; --i) tsd.push_back(std::nearbyint((double)i * ratio) + c.offset);
  } else {
    auto l = linspace(0.0, T - 1.0, steps);
    tsd.assign(l.rbegin(), l.rend());
  }
  std::vector<double> sigmas;
  for (double t : tsd) {  // numpy.interp over the integer grid
    double v;
    if (t <= 0) v = sig[0];
    else if (t >= T - 1) v = sig[c.T - 1];
    else {
      const int j = (int)std::floor(t);
      const double slope = (sig[j + 1] - sig[j]) / 1.0;
      v = slope * (t - (double)j) + sig[j];
    }
    sigmas.push_back(v);
    s.ts.push_back((int)t);
  }
  sigmas.push_back(0.0);
  double mx = 0;
  for (double v : sigmas) mx = std::max(mx, v);
  s.init_sigma = std::sqrt(mx * mx + 1.0);
  auto in_scale = [&](size_t i) { return 1.0 / std::sqrt(sigmas[i] * sigmas[i] + 1.0); };
  s.first_scale = in_scale(0);
  for (size_t i = 0; i < s.ts.size(); ++i) s.in_scale.push_back(in_scale(i));
  for (size_t i = 0; i < s.ts.size(); ++i) {
    const double sf = sigmas[i], st = sigmas[i + 1];
    const double up = std::sqrt(std::max(0.0, st * st * (sf * sf - st * st) / (sf * sf)));
    const double down = std::sqrt(std::max(0.0, st * st - up * up));
    const double S = i + 1 < s.ts.size() ? in_scale(i + 1) : 1.0;
    s.coef.push_back({1.f, (float)(down - sf), (float)up, (float)S});
  }
  return s;
}

// ---------------------------------------------------------------------------
// region allocator: the same call sequence gets the same addresses (graph-stable)
// ---------------------------------------------------------------------------
struct Arena {
  struct Chunk { char* p; size_t cap; };
  std::vector<Chunk> chunks;
  size_t ci = 0, off = 0, chunk_bytes = (size_t)1 << 30;
  bool frozen = false;  // during capture: no new chunks

  void* alloc(size_t n) {
    n = (n + 255) & ~(size_t)255;
    for (;;) {
      if (ci < chunks.size()) {
        if (off + n <= chunks[ci].cap) {
          void* r = chunks[ci].p + off;
          off += n;
          return r;
        }
        ++ci;
        off = 0;
        continue;
      }
      if (frozen) throw Error("activation arena exhausted inside a graph capture");
      const size_t cap = std::max(chunk_bytes, n);
      void* p = nullptr;
      hip_check(hipMalloc(&p, cap), "hipMalloc arena");
      chunks.push_back({static_cast<char*>(p), cap});
    }
  }
  void reset() { ci = 0; off = 0; }
  void release() {
    for (auto& c : chunks) (void)hipFree(c.p);
    chunks.clear();
    reset();
  }
};

uint32_t crc32(const std::string& s) {  // zlib.crc32
  uint32_t c = 0xFFFFFFFFu;
  for (unsigned char ch : s) {
    c ^= ch;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
  }
  return c ^ 0xFFFFFFFFu;
}

float half_to_f32(uint16_t h, bool bf16) {
  uint32_t bits;
  if (bf16) {
    bits = (uint32_t)h << 16;
  } else {
    const uint32_t s = (uint32_t)(h & 0x8000) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff;
    if (e == 0) {
      if (m == 0) bits = s;
      else {
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

const char* kPartNames[] = {"unet", "vae", "clip", "clip2"};

const char* kEpiNames[] = {"store", "resid32", "add16", "swiglu", "geglu", "partial", "store32",
                           "silu", "quick_gelu", "gelu"};
enum Epi { kStore = 0, kResid32 = 1, kAdd16 = 2, kGeglu = 4, kStore32 = 6, kSilu = 7,
           kQuickGelu = 8, kGelu = 9 };

// packed convolution weight: [OC][KH][KW][IC] (16-bit), bias [OC] (OC padded to 4 for the
// VAE's RGB output; the 1x1 few-channel form keeps [OC][IC])
struct ConvW {
  uint16_t* w = nullptr;
  uint16_t* b = nullptr;
  int OC = 0, IC = 0, K = 3, OCreal = 0;
  bool small1x1 = false;
};

struct ResnetW {
  std::string name;
  int cin, cout;
  uint16_t *n1w, *n1b, *n2w, *n2b;
  ConvW c1, c2, sc;
  bool has_sc = false;
  int toff = -1;  // column offset of its time bias in the stacked projection (UNet)
};

struct AttnBlockW {   // BasicTransformerBlock
  uint16_t *n1w, *n1b, *n2w, *n2b, *n3w, *n3b;
  uint16_t* qkv;      // [3C, C] self-attention q|k|v (no bias)
  uint16_t *o1w, *o1b;
  uint16_t* q2;       // [C, C] cross-attention q
  uint16_t* kv2;      // [2C, ctx] cross-attention k|v
  uint16_t *o2w, *o2b;
  uint16_t *ffi_w, *ffi_b, *ffo_w, *ffo_b;  // [8C, C] (GEGLU), [C, 4C]
  uint16_t* kv_cache = nullptr;  // [2, 77, 2C] of the current context
};

struct TransformerW {
  int ch, heads;
  uint16_t *nw, *nb;
  uint16_t *pin_w, *pin_b, *pout_w, *pout_b;  // [C, C] (1x1 conv or linear)
  std::vector<AttnBlockW> blocks;
};

struct DownW {
  std::vector<ResnetW> res;
  std::vector<TransformerW> att;
  bool has_ds = false;
  ConvW ds;
};
struct UpW {
  std::vector<ResnetW> res;
  std::vector<TransformerW> att;
  bool has_us = false;
  ConvW us;
};

struct VaeAttnW {
  uint16_t *nw, *nb, *qkv, *qkv_b, *ow, *ob;
  int C;
};

struct ClipLayerW {
  uint16_t *ln1w, *ln1b, *qkv, *qkv_b, *ow, *ob, *ln2w, *ln2b, *f1w, *f1b, *f2w, *f2b;
};
struct ClipW {
  ClipCfg cfg;
  uint16_t *tok, *pos, *fw, *fb;
  std::vector<ClipLayerW> layers;
};

// ---------------------------------------------------------------------------
// the engine
// ---------------------------------------------------------------------------
class SdEngine {
 public:
  SdEngine(const std::string& dir, const CakeSdOpts& o, const CakeSdSplitOpts* sp = nullptr)
      : dir_(dir) {
    dev_ = o.device;
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    hip_check(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking), "hipStreamCreate");
    dt_ = o.dtype == 0 ? 0 : 1;
    init_ = o.init;
    seed_ = o.seed;
    autotune_ = o.autotune != 0;
    std::string version = o.version ? o.version : "";
    std::string arch = o.tiny ? "tiny" : "full";
    try {  // cake_sd.json of a synthetic checkpoint names its version / architecture
      const Json j = Json::parse(read_file(dir + "/cake_sd.json"));
      if (version.empty() && j.has("version")) version = j.get("version").as_string();
      if (j.has("mini") && j.get("mini").type() == Json::Bool && j.get("mini").as_bool()) arch = "mini";
      if (j.has("tiny") && j.get("tiny").type() == Json::Bool && j.get("tiny").as_bool()) arch = "tiny";
    } catch (const std::exception&) {
    }
    if (version.empty()) version = "v1-5";
    cfg_ = make_config(version, arch);
    if (o.width > 0) cfg_.width = o.width;
    if (o.height > 0) cfg_.height = o.height;
    if (cfg_.width % 8 || cfg_.height % 8) throw Error("width / height must be multiples of 8");
    if (arch == "tiny")
      throw Error("the tiny test architecture has 32-channel convolutions the HIP kernels do "
                  "not take (use the mini architecture)");
    paths_[0] = o.unet_path ? o.unet_path : "";
    paths_[1] = o.vae_path ? o.vae_path : "";
    paths_[2] = o.clip_path ? o.clip_path : "";
    paths_[3] = o.clip2_path ? o.clip2_path : "";
    parts_ = o.parts ? o.parts : 15;
    if (!cfg_.xl) parts_ &= 7;
    if (sp && sp->world > 1) {
      srank_ = sp->rank;
      sworld_ = sp->world;
      if (srank_ < 0 || srank_ >= sworld_) throw Error("split UNet: bad rank");
      if (srank_ > 0) parts_ = 1;  // the UNet runs only: text, scheduler and VAE on rank 0
      else parts_ |= 1;
    }
    {
      const char* ra[4] = {o.remote_unet, o.remote_vae, o.remote_clip, o.remote_clip2};
      remote_timeout_ = o.remote_timeout_s > 0 ? o.remote_timeout_s : 120.0;
      for (int k = 0; k < 4; ++k)
        if (ra[k] && *ra[k]) {
          if (!cfg_.xl && k == 3) continue;
          remote_[k].addr = ra[k];
          parts_ &= ~(1 << k);  // served remotely: not loaded here
        }
      for (auto& r : remote_)
        if (!r.addr.empty()) connect_remote(r);
    }
    planner_.load(pkg_dir() + "/ops/gemm_tuned.json");
    zeros_ = dalloc(256);
    hip_check(hipMemset(zeros_, 0, 256), "memset");
    gn_tickets_ = static_cast<unsigned int*>(dalloc(256 * 4));
    hip_check(hipMemset(gn_tickets_, 0, 256 * 4), "memset");
    build_and_load();
    alloc_state();
    if (sworld_ > 1) connect_split(*sp);
  }

  ~SdEngine() {
    for (auto& r : remote_)
      if (r.fd >= 0) tcp_close(r.fd);
    for (int fd : speers_) {
      try {
        Json m = Json::object();
        m.set("cmd", Json::string("exit"));
        send_json(fd, m);
      } catch (const std::exception&) {
      }
      tcp_close(fd);
    }
    if (ctl_fd_ >= 0) tcp_close(ctl_fd_);
    for (auto& c : chans_) {
      if (c.inbox) (void)cake_hop_free(c.inbox);
      if (c.peer) (void)hipIpcCloseMemHandle(c.peer);
    }
    (void)hipSetDevice(dev_);
    (void)hipStreamSynchronize(st_);
    drop_graphs();
    unet_a_.release();
    text_a_.release();
    vae_a_.release();
    if (scratch_) (void)hipFree(scratch_);
    for (void* p : owned_) (void)hipFree(p);
    (void)hipStreamDestroy(st_);
  }

  const SdCfg& cfg() const { return cfg_; }
  int dtype() const { return dt_; }

  // ------------------------------------------------------------------ generation
  void generate(const CakeSdGenArgs& a, uint8_t* rgb, float* lat_out, double* step_s,
                CakeSdResult* res) {
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    for (int k = 0; k < (cfg_.xl ? 4 : 3); ++k)
      if (!(parts_ & (1 << k)) && remote_[k].addr.empty())
        throw Error(std::string("generate: component ") + kPartNames[k] +
                    " neither loaded nor served by a worker");
    const bool guide = a.uncond != nullptr && a.guidance > 1.0f;
    if (cfg_.xl && (a.cond2 == nullptr || (guide && a.uncond2 == nullptr)))
      throw Error("xl / turbo need the second tokenizer's ids (cond2 / uncond2)");
    const int bsize = std::max(1, a.bsize);
    if (bsize > 64) throw Error("bsize above 64");
    Schedule s = build_schedule(cfg_.sched, a.n_steps);
    int first = 0;  // index in the full schedule of the first step run
    if (a.init_latents) {  // img2img: the steps from t_start on (pipeline.py t_start)
      const int t0 = std::max(0, std::min(a.t_start, a.n_steps));
      if (t0 >= a.n_steps) throw Error("img2img: no step left after t_start");
      s.first_scale = s.in_scale.empty() ? 1.0 : s.in_scale[t0];
      s.ts.erase(s.ts.begin(), s.ts.begin() + t0);
      s.coef.erase(s.coef.begin(), s.coef.begin() + t0);
      first = t0;
    }
    const int n = (int)s.ts.size();
    const int B2 = (guide ? 2 : 1) * bsize;  // UNet rows
    if (sworld_ > 1 && srank_ != 0) throw Error("generate runs on split-UNet rank 0");
    if (split_active() && B2 > rows_cap_)
      throw Error("split UNet: bsize 1 (the device inboxes hold " + std::to_string(rows_cap_) +
                  " UNet rows)");
    if (split_active() && a.intermediary > 0)
      throw Error("split UNet: intermediary images are decoded on the single-rank engine");
    ensure_rows(B2);
    const auto t0 = std::chrono::steady_clock::now();
    // ---- text context [B2, 77, ctx]: rows [uncond; cond] x bsize
    text_context(a.cond, a.uncond, a.cond2, a.uncond2, guide, bsize);
    hook_ctx_.clear();  // ctx_ / the k|v caches now hold this generation's context
    const bool unet_remote = !remote_[0].addr.empty();
    if (!unet_remote) precompute_kv(B2);
    hip_check(hipStreamSynchronize(st_), "sync");
    const auto t1 = std::chrono::steady_clock::now();
    // ---- latents, tables
    const int h = cfg_.height / 8, w = cfg_.width / 8;
    const size_t nl1 = (size_t)4 * h * w, nl = nl1 * bsize;
    std::vector<float> x(nl);
    if (a.init_latents) {
      std::memcpy(x.data(), a.init_latents, nl * 4);
    } else if (a.init_noise) {
      for (size_t i = 0; i < nl; ++i) x[i] = a.init_noise[i] * (float)s.init_sigma;
    } else {  // engine-side noise: seeded host normals (parity with torch's stream unpinned)
      std::mt19937_64 rng(a.seed);
      std::normal_distribution<float> nd(0.f, 1.f);
      for (size_t i = 0; i < nl; ++i) x[i] = nd(rng) * (float)s.init_sigma;
    }
    hip_check(hipMemcpyAsync(x_, x.data(), nl * 4, hipMemcpyHostToDevice, st_), "H2D latents");
    std::vector<float> ttab(s.ts.size());
    for (size_t i = 0; i < s.ts.size(); ++i) ttab[i] = (float)s.ts[i];
    ensure_tables((int)s.ts.size() + 1);
    hip_check(hipMemcpyAsync(ttab_, ttab.data(), ttab.size() * 4, hipMemcpyHostToDevice, st_), "H2D");
    hip_check(hipMemcpyAsync(coef_, s.coef.data(), s.coef.size() * 16, hipMemcpyHostToDevice, st_),
              "H2D");
    hip_check(hipMemsetAsync(step_, 0, 4, st_), "memset");
    const uint64_t seed = a.seed & 0x7FFFFFFFFFFFFFFFULL;
    hip_check(hipMemcpyAsync(seed_dev_, &seed, 8, hipMemcpyHostToDevice, st_), "H2D");
    k_check(cake_scale_copy(dt_, x_, (long long)nl, (float)s.first_scale, guide ? 1 : 0, inp_, st_),
            "scale_copy");
    if (split_active()) split_start(n, B2, ttab);  // the worker ranks' step loops
    // ---- denoise: step 0 eager, then one graph replay per step
    std::vector<hipEvent_t> ev(2 * n);
    for (auto& e : ev) hip_check(hipEventCreate(&e), "event");
    const auto key = std::make_tuple(guide, a.guidance, B2);
    const size_t img_bytes = (size_t)cfg_.height * cfg_.width * 3;
    std::vector<uint8_t> mid;  // intermediary images (host)
    double mid_s = 0.0;
    try {
      for (int i = 0; i < n; ++i) {
        hip_check(hipEventRecord(ev[2 * i], st_), "event");
        if (unet_remote) {
          remote_step(B2, guide, a.guidance, ttab[i]);
        } else if (i == 0 || !a.use_graph) {
          step_body(B2, guide, a.guidance);
        } else {
          auto it = graphs_.find(key);
          if (it == graphs_.end())
            it = graphs_.emplace(key, capture_step(B2, guide, a.guidance)).first;
          hip_check(hipGraphLaunch(it->second.exec, st_), "hipGraphLaunch");
        }
        hip_check(hipEventRecord(ev[2 * i + 1], st_), "event");
        // the reference decodes the latents after step i when i % intermediary == 0
        // (sd.rs intermediary_images; pipeline.py _steps_eager / on_step)
        if (a.intermediary > 0 && a.on_image && (first + i) % a.intermediary == 0) {
          const auto m0 = std::chrono::steady_clock::now();
          mid.resize(img_bytes * bsize);
          decode_images(bsize, mid.data());
          a.on_image(a.cb_ctx, first + i, bsize, mid.data());
          mid_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - m0).count();
        }
      }
      hip_check(hipStreamSynchronize(st_), "sync");
      if (split_active()) split_finish();
    } catch (...) {
      (void)hipStreamSynchronize(st_);
      for (auto& e : ev) (void)hipEventDestroy(e);
      throw;
    }
    const auto t2 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) {
      float ms = 0;
      hip_check(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]), "elapsed");
      if (step_s) step_s[i] = ms / 1e3;
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    if (lat_out) hip_check(hipMemcpy(lat_out, x_, nl * 4, hipMemcpyDeviceToHost), "D2H latents");
    // ---- decode
    decode_images(bsize, rgb);
    const auto t3 = std::chrono::steady_clock::now();
    if (res) {
      res->width = cfg_.width;
      res->height = cfg_.height;
      res->n_steps = n;
      res->text_s = std::chrono::duration<double>(t1 - t0).count();
      res->denoise_s = std::chrono::duration<double>(t2 - t1).count() - mid_s;
      res->vae_s = std::chrono::duration<double>(t3 - t2).count();
    }
  }

  // the current latents x_ ([bsize, 4, h, w] f32) -> bsize RGB images on the host
  // ([bsize, height, width, 3] u8), one VAE decode per image
  void decode_images(int bsize, uint8_t* rgb) {
    const int h = cfg_.height / 8, w = cfg_.width / 8;
    const size_t nl1 = (size_t)4 * h * w;
    const size_t img_bytes = (size_t)cfg_.height * cfg_.width * 3;
    if (!remote_[1].addr.empty()) {  // the worker's VAE: pack([0 (decode), z]) -> image
      std::vector<float> z(nl1 * bsize);
      hip_check(hipMemcpyAsync(z.data(), x_, z.size() * 4, hipMemcpyDeviceToHost, st_), "D2H");
      hip_check(hipStreamSynchronize(st_), "sync");
      for (int b = 0; b < bsize; ++b) {
        std::vector<float> zb(z.begin() + b * nl1, z.begin() + (b + 1) * nl1);
        for (auto& v : zb) v = (float)(v / cfg_.vae_scale);
        const float dir = 0.f;
        const std::vector<float> pk =
            pack({{&dir, {1}}, {zb.data(), {1, 4, (uint64_t)h, (uint64_t)w}}});
        const std::vector<float> img = remote_call(remote_[1], "vae", pk, {(uint64_t)pk.size()},
                                                   (size_t)3 * cfg_.height * cfg_.width);
        const size_t hw = (size_t)cfg_.height * cfg_.width;
        uint8_t* dst = rgb + b * img_bytes;
        for (size_t p = 0; p < hw; ++p)  // [3, H, W] in [-1, 1] -> HWC u8 (cake_to_rgb8)
          for (int c = 0; c < 3; ++c) {
            const float v = std::min(1.f, std::max(0.f, img[c * hw + p] * 0.5f + 0.5f));
            dst[p * 3 + c] = (uint8_t)(v * 255.f);
          }
      }
      return;
    }
    for (int b = 0; b < bsize; ++b) {
      vae_a_.reset();
      uint16_t* z = new16(vae_a_, nl1);
      k_check(cake_scale_copy(dt_, x_ + b * nl1, (long long)nl1, (float)(1.0 / cfg_.vae_scale), 0,
                              z, st_), "scale_copy");
      const uint16_t* img = vae_decode(z);
      uint8_t* img8 = static_cast<uint8_t*>(vae_a_.alloc(img_bytes));
      k_check(cake_to_rgb8(dt_, img, 1, cfg_.height, cfg_.width, 0, img8, st_), "to_rgb8");
      hip_check(hipMemcpyAsync(rgb + b * img_bytes, img8, img_bytes, hipMemcpyDeviceToHost, st_),
                "D2H image");
      hip_check(hipStreamSynchronize(st_), "sync");  // the VAE arena is reused next
    }
  }

  // ------------------------------------------------------------------ remote components
  // The reference's Client (client.rs:23-133) for an image topology: one connection per
  // worker, Hello -> WorkerInfo at open, a SingleOp per call with the component's name.
  struct Remote {
    std::string addr;
    int fd = -1;
  };

  void connect_remote(Remote& r) {
    std::string host;
    int port = 0;
    split_host_port(r.addr, &host, &port);
    r.fd = tcp_connect(host, port, remote_timeout_);
    tcp_set_timeout(r.fd, remote_timeout_);
    Message hello;
    hello.type = MsgType::Hello;
    const std::string body = encode_body(hello);
    send_frame(r.fd, reinterpret_cast<const uint8_t*>(body.data()), (uint32_t)body.size());
    const std::string rep = recv_frame(r.fd);
    const Message info = decode_body(reinterpret_cast<const uint8_t*>(rep.data()), rep.size());
    if (info.type != MsgType::WorkerInfo)
      throw Error("SD worker " + r.addr + " did not answer Hello with WorkerInfo");
  }

  // SingleOp `name` on f32 `x` of `shape`; the reply as f32 (16-bit replies widened)
  std::vector<float> remote_call(Remote& r, const char* name, const std::vector<float>& x,
                                 std::vector<uint64_t> shape, size_t expect) {
    Message m;
    m.type = MsgType::SingleOp;
    m.layer_name = name;
    m.x.dtype = "f32";
    m.x.shape = std::move(shape);
    m.x.data = reinterpret_cast<const uint8_t*>(x.data());
    m.x.nbytes = x.size() * 4;
    const std::string body = encode_body(m);
    send_frame(r.fd, reinterpret_cast<const uint8_t*>(body.data()), (uint32_t)body.size());
    const std::string rep = recv_frame(r.fd);
    const Message t = decode_body(reinterpret_cast<const uint8_t*>(rep.data()), rep.size());
    if (t.type == MsgType::Error) throw Error("SD worker " + r.addr + " (" + name + "): " + t.error);
    if (t.type != MsgType::Tensor) throw Error("SD worker " + r.addr + ": unexpected reply");
    uint64_t cnt = 1;
    for (auto d : t.x.shape) cnt *= d;
    if (cnt != expect)
      throw Error("SD worker " + r.addr + " (" + name + "): " + std::to_string(cnt) +
                  " values, expected " + std::to_string(expect));
    std::vector<float> out(cnt);
    if (t.x.dtype == "f32" && t.x.nbytes == cnt * 4) {
      std::memcpy(out.data(), t.x.data, cnt * 4);
    } else if ((t.x.dtype == "f16" || t.x.dtype == "bf16") && t.x.nbytes == cnt * 2) {
      for (uint64_t i = 0; i < cnt; ++i) {
        uint16_t hv;
        std::memcpy(&hv, t.x.data + 2 * i, 2);
        out[i] = half_to_f32(hv, t.x.dtype == "bf16");
      }
    } else {
      throw Error("SD worker " + r.addr + ": unsupported reply tensor " + t.x.dtype);
    }
    return out;
  }

  // util.rs pack_tensors: [n, (ndim, dims..., values...) per tensor] as f32
  struct PackItem {
    const float* data;
    std::vector<uint64_t> shape;
  };
  static std::vector<float> pack(const std::vector<PackItem>& items) {
    std::vector<float> out{(float)items.size()};
    for (const auto& it : items) {
      out.push_back((float)it.shape.size());
      uint64_t n = 1;
      for (auto d : it.shape) {
        out.push_back((float)d);
        n *= d;
      }
      out.insert(out.end(), it.data, it.data + n);
    }
    return out;
  }

  // one denoising step through the worker's UNet: the model input and context down, the
  // prediction up, then the same fused CFG + scheduler update as the local step
  void remote_step(int B2, bool guide, float guidance, float t) {
    const int h = cfg_.height / 8, w = cfg_.width / 8;
    const size_t n = (size_t)B2 * 4 * h * w, nc = (size_t)B2 * kTok * cfg_.ctx_dim();
    std::vector<float> inp(n), ctx(nc);
    float* tmp = static_cast<float*>(text_scratch((n + nc) * 4));
    k_check(cake_widen16(dt_, inp_, (long long)n, tmp, st_), "widen16");
    k_check(cake_widen16(dt_, ctx_, (long long)nc, tmp + n, st_), "widen16");
    hip_check(hipMemcpyAsync(inp.data(), tmp, n * 4, hipMemcpyDeviceToHost, st_), "D2H");
    hip_check(hipMemcpyAsync(ctx.data(), tmp + n, nc * 4, hipMemcpyDeviceToHost, st_), "D2H");
    hip_check(hipStreamSynchronize(st_), "sync");
    const std::vector<float> pk = pack({{inp.data(), {(uint64_t)B2, 4, (uint64_t)h, (uint64_t)w}},
                                        {ctx.data(), {(uint64_t)B2, kTok, (uint64_t)cfg_.ctx_dim()}},
                                        {&t, {1}}});
    const std::vector<float> pred = remote_call(remote_[0], "unet", pk, {(uint64_t)pk.size()}, n);
    unet_a_.reset();
    uint16_t* p16 = new16(unet_a_, n);
    upload16(pred.data(), n, p16);
    k_check(cake_sched_step(dt_, x_, p16, (long long)(n / (guide ? 2 : 1)), guide ? 1 : 0, guidance,
                            coef_, step_, seed_dev_, inp_, st_), "sched_step");
    k_check(cake_step_advance(step_, st_), "step_advance");
  }

  std::array<Remote, 4> remote_;  // unet, vae, clip, clip2
  double remote_timeout_ = 120.0;

  // ------------------------------------------------------------------ component hooks
  void text_component(int which, const int32_t* ids, int B, float* out) {
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    if (which == 1 && !cfg_.xl) throw Error("this version has one text encoder");
    need(which == 0 ? 4 : 8, which == 0 ? "clip" : "clip2");
    const ClipW& cw = which == 0 ? clip_ : clip2_;
    for (int b = 0; b < B; ++b) {
      text_a_.reset();
      const uint16_t* y = clip_forward(cw, ids + (size_t)b * kTok);
      widen(y, (size_t)kTok * cw.cfg.D, out + (size_t)b * kTok * cw.cfg.D);
    }
  }

  // one UNet forward (the TCP worker's unet component, tests): eager the first time for
  // a batch size (convolution autotuning), captured the second, replayed after that; the
  // cross-attention k|v are recomputed only when the context changes
  void unet_component(const float* sample, int B, float t, const float* ctx, float* out) {
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    need(1, "unet");
    if (B < 1 || B > 128) throw Error("unet hook: batch 1..128");
    ensure_rows(B);
    const int h = cfg_.height / 8, w = cfg_.width / 8;
    const size_t n = (size_t)B * 4 * h * w, nc = (size_t)B * kTok * cfg_.ctx_dim();
    upload16(sample, n, inp_);
    if (hook_ctx_.size() != nc || std::memcmp(hook_ctx_.data(), ctx, nc * 4) != 0) {
      hook_ctx_.assign(ctx, ctx + nc);
      upload16(ctx, nc, ctx_);
      precompute_kv(B);
    }
    hip_check(hipMemcpyAsync(ttab_, &t, 4, hipMemcpyHostToDevice, st_), "H2D");
    HookGraph& hg = hook_[B];
    if (hg.calls == 0 || hg.exec == nullptr) {
      if (hg.calls == 0) {
        unet_a_.reset();
        hg.out = unet_forward(inp_, B, ttab_, nullptr);
      } else {  // capture, then replay below
        unet_a_.frozen = true;
        hip_check(hipStreamBeginCapture(st_, hipStreamCaptureModeThreadLocal), "BeginCapture");
        const uint16_t* y = nullptr;
        try {
          unet_a_.reset();
          y = unet_forward(inp_, B, ttab_, nullptr);
        } catch (...) {
          hipGraph_t junk = nullptr;
          (void)hipStreamEndCapture(st_, &junk);
          if (junk) (void)hipGraphDestroy(junk);
          unet_a_.frozen = false;
          throw;
        }
        hip_check(hipStreamEndCapture(st_, &hg.g), "EndCapture");
        unet_a_.frozen = false;
        hip_check(hipGraphInstantiate(&hg.exec, hg.g, nullptr, nullptr, 0), "GraphInstantiate");
        hg.out = y;
      }
    }
    if (hg.exec) hip_check(hipGraphLaunch(hg.exec, st_), "hipGraphLaunch");
    ++hg.calls;
    widen(hg.out, n, out);
  }

  void vae_encode_component(const float* img, float* moments) {
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    need(2, "vae");
    vae_a_.reset();
    const size_t n = (size_t)3 * cfg_.height * cfg_.width;
    uint16_t* x = new16(vae_a_, n);
    upload16(img, n, x);
    const uint16_t* y = vae_encode(x);
    widen(y, (size_t)2 * cfg_.vae.latent * (cfg_.height / 8) * (cfg_.width / 8), moments);
  }

  // img2img with the topology's VAE worker: pack([1 (encode), img]) -> the latent SAMPLE
  // [1, 4, h, w] (the worker draws the posterior noise, as the Python client path does)
  void vae_encode_remote(const float* img, float* sample) {
    if (remote_[1].addr.empty()) throw Error("no remote VAE in this engine");
    const float dir = 1.f;
    const std::vector<float> pk = pack(
        {{&dir, {1}}, {img, {1, 3, (uint64_t)cfg_.height, (uint64_t)cfg_.width}}});
    const size_t nl = (size_t)4 * (cfg_.height / 8) * (cfg_.width / 8);
    const std::vector<float> y = remote_call(remote_[1], "vae", pk, {(uint64_t)pk.size()}, nl);
    std::copy(y.begin(), y.end(), sample);
  }

  void vae_component(const float* zin, float* img) {
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    const int h = cfg_.height / 8, w = cfg_.width / 8;
    if (!remote_[1].addr.empty()) {  // the topology's VAE worker: pack([0 (decode), z])
      const float dir = 0.f;
      const std::vector<float> pk =
          pack({{&dir, {1}}, {zin, {1, 4, (uint64_t)h, (uint64_t)w}}});
      const std::vector<float> y = remote_call(remote_[1], "vae", pk, {(uint64_t)pk.size()},
                                               (size_t)3 * cfg_.height * cfg_.width);
      std::copy(y.begin(), y.end(), img);
      return;
    }
    need(2, "vae");
    vae_a_.reset();
    uint16_t* z = new16(vae_a_, (size_t)4 * h * w);
    upload16(zin, (size_t)4 * h * w, z);
    const uint16_t* y = vae_decode(z);
    widen(y, (size_t)3 * cfg_.height * cfg_.width, img);
  }

 private:
  // ------------------------------------------------------------------ memory
  void* dalloc(size_t bytes) {
    void* p = nullptr;
    hip_check(hipMalloc(&p, std::max<size_t>(bytes, 256)), "hipMalloc");
    owned_.push_back(p);
    return p;
  }
  uint16_t* dalloc16(size_t n) { return static_cast<uint16_t*>(dalloc(n * 2)); }
  void dfree(void* p) {
    if (!p) return;
    auto it = std::find(owned_.begin(), owned_.end(), p);
    if (it != owned_.end()) owned_.erase(it);
    (void)hipFree(p);
  }
  uint16_t* new16(Arena& a, size_t n) { return static_cast<uint16_t*>(a.alloc(n * 2)); }
  float* new32(Arena& a, size_t n) { return static_cast<float*>(a.alloc(n * 4)); }

  void upload16(const float* host, size_t n, uint16_t* dst) {
    float* tmp = static_cast<float*>(text_scratch(n * 4));
    hip_check(hipMemcpyAsync(tmp, host, n * 4, hipMemcpyHostToDevice, st_), "H2D");
    k_check(cake_cast16(2, dt_, tmp, dst, n, st_), "cast16");
    hip_check(hipStreamSynchronize(st_), "sync");
  }
  void widen(const uint16_t* src, size_t n, float* host) {
    float* tmp = static_cast<float*>(text_scratch(n * 4));
    k_check(cake_widen16(dt_, src, (long long)n, tmp, st_), "widen16");
    hip_check(hipMemcpyAsync(host, tmp, n * 4, hipMemcpyDeviceToHost, st_), "D2H");
    hip_check(hipStreamSynchronize(st_), "sync");
  }
  void* text_scratch(size_t bytes) {
    if (scratch_bytes_ < bytes) {
      if (scratch_) (void)hipFree(scratch_);
      scratch_ = nullptr;
      hip_check(hipMalloc(&scratch_, bytes), "hipMalloc scratch");
      scratch_bytes_ = bytes;
    }
    return scratch_;
  }

  // ------------------------------------------------------------------ weights
  std::string resolve(int comp) {
    static const char* rel[4] = {"unet/diffusion_pytorch_model", "vae/diffusion_pytorch_model",
                                 "text_encoder/model", "text_encoder_2/model"};
    if (!paths_[comp].empty()) return paths_[comp];
    for (const char* f : {".fp16", ""}) {
      const std::string p = dir_ + "/" + rel[comp] + f + ".safetensors";
      if (FILE* fp = std::fopen(p.c_str(), "rb")) {
        std::fclose(fp);
        return p;
      }
    }
    throw Error(std::string("no ") + rel[comp] + "[.fp16].safetensors under " + dir_);
  }

  struct Loader {
    SdEngine* e;
    std::unique_ptr<SafeTensorsFile> f;
    std::string comp;
    std::vector<uint8_t> host;

    const TensorView* find(const std::string& name) {
      if (!f) return nullptr;
      if (f->has(name)) return &f->tensor(name);
      // VAE legacy attention names (query / key / value / proj_attn)
      static const std::pair<const char*, const char*> legacy[] = {
          {".to_q.", ".query."}, {".to_k.", ".key."}, {".to_v.", ".value."},
          {".to_out.0.", ".proj_attn."}};
      for (const auto& l : legacy) {
        const auto at = name.find(l.first);
        if (at != std::string::npos) {
          std::string alt = name;
          alt.replace(at, std::strlen(l.first), l.second);
          if (f->has(alt)) return &f->tensor(alt);
        }
      }
      return nullptr;
    }

    // load `name` (numel elements in the file's layout; 4-D [O,I,1,1] accepted for 2-D)
    // into dst; pack = a conv weight [OC][IC][K][K] repacked to [OC][K][K][IC]
    void load(const std::string& name, const std::vector<int64_t>& shape, uint16_t* dst,
              bool pack = false, int pad_oc = 0) {
      size_t numel = 1;
      for (auto d : shape) numel *= (size_t)d;
      if (e->init_ == 1 || !f) {
        e->random_fill(comp + "/" + name, shape, dst, numel, pad_oc);
        return;
      }
      const TensorView* t = find(name);
      if (!t) throw Error(f->path() + ": missing tensor " + name);
      size_t n = 1;
      for (auto d : t->shape) n *= d;
      if (n != numel) throw Error(f->path() + ": " + name + " has " + std::to_string(n) +
                                  " elements, expected " + std::to_string(numel));
      int kind;
      if (t->dtype == "BF16") kind = 0;
      else if (t->dtype == "F16") kind = 1;
      else if (t->dtype == "F32") kind = 2;
      else throw Error(name + ": unsupported dtype " + t->dtype);
      const size_t es = kind == 2 ? 4 : 2;
      const uint8_t* src = t->data;
      if (pack && shape.size() == 4 && shape[2] * shape[3] > 1) {
        const int64_t OC = shape[0], IC = shape[1], KK = shape[2] * shape[3];
        host.resize(numel * es);
        for (int64_t o = 0; o < OC; ++o)
          for (int64_t i = 0; i < IC; ++i)
            for (int64_t k = 0; k < KK; ++k)
              std::memcpy(host.data() + ((o * KK + k) * IC + i) * es,
                          src + ((o * IC + i) * KK + k) * es, es);
        src = host.data();
      }
      const size_t total = (size_t)(pad_oc > 0 ? numel / shape[0] * pad_oc : numel);
      if (pad_oc > 0) hip_check(hipMemset(dst, 0, total * 2), "memset pad");
      if (kind == e->dt_) {
        hip_check(hipMemcpy(dst, src, numel * es, hipMemcpyHostToDevice), "weight H2D");
        return;
      }
      void* stage = e->text_scratch(numel * es);
      hip_check(hipMemcpy(stage, src, numel * es, hipMemcpyHostToDevice), "weight H2D");
      k_check(cake_cast16(kind, e->dt_, stage, dst, numel, e->st_), "cast16");
      hip_check(hipStreamSynchronize(e->st_), "sync");
    }
  };

  void random_fill(const std::string& key, const std::vector<int64_t>& shape, uint16_t* dst,
                   size_t numel, int pad_oc) {
    const std::string& name = key;
    const bool bias = name.size() > 5 && name.compare(name.size() - 5, 5, ".bias") == 0;
    if (pad_oc > 0) hip_check(hipMemset(dst, 0, numel / shape[0] * pad_oc * 2), "memset");
    if (bias) {
      hip_check(hipMemset(dst, 0, numel * 2), "memset");
      return;
    }
    if (shape.size() == 1) {  // norm weights: ones
      std::vector<uint16_t> ones(numel, dt_ == 0 ? 0x3F80 : 0x3C00);
      hip_check(hipMemcpy(dst, ones.data(), numel * 2, hipMemcpyHostToDevice), "H2D");
      return;
    }
    double std_;
    if (name.find("embedding") != std::string::npos) {
      std_ = name.find("token") != std::string::npos ? 0.02 : 0.01;
    } else {
      double fan = 1;
      for (size_t i = 1; i < shape.size(); ++i) fan *= (double)shape[i];
      std_ = 0.7 / std::sqrt(fan);
    }
    const unsigned long long k = seed_ * 1000003ULL + crc32(key);
    k_check(cake_fill_normal(dt_, dst, numel, 0.f, (float)std_, k, st_), "fill_normal");
  }

  uint16_t* param(Loader& L, const std::string& name, std::vector<int64_t> shape) {
    size_t n = 1;
    for (auto d : shape) n *= (size_t)d;
    uint16_t* p = dalloc16(n);
    L.load(name, shape, p);
    return p;
  }

  ConvW conv_param(Loader& L, const std::string& name, int cout, int cin, int k) {
    ConvW c;
    c.IC = cin;
    c.OC = cout;
    c.OCreal = cout;
    c.K = k;
    c.small1x1 = k == 1 && cin <= 16 && cout <= 16;
    const bool pad4 = cout < 4;
    if (pad4) c.OC = 4;
    c.w = dalloc16((size_t)c.OC * k * k * cin);
    L.load(name + ".weight", {cout, cin, k, k}, c.w, true, pad4 ? 4 : 0);
    c.b = dalloc16(c.OC);
    if (pad4) hip_check(hipMemset(c.b, 0, c.OC * 2), "memset");
    L.load(name + ".bias", {cout}, c.b);
    if (!c.small1x1 && !conv_ok(cin, c.OC, k))
      throw Error(name + ": a " + std::to_string(cin) + " -> " + std::to_string(cout) +
                  " convolution the HIP kernels do not take");
    return c;
  }

  static bool conv_ok(int IC, int OC, int k) {
    if (IC == 3 || IC == 4) return k == 3 && OC % 8 == 0 && 9 * IC * OC <= 18432;
    return IC % 64 == 0 && OC % 4 == 0;
  }

  ResnetW resnet_param(Loader& L, const std::string& name, int cin, int cout, int temb) {
    ResnetW r;
    r.name = name;
    r.cin = cin;
    r.cout = cout;
    r.n1w = param(L, name + ".norm1.weight", {cin});
    r.n1b = param(L, name + ".norm1.bias", {cin});
    r.c1 = conv_param(L, name + ".conv1", cout, cin, 3);
    r.n2w = param(L, name + ".norm2.weight", {cout});
    r.n2b = param(L, name + ".norm2.bias", {cout});
    r.c2 = conv_param(L, name + ".conv2", cout, cout, 3);
    if (cin != cout) {
      r.has_sc = true;
      r.sc = conv_param(L, name + ".conv_shortcut", cout, cin, 1);
    }
    if (temb > 0) {
      r.toff = temb_cols_;
      temb_list_.push_back({name, cout});
      temb_cols_ += cout;
    }
    return r;
  }

  TransformerW transformer_param(Loader& L, const std::string& name, int ch, int heads,
                                 int layers) {
    const UCfg& u = cfg_.unet;
    TransformerW t;
    t.ch = ch;
    t.heads = heads;
    t.nw = param(L, name + ".norm.weight", {ch});
    t.nb = param(L, name + ".norm.bias", {ch});
    auto proj = [&](const std::string& n, uint16_t*& w, uint16_t*& b) {
      w = dalloc16((size_t)ch * ch);
      if (u.linear_proj) L.load(n + ".weight", {ch, ch}, w);
      else L.load(n + ".weight", {ch, ch, 1, 1}, w);
      b = param(L, n + ".bias", {ch});
    };
    proj(name + ".proj_in", t.pin_w, t.pin_b);
    for (int i = 0; i < layers; ++i) {
      const std::string p = name + ".transformer_blocks." + std::to_string(i);
      AttnBlockW a;
      a.n1w = param(L, p + ".norm1.weight", {ch});
      a.n1b = param(L, p + ".norm1.bias", {ch});
      a.n2w = param(L, p + ".norm2.weight", {ch});
      a.n2b = param(L, p + ".norm2.bias", {ch});
      a.n3w = param(L, p + ".norm3.weight", {ch});
      a.n3b = param(L, p + ".norm3.bias", {ch});
      a.qkv = dalloc16((size_t)3 * ch * ch);
      L.load(p + ".attn1.to_q.weight", {ch, ch}, a.qkv);
      L.load(p + ".attn1.to_k.weight", {ch, ch}, a.qkv + (size_t)ch * ch);
      L.load(p + ".attn1.to_v.weight", {ch, ch}, a.qkv + (size_t)2 * ch * ch);
      a.o1w = param(L, p + ".attn1.to_out.0.weight", {ch, ch});
      a.o1b = param(L, p + ".attn1.to_out.0.bias", {ch});
      a.q2 = param(L, p + ".attn2.to_q.weight", {ch, ch});
      a.kv2 = dalloc16((size_t)2 * ch * u.ctx);
      L.load(p + ".attn2.to_k.weight", {ch, u.ctx}, a.kv2);
      L.load(p + ".attn2.to_v.weight", {ch, u.ctx}, a.kv2 + (size_t)ch * u.ctx);
      a.o2w = param(L, p + ".attn2.to_out.0.weight", {ch, ch});
      a.o2b = param(L, p + ".attn2.to_out.0.bias", {ch});
      a.ffi_w = param(L, p + ".ff.net.0.proj.weight", {8 * ch, ch});
      a.ffi_b = param(L, p + ".ff.net.0.proj.bias", {8 * ch});
      a.ffo_w = param(L, p + ".ff.net.2.weight", {ch, 4 * ch});
      a.ffo_b = param(L, p + ".ff.net.2.bias", {ch});
      a.kv_cache = dalloc16((size_t)2 * kTok * 2 * ch);
      t.blocks.push_back(a);
    }
    proj(name + ".proj_out", t.pout_w, t.pout_b);
    return t;
  }

  void need(int mask, const char* what) const {
    if ((parts_ & mask) != mask)
      throw Error(std::string("this engine was opened without the ") + what);
  }

  void build_and_load() {
    // ---------------- UNet (unet.py UNet2DConditionModel.__init__ / params)
    if (parts_ & 1) {
      Loader L{this, nullptr, "unet", {}};
      if (init_ != 1) L.f = std::make_unique<SafeTensorsFile>(resolve(0));
      const UCfg& u = cfg_.unet;
      std::vector<int> chans;
      for (const auto& b : u.blocks) chans.push_back(b.ch);
      const int C0 = chans[0], temb = C0 * 4;
      temb_dim_ = temb;
      conv_in_ = conv_param(L, "conv_in", C0, u.in_ch, 3);
      t1w_ = param(L, "time_embedding.linear_1.weight", {temb, C0});
      t1b_ = param(L, "time_embedding.linear_1.bias", {temb});
      t2w_ = param(L, "time_embedding.linear_2.weight", {temb, temb});
      t2b_ = param(L, "time_embedding.linear_2.bias", {temb});
      int cout = C0;
      for (size_t i = 0; i < u.blocks.size(); ++i) {
        const auto& b = u.blocks[i];
        const int cin = cout;
        cout = b.ch;
        DownW d;
        for (int j = 0; j < u.lpb; ++j) {
          const std::string rn = "down_blocks." + std::to_string(i) + ".resnets." + std::to_string(j);
          d.res.push_back(resnet_param(L, rn, j == 0 ? cin : cout, cout, temb));
          if (b.attn)
            d.att.push_back(transformer_param(
                L, "down_blocks." + std::to_string(i) + ".attentions." + std::to_string(j), cout,
                b.heads, b.layers));
        }
        if (i + 1 < u.blocks.size()) {
          d.has_ds = true;
          d.ds = conv_param(L, "down_blocks." + std::to_string(i) + ".downsamplers.0.conv", cout,
                            cout, 3);
        }
        down_.push_back(std::move(d));
      }
      const int cm = chans.back();
      const auto& mb = u.blocks.back();
      mid_res_[0] = resnet_param(L, "mid_block.resnets.0", cm, cm, temb);
      mid_att_ = transformer_param(L, "mid_block.attentions.0", cm, mb.heads, mb.layers);
      mid_res_[1] = resnet_param(L, "mid_block.resnets.1", cm, cm, temb);
      std::vector<int> rev(chans.rbegin(), chans.rend());
      int out_ch = rev[0];
      for (size_t i = 0; i < rev.size(); ++i) {
        const auto& b = u.blocks[u.blocks.size() - 1 - i];
        const int prev = out_ch;
        out_ch = rev[i];
        const int in_ch = rev[std::min(i + 1, rev.size() - 1)];
        UpW up;
        const int n = u.lpb + 1;
        for (int j = 0; j < n; ++j) {
          const int skip = j == n - 1 ? in_ch : out_ch;
          const int rin = j == 0 ? prev : out_ch;
          const std::string rn = "up_blocks." + std::to_string(i) + ".resnets." + std::to_string(j);
          up.res.push_back(resnet_param(L, rn, rin + skip, out_ch, temb));
          if (b.attn)
            up.att.push_back(transformer_param(
                L, "up_blocks." + std::to_string(i) + ".attentions." + std::to_string(j), out_ch,
                b.heads, b.layers));
        }
        if (i + 1 < rev.size()) {
          up.has_us = true;
          up.us = conv_param(L, "up_blocks." + std::to_string(i) + ".upsamplers.0.conv", out_ch,
                             out_ch, 3);
        }
        up_.push_back(std::move(up));
      }
      norm_out_w_ = param(L, "conv_norm_out.weight", {C0});
      norm_out_b_ = param(L, "conv_norm_out.bias", {C0});
      conv_out_ = conv_param(L, "conv_out", u.out_ch, C0, 3);
      // every resnet's time projection, stacked in resnets() order (down, mid, up): the
      // per-step time biases are ONE GEMM (unet.py _temb_all)
      tall_w_ = dalloc16((size_t)temb_cols_ * temb);
      tall_b_ = dalloc16((size_t)temb_cols_);
      for (const auto& e : temb_list_) {
        const int off = temb_off(e.first);
        L.load(e.first + ".time_emb_proj.weight", {e.second, temb}, tall_w_ + (size_t)off * temb);
        L.load(e.first + ".time_emb_proj.bias", {e.second}, tall_b_ + off);
      }
    }
    // ---------------- VAE (vae.py AutoencoderKL: the decoder, and the encoder for img2img)
    if (parts_ & 2) {
      Loader L{this, nullptr, "vae", {}};
      if (init_ != 1) L.f = std::make_unique<SafeTensorsFile>(resolve(1));
      const VCfg& v = cfg_.vae;
      {  // encoder
        e_in_ = conv_param(L, "encoder.conv_in", v.ch[0], 3, 3);
        int out = v.ch[0];
        for (size_t i = 0; i < v.ch.size(); ++i) {
          const int cin = out;
          out = v.ch[i];
          DownW d;
          for (int j = 0; j < v.lpb; ++j)
            d.res.push_back(resnet_param(L, "encoder.down_blocks." + std::to_string(i) +
                                                ".resnets." + std::to_string(j),
                                         j == 0 ? cin : out, out, 0));
          if (i + 1 < v.ch.size()) {
            d.has_ds = true;
            d.ds = conv_param(L, "encoder.down_blocks." + std::to_string(i) + ".downsamplers.0.conv",
                              out, out, 3);
          }
          e_down_.push_back(std::move(d));
        }
        for (int j = 0; j < 2; ++j)
          e_mid_[j] = resnet_param(L, "encoder.mid_block.resnets." + std::to_string(j),
                                   v.ch.back(), v.ch.back(), 0);
        e_att_ = vae_attn_param(L, "encoder.mid_block.attentions.0", v.ch.back());
        e_norm_w_ = param(L, "encoder.conv_norm_out.weight", {v.ch.back()});
        e_norm_b_ = param(L, "encoder.conv_norm_out.bias", {v.ch.back()});
        e_out_ = conv_param(L, "encoder.conv_out", 2 * v.latent, v.ch.back(), 3);
        quant_ = conv_param(L, "quant_conv", 2 * v.latent, 2 * v.latent, 1);
      }
      post_quant_ = conv_param(L, "post_quant_conv", v.latent, v.latent, 1);
      d_in_ = conv_param(L, "decoder.conv_in", v.ch.back(), v.latent, 3);
      for (int j = 0; j < 2; ++j)
        d_mid_[j] = resnet_param(L, "decoder.mid_block.resnets." + std::to_string(j), v.ch.back(),
                                 v.ch.back(), 0);
      d_att_ = vae_attn_param(L, "decoder.mid_block.attentions.0", v.ch.back());
      std::vector<int> rev(v.ch.rbegin(), v.ch.rend());
      int out = rev[0];
      for (size_t i = 0; i < rev.size(); ++i) {
        const int prev = out;
        out = rev[i];
        UpW up;
        for (int j = 0; j < v.lpb + 1; ++j)
          up.res.push_back(resnet_param(L, "decoder.up_blocks." + std::to_string(i) + ".resnets." +
                                               std::to_string(j),
                                        j == 0 ? prev : out, out, 0));
        if (i + 1 < rev.size()) {
          up.has_us = true;
          up.us = conv_param(L, "decoder.up_blocks." + std::to_string(i) + ".upsamplers.0.conv",
                             out, out, 3);
        }
        d_up_.push_back(std::move(up));
      }
      d_norm_w_ = param(L, "decoder.conv_norm_out.weight", {v.ch[0]});
      d_norm_b_ = param(L, "decoder.conv_norm_out.bias", {v.ch[0]});
      d_out_ = conv_param(L, "decoder.conv_out", v.out_ch, v.ch[0], 3);
    }
    // ---------------- text encoders (clip.py)
    if (parts_ & 4) clip_ = clip_param(2, cfg_.clip);
    if (cfg_.xl && (parts_ & 8)) clip2_ = clip_param(3, cfg_.clip2);
    hip_check(hipDeviceSynchronize(), "sync");
  }

  VaeAttnW vae_attn_param(Loader& L, const std::string& n, int C) {
    VaeAttnW a;
    a.C = C;
    a.nw = param(L, n + ".group_norm.weight", {C});
    a.nb = param(L, n + ".group_norm.bias", {C});
    a.qkv = dalloc16((size_t)3 * C * C);
    a.qkv_b = dalloc16((size_t)3 * C);
    const char* qkvn[3] = {".to_q", ".to_k", ".to_v"};
    for (int k = 0; k < 3; ++k) {
      load_linear_or_1x1(L, n + qkvn[k] + ".weight", C, C, a.qkv + (size_t)k * C * C);
      L.load(n + qkvn[k] + ".bias", {C}, a.qkv_b + (size_t)k * C);
    }
    a.ow = dalloc16((size_t)C * C);
    load_linear_or_1x1(L, n + ".to_out.0.weight", C, C, a.ow);
    a.ob = param(L, n + ".to_out.0.bias", {C});
    return a;
  }

  void load_linear_or_1x1(Loader& L, const std::string& name, int o, int i, uint16_t* dst) {
    const TensorView* t = L.f ? L.find(name) : nullptr;
    if (t && t->shape.size() == 4) L.load(name, {o, i, 1, 1}, dst);
    else L.load(name, {o, i}, dst);
  }

  int temb_off(const std::string& name) const {
    int o = 0;
    for (const auto& e : temb_list_) {
      if (e.first == name) return o;
      o += e.second;
    }
    throw Error("no time projection for " + name);
  }

  ClipW clip_param(int comp, const ClipCfg& c) {
    Loader L{this, nullptr, comp == 2 ? "clip" : "clip2", {}};
    if (init_ != 1) L.f = std::make_unique<SafeTensorsFile>(resolve(comp));
    ClipW w;
    w.cfg = c;
    const int D = c.D, I = c.I;
    w.tok = param(L, "text_model.embeddings.token_embedding.weight", {c.vocab, D});
    w.pos = param(L, "text_model.embeddings.position_embedding.weight", {kTok, D});
    w.fw = param(L, "text_model.final_layer_norm.weight", {D});
    w.fb = param(L, "text_model.final_layer_norm.bias", {D});
    for (int i = 0; i < c.L; ++i) {
      const std::string p = "text_model.encoder.layers." + std::to_string(i);
      ClipLayerW l;
      l.ln1w = param(L, p + ".layer_norm1.weight", {D});
      l.ln1b = param(L, p + ".layer_norm1.bias", {D});
      l.qkv = dalloc16((size_t)3 * D * D);
      l.qkv_b = dalloc16((size_t)3 * D);
      const char* n[3] = {"q_proj", "k_proj", "v_proj"};
      for (int k = 0; k < 3; ++k) {
        L.load(p + ".self_attn." + n[k] + ".weight", {D, D}, l.qkv + (size_t)k * D * D);
        L.load(p + ".self_attn." + n[k] + ".bias", {D}, l.qkv_b + (size_t)k * D);
      }
      l.ow = param(L, p + ".self_attn.out_proj.weight", {D, D});
      l.ob = param(L, p + ".self_attn.out_proj.bias", {D});
      l.ln2w = param(L, p + ".layer_norm2.weight", {D});
      l.ln2b = param(L, p + ".layer_norm2.bias", {D});
      l.f1w = param(L, p + ".mlp.fc1.weight", {I, D});
      l.f1b = param(L, p + ".mlp.fc1.bias", {I});
      l.f2w = param(L, p + ".mlp.fc2.weight", {D, I});
      l.f2b = param(L, p + ".mlp.fc2.bias", {D});
      w.layers.push_back(l);
    }
    return w;
  }

  void alloc_state() {
    const int h = cfg_.height / 8, w = cfg_.width / 8;
    const size_t nl = (size_t)4 * h * w;
    x_ = static_cast<float*>(dalloc(2 * nl * 4));
    inp_ = dalloc16(2 * nl);
    ctx_ = dalloc16((size_t)2 * kTok * cfg_.ctx_dim());
    seed_dev_ = dalloc(8);
    step_ = static_cast<int*>(dalloc(64));
    ensure_tables(1024);
  }

  // UNet rows the per-generation buffers hold (latents, UNet input, text context and the
  // cross-attention k|v of every transformer block): grown for bsize > 1 / larger hook
  // batches; the captured graphs point at the old buffers and are dropped
  int rows_cap_ = 2;
  void ensure_rows(int rows) {
    if (rows <= rows_cap_) return;
    hip_check(hipStreamSynchronize(st_), "sync");
    drop_graphs();
    hook_ctx_.clear();
    const int h = cfg_.height / 8, w = cfg_.width / 8;
    const size_t nl = (size_t)4 * h * w;
    dfree(x_);
    dfree(inp_);
    dfree(ctx_);
    x_ = static_cast<float*>(dalloc((size_t)rows * nl * 4));
    inp_ = dalloc16((size_t)rows * nl);
    ctx_ = dalloc16((size_t)rows * kTok * cfg_.ctx_dim());
    auto grow = [&](TransformerW& t) {
      for (auto& blk : t.blocks) {
        dfree(blk.kv_cache);
        blk.kv_cache = dalloc16((size_t)rows * kTok * 2 * t.ch);
      }
    };
    if (parts_ & 1) {
      for (auto& d : down_)
        for (auto& t : d.att) grow(t);
      grow(mid_att_);
      for (auto& u : up_)
        for (auto& t : u.att) grow(t);
    }
    rows_cap_ = rows;
  }

  void ensure_tables(int n) {
    if (n <= table_cap_) return;
    table_cap_ = n;
    ttab_ = static_cast<float*>(dalloc((size_t)n * 4));
    coef_ = static_cast<float*>(dalloc((size_t)n * 16));
    drop_graphs();  // the captured steps point at the old tables
  }

  // ------------------------------------------------------------------ ops
  float* gemm_ws(size_t n) {
    if (n > ws_n_) {
      if (unet_a_.frozen) throw Error("GEMM split-K workspace grew inside a capture");
      ws_n_ = std::max(n, (size_t)1 << 20);
      ws_ = static_cast<float*>(dalloc(ws_n_ * 4));
    }
    return ws_;
  }

  // y = epilogue(x W^T): x [M, K] (row stride lda), W [Nv, K]; out [M, N] (row stride ldc)
  void gemm(int epi, const uint16_t* x, long long lda, int M, int K, const uint16_t* w, int Nv,
            const uint16_t* bias, void* out, long long ldc, const void* resid = nullptr,
            long long ldr = 0) {
    const bool gated = epi == 3 || epi == kGeglu;
    const int N = gated ? Nv / 2 : Nv;
    const auto pl = planner_.plan_mfma(M, Nv, K, kEpiNames[epi]);  // no library path here
    float* ws = pl.second > 1
                    ? gemm_ws((size_t)cake_gemm_ws_floats(pl.first, pl.second, M, N, K, gated ? 1 : 0))
                    : nullptr;
    const bool f32out = epi == kResid32 || epi == kStore32;
    k_check(cake_gemm(dt_, epi, pl.first, pl.second, x, lda, w, K, f32out ? nullptr : out,
                      f32out ? 0 : ldc,
                      bias, f32out ? out : const_cast<void*>(resid), f32out ? ldc : ldr, ws,
                      zeros_, M, N, K, st_), "gemm");
  }

  uint16_t* group_norm(Arena& A, const uint16_t* x, const uint16_t* x2, int Cx, int N, int HW,
                       int C, const uint16_t* g, const uint16_t* b, int groups, float eps,
                       bool silu, uint16_t* cat = nullptr) {
    const int cg = C / groups;
    if (C % groups || C % 8 || C > 4096 || cg < 4 || !(cg >= 8 || 8 % cg == 0) || Cx % 8)
      throw Error("GroupNorm: unsupported C=" + std::to_string(C) + " groups=" +
                  std::to_string(groups));
    const int S = cake_groupnorm_nhwc_splits(HW);
    double* part = static_cast<double*>(A.alloc((size_t)N * S * groups * 2 * 8));
    float* stats = new32(A, (size_t)N * groups * 2);
    uint16_t* y = new16(A, (size_t)N * HW * C);
    k_check(cake_groupnorm_nhwc2(dt_, x, x2, Cx, cat, g, b, N, HW, C, groups, eps, silu ? 1 : 0,
                                 part, gn_tickets_, stats, y, st_), "groupnorm_nhwc");
    return y;
  }

  uint16_t* layer_norm(Arena& A, const uint16_t* x, long long rows, int C, const uint16_t* g,
                       const uint16_t* b, float eps) {
    uint16_t* y = new16(A, (size_t)rows * C);
    k_check(cake_layernorm(dt_, x, g, b, rows, C, eps, y, st_), "layernorm");
    return y;
  }

  // ops.attention over [B, rows, heads * D] views (row strides ldq / ldk / ldv, out dense)
  uint16_t* attention(Arena& A, const uint16_t* q, long long ldq, const uint16_t* k,
                      long long ldk, const uint16_t* v, long long ldv, int B, int N, int M,
                      int heads, int C, bool causal) {
    const int D = C / heads;
    uint16_t* o = new16(A, (size_t)B * N * C);
    const float scale = (float)(1.0 / std::sqrt((double)D));
    if (D <= 256) {
      const long long st[12] = {N * ldq, D, ldq, M * ldk, D, ldk, M * ldv, D, ldv,
                                (long long)N * C, D, C};
      void* ws = nullptr;
      long long wsb = 0;
      if (!causal) {
        const size_t need = (size_t)4 * B * heads * N * (D + 1);
        if (need > flash_ws_n_) {
          if (unet_a_.frozen) throw Error("flash workspace grew inside a capture");
          flash_ws_n_ = need;
          flash_ws_ = dalloc(need * 4);
        }
        ws = flash_ws_;
        wsb = (long long)flash_ws_n_ * 4;
      }
      k_check(cake_flash_attn_ws(dt_, q, k, v, o, B, heads, heads, N, M, D, st, scale,
                                 causal ? 1 : 0, 0, ws, wsb, st_), "flash_attn");
      return o;
    }
    if (D == 512 && heads == 1) {
      k_check(cake_attn512(dt_, q, k, v, o, B, N, M, ldq, ldk, ldv, C, N * ldq, M * ldk, M * ldv,
                           (long long)N * C, scale, zeros_, st_), "attn512");
      return o;
    }
    throw Error("attention: head dim " + std::to_string(D) + " is not supported");
  }

  static std::pair<int, int> halo_tile(int OH, int OW, int bn) {
    static const int t256[3][2] = {{16, 16}, {8, 32}, {32, 8}};
    static const int t128[4][2] = {{8, 16}, {16, 8}, {10, 12}, {12, 10}};
    static const int t64[3][2] = {{8, 8}, {4, 16}, {16, 4}};
    const int(*tab)[2] = bn == 256 ? t256 : bn == 128 ? t128 : t64;
    const int n = bn == 128 ? 4 : 3;
    std::pair<int, int> best{0, 0};
    long long ba = -1;
    int bw = 0;
    for (int i = 0; i < n; ++i) {
      const int th = tab[i][0], tw = tab[i][1];
      const long long area = (long long)((OH + th - 1) / th) * th * ((OW + tw - 1) / tw) * tw;
      if (ba < 0 || area < ba || (area == ba && tw > bw)) {
        ba = area;
        bw = tw;
        best = {th, tw};
      }
    }
    return best;
  }

  static std::pair<int, int> conv_plan(long long P, int OC, int ksteps) {
    static const int tiles[4][2] = {{128, 128}, {64, 128}, {128, 64}, {64, 64}};
    static const int slots[4] = {2, 3, 3, 5};
    static const double eff[4] = {1.0, 0.8, 0.8, 0.6};
    double best = -1;
    std::pair<int, int> out{0, 1};
    for (int cfg = 0; cfg < 4; ++cfg) {
      const int bm = tiles[cfg][0], bn = tiles[cfg][1];
      const long long nt = (long long)((OC + bm - 1) / bm) * ((P + bn - 1) / bn);
      for (int sp : {1, 2, 4, 8}) {
        if (sp > 1 && (ksteps / sp < 4 || nt * sp > 2LL * 256 * slots[cfg])) continue;
        const long long waves = (nt * sp + 256LL * slots[cfg] - 1) / (256LL * slots[cfg]);
        double cost = (double)waves * slots[cfg] * bm * bn * (double)((ksteps + sp - 1) / sp) / eff[cfg];
        if (sp > 1) cost += (double)P * OC * sp * 0.05;
        if (best < 0 || cost < best) { best = cost; out = {cfg, sp}; }
      }
    }
    return out;
  }

  // one launch of the NHWC implicit-GEMM convolution with variant (cfg, splits)
  int conv_launch(Arena& A, const ConvW& c, const uint16_t* x, int N, int H, int W, int stride,
                  int pad, bool up, const float* bias2, int bias2_ld, const uint16_t* resid,
                  int layout, uint16_t* out, int cfg, int splits) {
    const int KH = c.K;
    const int VH = H << (up ? 1 : 0), VW = W << (up ? 1 : 0);
    const int OH = (VH + 2 * pad - KH) / stride + 1, OW = (VW + 2 * pad - KH) / stride + 1;
    const long long P = (long long)N * OH * OW;
    int ksteps = KH * KH * c.IC / 64;
    if (c.IC % 64) { cfg = 14; splits = 1; ksteps = 1; }
    int th = 0, tw = 0;
    if (cfg >= 8 && cfg < 14) {
      if (stride != 1) return (int)hipErrorInvalidValue;
      splits = 1;
      const auto t = halo_tile(OH, OW, cfg >= 12 ? 256 : cfg < 10 ? 128 : 64);
      th = t.first;
      tw = t.second;
    }
    splits = std::max(1, std::min(splits, ksteps));
    const int kps = (ksteps + splits - 1) / splits;
    splits = (ksteps + kps - 1) / kps;
    float* ws = splits > 1 ? new32(A, (size_t)splits * P * c.OC) : nullptr;
    return cake_conv2d_nhwc2(dt_, x, c.w, c.b, bias2, resid, out, ws, zeros_, N, H, W, c.IC, c.OC,
                             KH, KH, stride, pad, up ? 1 : 0, cfg, splits, th, tw, bias2_ld,
                             layout, st_);
  }

  // ops.conv on the NHWC path (ops/conv.py: the autotuned variant per shape)
  uint16_t* conv(Arena& A, const ConvW& c, const uint16_t* x, int N, int H, int W, int stride,
                 int pad, bool up, const float* bias2 = nullptr, int bias2_ld = 0,
                 const uint16_t* resid = nullptr, bool in_nchw = false, bool out_nchw = false,
                 int* oh = nullptr, int* ow = nullptr) {
    const int VH = H << (up ? 1 : 0), VW = W << (up ? 1 : 0);
    const int OH = (VH + 2 * pad - c.K) / stride + 1, OW = (VW + 2 * pad - c.K) / stride + 1;
    if (oh) *oh = OH;
    if (ow) *ow = OW;
    uint16_t* out = new16(A, (size_t)N * OH * OW * c.OC);
    if (c.small1x1) {
      k_check(cake_conv1x1_small(dt_, x, c.w, c.b, out, N, H * W, c.IC, c.OC,
                                 (in_nchw ? 1 : 0) | (out_nchw ? 2 : 0), st_), "conv1x1_small");
      return out;
    }
    const int layout = (in_nchw ? 1 : 0) | (out_nchw ? 2 : 0);
    const auto key = std::make_tuple(N, H, W, c.IC, c.OC, c.K * 100 + stride * 10 + pad,
                                     (up ? 1 : 0) | (bias2 ? 2 : 0) | (resid ? 4 : 0) | (layout << 3));
    auto it = conv_cache_.find(key);
    if (it == conv_cache_.end()) {
      std::pair<int, int> choice;
      if (c.IC % 64) {
        choice = {14, 1};
      } else if (autotune_ && !unet_a_.frozen) {
        choice = autotune_conv(A, c, x, N, H, W, stride, pad, up, bias2, bias2_ld, resid, layout,
                               out);
      } else {
        choice = conv_plan((long long)N * OH * OW, c.OC, c.K * c.K * c.IC / 64);
      }
      it = conv_cache_.emplace(key, choice).first;
    }
    k_check(conv_launch(A, c, x, N, H, W, stride, pad, up, bias2, bias2_ld, resid, layout, out,
                        it->second.first, it->second.second), "conv2d_nhwc");
    return out;
  }

  std::pair<int, int> autotune_conv(Arena& A, const ConvW& c, const uint16_t* x, int N, int H,
                                    int W, int stride, int pad, bool up, const float* bias2,
                                    int bias2_ld, const uint16_t* resid, int layout,
                                    uint16_t* out) {
    std::vector<std::pair<int, int>> cands;
    if (stride == 1 && c.K > 1)
      for (int cfg = 8; cfg < 14; ++cfg) cands.push_back({cfg, 1});
    for (int cfg : {4, 5, 6, 7, 0, 1, 2, 3})
      for (int sp : {1, 2, 4, 8}) cands.push_back({cfg, sp});
    hipEvent_t e0, e1;
    hip_check(hipEventCreate(&e0), "event");
    hip_check(hipEventCreate(&e1), "event");
    float best = -1;
    std::pair<int, int> pick{0, 1};
    for (const auto& cs : cands) {
      // each try's split-K slab comes from the arena: rewind it after the try
      const size_t ci = A.ci, off = A.off;
      if (conv_launch(A, c, x, N, H, W, stride, pad, up, bias2, bias2_ld, resid, layout, out,
                      cs.first, cs.second) != 0) {
        (void)hipGetLastError();
        A.ci = ci;
        A.off = off;
        continue;
      }
      hip_check(hipEventRecord(e0, st_), "event");
      for (int i = 0; i < 3; ++i)
        k_check(conv_launch(A, c, x, N, H, W, stride, pad, up, bias2, bias2_ld, resid, layout,
                            out, cs.first, cs.second), "conv autotune");
      hip_check(hipEventRecord(e1, st_), "event");
      hip_check(hipEventSynchronize(e1), "event sync");
      float ms = 0;
      hip_check(hipEventElapsedTime(&ms, e0, e1), "elapsed");
      A.ci = ci;
      A.off = off;
      if (best < 0 || ms < best) { best = ms; pick = cs; }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return pick;
  }

  // ------------------------------------------------------------------ UNet
  struct Fm { uint16_t* p; int H, W, C; };  // NHWC feature map of batch B_

  Fm resnet(const ResnetW& r, Fm x, const float* tb, int tb_ld, const Fm* skip,
            int groups, float eps) {
    Arena& A = unet_a_;
    const int HW = x.H * x.W;
    uint16_t* h;
    Fm in = x;
    if (skip) {
      const int C = x.C + skip->C;
      uint16_t* cat = new16(A, (size_t)B_ * HW * C);
      h = group_norm(A, x.p, skip->p, x.C, B_, HW, C, r.n1w, r.n1b, groups, eps, true, cat);
      in = {cat, x.H, x.W, C};
    } else {
      h = group_norm(A, x.p, nullptr, x.C, B_, HW, x.C, r.n1w, r.n1b, groups, eps, true);
    }
    h = conv(A, r.c1, h, B_, x.H, x.W, 1, 1, false, tb, tb_ld);
    h = group_norm(A, h, nullptr, r.cout, B_, HW, r.cout, r.n2w, r.n2b, groups, eps, true);
    const uint16_t* shortcut = in.p;
    if (r.has_sc) shortcut = conv(A, r.sc, in.p, B_, x.H, x.W, 1, 0, false);
    uint16_t* y = conv(A, r.c2, h, B_, x.H, x.W, 1, 1, false, nullptr, 0, shortcut);
    return {y, x.H, x.W, r.cout};
  }

  Fm transformer(const TransformerW& t, Fm x) {
    Arena& A = unet_a_;
    const int C = t.ch, T = x.H * x.W;
    const long long rows = (long long)B_ * T;
    uint16_t* h = group_norm(A, x.p, nullptr, C, B_, T, C, t.nw, t.nb, cfg_.unet.groups, 1e-6f,
                             false);
    uint16_t* hp = new16(A, (size_t)rows * C);
    gemm(kStore, h, C, (int)rows, C, t.pin_w, C, t.pin_b, hp, C);
    h = hp;
    for (const auto& blk : t.blocks) {
      // self-attention: one q|k|v GEMM, flash attention, o-proj + residual
      uint16_t* n1 = layer_norm(A, h, rows, C, blk.n1w, blk.n1b, 1e-5f);
      uint16_t* qkv = new16(A, (size_t)rows * 3 * C);
      gemm(kStore, n1, C, (int)rows, C, blk.qkv, 3 * C, nullptr, qkv, 3 * C);
      uint16_t* a = attention(A, qkv, 3 * C, qkv + C, 3 * C, qkv + 2 * C, 3 * C, B_, T, T,
                              t.heads, C, false);
      uint16_t* x1 = new16(A, (size_t)rows * C);
      gemm(kAdd16, a, C, (int)rows, C, blk.o1w, C, blk.o1b, x1, C, h, C);
      // cross-attention on the cached context k|v
      uint16_t* n2 = layer_norm(A, x1, rows, C, blk.n2w, blk.n2b, 1e-5f);
      uint16_t* q = new16(A, (size_t)rows * C);
      gemm(kStore, n2, C, (int)rows, C, blk.q2, C, nullptr, q, C);
      uint16_t* a2 = attention(A, q, C, blk.kv_cache, 2 * C, blk.kv_cache + C, 2 * C, B_, T, kTok,
                               t.heads, C, false);
      uint16_t* x2 = new16(A, (size_t)rows * C);
      gemm(kAdd16, a2, C, (int)rows, C, blk.o2w, C, blk.o2b, x2, C, x1, C);
      // GEGLU feed-forward, residual in the output projection
      uint16_t* n3 = layer_norm(A, x2, rows, C, blk.n3w, blk.n3b, 1e-5f);
      uint16_t* ff = new16(A, (size_t)rows * 4 * C);
      gemm(kGeglu, n3, C, (int)rows, C, blk.ffi_w, 8 * C, blk.ffi_b, ff, 4 * C);
      uint16_t* x3 = new16(A, (size_t)rows * C);
      gemm(kAdd16, ff, 4 * C, (int)rows, 4 * C, blk.ffo_w, C, blk.ffo_b, x3, C, x2, C);
      h = x3;
    }
    uint16_t* y = new16(A, (size_t)rows * C);
    gemm(kAdd16, h, C, (int)rows, C, t.pout_w, C, t.pout_b, y, C, x.p, C);
    return {y, x.H, x.W, C};
  }

  // cross-attention k|v of the current context for every transformer block
  void precompute_kv(int B) {
    const int ctx = cfg_.unet.ctx;
    auto run = [&](TransformerW& t) {
      for (auto& blk : t.blocks)
        gemm(kStore, ctx_, ctx, B * kTok, ctx, blk.kv2, 2 * t.ch, nullptr, blk.kv_cache, 2 * t.ch);
    };
    for (auto& d : down_)
      for (auto& t : d.att) run(t);
    run(mid_att_);
    for (auto& u : up_)
      for (auto& t : u.att) run(t);
  }

  // ---- the UNet as stages (the split UNet's units: parallel/sd_split.py stage_names):
  // 0 .. nd-1 = down.i (down.0 also runs conv_in), nd = mid, nd+1 .. = up.i (the last one
  // also norm_out + conv_out).  Skip tensors are numbered in push order; an up stage pops
  // the highest live index first (the reference's LIFO skip stack), so every rank can
  // hold just the skips it produces or receives.
  int n_stages() const { return (int)down_.size() + 1 + (int)up_.size(); }
  int stage_pushes(int k) const {
    const int nd = (int)down_.size();
    if (k >= nd) return 0;
    return (k == 0 ? 1 : 0) + (int)down_[k].res.size() + (down_[k].has_ds ? 1 : 0);
  }
  int stage_pops(int k) const {
    const int nd = (int)down_.size();
    return k > nd ? (int)up_[k - nd - 1].res.size() : 0;
  }
  // live skips before stage k (the stack height)
  int stack_before(int k) const {
    int t = 0;
    for (int i = 0; i < k; ++i) t += stage_pushes(i) - stage_pops(i);
    return t;
  }
  int total_skips() const {
    int t = 0;
    for (int i = 0; i < n_stages(); ++i) t += stage_pushes(i);
    return t;
  }
  std::string stage_name(int k) const {
    const int nd = (int)down_.size();
    if (k < nd) return "down." + std::to_string(k);
    if (k == nd) return "mid";
    return "up." + std::to_string(k - nd - 1);
  }

  struct UnetRun {  // per-forward context of the stages
    float* tb;
    int tb_ld;  // the row stride of tb (0: one shared row)
  };

  // time biases: sinusoidal embedding -> linear_1 (+SiLU) -> linear_2 (+SiLU) -> every
  // resnet's projection as one GEMM (f32)
  UnetRun unet_begin(int B, const float* ttab, const int* tidx) {
    Arena& A = unet_a_;
    const UCfg& u = cfg_.unet;
    B_ = B;
    const int C0 = u.blocks[0].ch;
    uint16_t* emb = new16(A, (size_t)B * C0);
    k_check(cake_timestep_embed(dt_, ttab, tidx, B, C0, u.flip ? 1 : 0, (float)u.shift, 1, emb, st_),
            "timestep_embed");
    uint16_t* e1 = new16(A, (size_t)B * temb_dim_);
    gemm(kSilu, emb, C0, B, C0, t1w_, temb_dim_, t1b_, e1, temb_dim_);
    uint16_t* e2 = new16(A, (size_t)B * temb_dim_);
    gemm(kSilu, e1, temb_dim_, B, temb_dim_, t2w_, temb_dim_, t2b_, e2, temb_dim_);
    float* tb = new32(A, (size_t)B * temb_cols_);
    gemm(kStore32, e2, temb_dim_, B, temb_dim_, tall_w_, temb_cols_, tall_b_, tb, temb_cols_);
    return {tb, B > 1 ? temb_cols_ : 0};
  }

  // stage k: x in / out, pushes into / pops from sk at the stack height `top`; stage 0
  // reads the NCHW input `inp`, the last stage leaves the NCHW prediction in x.p
  void unet_stage(int k, const UnetRun& R, const uint16_t* inp, Fm& x, std::vector<Fm>& sk,
                  int& top) {
    Arena& A = unet_a_;
    const UCfg& u = cfg_.unet;
    const int G = u.groups;
    const float eps = (float)u.eps;
    auto tbias = [&](const ResnetW& r) { return R.tb + r.toff; };
    auto tld = [&](const ResnetW& r) { return B_ > 1 ? R.tb_ld : r.cout; };
    const int nd = (int)down_.size();
    if (k < nd) {
      if (k == 0) {  // down.0: conv_in reads the NCHW input
        const int h = cfg_.height / 8, w = cfg_.width / 8;
        x = Fm{conv(A, conv_in_, inp, B_, h, w, 1, 1, false, nullptr, 0, nullptr, true, false), h,
               w, u.blocks[0].ch};
        sk[top++] = x;
      }
      const DownW& d = down_[k];
      for (size_t j = 0; j < d.res.size(); ++j) {
        x = resnet(d.res[j], x, tbias(d.res[j]), tld(d.res[j]), nullptr, G, eps);
        if (!d.att.empty()) x = transformer(d.att[j], x);
        sk[top++] = x;
      }
      if (d.has_ds) {
        int oh, ow;
        uint16_t* y = conv(A, d.ds, x.p, B_, x.H, x.W, 2, 1, false, nullptr, 0, nullptr, false,
                           false, &oh, &ow);
        x = {y, oh, ow, d.ds.OC};
        sk[top++] = x;
      }
      return;
    }
    if (k == nd) {
      x = resnet(mid_res_[0], x, tbias(mid_res_[0]), tld(mid_res_[0]), nullptr, G, eps);
      x = transformer(mid_att_, x);
      x = resnet(mid_res_[1], x, tbias(mid_res_[1]), tld(mid_res_[1]), nullptr, G, eps);
      return;
    }
    const UpW& up = up_[k - nd - 1];
    for (size_t j = 0; j < up.res.size(); ++j) {
      const Fm s = sk[--top];
      x = resnet(up.res[j], x, tbias(up.res[j]), tld(up.res[j]), &s, G, eps);
      if (!up.att.empty()) x = transformer(up.att[j], x);
    }
    if (up.has_us) {
      int oh, ow;
      uint16_t* y = conv(A, up.us, x.p, B_, x.H, x.W, 1, 1, true, nullptr, 0, nullptr, false,
                         false, &oh, &ow);
      x = {y, oh, ow, up.us.OC};
    }
    if (k + 1 == n_stages()) {
      uint16_t* hN = group_norm(A, x.p, nullptr, x.C, B_, x.H * x.W, x.C, norm_out_w_,
                                norm_out_b_, G, eps, true);
      x.p = conv(A, conv_out_, hN, B_, x.H, x.W, 1, 1, false, nullptr, 0, nullptr, false, true);
      x.C = 4;
    }
  }

  // the UNet forward on inp [B, 4, h, w] (NCHW 16-bit): returns [B, 4, h, w] NCHW
  const uint16_t* unet_forward(const uint16_t* inp, int B, const float* ttab, const int* tidx) {
    const UnetRun R = unet_begin(B, ttab, tidx);
    std::vector<Fm> sk(total_skips());
    int top = 0;
    Fm x{nullptr, 0, 0, 0};
    for (int k = 0; k < n_stages(); ++k) unet_stage(k, R, inp, x, sk, top);
    return x.p;
  }

  // ------------------------------------------------------------------ split UNet
  // (sd_engine.h CakeSdSplitOpts).  Shapes of every stage output and skip tensor from the
  // weights' channel counts, the producer / consumer stage of every skip, the runs of
  // the ranks and the channels between them — the same on every rank.
  struct Shp { int H, W, C; };
  struct Chan {
    int src = 0, dst = 0;
    int x_after = -1;          // carries the feature map after this stage (-1: none)
    std::vector<int> skips;    // skip indices, ascending
    size_t cap = 0;            // inbox bytes (dst == this rank)
    void* inbox = nullptr;     // dst == this rank: its uncached inbox
    void* peer = nullptr;      // src == this rank: the receiver's inbox, IPC-mapped
    unsigned* ctr = nullptr;   // device: send seq, send count, recv seq
  };
  size_t fm_bytes(const Shp& x, int B) const { return ((size_t)B * x.H * x.W * x.C * 2 + 15) / 16 * 16; }

  void split_plan(const CakeSdSplitOpts& sp) {
    const int n = n_stages(), nd = (int)down_.size();
    // shapes (conv stride 2 pad 1: ceil(H / 2); the up blocks' nearest-2x conv: 2H)
    int H = cfg_.height / 8, W = cfg_.width / 8, C = conv_in_.OC;
    x_shp_.assign(n, Shp{0, 0, 0});
    skip_shp_.clear();
    skip_prod_.clear();
    skip_cons_.assign(total_skips(), -1);
    int top = 0;
    std::vector<int> stack;
    for (int k = 0; k < n; ++k) {
      auto push = [&](Shp x) {
        skip_shp_.push_back(x);
        skip_prod_.push_back(k);
        stack.push_back((int)skip_shp_.size() - 1);
        ++top;
      };
      if (k < nd) {
        if (k == 0) push({H, W, C});
        const DownW& d = down_[k];
        for (const auto& r : d.res) {
          C = r.cout;
          push({H, W, C});
        }
        if (d.has_ds) {
          H = (H - 1) / 2 + 1;
          W = (W - 1) / 2 + 1;
          C = d.ds.OC;
          push({H, W, C});
        }
      } else if (k == nd) {
        C = mid_res_[1].cout;
      } else {
        const UpW& u = up_[k - nd - 1];
        for (const auto& r : u.res) {
          skip_cons_[stack.back()] = k;
          stack.pop_back();
          --top;
          C = r.cout;
        }
        if (u.has_us) {
          H *= 2;
          W *= 2;
          C = u.us.OC;
        }
        if (k + 1 == n) C = 4;  // conv_out: the NCHW prediction
      }
      x_shp_[k] = {H, W, C};
    }
    // owners: contiguous runs, rank 0 first
    sused_ = std::min(sworld_, n);
    sowner_.assign(n, 0);
    if (sp.owners && sp.n_owners > 0) {
      if (sp.n_owners != n) throw Error("split UNet: owners must name every one of the " +
                                        std::to_string(n) + " stages");
      for (int k = 0; k < n; ++k) sowner_[k] = sp.owners[k];
      int used = 0;
      for (int k = 0; k < n; ++k) {
        if (sowner_[k] < 0 || sowner_[k] >= sworld_) throw Error("split UNet: owner out of range");
        const int want = k == 0 ? 0 : (sowner_[k] == sowner_[k - 1] ? sowner_[k - 1] : sowner_[k - 1] + 1);
        if (sowner_[k] != want) throw Error("split UNet: owners must be contiguous runs 0, 1, ...");
        used = sowner_[k] + 1;
      }
      sused_ = used;
    } else {
      for (int k = 0; k < n; ++k) sowner_[k] = (int)((long long)k * sused_ / n);
    }
    s_first_ = n;
    s_end_ = n;
    for (int k = 0; k < n; ++k)
      if (sowner_[k] == srank_) {
        s_first_ = std::min(s_first_, k);
        s_end_ = k + 1;
      }
    if (s_first_ >= s_end_) s_first_ = s_end_ = 0;
    // channels: the feature map run -> next run (and the prediction back to rank 0), every
    // skip producer -> consumer across ranks
    chans_.clear();
    auto chan = [&](int src, int dst) -> Chan& {
      for (auto& c : chans_)
        if (c.src == src && c.dst == dst) return c;
      chans_.push_back(Chan{});
      chans_.back().src = src;
      chans_.back().dst = dst;
      return chans_.back();
    };
    for (int k = 1; k < n; ++k)
      if (sowner_[k] != sowner_[k - 1]) chan(sowner_[k - 1], sowner_[k]).x_after = k - 1;
    if (sowner_[n - 1] != 0) chan(sowner_[n - 1], 0).x_after = n - 1;
    for (size_t i = 0; i < skip_shp_.size(); ++i) {
      const int src = sowner_[skip_prod_[i]], dst = sowner_[skip_cons_[i]];
      if (src != dst) chan(src, dst).skips.push_back((int)i);
    }
    std::sort(chans_.begin(), chans_.end(), [](const Chan& a, const Chan& b) {
      return a.src != b.src ? a.src < b.src : a.dst < b.dst;
    });
  }

  // segment byte sizes of a channel's message at B rows: [feature map] + skips
  std::vector<size_t> chan_segs(const Chan& c, int B) const {
    std::vector<size_t> v;
    if (c.x_after >= 0) v.push_back(fm_bytes(x_shp_[c.x_after], B));
    for (int i : c.skips) v.push_back(fm_bytes(skip_shp_[i], B));
    return v;
  }
  size_t chan_bytes(const Chan& c, int B) const {
    size_t t = 0;
    for (size_t b : chan_segs(c, B)) t += b;
    return t;
  }

  // inboxes (uncached device memory, hop.hip bulk messages) for the channels into this
  // rank, exchanged as IPC handles through rank 0; then every channel's sender maps its
  // receiver's inbox
  void connect_split(const CakeSdSplitOpts& sp) {
    split_plan(sp);
    stimeout_ = sp.timeout_s > 0 ? sp.timeout_s : 60.0;
    std::string host;
    int port = 0;
    split_host_port(sp.master_addr ? sp.master_addr : "127.0.0.1:29533", &host, &port);
    serr_ = static_cast<int*>(dalloc(64));
    hip_check(hipMemset(serr_, 0, 64), "memset");
    Json me = Json::object();
    me.set("rank", Json::integer(srank_));
    Json boxes = Json::array();
    for (size_t i = 0; i < chans_.size(); ++i) {
      Chan& c = chans_[i];
      c.ctr = static_cast<unsigned*>(dalloc(64));  // send seq, send count, recv seq
      hip_check(hipMemset(c.ctr, 0, 64), "memset");
      if (c.dst != srank_) continue;
      c.cap = chan_bytes(c, rows_cap_);
      k_check(cake_hop_alloc(c.cap + 256, &c.inbox), "hop_alloc");
      hip_check(hipMemset(c.inbox, 0, c.cap + 256), "memset inbox");
      hipIpcMemHandle_t h;
      hip_check(hipIpcGetMemHandle(&h, c.inbox), "IpcGetMemHandle");
      Json e = Json::array();
      e.push(Json::integer((int64_t)i));
      e.push(Json::string(hex_of(&h, sizeof(h))));
      boxes.push(e);
    }
    me.set("inboxes", boxes);
    std::vector<Json> table(sworld_);
    if (srank_ == 0) {
      const int lfd = tcp_listen(host, port);
      table[0] = me;
      speers_.assign(sworld_ - 1, -1);
      try {
        for (int i = 1; i < sworld_; ++i) {
          std::string peer;
          const int fd = tcp_accept(lfd, &peer);
          tcp_set_timeout(fd, 0);
          const Json j = recv_json(fd);
          const int r = (int)j.get("rank").as_int();
          if (r < 1 || r >= sworld_ || speers_[r - 1] >= 0) throw Error("split UNet: bad rank hello");
          speers_[r - 1] = fd;
          table[r] = j;
        }
      } catch (...) {
        tcp_close(lfd);
        throw;
      }
      tcp_close(lfd);
      Json all = Json::array();
      for (const auto& t : table) all.push(t);
      Json m = Json::object();
      m.set("table", all);
      for (int fd : speers_) send_json(fd, m);
    } else {
      const double ct = sp.connect_timeout_s > 0 ? sp.connect_timeout_s : 600.0;
      const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(ct);
      for (;;) {
        try {
          ctl_fd_ = tcp_connect(host, port, 2.0);
          break;
        } catch (const std::exception&) {
          if (std::chrono::steady_clock::now() > deadline) throw;
          std::this_thread::sleep_for(std::chrono::milliseconds(200));
        }
      }
      tcp_set_timeout(ctl_fd_, 0);
      send_json(ctl_fd_, me);
      const Json m = recv_json(ctl_fd_);
      for (int r = 0; r < sworld_; ++r) table[r] = m.get("table").at(r);
    }
    for (size_t i = 0; i < chans_.size(); ++i) {
      Chan& c = chans_[i];
      if (c.src != srank_) continue;
      bool found = false;
      for (const auto& x : table[c.dst].get("inboxes").items()) {
        if ((size_t)x.at(0).as_int() != i) continue;
        hipIpcMemHandle_t h;
        unhex(x.at(1).as_string(), &h, sizeof(h));
        hip_check(hipIpcOpenMemHandle(&c.peer, h, hipIpcMemLazyEnablePeerAccess), "IpcOpen inbox");
        found = true;
      }
      if (!found) throw Error("split UNet: rank " + std::to_string(c.dst) + " published no inbox");
    }
  }

  // this rank's part of one denoise step of the split UNet on B rows: receive, its stages,
  // send; rank 0 (stage 0 reads inp) then receives the prediction and returns it
  const uint16_t* split_unet(int B, const uint16_t* inp) {
    const UnetRun R = unet_begin(B, ttab_, step_);
    std::vector<Fm> sk(total_skips());
    Fm x{nullptr, 0, 0, 0};
    auto recv = [&](const Chan& c) {
      const std::vector<size_t> segs = chan_segs(c, B);
      const size_t bytes = chan_bytes(c, B);
      uint8_t* buf = static_cast<uint8_t*>(unet_a_.alloc(bytes));
      k_check(cake_bulk_recv(c.inbox, bytes, buf, c.ctr + 2, serr_, stimeout_, st_), "bulk_recv");
      size_t o = 0, si = 0;
      if (c.x_after >= 0) {
        const Shp& xs = x_shp_[c.x_after];
        x = Fm{reinterpret_cast<uint16_t*>(buf), xs.H, xs.W, xs.C};
        o += segs[si++];
      }
      for (int i : c.skips) {
        const Shp& q = skip_shp_[i];
        sk[i] = Fm{reinterpret_cast<uint16_t*>(buf + o), q.H, q.W, q.C};
        o += segs[si++];
      }
    };
    const bool pred_chan_rank0 = srank_ == 0;
    for (const auto& c : chans_)
      if (c.dst == srank_ && !(pred_chan_rank0 && c.x_after == n_stages() - 1)) recv(c);
    int top = stack_before(s_first_);
    for (int k = s_first_; k < s_end_; ++k) unet_stage(k, R, inp, x, sk, top);
    for (const auto& c : chans_) {
      if (c.src != srank_) continue;
      const std::vector<size_t> segs = chan_segs(c, B);
      std::vector<const void*> src;
      std::vector<unsigned long long> nb, off;
      size_t o = 0, si = 0;
      auto add = [&](const void* p) {
        src.push_back(p);
        nb.push_back(segs[si]);
        off.push_back(o);
        o += segs[si++];
      };
      if (c.x_after >= 0) add(x.p);
      for (int i : c.skips) add(sk[i].p);
      k_check(cake_bulk_send(src.data(), nb.data(), off.data(), (int)src.size(), c.peer, o, c.ctr,
                             c.ctr + 1, st_), "bulk_send");
    }
    if (srank_ != 0) return nullptr;
    for (const auto& c : chans_)
      if (c.dst == 0 && c.x_after == n_stages() - 1) recv(c);
    return x.p;
  }

  // one step of a worker rank (graph-captured after the first): its stages, step += 1
  void split_worker_step(int B) {
    unet_a_.reset();
    split_unet(B, nullptr);
    k_check(cake_step_advance(step_, st_), "step_advance");
  }

  bool split_active() const { return sworld_ > 1 && sused_ > 1; }

  // rank 0, at the start of a generation's denoise loop: each used worker rank gets the
  // step count, the UNet rows, the timestep table and the text context
  void split_start(int n_steps, int B2, const std::vector<float>& ttab) {
    const size_t ctx_bytes = (size_t)B2 * kTok * cfg_.ctx_dim() * 2;
    std::vector<uint8_t> ctx(ctx_bytes);
    hip_check(hipMemcpyAsync(ctx.data(), ctx_, ctx_bytes, hipMemcpyDeviceToHost, st_), "D2H ctx");
    hip_check(hipStreamSynchronize(st_), "sync");
    Json m = Json::object();
    m.set("cmd", Json::string("gen"));
    m.set("n", Json::integer(n_steps));
    m.set("B", Json::integer(B2));
    Json tt = Json::array();
    for (float t : ttab) tt.push(Json::number(t));
    m.set("ttab", tt);
    for (int r = 1; r < sused_; ++r) {
      send_json(speers_[r - 1], m);
      send_frame(speers_[r - 1], ctx.data(), (uint32_t)ctx.size());
    }
  }

  // rank 0, after its denoise loop: every used worker's verdict
  void split_finish() {
    std::string bad;
    for (int r = 1; r < sused_; ++r) {
      const Json a = recv_json(speers_[r - 1]);
      if (bad.empty() && a.has("error")) bad = "split UNet rank " + std::to_string(r) + ": " +
                                                a.get("error").as_string();
    }
    int e = 0;
    hip_check(hipMemcpy(&e, serr_, sizeof(int), hipMemcpyDeviceToHost), "D2H err");
    if (e) {
      hip_check(hipMemset(serr_, 0, sizeof(int)), "memset");
      if (bad.empty()) bad = "split UNet: a hop into rank 0 timed out";
    }
    if (!bad.empty()) throw Error(bad);
  }

 public:
  // ranks > 0: serve rank 0's generations (gen: the steps of one image) until it exits
  void serve() {
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    if (sworld_ < 2 || srank_ == 0) throw Error("serve() runs on split-UNet ranks > 0");
    for (;;) {
      const Json m = recv_json(ctl_fd_);
      const std::string cmd = m.get("cmd").as_string();
      if (cmd == "exit") return;
      if (cmd != "gen") throw Error("split UNet: unknown control message " + cmd);
      const int n = (int)m.get("n").as_int(), B = (int)m.get("B").as_int();
      const std::string ctx = recv_frame(ctl_fd_);
      Json ack = Json::object();
      try {
        if (B < 1 || B > rows_cap_) throw Error("split UNet: " + std::to_string(B) +
                                               " UNet rows (the inboxes hold " +
                                               std::to_string(rows_cap_) + ")");
        if (ctx.size() != (size_t)B * kTok * cfg_.ctx_dim() * 2) throw Error("split UNet: context size");
        std::vector<float> tt;
        for (const auto& v : m.get("ttab").items()) tt.push_back((float)v.as_double());
        ensure_tables((int)tt.size() + 1);
        hip_check(hipMemcpyAsync(ttab_, tt.data(), tt.size() * 4, hipMemcpyHostToDevice, st_), "H2D");
        hip_check(hipMemcpyAsync(ctx_, ctx.data(), ctx.size(), hipMemcpyHostToDevice, st_), "H2D");
        hip_check(hipMemsetAsync(step_, 0, 4, st_), "memset");
        precompute_kv(B);
        for (int i = 0; i < n; ++i) {
          if (i == 0) {
            split_worker_step(B);
          } else {
            auto it = wgraphs_.find(B);
            if (it == wgraphs_.end()) it = wgraphs_.emplace(B, capture_worker(B)).first;
            hip_check(hipGraphLaunch(it->second.exec, st_), "hipGraphLaunch");
          }
        }
        hip_check(hipStreamSynchronize(st_), "sync");
        int e = 0;
        hip_check(hipMemcpy(&e, serr_, sizeof(int), hipMemcpyDeviceToHost), "D2H err");
        if (e) {
          hip_check(hipMemset(serr_, 0, sizeof(int)), "memset");
          throw Error("a hop into this rank timed out");
        }
      } catch (const std::exception& x) {
        (void)hipStreamSynchronize(st_);
        ack.set("error", Json::string(x.what()));
      }
      send_json(ctl_fd_, ack);
    }
  }

  void split_info(int32_t* o) const {
    o[0] = srank_;
    o[1] = sworld_;
    o[2] = n_stages();
    o[3] = sused_;
    o[4] = s_first_;
    o[5] = s_end_;
  }

 private:
  void step_body(int B2, bool guide, float guidance) {
    unet_a_.reset();
    const uint16_t* pred = split_active() ? split_unet(B2, inp_) : unet_forward(inp_, B2, ttab_, step_);
    const int h = cfg_.height / 8, w = cfg_.width / 8;
    const long long nl = (long long)4 * h * w * (guide ? B2 / 2 : B2);
    k_check(cake_sched_step(dt_, x_, pred, nl, guide ? 1 : 0, guidance, coef_, step_, seed_dev_,
                            inp_, st_), "sched_step");
    k_check(cake_step_advance(step_, st_), "step_advance");
  }

  struct Graph {
    hipGraph_t g = nullptr;
    hipGraphExec_t exec = nullptr;
  };
  std::map<std::tuple<bool, float, int>, Graph> graphs_;  // (guidance on, scale, UNet rows)

  Graph capture_step(int B2, bool guide, float guidance) {
    Graph gr;
    unet_a_.frozen = true;
    hip_check(hipStreamBeginCapture(st_, hipStreamCaptureModeThreadLocal), "BeginCapture");
    try {
      step_body(B2, guide, guidance);
    } catch (...) {
      hipGraph_t junk = nullptr;
      (void)hipStreamEndCapture(st_, &junk);
      if (junk) (void)hipGraphDestroy(junk);
      unet_a_.frozen = false;
      throw;
    }
    hip_check(hipStreamEndCapture(st_, &gr.g), "EndCapture");
    unet_a_.frozen = false;
    hip_check(hipGraphInstantiate(&gr.exec, gr.g, nullptr, nullptr, 0), "GraphInstantiate");
    return gr;
  }

  Graph capture_worker(int B) {
    Graph gr;
    unet_a_.frozen = true;
    hip_check(hipStreamBeginCapture(st_, hipStreamCaptureModeThreadLocal), "BeginCapture");
    try {
      split_worker_step(B);
    } catch (...) {
      hipGraph_t junk = nullptr;
      (void)hipStreamEndCapture(st_, &junk);
      if (junk) (void)hipGraphDestroy(junk);
      unet_a_.frozen = false;
      throw;
    }
    hip_check(hipStreamEndCapture(st_, &gr.g), "EndCapture");
    unet_a_.frozen = false;
    hip_check(hipGraphInstantiate(&gr.exec, gr.g, nullptr, nullptr, 0), "GraphInstantiate");
    return gr;
  }

  struct HookGraph {
    hipGraph_t g = nullptr;
    hipGraphExec_t exec = nullptr;
    const uint16_t* out = nullptr;
    long calls = 0;
  };
  std::map<int, HookGraph> hook_;  // by batch
  std::vector<float> hook_ctx_;

  void drop_graphs() {
    for (auto& kv : hook_) {
      if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
      if (kv.second.g) (void)hipGraphDestroy(kv.second.g);
    }
    hook_.clear();
    for (auto& kv : graphs_) {
      if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
      if (kv.second.g) (void)hipGraphDestroy(kv.second.g);
    }
    for (auto& kv : wgraphs_) {
      if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
      if (kv.second.g) (void)hipGraphDestroy(kv.second.g);
    }
    wgraphs_.clear();
    graphs_.clear();
  }

  // ------------------------------------------------------------------ text
  const uint16_t* clip_forward(const ClipW& cw, const int32_t* ids_host) {
    Arena& A = text_a_;
    const ClipCfg& c = cw.cfg;
    const int D = c.D, T = kTok;
    int* ids = static_cast<int*>(A.alloc(T * 4));
    hip_check(hipMemcpyAsync(ids, ids_host, T * 4, hipMemcpyHostToDevice, st_), "H2D ids");
    uint16_t* x = new16(A, (size_t)T * D);
    k_check(cake_clip_embed(dt_, cw.tok, cw.pos, ids, T, T, D, c.vocab, x, st_), "clip_embed");
    for (const auto& l : cw.layers) {
      uint16_t* h = layer_norm(A, x, T, D, l.ln1w, l.ln1b, (float)c.eps);
      uint16_t* qkv = new16(A, (size_t)T * 3 * D);
      gemm(kStore, h, D, T, D, l.qkv, 3 * D, l.qkv_b, qkv, 3 * D);
      uint16_t* a = attention(A, qkv, 3 * D, qkv + D, 3 * D, qkv + 2 * D, 3 * D, 1, T, T, c.heads,
                              D, true);
      uint16_t* x1 = new16(A, (size_t)T * D);
      gemm(kAdd16, a, D, T, D, l.ow, D, l.ob, x1, D, x, D);
      h = layer_norm(A, x1, T, D, l.ln2w, l.ln2b, (float)c.eps);
      uint16_t* m = new16(A, (size_t)T * c.I);
      gemm(c.quick_gelu ? kQuickGelu : kGelu, h, D, T, D, l.f1w, c.I, l.f1b, m, c.I);
      uint16_t* x2 = new16(A, (size_t)T * D);
      gemm(kAdd16, m, c.I, T, c.I, l.f2w, D, l.f2b, x2, D, x1, D);
      x = x2;
    }
    return layer_norm(A, x, T, D, cw.fw, cw.fb, (float)c.eps);
  }

  // ctx_ rows [uncond; cond] (or [cond]) of [77, D1 (+ D2)], repeated bsize times as the
  // reference's text_embeddings.repeat((bsize, 1, 1)) (sd.rs; pipeline.py text_emb)
  void text_context(const int32_t* cond, const int32_t* uncond, const int32_t* cond2,
                    const int32_t* uncond2, bool guide, int bsize = 1) {
    const int D1 = cfg_.clip.D, Dc = cfg_.ctx_dim();
    const int per = guide ? 2 : 1;
    auto put = [&](const ClipW& cw, const int32_t* ids, int row, int col) {
      text_a_.reset();
      const int which = &cw == &clip_ ? 0 : 1;
      const int D = which == 0 ? cfg_.clip.D : cfg_.clip2.D;
      const uint16_t* y;
      if (!remote_[2 + which].addr.empty()) {  // the worker's encoder: ids [1, 77] -> [1, 77, D]
        std::vector<float> fid(kTok);
        for (int t = 0; t < kTok; ++t) fid[t] = (float)ids[t];
        const std::vector<float> e = remote_call(remote_[2 + which], which ? "clip2" : "clip", fid,
                                                 {1, (uint64_t)kTok}, (size_t)kTok * D);
        uint16_t* e16 = new16(text_a_, (size_t)kTok * D);
        upload16(e.data(), e.size(), e16);
        y = e16;
      } else {
        y = clip_forward(cw, ids);
      }
      for (int b = 0; b < bsize; ++b)
        hip_check(hipMemcpy2DAsync(ctx_ + (size_t)(b * per + row) * kTok * Dc + col,
                                   (size_t)Dc * 2, y, (size_t)D * 2, (size_t)D * 2, kTok,
                                   hipMemcpyDeviceToDevice, st_), "ctx copy");
      hip_check(hipStreamSynchronize(st_), "sync");  // the text arena is reused next
    };
    const int rc = guide ? 1 : 0;
    put(clip_, cond, rc, 0);
    if (guide) put(clip_, uncond, 0, 0);
    if (cfg_.xl) {
      put(clip2_, cond2, rc, D1);
      if (guide) put(clip2_, uncond2, 0, D1);
    }
  }

  // ------------------------------------------------------------------ VAE
  Fm vae_resnet(const ResnetW& r, Fm x) {
    Arena& A = vae_a_;
    const int G = cfg_.vae.groups, HW = x.H * x.W;
    uint16_t* h = group_norm(A, x.p, nullptr, x.C, 1, HW, x.C, r.n1w, r.n1b, G, 1e-6f, true);
    h = conv(A, r.c1, h, 1, x.H, x.W, 1, 1, false);
    h = group_norm(A, h, nullptr, r.cout, 1, HW, r.cout, r.n2w, r.n2b, G, 1e-6f, true);
    const uint16_t* sc = x.p;
    if (r.has_sc) sc = conv(A, r.sc, x.p, 1, x.H, x.W, 1, 0, false);
    return {conv(A, r.c2, h, 1, x.H, x.W, 1, 1, false, nullptr, 0, sc), x.H, x.W, r.cout};
  }

  // mid-block attention: one head of dim C, residual in the output projection
  Fm vae_attention(const VaeAttnW& at, Fm x) {
    Arena& A = vae_a_;
    const int C = at.C, T = x.H * x.W;
    uint16_t* hn = group_norm(A, x.p, nullptr, C, 1, T, C, at.nw, at.nb, cfg_.vae.groups, 1e-6f,
                              false);
    uint16_t* qkv = new16(A, (size_t)T * 3 * C);
    gemm(kStore, hn, C, T, C, at.qkv, 3 * C, at.qkv_b, qkv, 3 * C);
    uint16_t* a = attention(A, qkv, 3 * C, qkv + C, 3 * C, qkv + 2 * C, 3 * C, 1, T, T, 1, C,
                            false);
    uint16_t* y = new16(A, (size_t)T * C);
    gemm(kAdd16, a, C, T, C, at.ow, C, at.ob, y, C, x.p, C);
    return {y, x.H, x.W, C};
  }

  // vae.py _encode: image [1, 3, H, W] (NCHW) -> moments [1, 8, h, w] (NCHW)
  const uint16_t* vae_encode(const uint16_t* img) {
    Arena& A = vae_a_;
    const VCfg& v = cfg_.vae;
    int H = cfg_.height, W = cfg_.width;
    Fm x{conv(A, e_in_, img, 1, H, W, 1, 1, false, nullptr, 0, nullptr, true, false), H, W,
         v.ch[0]};
    for (const auto& d : e_down_) {
      for (const auto& r : d.res) x = vae_resnet(r, x);
      if (d.has_ds) {  // pad one zero row (bottom) and column (right), conv 3x3 stride 2
        const int C = x.C;
        uint16_t* pad = new16(A, (size_t)(x.H + 1) * (x.W + 1) * C);
        hip_check(hipMemsetAsync(pad, 0, (size_t)(x.H + 1) * (x.W + 1) * C * 2, st_), "memset");
        hip_check(hipMemcpy2DAsync(pad, (size_t)(x.W + 1) * C * 2, x.p, (size_t)x.W * C * 2,
                                   (size_t)x.W * C * 2, x.H, hipMemcpyDeviceToDevice, st_),
                  "pad copy");
        int oh, ow;
        uint16_t* y = conv(A, d.ds, pad, 1, x.H + 1, x.W + 1, 2, 0, false, nullptr, 0, nullptr,
                           false, false, &oh, &ow);
        x = {y, oh, ow, d.ds.OC};
      }
    }
    x = vae_resnet(e_mid_[0], x);
    x = vae_attention(e_att_, x);
    x = vae_resnet(e_mid_[1], x);
    uint16_t* hn = group_norm(A, x.p, nullptr, x.C, 1, x.H * x.W, x.C, e_norm_w_, e_norm_b_,
                              v.groups, 1e-6f, true);
    uint16_t* mo = conv(A, e_out_, hn, 1, x.H, x.W, 1, 1, false);
    return conv(A, quant_, mo, 1, x.H, x.W, 1, 0, false, nullptr, 0, nullptr, false, true);
  }

  const uint16_t* vae_decode(const uint16_t* z) {
    Arena& A = vae_a_;
    const VCfg& v = cfg_.vae;
    const int h = cfg_.height / 8, w = cfg_.width / 8;
    uint16_t* pq = conv(A, post_quant_, z, 1, h, w, 1, 0, false, nullptr, 0, nullptr, true, false);
    Fm x{conv(A, d_in_, pq, 1, h, w, 1, 1, false), h, w, v.ch.back()};
    x = vae_resnet(d_mid_[0], x);
    x = vae_attention(d_att_, x);
    x = vae_resnet(d_mid_[1], x);
    for (const auto& up : d_up_) {
      for (const auto& r : up.res) x = vae_resnet(r, x);
      if (up.has_us) {
        int oh, ow;
        uint16_t* y = conv(A, up.us, x.p, 1, x.H, x.W, 1, 1, true, nullptr, 0, nullptr, false,
                           false, &oh, &ow);
        x = {y, oh, ow, up.us.OC};
      }
    }
    uint16_t* hn = group_norm(A, x.p, nullptr, x.C, 1, x.H * x.W, x.C, d_norm_w_, d_norm_b_,
                              v.groups, 1e-6f, true);
    // [1, 4, H, W] NCHW (the padded 4th channel is never read: RGB = the first 3 planes)
    return conv(A, d_out_, hn, 1, x.H, x.W, 1, 1, false, nullptr, 0, nullptr, false, true);
  }

  // ------------------------------------------------------------------ state
  std::string dir_;
  std::string paths_[4];
  SdCfg cfg_;
  int dev_ = 0, dt_ = 1, init_ = 0, parts_ = 15;
  uint64_t seed_ = 0;
  bool autotune_ = true;
  hipStream_t st_ = nullptr;
  GemmPlanner planner_;
  std::vector<void*> owned_;
  void* scratch_ = nullptr;
  size_t scratch_bytes_ = 0;
  void* zeros_ = nullptr;
  unsigned int* gn_tickets_ = nullptr;
  float* ws_ = nullptr;
  size_t ws_n_ = 0;
  void* flash_ws_ = nullptr;
  size_t flash_ws_n_ = 0;
  Arena unet_a_, text_a_, vae_a_;
  std::map<std::tuple<int, int, int, int, int, int, int>, std::pair<int, int>> conv_cache_;
  int B_ = 2;
  // UNet
  ConvW conv_in_, conv_out_;
  uint16_t *t1w_, *t1b_, *t2w_, *t2b_, *tall_w_, *tall_b_, *norm_out_w_, *norm_out_b_;
  int temb_dim_ = 0, temb_cols_ = 0;
  std::vector<std::pair<std::string, int>> temb_list_;
  std::vector<DownW> down_;
  ResnetW mid_res_[2];
  TransformerW mid_att_;
  std::vector<UpW> up_;
  // VAE
  ConvW e_in_, e_out_, quant_;
  std::vector<DownW> e_down_;
  ResnetW e_mid_[2];
  VaeAttnW e_att_;
  uint16_t *e_norm_w_, *e_norm_b_;
  ConvW post_quant_, d_in_, d_out_;
  ResnetW d_mid_[2];
  VaeAttnW d_att_;
  std::vector<UpW> d_up_;
  uint16_t *d_norm_w_, *d_norm_b_;
  // text
  ClipW clip_, clip2_;
  // per-generation state
  float* x_ = nullptr;
  uint16_t* inp_ = nullptr;
  uint16_t* ctx_ = nullptr;
  void* seed_dev_ = nullptr;
  int* step_ = nullptr;
  float* ttab_ = nullptr;
  float* coef_ = nullptr;
  int table_cap_ = 0;
  // split UNet (connect_split): this rank, its stages, the channels
  int srank_ = 0, sworld_ = 1, sused_ = 1, s_first_ = 0, s_end_ = 0;
  double stimeout_ = 60.0;
  int ctl_fd_ = -1;
  std::vector<int> speers_;
  std::vector<int> sowner_, skip_prod_, skip_cons_;
  std::vector<Shp> x_shp_, skip_shp_;
  std::vector<Chan> chans_;
  int* serr_ = nullptr;
  std::map<int, Graph> wgraphs_;  // worker step graphs by UNet rows
};

void set_err(char* err, int32_t n, const std::string& m) {
  if (err && n > 0) std::snprintf(err, (size_t)n, "%s", m.c_str());
}

}  // namespace
}  // namespace cake

using cake::SdEngine;

CAKE_API void* cake_sd_open(const char* model_dir, const CakeSdOpts* o, char* err, int32_t n) {
  try {
    CakeSdOpts d{};
    d.dtype = 1;
    d.autotune = 1;
    return new SdEngine(model_dir ? model_dir : ".", o ? *o : d);
  } catch (const std::exception& e) {
    cake::set_err(err, n, e.what());
    return nullptr;
  }
}

CAKE_API void* cake_sd_open_split(const char* model_dir, const CakeSdOpts* o,
                                  const CakeSdSplitOpts* sp, char* err, int32_t n) {
  try {
    if (!sp) throw cake::Error("cake_sd_open_split: null split options");
    CakeSdOpts d{};
    d.dtype = 1;
    d.autotune = 1;
    return new SdEngine(model_dir ? model_dir : ".", o ? *o : d, sp);
  } catch (const std::exception& e) {
    cake::set_err(err, n, e.what());
    return nullptr;
  }
}

CAKE_API int32_t cake_sd_serve(void* eng, char* err, int32_t n) {
  try {
    if (!eng) throw cake::Error("cake_sd_serve: null engine");
    static_cast<SdEngine*>(eng)->serve();
    return 0;
  } catch (const std::exception& e) {
    cake::set_err(err, n, e.what());
    return 1;
  }
}

CAKE_API void cake_sd_split_info(void* eng, int32_t* out6) {
  if (eng && out6) static_cast<SdEngine*>(eng)->split_info(out6);
}

CAKE_API int32_t cake_sd_generate(void* eng, const CakeSdGenArgs* a, uint8_t* rgb, float* lat,
                                  double* step_s, CakeSdResult* res, char* err, int32_t n) {
  try {
    if (!eng || !a || !rgb || !a->cond) throw cake::Error("cake_sd_generate: null argument");
    static_cast<SdEngine*>(eng)->generate(*a, rgb, lat, step_s, res);
    return 0;
  } catch (const std::exception& e) {
    cake::set_err(err, n, e.what());
    return 1;
  }
}

CAKE_API void cake_sd_close(void* eng) { delete static_cast<SdEngine*>(eng); }

CAKE_API void cake_sd_info(void* eng, int32_t* out6) {
  const auto* e = static_cast<SdEngine*>(eng);
  out6[0] = e->cfg().width;
  out6[1] = e->cfg().height;
  out6[2] = e->cfg().ctx_dim();
  out6[3] = e->dtype();
  out6[4] = e->cfg().clip.D;
  out6[5] = e->cfg().xl ? e->cfg().clip2.D : 0;
}

CAKE_API int32_t cake_sd_text(void* eng, int32_t which, const int32_t* ids, int32_t B, float* out,
                              char* err, int32_t n) {
  try {
    static_cast<SdEngine*>(eng)->text_component(which, ids, B, out);
    return 0;
  } catch (const std::exception& e) {
    cake::set_err(err, n, e.what());
    return 1;
  }
}

CAKE_API int32_t cake_sd_unet(void* eng, const float* sample, int32_t B, float t, const float* ctx,
                              float* out, char* err, int32_t n) {
  try {
    static_cast<SdEngine*>(eng)->unet_component(sample, B, t, ctx, out);
    return 0;
  } catch (const std::exception& e) {
    cake::set_err(err, n, e.what());
    return 1;
  }
}

CAKE_API int32_t cake_sd_vae_decode(void* eng, const float* z, float* img, char* err, int32_t n) {
  try {
    static_cast<SdEngine*>(eng)->vae_component(z, img);
    return 0;
  } catch (const std::exception& e) {
    cake::set_err(err, n, e.what());
    return 1;
  }
}

CAKE_API int32_t cake_sd_vae_encode_remote(void* eng, const float* img, float* sample, char* err,
                                           int32_t n) {
  try {
    static_cast<SdEngine*>(eng)->vae_encode_remote(img, sample);
    return 0;
  } catch (const std::exception& e) {
    cake::set_err(err, n, e.what());
    return 1;
  }
}

CAKE_API int32_t cake_sd_vae_encode(void* eng, const float* img, float* moments, char* err,
                                    int32_t n) {
  try {
    static_cast<SdEngine*>(eng)->vae_encode_component(img, moments);
    return 0;
  } catch (const std::exception& e) {
    cake::set_err(err, n, e.what());
    return 1;
  }
}
