// Native Llama engine (see llama_engine.h): host orchestration in C++ over the gfx950
// kernels' C entry points — what models/llama3/{blocks,model}.py + decode_loop.py do
// through PyTorch, with no interpreter, no torch allocator and no torch graphs:
//
//   * weights: HF safetensors (mmap, csrc/runtime/safetensors.cpp) uploaded once into
//     hipMalloc'd buffers in the model dtype (bf16 / f16; other checkpoint dtypes
//     converted on the device by cake_cast16).  q|k|v rows and gate|up rows are packed
//     into one matrix each: the prefill GEMMs read them as one operand, the decode
//     GEMVs take the three / two row blocks as separate pointers.
//   * prefill: embed -> per layer RMSNorm, q|k|v GEMM, RoPE + KV write, causal flash
//     attention, o_proj GEMM (+residual epilogue), RMSNorm, gate|up GEMM (SwiGLU
//     epilogue), down GEMM (+residual) -> final-norm lm_head GEMV on the last row
//     (reference: llama.rs:72-138, transformer.rs:51-73).  GEMM tiles come from the
//     same cost model + measured table (ops/gemm_tuned.json) as ops/gemm.py.
//   * decode: one step = 5 launches per layer + the head; captured with
//     hipStreamBeginCapture into one graph per attention split-cap bucket (the live
//     length picks the bucket), replayed by the native loop (graph_loop.cpp).  Greedy
//     steps end in the fused head_select launch (lm_head + penalty + argmax + the next
//     step's embedding row); sampled steps in threshold + Gumbel-max draws keyed by
//     (seed, step) — the same kernels and launch order as DeviceDecoder, so tokens match
//     the Python engine exactly (tests/test_engine_gpu.py).
#include "llama_engine.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <list>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "../driver/graph_loop.h"
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
int cake_embed(int dt, const void* table, const int* tok, int T, int H, float* out, hipStream_t st);
int cake_rmsnorm(int dt, const float* x, const void* w, float eps, int T, int H, void* out,
                 hipStream_t st);
int cake_rope_kv(int dt, void* q, const void* k, const void* v, int ldq, int ld, int T, int nh,
                 int nkv, int hd, const float* inv_freq, int pos0, int S, void* kc, void* vc,
                 hipStream_t st);
int cake_flash_attn(int dt, const void* q, const void* k, const void* v, void* o, int B, int H,
                    int Hkv, int N, int M, int D, const long long* strides, float scale,
                    int causal, int pos0, hipStream_t st);
long long cake_gemm_ws_floats(int cfg, int splits, int M, int N, int K, int gated);
int cake_gemm(int dt, int epi, int cfg, int splits, const void* a, long long lda, const void* b,
              long long ldb, void* c, long long ldc, const void* bias, void* resid,
              long long ldr, float* ws, const void* zeros, int M, int N, int K, hipStream_t st);
int cake_blaslt_gemm(int dt, int out, const void* a, long long lda, const void* w, long long ldw,
                     void* c, long long ldc, int M, int N, int K, void* ws, size_t ws_bytes,
                     hipStream_t st);
int cake_silu_mul_rows(int dt, const void* gu, size_t T, int I, void* out, hipStream_t st);
int cake_qkv_rope(int dt, const float* resid, const void* norm_w, float eps, const void* wq,
                  const void* wk, const void* wv, int K, int nh, int nkv, int hd,
                  const float* inv_freq, const int* pos, float* q_out, void* kcache,
                  void* vcache, int S, hipStream_t st);
int cake_attn_decode(int dt, const float* q, const void* kc, const void* vc, const int* pos,
                     int S, int nh, int nkv, int hd, float scale, float* part,
                     unsigned int* tickets, void* out, hipStream_t st);
int cake_attn_set_split_cap(int cap);
int cake_attn_set_heads(int max_keys, int waves);
int cake_attn_set_head_prefetch(int pfd);
int cake_attn_decode_heads(int dt, const float* q, const void* kc, const void* vc, const int* pos,
                           int S, int nh, int nkv, int hd, float scale, void* out, hipStream_t st);
int cake_attn_splits(int Tk);
int cake_attn_max_split(int S);
int cake_gemv_x16(int dt, const void* x, const void* w, int K, int N, float* out, int accumulate,
                  hipStream_t st);
int cake_swiglu(int dt, const float* resid, const void* norm_w, float eps, const void* wg,
                const void* wu, int K, int I, void* act, hipStream_t st);
int cake_gemv_norm_f32(int dt, const float* resid, const void* norm_w, float eps, const void* w,
                       int K, int N, float* out, hipStream_t st);
int cake_head_select(int dt, const float* resid, const void* norm_w, float eps, const void* w,
                     int K, int N, float* out, int* hist, int* hist_len, int last_n,
                     float penalty, unsigned long long* slot, unsigned int* ticket, int* tok,
                     int* pos, int max_hist, const void* embed, float* emb_out, hipStream_t st);
int cake_repeat_penalty(float* logits, const int* hist, const int* hist_len, int last_n,
                        float penalty, hipStream_t st);
int cake_argmax(const float* logits, int V, unsigned long long* slot, hipStream_t st);
int cake_sample_threshold(const float* logits, int V, float temperature, int top_k, float top_p,
                          unsigned int* thr, hipStream_t st);
int cake_gumbel_argmax(const float* logits, int V, float temperature, unsigned long long seed,
                       const int* step, const unsigned int* thr, unsigned long long* slot,
                       hipStream_t st);
int cake_finalize_token(unsigned long long* slot, int* tok, int* hist, int* hist_len, int* pos,
                        int max_hist, hipStream_t st);
int cake_hop_alloc(size_t bytes, void** ptr);
int cake_sum_slices(float* out, const float* src, int W, long long stride, long long n,
                    int accumulate, hipStream_t st);
long long cake_ar_inbox_words(int world, int n);
int cake_ar_sum(const float* partial, float* out, int n, int accumulate, void* const* peers,
                const void* inbox, unsigned int* seq, int* err, int rank, int world,
                double timeout_s, hipStream_t st);
int cake_ar_max_key(unsigned long long* slot, void* const* peers, const void* inbox,
                    unsigned int* seq, int* err, int rank, int world, double timeout_s,
                    hipStream_t st);
int cake_ar_gather(const float* shard, int off, int n_local, float* full, int n,
                   void* const* peers, const void* inbox, unsigned int* seq, int* err, int rank,
                   int world, double timeout_s, hipStream_t st);
int cake_select_shard(float* logits, int V, int off, const int* hist, const int* hist_len,
                      int last_n, float penalty, float temperature, unsigned long long seed,
                      unsigned long long* slot, hipStream_t st);
int cake_hop_free(void* ptr);
int cake_hop_words(int H, int nhdr, int bf16);
int cake_hop_send(const float* src, int H, int nhdr, int bf16, void* dst_inbox, unsigned int* seq,
                  hipStream_t st);
int cake_hop_recv(const void* inbox, int H, int nhdr, int bf16, float* dst, unsigned int* seq,
                  int* err, double timeout_s, hipStream_t st);
}

namespace cake {
namespace {

// Entry points of csrc/experimental/attn_oproj.hip, found in the loaded kernel library
// (the one that holds cake_attn_decode) when it was built with CAKE_BUILD_EXPERIMENTAL=1;
// all null otherwise.
struct AoFns {
  int (*supported)(int, int, int, int) = nullptr;
  long long (*ws_floats)(int, int) = nullptr;
  long long (*ticket_words)(int, int) = nullptr;
  int (*run)(int, const float*, const void*, const void*, const int*, int, int, int, int, float,
             const void*, int, int, float*, int, float*, unsigned int*, unsigned int*,
             hipStream_t) = nullptr;
};

AoFns ao_fns() {
  AoFns f;
  Dl_info info;
  if (!dladdr(reinterpret_cast<void*>(&cake_attn_decode), &info) || !info.dli_fname) return f;
  void* h = dlopen(info.dli_fname, RTLD_LAZY | RTLD_NOLOAD);
  if (!h) return f;
  f.supported = reinterpret_cast<decltype(f.supported)>(dlsym(h, "cake_attn_oproj_supported"));
  f.ws_floats = reinterpret_cast<decltype(f.ws_floats)>(dlsym(h, "cake_attn_oproj_ws_floats"));
  f.ticket_words =
      reinterpret_cast<decltype(f.ticket_words)>(dlsym(h, "cake_attn_oproj_ticket_words"));
  f.run = reinterpret_cast<decltype(f.run)>(dlsym(h, "cake_attn_oproj"));
  if (!f.supported || !f.ws_floats || !f.ticket_words || !f.run) f = AoFns{};
  return f;
}

constexpr int kHeadSelectMaxLastN = 256;  // gemv.hip head_select window bound
constexpr int kAttnMaxSplit = 64;         // attention.hip kMaxSplit


// ---------------------------------------------------------------------------
// model config (config.json; models/llama3/config.py from_dict)
// ---------------------------------------------------------------------------
struct Cfg {
  int H = 0, I = 0, V = 0, L = 0, nh = 0, nkv = 0, hd = 0;
  double eps = 1e-5, theta = 10000.0;
  bool tie = false;
  std::vector<int> eos;
  Json rope_scaling;

  static Cfg parse(const Json& d) {
    auto num = [&](const char* k, double def) {
      return d.has(k) && d.get(k).is_number() ? d.get(k).as_double() : def;
    };
    Cfg c;
    c.H = (int)d.get("hidden_size").as_int();
    c.I = (int)d.get("intermediate_size").as_int();
    c.V = (int)d.get("vocab_size").as_int();
    c.L = (int)d.get("num_hidden_layers").as_int();
    c.nh = (int)d.get("num_attention_heads").as_int();
    c.nkv = d.has("num_key_value_heads") && d.get("num_key_value_heads").is_number()
                ? (int)d.get("num_key_value_heads").as_int() : c.nh;
    c.hd = c.H / c.nh;
    c.eps = num("rms_norm_eps", 1e-5);
    c.theta = num("rope_theta", 10000.0);
    c.tie = d.has("tie_word_embeddings") && d.get("tie_word_embeddings").type() == Json::Bool &&
            d.get("tie_word_embeddings").as_bool();
    if (d.has("eos_token_id")) {
      const Json& e = d.get("eos_token_id");
      if (e.is_array()) {
        for (const auto& x : e.items()) c.eos.push_back((int)x.as_int());
      } else if (e.is_number()) {
        c.eos.push_back((int)e.as_int());
      }
    }
    if (d.has("rope_scaling")) c.rope_scaling = d.get("rope_scaling");
    return c;
  }

  // theta_i = 1 / theta^(2i/d) with optional Llama-3.1 "llama3" scaling (f64, as
  // ops/reference.py inv_freq)
  std::vector<float> inv_freq() const {
    std::vector<float> out(hd / 2);
    const bool l3 = rope_scaling.is_object() &&
                    ((rope_scaling.has("rope_type") && rope_scaling.get("rope_type").is_string() &&
                      rope_scaling.get("rope_type").as_string() == "llama3") ||
                     (rope_scaling.has("type") && rope_scaling.get("type").is_string() &&
                      rope_scaling.get("type").as_string() == "llama3"));
    auto rs = [&](const char* k, double def) {
      return rope_scaling.has(k) && rope_scaling.get(k).is_number() ? rope_scaling.get(k).as_double()
                                                                    : def;
    };
    for (int i = 0; i < hd / 2; ++i) {
      double f = 1.0 / std::pow(theta, (double)(2 * i) / (double)hd);
      if (l3) {
        const double factor = rs("factor", 8.0), lo = rs("low_freq_factor", 1.0),
                     hi = rs("high_freq_factor", 4.0),
                     old = rs("original_max_position_embeddings", 8192.0);
        const double lo_wl = old / lo, hi_wl = old / hi, wl = 2.0 * M_PI / f;
        const double o = wl > lo_wl ? f / factor : f;
        const double smooth = (old / wl - lo) / (hi - lo);
        const double mid = (1.0 - smooth) * o / factor + smooth * o;
        f = (wl >= hi_wl && wl <= lo_wl) ? mid : o;
      }
      out[i] = (float)f;
    }
    return out;
  }
};


constexpr int kEpiStore = 0, kEpiResid32 = 1, kEpiSwiglu = 3, kEpiStore32 = 6;

// Contiguous layer shards, rank 0 lighter by the head's weight in blocks
// (parallel/pipeline.py shard_layers + head_cost_in_layers).
std::vector<std::pair<int, int>> shard_layers(const Cfg& c, int world) {
  std::vector<std::pair<int, int>> out;
  if (world <= 1) {
    out.push_back({0, c.L});
    return out;
  }
  if (world > c.L) {  // one layer per rank, the ranks past the last layer idle
    for (int r = 0; r < world; ++r) out.push_back(r < c.L ? std::make_pair(r, r + 1)
                                                          : std::make_pair(c.L, c.L));
    return out;
  }
  const double layer_bytes = 2.0 * ((double)c.H * (c.nh + 2 * c.nkv) * c.hd +
                                    (double)c.nh * c.hd * c.H + 3.0 * c.H * c.I + 2.0 * c.H);
  const double head = 2.0 * (double)c.V * c.H / layer_bytes;
  const double total = c.L + head;
  int start = 0;
  for (int r = 0; r < world; ++r) {
    int end = r < world - 1 ? (int)std::nearbyint((r + 1) * total / world - head) : c.L;
    end = std::max(start + (c.L - start >= world - r ? 1 : 0), std::min(end, c.L - (world - 1 - r)));
    out.push_back({start, end});
    start = end;
  }
  return out;
}

// [start, end) of rank's contiguous share of n items (parallel/tensor_parallel.py)
std::pair<int, int> split_range(int n, int world, int rank) {
  const int q = n / world, r = n % world;
  const int a = rank * q + std::min(rank, r);
  return {a, a + q + (rank < r ? 1 : 0)};
}

// CAKE_ENGINE_TRACE=1: control-plane progress on stderr (rank-tagged, seconds since the
// process's first trace line) — where a multi-rank start or generation stands
bool trace_on() {
  static const bool on = [] {
    const char* v = std::getenv("CAKE_ENGINE_TRACE");
    return v && *v && std::string(v) != "0";
  }();
  return on;
}
void trace(int rank, const std::string& what) {
  if (!trace_on()) return;
  static const auto t0 = std::chrono::steady_clock::now();
  const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::fprintf(stderr, "[engine r%d +%.3fs] %s\n", rank, t, what.c_str());
  std::fflush(stderr);
}

Json msg(const char* cmd) {
  Json j = Json::object();
  j.set("cmd", Json::string(cmd));
  return j;
}

// ---------------------------------------------------------------------------
// the engine
// ---------------------------------------------------------------------------
class Llama {
 public:
  Llama(const std::string& dir, const CakeEngineOpts& o, const CakePipeOpts* pp = nullptr,
        const std::vector<int>* layers = nullptr, const CakeTPOpts* tp = nullptr,
        const CakeRemoteOpts* remote = nullptr)
      : dt_(o.dtype), dev_(o.device), init_(o.init), seed_(o.seed) {
    if (dt_ != 0 && dt_ != 1) throw Error("dtype must be 0 (bf16) or 1 (f16)");
    if (init_ != 0 && init_ != 1) throw Error("init must be 0 (checkpoint) or 1 (random)");
    if (tp) {
      tp_ = tp->world;
      tp_rank_ = tp->rank;
      hop_timeout_ = tp->timeout_s > 0 ? tp->timeout_s : 30.0;
      if (tp_ < 1 || tp_ > 8 || tp_rank_ < 0 || tp_rank_ >= tp_) throw Error("bad TP rank / world");
      int n = 0;
      hip_check(hipGetDeviceCount(&n), "hipGetDeviceCount");
      if (n > 0) dev_ %= n;
    }
    if (pp) {
      rank_ = pp->rank;
      world_ = pp->world;
      hop_bf16_ = pp->hop_bf16 != 0;
      hop_timeout_ = pp->hop_timeout_s > 0 ? pp->hop_timeout_s : 30.0;
      if (world_ < 1 || rank_ < 0 || rank_ >= world_) throw Error("bad rank / world");
      // one process per GPU; more ranks than GPUs share them round-robin (rehearsals on
      // a one-GPU box, as parallel/pipeline_bench.py DistEnv)
      int n = 0;
      hip_check(hipGetDeviceCount(&n), "hipGetDeviceCount");
      if (n > 0) dev_ %= n;
    }
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    hip_check(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking), "hipStreamCreate");
    cfg_ = Cfg::parse(Json::parse(read_file(dir + "/config.json")));
    S_ = o.max_seq > 0 ? o.max_seq : 4096;
    k_ = std::max(1, o.steps_per_graph);
    if (cfg_.H % 8 || cfg_.hd % 2 || cfg_.nh % cfg_.nkv) throw Error("unsupported model shape");
    // this rank's compute shapes: the whole model, or its tensor-parallel slice
    lc_ = cfg_;
    if (tp_ > 1) {
      if (cfg_.nh % tp_ || cfg_.nkv % tp_)
        throw Error("tensor-parallel degree must divide the query and KV heads");
      lc_.nh = cfg_.nh / tp_;
      lc_.nkv = cfg_.nkv / tp_;
      const auto ir = split_range(cfg_.I, tp_, tp_rank_);
      const auto vr = split_range(cfg_.V, tp_, tp_rank_);
      i0_ = ir.first;
      lc_.I = ir.second - ir.first;
      voff_ = vr.first;
      lc_.V = vr.second - vr.first;
      if (lc_.I % 8 || (lc_.nh * cfg_.hd) % 8) throw Error("tensor-parallel slice not 8-aligned");
    }
    if (layers) {  // a TCP worker: the topology node's layers, no embedding / head
      owned_ = *layers;
      std::sort(owned_.begin(), owned_.end());
      owned_.erase(std::unique(owned_.begin(), owned_.end()), owned_.end());
      if (owned_.empty() || owned_.front() < 0 || owned_.back() >= cfg_.L)
        throw Error("worker layers outside the model");
      head_ = false;
    } else {
      // layer -> rank: the topology's owner map, or contiguous shards
      const bool placed = pp && pp->owners && pp->n_owners > 0;
      owner_.assign(cfg_.L, 0);
      if (placed) {
        if (pp->n_owners != cfg_.L)
          throw Error("owner map has " + std::to_string(pp->n_owners) + " entries for " +
                      std::to_string(cfg_.L) + " layers");
        for (int l = 0; l < cfg_.L; ++l) {
          if (pp->owners[l] < 0 || pp->owners[l] >= world_)
            throw Error("layer " + std::to_string(l) + " placed on rank " +
                        std::to_string(pp->owners[l]) + " outside the world of " +
                        std::to_string(world_));
          owner_[l] = pp->owners[l];
        }
      } else {
        const auto sh = shard_layers(cfg_, world_);
        for (int r = 0; r < world_; ++r)
          for (int l = sh[r].first; l < sh[r].second; ++l) owner_[l] = r;
      }
      if (remote) {  // TCP workers: layer -> worker index, -1 = local
        if (remote->n_layers != cfg_.L || !remote->worker_of)
          throw Error("remote placement must name every layer (-1 = local)");
        remote_of_.assign(remote->worker_of, remote->worker_of + cfg_.L);
        for (int l = 0; l < cfg_.L; ++l)
          if (remote_of_[l] < -1 || remote_of_[l] >= remote->n_workers)
            throw Error("layer " + std::to_string(l) + " placed on an unknown worker");
        for (int w = 0; w < remote->n_workers; ++w)
          remotes_.push_back({remote->workers[w] ? remote->workers[w] : "", -1});
        remote_timeout_ = remote->timeout_s > 0 ? remote->timeout_s : 60.0;
      }
      for (int l = 0; l < cfg_.L; ++l)
        if (owner_[l] == rank_ && (remote_of_.empty() || remote_of_[l] < 0)) owned_.push_back(l);
      head_ = rank_ == 0;
    }
    lo_ = owned_.empty() ? 0 : owned_.front();
    hi_ = owned_.empty() ? 0 : owned_.back() + 1;
    local_.assign(cfg_.L, -1);
    for (size_t i = 0; i < owned_.size(); ++i) local_[owned_[i]] = (int)i;
    if (!layers) plan_walk();
    planner_.load(pkg_dir() + "/ops/gemm_tuned.json");
    load_weights(dir);
    alloc_state();
    warm_library();
    {
      size_t fr = 0, tot = 0;
      (void)hipMemGetInfo(&fr, &tot);
      trace(rank(), "weights + state ready (" + std::to_string(owned_.size()) + " layers), " +
                        std::to_string(fr >> 20) + " of " + std::to_string(tot >> 20) +
                        " MiB free");
    }
    if (world_ > 1) {
      connect_pipeline(pp->master_addr ? pp->master_addr : "127.0.0.1:29517",
                       pp->connect_timeout_s > 0 ? pp->connect_timeout_s : 600.0);
      trace(rank_, "pipeline connected: walk " + walk_str() + ", " +
                       std::to_string(edges_.size()) + " edges");
      selftest_pipeline();
      trace(rank_, "pipeline self-test passed");
    }
    if (tp_ > 1) {
      connect_tp(tp->master_addr ? tp->master_addr : "127.0.0.1:29517",
                 tp->connect_timeout_s > 0 ? tp->connect_timeout_s : 600.0);
      trace(rank(), "tensor-parallel channels mapped");
      selftest_tp();
      trace(rank(), "tensor-parallel self-test passed");
    }
    if (!remotes_.empty()) connect_remotes();
  }

  ~Llama() {
    (void)hipSetDevice(dev_);
    (void)hipStreamSynchronize(st_);
    if (rank_ == 0 && tp_rank_ == 0)
      for (int fd : peers_) {
        try {
          send_json(fd, msg("exit"));
        } catch (const std::exception&) {
        }
      }
    for (int fd : peers_) tcp_close(fd);
    if (ctl_fd_ >= 0) tcp_close(ctl_fd_);
    for (auto& r : remotes_)
      if (r.fd >= 0) tcp_close(r.fd);
    drop_graphs();
    for (void* p : tp_mapped_) (void)hipIpcCloseMemHandle(p);
    for (void* p : tp_owned_) (void)cake_hop_free(p);
    for (auto& kv : out_inbox_) (void)hipIpcCloseMemHandle(kv.second);
    for (auto& kv : peer_pbuf_) (void)hipIpcCloseMemHandle(kv.second);
    for (auto& kv : my_inbox_) (void)cake_hop_free(kv.second);
    if (relay_) (void)cake_hop_free(relay_);
    for (void* p : allocs_) (void)hipFree(p);
    (void)hipStreamDestroy(st_);
  }

  int rank() const { return tp_ > 1 ? tp_rank_ : rank_; }
  int world() const { return tp_ > 1 ? tp_ : world_; }
  std::pair<int, int> layer_range() const { return {lo_, hi_}; }

  const Cfg& cfg() const { return cfg_; }
  int max_seq() const { return S_; }

  void prefill_logits(const int32_t* prompt, int T, float* host_logits) {
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    if (!head_) throw Error("prefill_logits() runs on pipeline rank 0");
    prefill(prompt, T);
    hip_check(hipMemcpyAsync(host_logits, logits_, sizeof(float) * cfg_.V, hipMemcpyDeviceToHost,
                             st_), "logits D2H");
    hip_check(hipStreamSynchronize(st_), "sync");
  }

  void forced_logits(const int32_t* prompt, int T, const int32_t* forced, int n, float* out) {
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    if (!head_ || tp_rank_ != 0) throw Error("forced_logits() runs on rank 0");
    if (T <= 0 || n < 0 || T + n + 1 > S_) throw Error("prompt + forced tokens exceed max_seq");
    forced_run(prompt, T, forced, n, out);
  }

  void generate(const int32_t* prompt, int T, int max_new, const CakeEngineSampling& smp,
                const int32_t* eos, int n_eos, cake_engine_token_cb cb, void* ctx, int32_t* out,
                int out_cap, CakeEngineStats* stats) {
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    if (!head_) throw Error("generate() runs on pipeline rank 0");
    if (tp_ > 1 && tp_rank_ != 0) throw Error("generate() runs on tensor-parallel rank 0");
    if (T <= 0) throw Error("empty prompt");
    if (max_new <= 0) return;
    if (T + max_new + k_ + 1 > S_) throw Error("prompt + max_new exceeds max_seq");
    if (out_cap < max_new) throw Error("output buffer smaller than max_new");
    if (tp_ > 1) {  // every tensor-parallel rank runs the same steps: tell them what
      Json m = msg("generate");
      Json pr = Json::array();
      for (int i = 0; i < T; ++i) pr.push(Json::integer(prompt[i]));
      m.set("prompt", pr);
      m.set("max_new", Json::integer(max_new));
      m.set("temperature", Json::number(smp.temperature));
      m.set("top_k", Json::integer(smp.top_k));
      m.set("top_p", Json::number(smp.top_p));
      m.set("seed", Json::string(std::to_string(smp.seed)));
      m.set("penalty", Json::number(smp.repeat_penalty));
      m.set("last_n", Json::integer(smp.repeat_last_n));
      m.set("eos", eos_json(eos, n_eos));
      for (int fd : peers_) send_json(fd, m);
    }
    run_generation(prompt, T, max_new, smp, eos, n_eos, cb, ctx, out, out_cap, stats, true);
  }

  // More tokens after the last generate / continue: the device history, position and
  // graphs (same sampling mode) are where that call left them.
  void continue_gen(int max_new, const int32_t* eos, int n_eos, cake_engine_token_cb cb,
                    void* ctx, int32_t* out, int out_cap, CakeEngineStats* stats) {
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    if (!head_) throw Error("continue() runs on pipeline rank 0");
    if (tp_ > 1 && tp_rank_ != 0) throw Error("continue() runs on tensor-parallel rank 0");
    if (!have_graphs_) throw Error("continue() needs a previous generate()");
    if (max_new <= 0) return;
    if (out_cap < max_new) throw Error("output buffer smaller than max_new");
    const int L = read_i32(hist_len_);
    if (L + max_new + k_ + 1 > S_) throw Error("context + max_new exceeds max_seq");
    if (tp_ > 1) {
      Json m = msg("continue");
      m.set("max_new", Json::integer(max_new));
      m.set("eos", eos_json(eos, n_eos));
      for (int fd : peers_) send_json(fd, m);
    }
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<float> ms;
    const int n_out = remote_mode()
                          ? decode_eager(L - 1, max_new, last_mode_, eos, n_eos, cb, ctx, out,
                                         out_cap, &ms)
                          : decode_tokens(L, max_new, eos, n_eos, cb, ctx, out, out_cap, true, &ms);
    const auto t1 = std::chrono::steady_clock::now();
    if (stats) {
      fill_stats(stats, L, n_out, 0.0, std::chrono::duration<double>(t1 - t0).count(), ms);
      // every token of a continuation is a decode step: the rate counts all of them
      stats->tokens_per_s = stats->decode_s > 0 ? n_out / stats->decode_s : 0.0;
    }
  }

  // A tensor-parallel rank's callback never stops the generation (every rank must replay
  // the same steps: they all stop at the same EOS token, which each reads back itself);
  // the lead's callback only sees the tokens.
  struct TpStop {
    cake_engine_token_cb cb;
    void* ctx;
    bool stopped;
  };
  static int32_t tp_token_cb(void* vctx, int32_t tok) {
    auto* t = static_cast<TpStop*>(vctx);
    if (!t->stopped && t->cb && t->cb(t->ctx, tok) != 0) t->stopped = true;
    return 0;
  }

  static Json eos_json(const int32_t* eos, int n_eos) {
    Json a = Json::array();
    for (int i = 0; i < n_eos; ++i) a.push(Json::integer(eos[i]));
    return a;
  }

  // n tokens of graph replays after history length L (device position L - 1); 0 or the
  // tokens kept (lead: written to out, EOS inclusive); per-token device ms in *ms_out
  int decode_tokens(int L, int n, const int32_t* eos, int n_eos, cake_engine_token_cb cb,
                    void* ctx, int32_t* out, int out_cap, bool lead, std::vector<float>* ms_out) {
    std::vector<int32_t> toks(n);
    std::vector<float> ms(n, 0.f);
    CakeLoopSpec spec{};
    std::vector<void*> execs(execs_.begin(), execs_.end());
    spec.execs = execs.data();
    spec.n_execs = (int32_t)execs.size();
    spec.bucket_of = bucket_of_.data();
    spec.n_len = (int32_t)bucket_of_.size();
    spec.k = k_;
    spec.hist = hist_;
    spec.base = L;      // history index of the first token of this run
    spec.pos = L - 1;   // device position (last written row)
    spec.n = n;
    spec.chunk = 0;
    AnnounceCtx actx{this, L - 1};
    if (world_ > 1) {  // the workers enqueue each chunk of replays when told
      spec.chunk = kAnnounceChunk;
      spec.announce = &Llama::announce_cb;
      spec.announce_ctx = &actx;
    }
    spec.eos = eos;
    spec.n_eos = n_eos;
    spec.on_token = cb;
    spec.token_ctx = ctx;
    spec.stream = st_;
    spec.out_tokens = toks.data();
    spec.out_ms = ms.data();
    spec.out_cap = n;
    TpStop tps{cb, ctx, false};
    if (tp_ > 1) {  // lock step: every rank reads the tokens back and stops at EOS
      spec.on_token = lead ? &Llama::tp_token_cb : nullptr;
      spec.token_ctx = &tps;
    }
    CakeLoopResult res{};
    trace(rank(), "decode " + std::to_string(n) + " tokens from length " + std::to_string(L));
    const int rc = cake_graph_decode(&spec, &res);
    trace(rank(), "decode loop done: " + std::to_string(res.n_tokens) + " tokens, " +
                      std::to_string(res.replays) + " replays, rc " + std::to_string(rc));
    if (world_ > 1) sync_workers();
    if (tp_ > 1 && lead) sync_tp_workers();
    k_check(rc, "graph_decode");
    if (lead) check_attn_error("rank " + std::to_string(rank()));  // TP workers: in "sync"
    int n_out = 0;
    if (lead)
      for (int i = 0; i < res.n_tokens && n_out < out_cap; ++i) out[n_out++] = toks[i];
    ms.resize(lead ? res.n_tokens : 0);
    if (ms_out) *ms_out = std::move(ms);
    return n_out;
  }

  void fill_stats(CakeEngineStats* stats, int n_prompt, int n_out, double prefill_s,
                  double decode_s, const std::vector<float>& ms) const {
    stats->n_prompt = n_prompt;
    stats->n_generated = n_out;
    stats->prefill_s = prefill_s;
    stats->decode_s = decode_s;
    stats->tokens_per_s = n_out > 1 && decode_s > 0 ? (n_out - 1) / decode_s : 0.0;
    std::vector<float> s = ms;
    std::sort(s.begin(), s.end());
    auto pct = [&](double q) {
      if (s.empty()) return 0.f;
      const size_t i = std::min(s.size() - 1, (size_t)std::llround(q / 100.0 * (s.size() - 1)));
      return s[i];
    };
    stats->p50_ms = pct(50);
    stats->p99_ms = pct(99);
  }

  void run_generation(const int32_t* prompt, int T, int max_new, const CakeEngineSampling& smp,
                      const int32_t* eos, int n_eos, cake_engine_token_cb cb, void* ctx,
                      int32_t* out, int out_cap, CakeEngineStats* stats, bool lead) {
    const auto t0 = std::chrono::steady_clock::now();
    prefill_body(prompt, T);
    // the prefill position bookkeeping of DeviceDecoder.start: history = prompt,
    // pos = T - 1 (the last written row), slot cleared
    std::vector<int32_t> h(prompt, prompt + T);
    hip_check(hipMemcpyAsync(hist_, h.data(), sizeof(int32_t) * T, hipMemcpyHostToDevice, st_),
              "hist H2D");
    set_i32(hist_len_, T);
    set_i32(pos_, T - 1);
    hip_check(hipMemsetAsync(slot_, 0, sizeof(unsigned long long), st_), "slot");
    Mode mode = mode_of(smp);
    // first token from the prefill logits (DeviceDecoder._select_first)
    if (tp_ > 1) {
      head_tp(hidden_ + (size_t)(T - 1) * cfg_.H, mode);
    } else {
      k_check(cake_gemv_norm_f32(dt_, hidden_ + (size_t)(T - 1) * cfg_.H, norm_, (float)lc_.eps,
                                 lm_head_, lc_.H, lc_.V, logits_, st_), "lm_head");
      select_tail(mode);
    }
    if (mode.fused) k_check(cake_embed(dt_, embed_, tok_, 1, cfg_.H, resid_, st_), "embed");
    int32_t first = 0;
    hip_check(hipMemcpyAsync(&first, tok_, sizeof(int32_t), hipMemcpyDeviceToHost, st_), "tok");
    hip_check(hipStreamSynchronize(st_), "sync");
    const auto t1 = std::chrono::steady_clock::now();
    int n_out = 0;
    bool stop = false;
    for (int e = 0; e < n_eos && !stop; ++e)
      if (eos[e] == first) stop = true;
    if (lead) {
      out[n_out++] = first;
      const bool cb_stop = cb && cb(ctx, first) != 0;
      if (tp_ == 1) stop = stop || cb_stop;  // TP: only EOS stops (all ranks alike)
    }
    std::vector<float> ms;
    last_mode_ = mode;
    if (remote_mode()) {  // host round trips inside the step: eager
      have_graphs_ = true;  // continue() may follow
      if (!stop && max_new > 1)
        n_out += decode_eager(T, max_new - 1, mode, eos, n_eos, cb, ctx, out + n_out,
                              out_cap - n_out, &ms);
    } else {
      // graphs exist after every generation (continue() replays them), even a 1-token one
      ensure_graphs(mode);
      if (!stop && max_new > 1)
        n_out += decode_tokens(T + 1, max_new - 1, eos, n_eos, cb, ctx,
                               lead ? out + n_out : nullptr, lead ? out_cap - n_out : 0, lead, &ms);
    }
    const auto t2 = std::chrono::steady_clock::now();
    if (stats)
      fill_stats(stats, T, n_out, std::chrono::duration<double>(t1 - t0).count(),
                 std::chrono::duration<double>(t2 - t1).count(), ms);
  }

  int read_i32(const int* p) {
    int v = 0;
    hip_check(hipMemcpyAsync(&v, p, sizeof(int), hipMemcpyDeviceToHost, st_), "i32 D2H");
    hip_check(hipStreamSynchronize(st_), "sync");
    return v;
  }

  // the split-K attention merge's error word (tickets[2 nkv], attn_core2.h): a merge
  // that gave up waiting for its partials left that launch's outputs invalid
  void check_attn_error(const std::string& who) {
    unsigned int w = 0;
    hip_check(hipMemcpyAsync(&w, tickets_ + 2 * lc_.nkv, sizeof(w), hipMemcpyDeviceToHost, st_),
              "attn err D2H");
    hip_check(hipStreamSynchronize(st_), "sync");
    if (w) {
      hip_check(hipMemsetAsync(tickets_ + 2 * lc_.nkv, 0, sizeof(unsigned int), st_), "attn err");
      hip_check(hipStreamSynchronize(st_), "sync");
      throw Error(who + ": decode attention split merge timed out waiting for its partials; "
                        "the tokens of that generation are invalid");
    }
  }

 private:
  struct LayerW { void *ln1, *wqkv, *wo, *ln2, *wgu, *wd; };
  struct Mode {
    bool fused = true;  // greedy with the fused head_select tail
    bool greedy = true;
    float temperature = 0.f, top_p = 0.f, penalty = 1.f;
    int top_k = 0, last_n = 0;
    unsigned long long seed = 0;
    bool operator==(const Mode& o) const {
      return std::tie(fused, greedy, temperature, top_p, penalty, top_k, last_n, seed) ==
             std::tie(o.fused, o.greedy, o.temperature, o.top_p, o.penalty, o.top_k, o.last_n,
                      o.seed);
    }
  };

  int dt_, dev_, init_ = 0;
  bool forced_ = false;  // teacher-forcing steps: the head writes full logits
  // fused decode attention + o_proj (attn_oproj.hip) for one-split live lengths: the
  // short-context graph bucket and eager steps at such a position
  // fused attention + o_proj (csrc/experimental/attn_oproj.hip, CAKE_BUILD_EXPERIMENTAL=1;
  // measured slower than the pair: profiles/r5_attn_oproj_ab.md), looked up at run time
  AoFns ao_;
  bool ao_ok_ = false, short_step_ = false;
  int heads_max_ = 0;  // live lengths <= this: head-parallel attention (attn_head_kernel)
  float* ao_ws_ = nullptr;
  unsigned int* ao_tickets_ = nullptr;
  uint64_t seed_ = 0;
  int rank_ = 0, world_ = 1, lo_ = 0, hi_ = 0;
  bool head_ = true, hop_bf16_ = false;
  double hop_timeout_ = 30.0;
  // The token's walk (llama.rs:81-117): embedding on rank 0, then every maximal run of
  // consecutive layers on one rank, then the head on rank 0.  An edge joins consecutive
  // stops on different ranks; each edge has its own inbox on the receiving rank and its
  // own sequence words (seq_[2e] send side, seq_[2e + 1] receive side).
  enum StopKind { kEmbedStop, kRunStop, kHeadStop, kRemoteStop };
  struct Stop {
    StopKind kind;
    int rank;
    std::vector<int> layers;  // global ids (runs)
    std::vector<int> sel;     // the same as this rank's local layer slots
    int remote = -1;          // kRemoteStop: index into remotes_
  };
  // TCP workers (master side): one connection each, Hello -> WorkerInfo at open
  struct RemoteWorker {
    std::string addr;
    int fd;
  };
  std::vector<RemoteWorker> remotes_;
  std::vector<int> remote_of_;  // layer -> remote worker, -1 = local
  double remote_timeout_ = 60.0;
  std::vector<float> host_rows_;  // staging of the hidden rows a remote run transforms
  std::vector<Stop> walk_;
  std::vector<int> edge_in_;                // per stop: the edge feeding it, or -1
  std::vector<std::pair<int, int>> edges_;  // (src rank, dst rank)
  std::vector<int> owner_;                  // layer -> pipeline rank
  std::map<int, void*> my_inbox_;           // edge -> own inbox (edges into this rank)
  std::map<int, void*> out_inbox_;          // edge -> IPC-mapped inbox of the receiver
  std::map<int, void*> peer_pbuf_;          // rank -> IPC-mapped prefill relay buffer
  // prefill rows a peer hands to this rank land here (uncached device memory, IPC-exported,
  // written over xGMI by the sender's copy), then one local copy moves them into hidden_:
  // hidden_ itself stays ordinary cached memory for the GEMM epilogues, and no L2 line of
  // this device can hold a stale copy of what the peer wrote
  float* relay_ = nullptr;
  unsigned int* seq_ = nullptr;
  int* hop_err_ = nullptr;
  std::vector<int> peers_;  // rank 0: control sockets of ranks 1..world-1
  // tensor parallel
  struct ArChan {
    void* inbox = nullptr;
    std::vector<void*> peers;  // peer inboxes (IPC-mapped), own slot unused
  };

  int tp_ = 1, tp_rank_ = 0, i0_ = 0, voff_ = 0, slab_bank_ = 0;
  // rows of one prefill all-reduce round: the slab (2 banks x tp slots x rows x H f32,
  // uncached, IPC-mapped by every peer) is sized for this many rows, a longer prefill
  // runs in rounds — a slab sized for max_seq (2 GB per rank at 70B tp8, 4096 keys) made
  // the eight peer imports stall on one shared GPU
  static constexpr int kSlabRows = 512;
  Cfg lc_;                   // this rank's compute shapes (the whole model unless TP)
  ArChan ch_sum_, ch_key_, ch_gat_;
  float *partial_ = nullptr, *ppart_ = nullptr, *full_logits_ = nullptr, *slab_ = nullptr;
  unsigned int* ar_seq_ = nullptr;
  int* ar_err_ = nullptr;
  std::vector<void*> peer_slab_, tp_mapped_, tp_owned_;
  int ctl_fd_ = -1;         // workers: control socket to rank 0
  hipStream_t st_ = nullptr;
  Cfg cfg_;
  int S_ = 0, k_ = 1;
  GemmPlanner planner_;
  std::vector<void*> allocs_;
  void *embed_ = nullptr, *norm_ = nullptr, *lm_head_ = nullptr;
  std::vector<LayerW> layers_;
  struct KV { uint16_t *k, *v; };           // [local layers][nkv][S][hd]
  std::map<uint64_t, KV> kv_;
  std::list<uint64_t> lru_;
  KV cur_{nullptr, nullptr};
  std::vector<int> owned_, local_;          // global layer ids served here / inverse map
  float* inv_freq_ = nullptr;
  // decode state (graph-stable addresses; DecodeBuffers)
  float *resid_ = nullptr, *q_ = nullptr, *part_ = nullptr, *logits_ = nullptr;
  void *attn_out_ = nullptr, *act_ = nullptr;
  unsigned int *tickets_ = nullptr, *thr_ = nullptr, *sel_ticket_ = nullptr;
  int *pos_ = nullptr, *tok_ = nullptr, *hist_ = nullptr, *hist_len_ = nullptr;
  unsigned long long* slot_ = nullptr;
  int* scratch_i32_ = nullptr;  // warm-up snapshot: tok, pos, hist_len
  float* scratch_resid_ = nullptr;
  int32_t* zeros_ = nullptr;    // 64 zero words (GEMM LDS-DMA padding source)
  // prefill buffers (grown to the longest prompt)
  int pre_T_ = 0;
  float* hidden_ = nullptr;
  void *x16_ = nullptr, *qkv_ = nullptr, *att_ = nullptr, *pact_ = nullptr;
  int32_t* ptok_ = nullptr;
  float* ws_ = nullptr;
  size_t ws_n_ = 0;
  static constexpr size_t kLibWsBytes = 32u << 20;
  uint8_t* lib_ws_ = nullptr;   // hipBLASLt workspace (first library GEMM)
  uint16_t* pgu_ = nullptr;     // [T, 2I] gate|up product of a library SwiGLU GEMM
  size_t pgu_n_ = 0;
  // decode graphs
  std::vector<hipGraphExec_t> execs_;
  std::vector<hipGraph_t> graphs_;
  std::vector<int32_t> bucket_of_;
  Mode graph_mode_, last_mode_;
  bool have_graphs_ = false;

  template <class T> T* dalloc(size_t n) {
    void* p = nullptr;
    hip_check(hipMalloc(&p, std::max<size_t>(n * sizeof(T), 16)), "hipMalloc");
    allocs_.push_back(p);
    return reinterpret_cast<T*>(p);
  }
  void dfree(void* p) {
    if (!p) return;
    auto it = std::find(allocs_.begin(), allocs_.end(), p);
    if (it != allocs_.end()) allocs_.erase(it);
    (void)hipFree(p);
  }

  void set_i32(int* p, int v) {
    hip_check(hipMemcpyAsync(p, &v, sizeof(int), hipMemcpyHostToDevice, st_), "i32 H2D");
    hip_check(hipStreamSynchronize(st_), "sync");  // &v is a stack value
  }

  // ---- weights
  void upload(Checkpoint& ck, const std::string& name, void* dst, size_t numel, void*& stage,
              size_t& stage_bytes) {
    const TensorView& t = ck.tensor(name);
    size_t n = 1;
    for (auto d : t.shape) n *= d;
    if (n != numel) throw Error(name + ": " + std::to_string(n) + " elements, expected " +
                                std::to_string(numel));
    const size_t R = t.shape.empty() ? 1 : t.shape[0];
    upload_slice(ck, name, dst, 0, R, 0, n / R, stage, stage_bytes);
  }

  // rows [r0, r0 + nr) x columns [c0, c0 + nc) of a 2-D tensor (1-D: one column) into
  // dst as a dense [nr, nc] block in the model dtype (column slices gathered on the host)
  void upload_slice(Checkpoint& ck, const std::string& name, void* dst, size_t r0, size_t nr,
                    size_t c0, size_t nc, void*& stage, size_t& stage_bytes) {
    const TensorView& t = ck.tensor(name);
    int kind;
    if (t.dtype == "BF16") kind = 0;
    else if (t.dtype == "F16") kind = 1;
    else if (t.dtype == "F32") kind = 2;
    else throw Error(name + ": unsupported dtype " + t.dtype);
    const size_t es = kind == 2 ? 4 : 2;
    const size_t R = t.shape.empty() ? 1 : t.shape[0];
    const size_t C = R ? (t.nbytes / es) / R : 0;
    if (r0 + nr > R || c0 + nc > C) throw Error(name + ": slice outside the tensor");
    const uint8_t* src = t.data + (r0 * C + c0) * es;
    std::vector<uint8_t> tmp;
    if (nc != C) {
      tmp.resize(nr * nc * es);
      for (size_t r = 0; r < nr; ++r)
        std::memcpy(tmp.data() + r * nc * es, t.data + ((r0 + r) * C + c0) * es, nc * es);
      src = tmp.data();
    }
    const size_t bytes = nr * nc * es, n = nr * nc;
    if (kind == dt_) {
      hip_check(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice), "weight H2D");
      return;
    }
    if (stage_bytes < bytes) {
      if (stage) (void)hipFree(stage);
      hip_check(hipMalloc(&stage, bytes), "hipMalloc stage");
      stage_bytes = bytes;
    }
    hip_check(hipMemcpy(stage, src, bytes, hipMemcpyHostToDevice), "weight H2D");
    k_check(cake_cast16(kind, dt_, stage, dst, n, st_), "cast16");
    hip_check(hipStreamSynchronize(st_), "sync");
  }

  // weights of this rank: all of the model, its pipeline layers, or (tensor parallel) its
  // slices — q / k / v rows of its heads, o_proj columns of its heads, gate / up rows and
  // down_proj columns of its intermediate range, lm_head rows of its vocabulary range
  // (parallel/tensor_parallel.py shard_block / shard_head)
  // init = 1: this rank's tensors (same shapes and packing as a checkpoint load) drawn
  // on the device — N(0, 0.02) linears and lm_head, N(0, 1) embedding, N(1, 0.05) norms
  // (models/llama3/weights.py random) — keyed by (seed, layer, tensor)
  void load_random() {
    const Cfg& c = cfg_;
    const size_t H = c.H, V = c.V, hd = c.hd;
    const size_t nq = (size_t)lc_.nh * hd, nk = (size_t)lc_.nkv * hd, I = lc_.I;
    auto fill = [&](void* p, size_t n, float mean, float std, uint64_t tag) {
      const uint64_t key = seed_ * 0x9e3779b97f4a7c15ULL + tag * 0xc2b2ae3d27d4eb4fULL +
                           (uint64_t)tp_rank_ * 0x165667b19e3779f9ULL;
      k_check(cake_fill_normal(dt_, p, n, mean, std, key, st_), "fill_normal");
    };
    if (head_) {
      embed_ = dalloc<uint16_t>(V * H);
      fill(embed_, V * H, 0.f, 1.f, 1);
      norm_ = dalloc<uint16_t>(H);
      fill(norm_, H, 1.f, 0.05f, 2);
      if (c.tie && tp_ == 1) {
        lm_head_ = embed_;
      } else {
        lm_head_ = dalloc<uint16_t>((size_t)lc_.V * H);
        fill(lm_head_, (size_t)lc_.V * H, 0.f, 0.02f, 3);
      }
    }
    layers_.resize(owned_.size());
    for (int l : owned_) {
      LayerW& w = layers_[local_[l]];
      const uint64_t t = 16 + 16 * (uint64_t)l;
      w.ln1 = dalloc<uint16_t>(H);
      fill(w.ln1, H, 1.f, 0.05f, t);
      w.wqkv = dalloc<uint16_t>((nq + 2 * nk) * H);
      fill(w.wqkv, (nq + 2 * nk) * H, 0.f, 0.02f, t + 1);
      w.wo = dalloc<uint16_t>(H * nq);
      fill(w.wo, H * nq, 0.f, 0.02f, t + 2);
      w.ln2 = dalloc<uint16_t>(H);
      fill(w.ln2, H, 1.f, 0.05f, t + 3);
      w.wgu = dalloc<uint16_t>(2 * I * H);
      fill(w.wgu, 2 * I * H, 0.f, 0.02f, t + 4);
      w.wd = dalloc<uint16_t>(H * I);
      fill(w.wd, H * I, 0.f, 0.02f, t + 5);
    }
    hip_check(hipStreamSynchronize(st_), "sync");
  }

  void load_weights(const std::string& dir) {
    if (init_ == 1) {
      load_random();
      return;
    }
    Checkpoint ck(dir);
    const Cfg& c = cfg_;
    const size_t H = c.H, V = c.V, hd = c.hd;
    const size_t nq = (size_t)lc_.nh * hd, nk = (size_t)lc_.nkv * hd, I = lc_.I;
    const size_t q0 = (size_t)tp_rank_ * lc_.nh * hd, k0 = (size_t)tp_rank_ * lc_.nkv * hd;
    const size_t i0 = i0_;
    void* stage = nullptr;
    size_t stage_bytes = 0;
    try {
      if (head_) {
        embed_ = dalloc<uint16_t>(V * H);
        upload(ck, "model.embed_tokens.weight", embed_, V * H, stage, stage_bytes);
        norm_ = dalloc<uint16_t>(H);
        upload(ck, "model.norm.weight", norm_, H, stage, stage_bytes);
        const bool own_head = ck.has("lm_head.weight") && !c.tie;
        const char* hn = own_head ? "lm_head.weight" : "model.embed_tokens.weight";
        if (tp_ > 1) {
          lm_head_ = dalloc<uint16_t>((size_t)lc_.V * H);
          upload_slice(ck, hn, lm_head_, voff_, lc_.V, 0, H, stage, stage_bytes);
        } else if (own_head) {
          lm_head_ = dalloc<uint16_t>(V * H);
          upload(ck, hn, lm_head_, V * H, stage, stage_bytes);
        } else {
          lm_head_ = embed_;  // tied embeddings
        }
      }
      layers_.resize(owned_.size());
      for (int l : owned_) {
        const std::string p = "model.layers." + std::to_string(l) + ".";
        LayerW& w = layers_[local_[l]];
        w.ln1 = dalloc<uint16_t>(H);
        upload(ck, p + "input_layernorm.weight", w.ln1, H, stage, stage_bytes);
        w.wqkv = dalloc<uint16_t>((nq + 2 * nk) * H);
        uint16_t* qkv = reinterpret_cast<uint16_t*>(w.wqkv);
        upload_slice(ck, p + "self_attn.q_proj.weight", qkv, q0, nq, 0, H, stage, stage_bytes);
        upload_slice(ck, p + "self_attn.k_proj.weight", qkv + nq * H, k0, nk, 0, H, stage,
                     stage_bytes);
        upload_slice(ck, p + "self_attn.v_proj.weight", qkv + (nq + nk) * H, k0, nk, 0, H, stage,
                     stage_bytes);
        w.wo = dalloc<uint16_t>(H * nq);
        upload_slice(ck, p + "self_attn.o_proj.weight", w.wo, 0, H, q0, nq, stage, stage_bytes);
        w.ln2 = dalloc<uint16_t>(H);
        upload(ck, p + "post_attention_layernorm.weight", w.ln2, H, stage, stage_bytes);
        w.wgu = dalloc<uint16_t>(2 * I * H);
        uint16_t* gu = reinterpret_cast<uint16_t*>(w.wgu);
        upload_slice(ck, p + "mlp.gate_proj.weight", gu, i0, I, 0, H, stage, stage_bytes);
        upload_slice(ck, p + "mlp.up_proj.weight", gu + I * H, i0, I, 0, H, stage, stage_bytes);
        w.wd = dalloc<uint16_t>(H * I);
        upload_slice(ck, p + "mlp.down_proj.weight", w.wd, 0, H, i0, I, stage, stage_bytes);
      }
    } catch (...) {
      if (stage) (void)hipFree(stage);
      throw;
    }
    if (stage) (void)hipFree(stage);
  }


  void alloc_state() {
    const Cfg& c = lc_;
    kv_session(0);  // session 0: generation / pipeline
    const std::vector<float> f = c.inv_freq();
    inv_freq_ = dalloc<float>(f.size());
    hip_check(hipMemcpy(inv_freq_, f.data(), f.size() * sizeof(float), hipMemcpyHostToDevice),
              "inv_freq");
    const size_t nq = (size_t)c.nh * c.hd;
    // [H f32 | pos | pad]: a pipeline hop carries the position as its header word
    resid_ = dalloc<float>(c.H + 4);
    hidden_ = dalloc<float>((size_t)S_ * c.H);  // prefill hidden (peer-written in a pipeline)
    q_ = dalloc<float>(nq);
    part_ = dalloc<float>(2 * (size_t)c.nh * kAttnMaxSplit * (c.hd + 2));
    logits_ = dalloc<float>(c.V);
    attn_out_ = dalloc<uint16_t>(nq);
    act_ = dalloc<uint16_t>(c.I);
    tickets_ = dalloc<unsigned int>(2 * c.nkv + 2);
    thr_ = dalloc<unsigned int>(1);
    sel_ticket_ = dalloc<unsigned int>(1);
    pos_ = reinterpret_cast<int*>(resid_ + c.H);
    tok_ = dalloc<int>(1);
    hist_ = dalloc<int>(S_);
    hist_len_ = dalloc<int>(1);
    slot_ = dalloc<unsigned long long>(1);
    scratch_i32_ = dalloc<int>(4);
    scratch_resid_ = dalloc<float>(c.H + 4);  // + the hop header (self-tests)
    zeros_ = dalloc<int32_t>(64);
    hip_check(hipMemset(tickets_, 0, sizeof(unsigned int) * (2 * c.nkv + 2)), "memset");
    hip_check(hipMemset(part_, 0, sizeof(float) * 2 * c.nh * kAttnMaxSplit * (c.hd + 2)), "memset");
    hip_check(hipMemset(sel_ticket_, 0, sizeof(unsigned int)), "memset");
    hip_check(hipMemset(slot_, 0, sizeof(unsigned long long)), "memset");
    hip_check(hipMemset(zeros_, 0, sizeof(int32_t) * 64), "memset");
    hip_check(hipMemset(hist_, 0, sizeof(int) * S_), "memset");
    hip_check(hipMemset(resid_, 0, sizeof(float) * (c.H + 4)), "memset");
    // opt-in (CAKE_ATTN_OPROJ=1): measured slower than the attention + o_proj pair on
    // MI355X (profiles/r5_attn_oproj_ab.md), kept for the A/B
    {
      const char* e = std::getenv("CAKE_ATTN_OPROJ");
      if (e && std::string(e) == "1") ao_ = ao_fns();
      ao_ok_ = ao_.run != nullptr && ao_.supported(c.nh, c.nkv, c.hd, c.H) != 0;
    }
    // CAKE_ATTN_HEADS=<max keys>[:<waves>]: the head-parallel short-context attention
    if (!ao_ok_) {
      const char* e = std::getenv("CAKE_ATTN_HEADS");
      int mx = 0, nw = 2, pfd = 2;
      if (e && *e) std::sscanf(e, "%d:%d:%d", &mx, &nw, &pfd);
      if (mx > 0 && cake_attn_set_heads(mx, nw) == 0 && cake_attn_set_head_prefetch(pfd) == 0)
        heads_max_ = mx;
    }
    if (ao_ok_) {
      ao_ws_ = dalloc<float>((size_t)ao_.ws_floats(c.nkv, c.H));
      const size_t tw = (size_t)ao_.ticket_words(c.nkv, c.H);
      ao_tickets_ = dalloc<unsigned int>(tw);
      hip_check(hipMemset(ao_tickets_, 0, sizeof(unsigned int) * tw), "memset");
    }
    const size_t nseq = 2 * edges_.size() + 2;  // per edge: send, receive sequence
    seq_ = dalloc<unsigned int>(nseq);
    hop_err_ = dalloc<int>(4);
    hip_check(hipMemset(seq_, 0, sizeof(unsigned int) * nseq), "memset");
    hip_check(hipMemset(hop_err_, 0, sizeof(int) * 4), "memset");
    if (tp_ > 1) {
      partial_ = dalloc<float>(c.H);
      ppart_ = dalloc<float>((size_t)S_ * c.H);
      full_logits_ = dalloc<float>(cfg_.V);
      ar_seq_ = dalloc<unsigned int>(8);  // [channel][tag, ticket]
      ar_err_ = dalloc<int>(4);
      hip_check(hipMemset(ar_seq_, 0, sizeof(unsigned int) * 8), "memset");
      hip_check(hipMemset(ar_err_, 0, sizeof(int) * 4), "memset");
    }
    hip_check(hipDeviceSynchronize(), "sync");  // null-stream memsets before st_ work
  }

  uint16_t* kc(int l) const { return cur_.k + (size_t)l * lc_.nkv * S_ * lc_.hd; }
  uint16_t* vc(int l) const { return cur_.v + (size_t)l * lc_.nkv * S_ * lc_.hd; }

  // KV cache of one session (a master connection of a TCP worker; 0 = generation):
  // allocated on first use, least recently used dropped past kMaxSessions (P4)
  static constexpr size_t kMaxSessions = 8;
  void kv_session(uint64_t id) {
    auto it = kv_.find(id);
    if (it == kv_.end()) {
      if (kv_.size() >= kMaxSessions) {
        uint64_t victim = lru_.front();
        for (uint64_t x : lru_)
          if (x != 0) { victim = x; break; }
        drop_session(victim);
      }
      const size_t n = owned_.size() * (size_t)lc_.nkv * S_ * lc_.hd;
      KV kv{dalloc<uint16_t>(n), dalloc<uint16_t>(n)};
      it = kv_.emplace(id, kv).first;
    }
    lru_.remove(id);
    lru_.push_back(id);
    cur_ = it->second;
  }

 public:
  void drop_session(uint64_t id) {
    auto it = kv_.find(id);
    if (it == kv_.end() || id == 0) return;
    hip_check(hipStreamSynchronize(st_), "sync");
    dfree(it->second.k);
    dfree(it->second.v);
    kv_.erase(it);
    lru_.remove(id);
    if (kv_.count(0)) cur_ = kv_[0];
  }

  // TCP worker compute: `layers` (global indices, this worker's) over hidden [T, H] f32
  // (host, in place) at positions pos0.., with the session's KV cache (worker.rs:236-252;
  // parallel/worker.py _run_ops)
  void forward_host(uint64_t session, const std::vector<int>& layers, int pos0, float* h, int T) {
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    const Cfg& c = lc_;
    if (T < 1 || pos0 < 0 || (int64_t)pos0 + T > S_) throw Error("positions exceed the KV cache");
    std::vector<int> sel;
    for (int l : layers) {
      if (l < 0 || l >= c.L || local_[l] < 0)
        throw Error("layer " + std::to_string(l) + " is not served here");
      sel.push_back(local_[l]);
    }
    kv_session(session);
    if (T == 1) {
      hip_check(hipMemcpyAsync(resid_, h, sizeof(float) * c.H, hipMemcpyHostToDevice, st_), "H2D");
      hip_check(hipMemcpyAsync(pos_, &pos0, sizeof(int), hipMemcpyHostToDevice, st_), "H2D");
      short_step_ = short_at(pos0);
      try {
        step_layers(&sel);
      } catch (...) {
        short_step_ = false;
        throw;
      }
      short_step_ = false;
      hip_check(hipMemcpyAsync(h, resid_, sizeof(float) * c.H, hipMemcpyDeviceToHost, st_), "D2H");
    } else {
      const size_t bytes = sizeof(float) * (size_t)T * c.H;
      hip_check(hipMemcpyAsync(hidden_, h, bytes, hipMemcpyHostToDevice, st_), "H2D");
      prefill_layers(T, pos0, &sel);
      hip_check(hipMemcpyAsync(h, hidden_, bytes, hipMemcpyDeviceToHost, st_), "D2H");
    }
    hip_check(hipStreamSynchronize(st_), "sync");
    if (kv_.count(0)) cur_ = kv_[0];
    if (T == 1) check_attn_error("worker");
  }

 private:
  float scale() const { return 1.0f / std::sqrt((float)cfg_.hd); }

  // an eager step at device position `pos` takes the fused attention + o_proj launch
  // exactly when a one-step graph replay there would (bucket of length pos + 2)
  bool short_at(int pos) const { return short_len(pos + 2); }
  // live lengths served by the cap-1 graph bucket: one split with attention + o_proj fused,
  // or up to heads_max_ keys on the head-parallel attention launch
  bool short_len(int t) const {
    if (ao_ok_) return cake_attn_splits(t) == 1;
    return heads_max_ > 0 && t <= heads_max_;
  }

  // ---- prefill
  void grow_prefill(int T) {
    if (T <= pre_T_) return;
    const Cfg& c = lc_;
    for (void* p : {x16_, qkv_, att_, pact_, (void*)ptok_}) dfree(p);
    const size_t nq = (size_t)c.nh * c.hd, nk = (size_t)c.nkv * c.hd;
    x16_ = dalloc<uint16_t>((size_t)T * c.H);
    qkv_ = dalloc<uint16_t>((size_t)T * (nq + 2 * nk));
    att_ = dalloc<uint16_t>((size_t)T * nq);
    pact_ = dalloc<uint16_t>((size_t)T * c.I);
    ptok_ = dalloc<int32_t>(T);
    pre_T_ = T;
  }

  void gemm(int epi, const void* a, long long lda, const void* b, long long ldb, void* cptr,
            long long ldc, float* resid, long long ldr, int M, int N, int K, const char* what) {
    const bool gated = epi == kEpiSwiglu;
    const long long Nv = gated ? 2LL * N : N;
    static const char* names[] = {"store", "resid32", "add16", "swiglu", "geglu", "partial",
                                  "store32"};
    auto p = planner_.plan(M, Nv, K, names[epi]);
    if (p.first == kGemmLib) {  // the table names the library GEMM (CAKE_GEMM_LIB=1 only)
      if ((epi != kEpiSwiglu || ldc == N) &&
          lib_gemm(epi, a, lda, b, ldb, cptr, ldc, resid, ldr, M, N, K, what))
        return;
      // a strided SwiGLU output or a library failure: the MFMA kernel's plan
      p = planner_.plan_mfma(M, Nv, K, names[epi]);
    }
    const int splits = p.second;
    float* ws = nullptr;
    if (splits > 1) {
      const size_t need = (size_t)cake_gemm_ws_floats(p.first, splits, M, N, K, gated ? 1 : 0);
      if (need > ws_n_) {
        dfree(ws_);
        ws_ = dalloc<float>(need);
        ws_n_ = need;
      }
      ws = ws_;
    }
    k_check(cake_gemm(dt_, epi, p.first, splits, a, lda, b, ldb, cptr, ldc, nullptr, resid, ldr,
                      ws, zeros_, M, N, K, st_), what);
  }

  // hipBLASLt's first call in a process costs ~175 ms (library init; a new shape after it
  // ~0.3 ms: scripts/gpu_runs/gpu_r5_ax.sh): paid here at open, not by the first request's TTFT
  void warm_library() {
    if (!planner_.has_lib()) return;
    if (!lib_ws_) lib_ws_ = dalloc<uint8_t>(kLibWsBytes);
    const size_t n = 64 * 64 + 2 * 8 * 64;  // W [64, 64], A [8, 64], C [8, 64]
    uint16_t* t = dalloc<uint16_t>(n);
    hip_check(hipMemsetAsync(t, 0, n * 2, st_), "memset");
    const int rc = cake_blaslt_gemm(dt_, 0, t + 4096, 64, t, 64, t + 4096 + 512, 64, 8, 64, 64,
                                    lib_ws_, kLibWsBytes, st_);
    hip_check(hipStreamSynchronize(st_), "sync");
    dfree(t);
    if (rc)  // best effort: a library that cannot start leaves every shape on the MFMA kernel
      std::fprintf(stderr, "cake engine: hipBLASLt warm-up failed (rc %d); MFMA GEMMs only\n", rc);
  }

  // store -> 16-bit C; store32 / resid32 -> f32 C with beta 0 / 1; swiglu -> the [M, 2N]
  // product into pgu_, then silu(gate) * up into C.  false (nothing written) when the
  // library refuses the shape: the caller runs the MFMA kernel instead
  bool lib_gemm(int epi, const void* a, long long lda, const void* b, long long ldb, void* cptr,
                long long ldc, float* resid, long long ldr, int M, int N, int K,
                const char* what) {
    if (!lib_ws_) lib_ws_ = dalloc<uint8_t>(kLibWsBytes);
    auto run = [&](int mode, void* c, long long ld, int n) {
      return cake_blaslt_gemm(dt_, mode, a, lda, b, ldb, c, ld, M, n, K, lib_ws_, kLibWsBytes,
                              st_) == 0;
    };
    if (epi == kEpiStore) {
      return run(0, cptr, ldc, N);
    } else if (epi == kEpiStore32 || epi == kEpiResid32) {
      return run(epi == kEpiStore32 ? 1 : 2, resid, ldr, N);
    } else if (epi == kEpiSwiglu && ldc == N) {
      const size_t need = (size_t)M * 2 * N;
      if (need > pgu_n_) {
        dfree(pgu_);
        pgu_ = dalloc<uint16_t>(need);
        pgu_n_ = need;
      }
      if (!run(0, pgu_, 2LL * N, 2 * N)) return false;
      k_check(cake_silu_mul_rows(dt_, pgu_, M, N, cptr, st_), what);
      return true;
    } else {
      throw Error(std::string(what) + ": no library form of this epilogue");
    }
  }

  // embed -> this rank's layers -> (pipeline: the other ranks' layers, hidden rows
  // handed rank to rank through the peers' IPC-mapped prefill buffers) -> head
  void prefill(const int32_t* prompt, int T) {
    prefill_body(prompt, T);
    const Cfg& c = lc_;
    k_check(cake_gemv_norm_f32(dt_, hidden_ + (size_t)(T - 1) * c.H, norm_, (float)c.eps,
                               lm_head_, c.H, c.V, logits_, st_), "lm_head");
  }

  void prefill_body(const int32_t* prompt, int T) {
    const Cfg& c = cfg_;
    if (T > S_) throw Error("prompt longer than max_seq");
    hip_check(hipMemcpyAsync(ptok_buf(T), prompt, sizeof(int32_t) * T, hipMemcpyHostToDevice, st_),
              "prompt H2D");
    k_check(cake_embed(dt_, embed_, ptok_, T, c.H, hidden_, st_), "embed");
    // the walk: rank 0 runs its stops, tells each worker when its stop is due; every
    // stop hands its rows to the next stop's rank (the last one back to this rank)
    for (size_t i = 0; i + 1 < walk_.size(); ++i) {
      const Stop& s = walk_[i];
      if (s.kind == kRemoteStop) {
        remote_rows(s, 0, hidden_, T);
        continue;
      }
      if (s.rank == 0) {
        if (i > 0 && edge_in_[i] >= 0) take_relay(T);  // rows handed back by a worker rank
        if (s.kind == kRunStop) prefill_layers(T, 0, &s.sel);
        if (edge_in_[i + 1] >= 0) forward_hidden(T, walk_[i + 1].rank);
        continue;
      }
      Json m = msg("prefill");
      m.set("T", Json::integer(T));
      m.set("stop", Json::integer((int64_t)i));
      trace(rank_, "prefill stop " + std::to_string(i) + " -> rank " + std::to_string(s.rank));
      send_json(peers_[s.rank - 1], m);
      const Json ack = recv_json(peers_[s.rank - 1]);
      if (!ack.has("ok") || !ack.get("ok").as_bool())
        throw Error("pipeline rank " + std::to_string(s.rank) + " prefill failed: " +
                    (ack.has("error") ? ack.get("error").as_string() : std::string("?")));
    }
    if (edge_in_.back() >= 0) take_relay(T);  // the last worker's rows, for the head
  }

  int32_t* ptok_buf(int T) {
    grow_prefill(T);
    return ptok_;
  }

  // rows [0, T) a peer wrote into this rank's relay buffer -> hidden_ (the copy reads the
  // uncached relay from memory)
  void take_relay(int T) {
    if (!relay_) throw Error("no prefill relay buffer on this rank");
    hip_check(hipMemcpyAsync(hidden_, relay_, sizeof(float) * (size_t)T * cfg_.H,
                             hipMemcpyDeviceToDevice, st_), "prefill relay");
  }

  // hidden_ rows [0, T) -> rank dst's prefill relay buffer (device to device over the IPC
  // mapping), complete before the control message that announces them
  void forward_hidden(int T, int dst) {
    auto it = peer_pbuf_.find(dst);
    if (it == peer_pbuf_.end()) throw Error("no prefill mapping to rank " + std::to_string(dst));
    hip_check(hipMemcpyAsync(it->second, hidden_, sizeof(float) * (size_t)T * cfg_.H,
                             hipMemcpyDeviceToDevice, st_), "prefill hop");
    hip_check(hipStreamSynchronize(st_), "sync");
  }

  void prefill_layers(int T, int pos0 = 0, const std::vector<int>* sel = nullptr) {
    const Cfg& c = lc_;
    grow_prefill(T);
    const int nq = c.nh * c.hd, nk = c.nkv * c.hd, nqkv = nq + 2 * nk;
    const int Tk = pos0 + T;
    const int nl = sel ? (int)sel->size() : (int)layers_.size();
    for (int i = 0; i < nl; ++i) {
      const int l = sel ? (*sel)[i] : i;
      const LayerW& w = layers_[l];
      k_check(cake_rmsnorm(dt_, hidden_, w.ln1, (float)c.eps, T, c.H, x16_, st_), "rmsnorm");
      gemm(kEpiStore, x16_, c.H, w.wqkv, c.H, qkv_, nqkv, nullptr, 0, T, nqkv, c.H, "gemm qkv");
      uint16_t* q = reinterpret_cast<uint16_t*>(qkv_);
      k_check(cake_rope_kv(dt_, q, q + nq, q + nq + nk, nqkv, nqkv, T, c.nh, c.nkv, c.hd,
                           inv_freq_, pos0, S_, kc(l), vc(l), st_), "rope_kv");
      // [B, H, rows, D] strides of q (a column block of qkv), the layer's cache, the output
      const long long Sh = (long long)S_ * c.hd;
      const long long strides[12] = {(long long)T * nqkv, c.hd, nqkv,
                                     (long long)c.nkv * Sh, Sh, c.hd,
                                     (long long)c.nkv * Sh, Sh, c.hd,
                                     (long long)T * nq, c.hd, nq};
      k_check(cake_flash_attn(dt_, q, kc(l), vc(l), att_, 1, c.nh, c.nkv, T, Tk, c.hd, strides,
                              scale(), 1, pos0, st_), "flash_attn");
      if (tp_ > 1) {  // partial o_proj over this rank's heads, summed over the ranks
        gemm(kEpiStore32, att_, nq, w.wo, nq, nullptr, 0, ppart_, c.H, T, c.H, nq, "gemm o");
        dense_allreduce(T);
      } else {
        gemm(kEpiResid32, att_, nq, w.wo, nq, nullptr, 0, hidden_, c.H, T, c.H, nq, "gemm o");
      }
      k_check(cake_rmsnorm(dt_, hidden_, w.ln2, (float)c.eps, T, c.H, x16_, st_), "rmsnorm");
      gemm(kEpiSwiglu, x16_, c.H, w.wgu, c.H, pact_, c.I, nullptr, 0, T, c.I, c.H, "gemm gate|up");
      if (tp_ > 1) {
        gemm(kEpiStore32, pact_, c.I, w.wd, c.I, nullptr, 0, ppart_, c.H, T, c.H, c.I, "gemm down");
        dense_allreduce(T);
      } else {
        gemm(kEpiResid32, pact_, c.I, w.wd, c.I, nullptr, 0, hidden_, c.H, T, c.H, c.I, "gemm down");
      }
    }
  }

  // ---- token selection / decode step
  Mode mode_of(const CakeEngineSampling& s) const {
    Mode m;
    m.greedy = s.temperature <= 0.f;
    m.penalty = s.repeat_penalty;
    m.last_n = s.repeat_last_n;
    if (!m.greedy) {
      m.temperature = s.temperature;
      m.top_k = s.top_k > 0 ? s.top_k : 0;
      m.top_p = (s.top_p > 0.f && s.top_p < 1.f) ? s.top_p : 0.f;
      m.seed = s.seed;
    }
    m.fused = m.greedy && (m.penalty == 1.f || m.last_n <= kHeadSelectMaxLastN) && tp_ == 1;
    return m;
  }

  // logits -> penalty -> argmax / draw -> finalize (tok, history, pos)
  void select_tail(const Mode& m) {
    if (m.penalty != 1.f)
      k_check(cake_repeat_penalty(logits_, hist_, hist_len_, m.last_n, m.penalty, st_), "penalty");
    if (m.greedy) {
      k_check(cake_argmax(logits_, lc_.V, slot_, st_), "argmax");
    } else {
      const bool restrict = m.top_k > 0 || m.top_p > 0.f;
      if (restrict)
        k_check(cake_sample_threshold(logits_, lc_.V, m.temperature, m.top_k, m.top_p, thr_, st_),
                "sample_threshold");
      k_check(cake_gumbel_argmax(logits_, lc_.V, m.temperature, m.seed, hist_len_,
                                 restrict ? thr_ : nullptr, slot_, st_), "gumbel_argmax");
    }
    k_check(cake_finalize_token(slot_, tok_, hist_, hist_len_, pos_, S_, st_), "finalize");
  }

  // one decode step of this rank: its stops of the walk in order — receive (when the
  // previous stop is another rank's), the stop's work (embedding / layer run / head),
  // send (when the next stop is another rank's); the hop carries [hidden | position]
  void step_body(const Mode& m) {
    for (size_t i = 0; i < walk_.size(); ++i) {
      const Stop& s = walk_[i];
      if (s.rank != rank_) continue;
      if (edge_in_[i] >= 0) hop_recv(edge_in_[i]);
      if (s.kind == kEmbedStop) {
        if (!m.fused) k_check(cake_embed(dt_, embed_, tok_, 1, cfg_.H, resid_, st_), "embed");
      } else if (s.kind == kRunStop) {
        step_layers(&s.sel);
      } else if (s.kind == kRemoteStop) {
        remote_step(s);
      } else {
        step_head(m);
      }
      if (i + 1 < walk_.size() && edge_in_[i + 1] >= 0) hop_send(edge_in_[i + 1]);
    }
  }

  bool has_stops() const {
    for (const Stop& s : walk_)
      if (s.rank == rank_) return true;
    return false;
  }

  void hop_send(int e) {
    k_check(cake_hop_send(resid_, cfg_.H, 1, hop_bf16_ ? 1 : 0, out_inbox_.at(e), seq_ + 2 * e, st_),
            "hop_send");
  }
  void hop_recv(int e) {
    k_check(cake_hop_recv(my_inbox_.at(e), cfg_.H, 1, hop_bf16_ ? 1 : 0, resid_, seq_ + 2 * e + 1,
                          hop_err_, hop_timeout_, st_), "hop_recv");
  }

  // the walk of one token over the owner map (the placement loop llama.rs:205-220 and
  // the contiguous-run coalescing of llama.rs:95-114)
  void plan_walk() {
    walk_.clear();
    walk_.push_back({kEmbedStop, 0, {}, {}});
    for (int l = 0; l < cfg_.L; ++l) {
      const int w = remote_of_.empty() ? -1 : remote_of_[l];
      if (w >= 0) {  // a TCP worker's run: coalesced while the worker stays the same
        if (walk_.back().kind != kRemoteStop || walk_.back().remote != w)
          walk_.push_back({kRemoteStop, 0, {}, {}, w});
        walk_.back().layers.push_back(l);
        continue;
      }
      const int r = owner_.empty() ? 0 : owner_[l];
      if (walk_.back().kind != kRunStop || walk_.back().rank != r) walk_.push_back({kRunStop, r, {}, {}});
      walk_.back().layers.push_back(l);
      if (r == rank_) walk_.back().sel.push_back(local_[l]);
    }
    walk_.push_back({kHeadStop, 0, {}, {}});
    edge_in_.assign(walk_.size(), -1);
    edges_.clear();
    for (size_t i = 1; i < walk_.size(); ++i)
      if (walk_[i].rank != walk_[i - 1].rank) {
        edge_in_[i] = (int)edges_.size();
        edges_.push_back({walk_[i - 1].rank, walk_[i].rank});
      }
  }

 public:
  // "r:l0-l1,..." of the walk (logs / tests)
  std::string walk_str() const {
    std::string s;
    for (const Stop& st : walk_)
      if (st.kind == kRunStop || st.kind == kRemoteStop) {
        if (!s.empty()) s += ",";
        s += (st.kind == kRemoteStop ? "w" + std::to_string(st.remote) : std::to_string(st.rank)) +
             ":" + std::to_string(st.layers.front()) + "-" + std::to_string(st.layers.back());
      }
    return s;
  }
  int n_edges() const { return (int)edges_.size(); }

 private:

  void step_layers(const std::vector<int>* sel = nullptr) {
    const Cfg& c = lc_;
    const int nq = c.nh * c.hd, nk = c.nkv * c.hd;
    const int nl = sel ? (int)sel->size() : (int)layers_.size();
    for (int i = 0; i < nl; ++i) {
      const int l = sel ? (*sel)[i] : i;
      const LayerW& w = layers_[l];
      const uint16_t* wqkv = reinterpret_cast<const uint16_t*>(w.wqkv);
      k_check(cake_qkv_rope(dt_, resid_, w.ln1, (float)c.eps, wqkv, wqkv + (size_t)nq * c.H,
                            wqkv + (size_t)(nq + nk) * c.H, c.H, c.nh, c.nkv, c.hd, inv_freq_,
                            pos_, q_, kc(l), vc(l), S_, st_), "qkv_rope");
      if (short_step_ && ao_ok_) {  // one split: attention + o_proj in one launch
        k_check(ao_.run(dt_, q_, kc(l), vc(l), pos_, S_, c.nh, c.nkv, c.hd, scale(), w.wo,
                                nq, c.H, tp_ > 1 ? partial_ : resid_, tp_ > 1 ? 0 : 1, ao_ws_,
                                ao_tickets_, tickets_ + 2 * c.nkv, st_), "attn_oproj");
        if (tp_ > 1) ar_sum();
      } else {
        if (short_step_)  // head-parallel short-context attention
          k_check(cake_attn_decode_heads(dt_, q_, kc(l), vc(l), pos_, S_, c.nh, c.nkv, c.hd,
                                         scale(), attn_out_, st_), "attn_heads");
        else
          k_check(cake_attn_decode(dt_, q_, kc(l), vc(l), pos_, S_, c.nh, c.nkv, c.hd, scale(),
                                 part_, tickets_, attn_out_, st_), "attn_decode");
        if (tp_ > 1) {
          k_check(cake_gemv_x16(dt_, attn_out_, w.wo, nq, c.H, partial_, 0, st_), "o_proj");
          ar_sum();
        } else {
          k_check(cake_gemv_x16(dt_, attn_out_, w.wo, nq, c.H, resid_, 1, st_), "o_proj");
        }
      }
      const uint16_t* wgu = reinterpret_cast<const uint16_t*>(w.wgu);
      k_check(cake_swiglu(dt_, resid_, w.ln2, (float)c.eps, wgu, wgu + (size_t)c.I * c.H, c.H,
                          c.I, act_, st_), "swiglu");
      if (tp_ > 1) {
        k_check(cake_gemv_x16(dt_, act_, w.wd, c.I, c.H, partial_, 0, st_), "down_proj");
        ar_sum();
      } else {
        k_check(cake_gemv_x16(dt_, act_, w.wd, c.I, c.H, resid_, 1, st_), "down_proj");
      }
    }
  }

  void step_head(const Mode& m) {
    const Cfg& c = lc_;
    if (forced_) {  // teacher forcing: the full logits, no token choice
      head_logits(resid_);
      return;
    }
    if (tp_ > 1) {
      head_tp(resid_, m);
      return;
    }
    if (m.fused) {
      k_check(cake_head_select(dt_, resid_, norm_, (float)c.eps, lm_head_, c.H, c.V, logits_,
                               hist_, hist_len_, m.penalty != 1.f ? m.last_n : 0, m.penalty,
                               slot_, sel_ticket_, tok_, pos_, S_, embed_, resid_, st_),
              "head_select");
      return;
    }
    k_check(cake_gemv_norm_f32(dt_, resid_, norm_, (float)c.eps, lm_head_, c.H, c.V, logits_, st_),
            "lm_head");
    select_tail(m);
  }

  // f32 logits of the whole vocabulary for one hidden row: logits_ (one rank), or this
  // rank's vocabulary shard gathered into full_logits_ on every tensor-parallel rank
  float* head_logits(const float* row) {
    const Cfg& c = lc_;
    k_check(cake_gemv_norm_f32(dt_, row, norm_, (float)c.eps, lm_head_, c.H, c.V, logits_, st_),
            "lm_head");
    if (tp_ == 1) return logits_;
    k_check(cake_ar_gather(logits_, voff_, c.V, full_logits_, cfg_.V, ch_gat_.peers.data(),
                           ch_gat_.inbox, ar_seq_ + 4, ar_err_ + 2, tp_rank_, tp_, hop_timeout_,
                           st_), "ar_gather");
    return full_logits_;
  }

  // Teacher forcing: prefill `prompt`, then feed forced[0..n) one decode step each
  // (eager launches of the same decode kernels, hops and all-reduces as the captured
  // step); out[(n + 1) x V] = the logits after the prompt and after every forced token.
  // Rank 0 drives; pipeline workers run their stops on "fstep", tensor-parallel workers
  // the whole sequence on "forced".
  void forced_run(const int32_t* prompt, int T, const int32_t* forced, int n, float* out) {
    const bool lead = rank_ == 0 && tp_rank_ == 0;
    grow_prefill(T);
    if (tp_ > 1 && lead) {
      Json m = msg("forced");
      Json pr = Json::array(), fr = Json::array();
      for (int i = 0; i < T; ++i) pr.push(Json::integer(prompt[i]));
      for (int i = 0; i < n; ++i) fr.push(Json::integer(forced[i]));
      m.set("prompt", pr);
      m.set("forced", fr);
      for (int fd : peers_) send_json(fd, m);
    }
    prefill_body(prompt, T);
    const size_t V = cfg_.V;
    float* lg = head_logits(hidden_ + (size_t)(T - 1) * cfg_.H);
    if (out) hip_check(hipMemcpyAsync(out, lg, sizeof(float) * V, hipMemcpyDeviceToHost, st_), "D2H");
    hip_check(hipStreamSynchronize(st_), "sync");
    Mode m;
    m.fused = false;
    forced_ = true;
    try {
      for (int i = 0; i < n; ++i) {
        if (world_ > 1)
          for (int fd : peers_) {
            Json st = msg("fstep");
            st.set("pos", Json::integer(T + i));
            send_json(fd, st);
          }
        set_i32(tok_, forced[i]);
        set_i32(pos_, T + i);
        short_step_ = short_at(T + i);
        step_body(m);
        short_step_ = false;
        if (out)
          hip_check(hipMemcpyAsync(out + (size_t)(i + 1) * V, tp_ > 1 ? full_logits_ : logits_,
                                   sizeof(float) * V, hipMemcpyDeviceToHost, st_), "D2H");
        hip_check(hipStreamSynchronize(st_), "sync");
      }
    } catch (...) {
      forced_ = false;
      short_step_ = false;
      throw;
    }
    forced_ = false;
    if (world_ > 1) sync_workers();
    if (tp_ > 1 && lead) sync_tp_workers();
    if (lead) check_attn_error("rank " + std::to_string(rank()));
  }

  // ---- TCP workers (master side; the reference's Client, client.rs:23-133)
  void connect_remotes() {
    for (auto& w : remotes_) {
      std::string host;
      int port = 0;
      split_host_port(w.addr, &host, &port);
      w.fd = tcp_connect(host, port, remote_timeout_);
      tcp_set_timeout(w.fd, remote_timeout_);
      Message hello;
      hello.type = MsgType::Hello;
      const std::string body = encode_body(hello);
      send_frame(w.fd, reinterpret_cast<const uint8_t*>(body.data()), (uint32_t)body.size());
      const std::string rep = recv_frame(w.fd);
      const Message info = decode_body(reinterpret_cast<const uint8_t*>(rep.data()), rep.size());
      if (info.type != MsgType::WorkerInfo)
        throw Error("worker " + w.addr + " did not answer Hello with WorkerInfo");
      trace(0, "worker " + w.addr + ": " + info.info.device + " " + info.info.dtype + " (" +
                   info.info.os + "/" + info.info.arch + "), handshake " +
                   std::to_string(info.info.latency_lo) + " ms");
    }
  }

  static float wire_to_f32(uint16_t h, bool bf16) {
    uint32_t bits;
    if (bf16) {
      bits = (uint32_t)h << 16;
    } else {
      const uint32_t sg = (uint32_t)(h & 0x8000) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff;
      if (e == 0) {
        if (m == 0) {
          bits = sg;
        } else {
          int ee = -1;
          uint32_t mm = m;
          do { ++ee; mm <<= 1; } while (!(mm & 0x400));
          bits = sg | ((uint32_t)(127 - 15 - ee) << 23) | ((mm & 0x3ff) << 13);
        }
      } else if (e == 31) {
        bits = sg | 0x7f800000u | (m << 13);
      } else {
        bits = sg | ((e + 127 - 15) << 23) | (m << 13);
      }
    }
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
  }

  // one Batch round trip: host_rows_ [T, H] f32 at positions pos0.. through the worker's
  // run of layers (one (model.layers.l, pos0, l) item per layer), replaced by the reply
  void remote_call(const Stop& s, int pos0, int T) {
    RemoteWorker& w = remotes_.at(s.remote);
    const size_t n = (size_t)T * cfg_.H;
    Message m;
    m.type = MsgType::Batch;
    m.x.dtype = "f32";
    m.x.shape = {1, (uint64_t)T, (uint64_t)cfg_.H};
    m.x.data = reinterpret_cast<const uint8_t*>(host_rows_.data());
    m.x.nbytes = n * 4;
    for (int l : s.layers)
      m.batch.push_back({"model.layers." + std::to_string(l), (uint64_t)pos0, (uint64_t)l});
    const std::string body = encode_body(m);
    send_frame(w.fd, reinterpret_cast<const uint8_t*>(body.data()), (uint32_t)body.size());
    const std::string rep = recv_frame(w.fd);
    const Message r = decode_body(reinterpret_cast<const uint8_t*>(rep.data()), rep.size());
    if (r.type == MsgType::Error) throw Error("worker " + w.addr + ": " + r.error);
    if (r.type != MsgType::Tensor) throw Error("worker " + w.addr + ": unexpected reply");
    uint64_t cnt = 1;
    for (auto d : r.x.shape) cnt *= d;
    if (cnt != n) throw Error("worker " + w.addr + ": reply of " + std::to_string(cnt) +
                              " values, expected " + std::to_string(n));
    if (r.x.dtype == "f32" && r.x.nbytes == n * 4) {
      std::memcpy(host_rows_.data(), r.x.data, n * 4);
    } else if ((r.x.dtype == "f16" || r.x.dtype == "bf16") && r.x.nbytes == n * 2) {
      const bool bf = r.x.dtype == "bf16";
      for (size_t i = 0; i < n; ++i) {
        uint16_t h;
        std::memcpy(&h, r.x.data + 2 * i, 2);
        host_rows_[i] = wire_to_f32(h, bf);
      }
    } else {
      throw Error("worker " + w.addr + ": unsupported reply tensor " + r.x.dtype);
    }
  }

  // prefill rows [T, H] (device) through a remote run
  void remote_rows(const Stop& s, int pos0, float* rows, int T) {
    const size_t n = (size_t)T * cfg_.H;
    host_rows_.resize(n);
    hip_check(hipMemcpyAsync(host_rows_.data(), rows, n * 4, hipMemcpyDeviceToHost, st_), "D2H");
    hip_check(hipStreamSynchronize(st_), "sync");
    remote_call(s, pos0, T);
    hip_check(hipMemcpyAsync(rows, host_rows_.data(), n * 4, hipMemcpyHostToDevice, st_), "H2D");
    hip_check(hipStreamSynchronize(st_), "sync");
  }

  // the decode row through a remote run; its position rides in resid_'s header word
  void remote_step(const Stop& s) {
    const int H = cfg_.H;
    host_rows_.resize((size_t)H + 1);
    hip_check(hipMemcpyAsync(host_rows_.data(), resid_, sizeof(float) * (H + 1),
                             hipMemcpyDeviceToHost, st_), "D2H");
    hip_check(hipStreamSynchronize(st_), "sync");
    int pos = 0;
    std::memcpy(&pos, &host_rows_[H], 4);
    remote_call(s, pos, 1);
    hip_check(hipMemcpyAsync(resid_, host_rows_.data(), sizeof(float) * H, hipMemcpyHostToDevice,
                             st_), "H2D");
    hip_check(hipStreamSynchronize(st_), "sync");
  }

  // decode with TCP workers in the walk: every step eagerly (host round trips inside it),
  // the token read back after each; per-token host wall time
  int decode_eager(int pos0, int n, const Mode& m, const int32_t* eos, int n_eos,
                   cake_engine_token_cb cb, void* ctx, int32_t* out, int out_cap,
                   std::vector<float>* ms_out) {
    std::vector<float> ms;
    int n_out = 0;
    for (int i = 0; i < n; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      short_step_ = short_at(pos0 + i);
      try {
        step_body(m);
      } catch (...) {
        short_step_ = false;
        throw;
      }
      short_step_ = false;
      int32_t tok = 0;
      hip_check(hipMemcpyAsync(&tok, tok_, sizeof(tok), hipMemcpyDeviceToHost, st_), "tok");
      hip_check(hipStreamSynchronize(st_), "sync");
      ms.push_back((float)(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0)
                               .count() * 1e3));
      if (n_out < out_cap) out[n_out++] = tok;
      bool stop = cb && cb(ctx, tok) != 0;
      for (int e = 0; e < n_eos && !stop; ++e)
        if (eos[e] == tok) stop = true;
      if (stop) break;
    }
    check_attn_error("rank 0");
    if (ms_out) *ms_out = std::move(ms);
    return n_out;
  }

  bool remote_mode() const { return !remotes_.empty(); }

  // ---- pipeline (one process per GPU, layer shards, device-side hops)
  static constexpr int kAnnounceChunk = 8;  // replays per worker announcement
  struct AnnounceCtx {
    Llama* self;
    int pos0;  // device position before the first replay of this run
  };
  static int32_t announce_cb(void* vctx, int32_t first, int32_t count) {
    auto* a = static_cast<AnnounceCtx*>(vctx);
    try {
      Json m = msg("replays");
      m.set("count", Json::integer(count));
      m.set("pos", Json::integer(a->pos0 + (int64_t)first * a->self->k_));
      for (int fd : a->self->peers_) send_json(fd, m);
      return 0;
    } catch (const std::exception&) {
      return 1;
    }
  }

  // every worker drained its stream; any hop that gave up waiting is an error
  void sync_workers() {
    std::string err;
    for (size_t i = 0; i < peers_.size(); ++i) {
      try {
        send_json(peers_[i], msg("sync"));
        const Json r = recv_json(peers_[i]);
        if (r.has("hop_err") && r.get("hop_err").as_int() != 0)
          err = "pipeline rank " + std::to_string(i + 1) + ": hop receive timed out";
        if (r.has("error")) err = "pipeline rank " + std::to_string(i + 1) + ": " +
                                  r.get("error").as_string();
      } catch (const std::exception& e) {
        err = e.what();
      }
    }
    int own = 0;
    hip_check(hipMemcpy(&own, hop_err_, sizeof(int), hipMemcpyDeviceToHost), "hop_err");
    if (own) {
      (void)hipMemset(hop_err_, 0, sizeof(int));
      err = "pipeline rank 0: hop receive timed out";
    }
    if (!err.empty()) throw Error(err);
  }

 public:
  // worker rank: serve the master's control messages until it says exit
  void serve() {
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    if (tp_ > 1) {
      if (tp_rank_ == 0) throw Error("serve() runs on tensor-parallel workers (rank > 0)");
      serve_tp();
      return;
    }
    if (head_) throw Error("serve() runs on pipeline workers (rank > 0)");
    const bool active = has_stops();  // a rank the placement left idle only answers
    if (active) ensure_graphs(Mode{});
    std::vector<void*> execs(execs_.begin(), execs_.end());
    for (;;) {
      const Json m = recv_json(ctl_fd_);
      const std::string cmd = m.get("cmd").as_string();
      trace(rank_, "control: " + m.dump().substr(0, 120));
      if (cmd == "exit") break;
      if (cmd == "prefill") {
        Json r = Json::object();
        try {
          const int T = (int)m.get("T").as_int();
          const int i = (int)m.get("stop").as_int();
          if (T < 1 || T > S_) throw Error("bad prefill length");
          if (i < 1 || i + 1 >= (int)walk_.size() || walk_[i].rank != rank_)
            throw Error("prefill stop " + std::to_string(i) + " is not this rank's");
          if (edge_in_[i] >= 0) take_relay(T);
          prefill_layers(T, 0, &walk_[i].sel);
          if (edge_in_[i + 1] >= 0) forward_hidden(T, walk_[i + 1].rank);
          r.set("ok", Json::boolean(true));
        } catch (const std::exception& e) {
          r.set("ok", Json::boolean(false));
          r.set("error", Json::string(e.what()));
        }
        send_json(ctl_fd_, r);
      } else if (cmd == "fstep") {  // one eager teacher-forced step of this rank's stops
        if (!active) continue;
        Mode fm;
        fm.fused = false;
        short_step_ = short_at((int)m.get("pos").as_int());
        step_body(fm);
        short_step_ = false;
      } else if (cmd == "replays") {
        if (!active) continue;
        CakeLoopSpec spec{};
        spec.execs = execs.data();
        spec.n_execs = (int32_t)execs.size();
        spec.bucket_of = bucket_of_.data();
        spec.n_len = (int32_t)bucket_of_.size();
        spec.k = k_;
        spec.pos = (int32_t)m.get("pos").as_int();
        spec.n = (int32_t)m.get("count").as_int() * k_;
        spec.stream = st_;
        CakeLoopResult res{};
        k_check(cake_graph_decode(&spec, &res), "graph_decode");  // enqueue only
      } else if (cmd == "sync") {
        Json r = Json::object();
        const hipError_t e = hipStreamSynchronize(st_);
        int herr = 0;
        (void)hipMemcpy(&herr, hop_err_, sizeof(int), hipMemcpyDeviceToHost);
        if (herr) (void)hipMemset(hop_err_, 0, sizeof(int));
        r.set("ok", Json::boolean(e == hipSuccess));
        r.set("hop_err", Json::integer(herr));
        if (e != hipSuccess) r.set("error", Json::string(hipGetErrorString(e)));
        try {
          check_attn_error("attention");
        } catch (const std::exception& x) {
          r.set("error", Json::string(x.what()));
        }
        send_json(ctl_fd_, r);
      } else {
        throw Error("unknown control message " + cmd);
      }
    }
  }

 private:
  // inboxes (uncached device memory, device-side hops) and prefill buffers exchanged as
  // IPC handles over the TCP control plane; ring: rank r sends to (r + 1) % world
  void connect_pipeline(const std::string& addr, double timeout_s) {
    std::string host;
    int port = 0;
    split_host_port(addr, &host, &port);
    const int words = cake_hop_words(cfg_.H, 1, hop_bf16_ ? 1 : 0);
    // this rank's handles: its prefill buffer and one inbox per edge into it
    Json me = Json::object();
    me.set("rank", Json::integer(rank_));
    {
      void* rp = nullptr;
      k_check(cake_hop_alloc(sizeof(float) * (size_t)S_ * cfg_.H, &rp), "relay alloc");
      relay_ = static_cast<float*>(rp);
      hipIpcMemHandle_t hp;
      hip_check(hipIpcGetMemHandle(&hp, relay_), "IpcGetMemHandle");
      me.set("pbuf", Json::string(hex_of(&hp, sizeof(hp))));
      Json ib = Json::array();
      for (size_t e = 0; e < edges_.size(); ++e) {
        if (edges_[e].second != rank_) continue;
        void* p = nullptr;
        k_check(cake_hop_alloc((size_t)words * 8, &p), "hop_alloc");
        my_inbox_[(int)e] = p;
        hipIpcMemHandle_t hi;
        hip_check(hipIpcGetMemHandle(&hi, p), "IpcGetMemHandle");
        Json x = Json::array();
        x.push(Json::integer((int64_t)e));
        x.push(Json::string(hex_of(&hi, sizeof(hi))));
        ib.push(x);
      }
      me.set("inboxes", ib);
    }
    std::vector<Json> table(world_);
    if (rank_ == 0) {
      const int lfd = tcp_listen(host, port);
      table[0] = me;
      peers_.assign(world_ - 1, -1);
      try {
        for (int i = 1; i < world_; ++i) {
          std::string peer;
          const int fd = tcp_accept(lfd, &peer);
          tcp_set_timeout(fd, 0);
          const Json j = recv_json(fd);
          const int r = (int)j.get("rank").as_int();
          if (r < 1 || r >= world_ || peers_[r - 1] >= 0) throw Error("bad pipeline rank hello");
          peers_[r - 1] = fd;
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
      for (int fd : peers_) send_json(fd, m);
    } else {
      const auto deadline =
          std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
      for (;;) {
        try {
          ctl_fd_ = tcp_connect(host, port, 2.0);
          break;
        } catch (const std::exception&) {
          if (std::chrono::steady_clock::now() > deadline) throw;
          usleep(200000);
        }
      }
      tcp_set_timeout(ctl_fd_, 0);
      send_json(ctl_fd_, me);
      const Json m = recv_json(ctl_fd_);
      for (int r = 0; r < world_; ++r) table[r] = m.get("table").at(r);
    }
    // map the receivers of this rank's outgoing edges: their inbox, their prefill buffer
    for (size_t e = 0; e < edges_.size(); ++e) {
      if (edges_[e].first != rank_) continue;
      const int dst = edges_[e].second;
      const Json& t = table[dst];
      bool found = false;
      for (const auto& x : t.get("inboxes").items()) {
        if ((int)x.at(0).as_int() != (int)e) continue;
        hipIpcMemHandle_t h;
        unhex(x.at(1).as_string(), &h, sizeof(h));
        void* p = nullptr;
        hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "IpcOpen inbox");
        out_inbox_[(int)e] = p;
        found = true;
      }
      if (!found) throw Error("rank " + std::to_string(dst) + " published no inbox for edge " +
                              std::to_string(e));
      if (!peer_pbuf_.count(dst)) {
        hipIpcMemHandle_t h;
        unhex(t.get("pbuf").as_string(), &h, sizeof(h));
        void* p = nullptr;
        hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "IpcOpen pbuf");
        peer_pbuf_[dst] = p;
      }
    }
  }

  // Start-up self-test of every edge (before any graph exists): each rank pushes a
  // tagged pattern through each outgoing edge (non-blocking peer stores), then receives
  // on each incoming edge (bounded device wait) and checks every word; every rank's
  // verdict goes to rank 0, which fails the start with the rank and peer named.  A
  // mapping that does not carry stores across the devices fails here, not as a hop
  // timeout in the middle of the first generation.
  static float selftest_value(int e, int i) { return (float)(((i * 7 + e * 13) % 251) - 125); }

  static bool selftest_forced_fail() {  // test hook: the fallback path of bench / cake-cli
    const char* e = std::getenv("CAKE_IPC_SELFTEST_FAIL");
    return e && *e == '1';
  }

  // every rank reaches this point, then every rank leaves it (rank 0 is the hub)
  void ctl_barrier() {
    if (rank_ == 0) {
      for (int fd : peers_) (void)recv_json(fd);
      for (int fd : peers_) send_json(fd, Json::object());
    } else {
      send_json(ctl_fd_, Json::object());
      (void)recv_json(ctl_fd_);
    }
  }

  // Each outgoing edge writes a pattern row into the receiver's relay buffer the way
  // forward_hidden does (device copy over the IPC mapping, synchronized before the
  // control message); after a barrier the receiver moves it out with take_relay's copy
  // and checks every word.  Round 2 writes a new pattern over rows the receiver has
  // already read, so a receiver that kept the old contents in a cache fails here.
  void selftest_relay(std::string& bad) {
    const int H = cfg_.H;
    std::vector<float> pat(H), got(H);
    for (int round = 1; round <= 2; ++round) {
      for (size_t e = 0; e < edges_.size(); ++e) {
        if (edges_[e].first != rank_ || (int)e >= S_) continue;
        for (int i = 0; i < H; ++i) pat[i] = selftest_value((int)e + 64 * round, i);
        hip_check(hipMemcpyAsync(hidden_, pat.data(), sizeof(float) * H, hipMemcpyHostToDevice,
                                 st_), "selftest H2D");
        float* dst = static_cast<float*>(peer_pbuf_.at(edges_[e].second)) + e * (size_t)H;
        hip_check(hipMemcpyAsync(dst, hidden_, sizeof(float) * H, hipMemcpyDeviceToDevice, st_),
                  "selftest relay");
        hip_check(hipStreamSynchronize(st_), "selftest sync");
      }
      ctl_barrier();
      for (size_t e = 0; e < edges_.size(); ++e) {
        if (edges_[e].second != rank_ || (int)e >= S_) continue;
        hip_check(hipMemcpyAsync(hidden_ + H, relay_ + e * (size_t)H, sizeof(float) * H,
                                 hipMemcpyDeviceToDevice, st_), "selftest relay read");
        hip_check(hipMemcpyAsync(got.data(), hidden_ + H, sizeof(float) * H,
                                 hipMemcpyDeviceToHost, st_), "selftest D2H");
        hip_check(hipStreamSynchronize(st_), "selftest sync");
        int wrong = 0;
        for (int i = 0; i < H; ++i)
          if (got[i] != selftest_value((int)e + 64 * round, i)) ++wrong;
        if (wrong && bad.empty())
          bad = "rank " + std::to_string(rank_) + ": prefill relay from rank " +
                std::to_string(edges_[e].first) + " (edge " + std::to_string(e) + ", round " +
                std::to_string(round) + ") delivered " + std::to_string(wrong) + " wrong words";
      }
      ctl_barrier();
    }
  }

  void selftest_pipeline() {
    const int H = cfg_.H;
    std::string bad;
    std::vector<float> pat(H + 4, 0.f);
    for (size_t e = 0; e < edges_.size(); ++e) {
      if (edges_[e].first != rank_) continue;
      for (int i = 0; i < H; ++i) pat[i] = selftest_value((int)e, i);
      const uint32_t tag = 0xC0DE0000u + (uint32_t)e;
      std::memcpy(&pat[H], &tag, 4);
      hip_check(hipMemcpyAsync(scratch_resid_, pat.data(), sizeof(float) * (H + 1),
                               hipMemcpyHostToDevice, st_), "selftest H2D");
      k_check(cake_hop_send(scratch_resid_, H, 1, hop_bf16_ ? 1 : 0, out_inbox_.at((int)e),
                            seq_ + 2 * e, st_), "selftest send");
      hip_check(hipStreamSynchronize(st_), "selftest sync");
    }
    for (size_t e = 0; e < edges_.size(); ++e) {
      if (edges_[e].second != rank_) continue;
      hip_check(hipMemsetAsync(scratch_resid_, 0, sizeof(float) * (H + 1), st_), "memset");
      k_check(cake_hop_recv(my_inbox_.at((int)e), H, 1, hop_bf16_ ? 1 : 0, scratch_resid_,
                            seq_ + 2 * e + 1, hop_err_, hop_timeout_, st_), "selftest recv");
      std::vector<float> got(H + 1);
      hip_check(hipMemcpyAsync(got.data(), scratch_resid_, sizeof(float) * (H + 1),
                               hipMemcpyDeviceToHost, st_), "selftest D2H");
      int herr = 0;
      hip_check(hipMemcpyAsync(&herr, hop_err_, sizeof(int), hipMemcpyDeviceToHost, st_), "err");
      hip_check(hipStreamSynchronize(st_), "selftest sync");
      const int src = edges_[e].first;
      uint32_t tag = 0;
      std::memcpy(&tag, &got[H], 4);
      int wrong = 0;
      for (int i = 0; i < H; ++i)
        if (got[i] != selftest_value((int)e, i)) ++wrong;
      if (herr) {
        bad = "rank " + std::to_string(rank_) + ": hop from rank " + std::to_string(src) +
              " (edge " + std::to_string(e) + ") timed out in the start-up self-test";
        hip_check(hipMemset(hop_err_, 0, sizeof(int)), "memset");
        break;
      }
      if (wrong || tag != 0xC0DE0000u + (uint32_t)e) {
        bad = "rank " + std::to_string(rank_) + ": hop from rank " + std::to_string(src) +
              " (edge " + std::to_string(e) + ") delivered " + std::to_string(wrong) +
              " wrong words in the start-up self-test";
        break;
      }
    }
    // the prefill relay buffers: every rank takes part whatever the hops found (the
    // rounds are lock-stepped through rank 0)
    selftest_relay(bad);
    if (bad.empty() && selftest_forced_fail())
      bad = "rank " + std::to_string(rank_) + ": failure forced by CAKE_IPC_SELFTEST_FAIL=1";
    // verdicts to rank 0 (which fails the start naming every bad edge)
    if (rank_ == 0) {
      for (size_t i = 0; i < peers_.size(); ++i) {
        const Json r = recv_json(peers_[i]);
        if (r.has("bad") && bad.empty()) bad = r.get("bad").as_string();
      }
      Json v = Json::object();
      v.set("ok", Json::boolean(bad.empty()));
      if (!bad.empty()) v.set("bad", Json::string(bad));
      for (int fd : peers_) send_json(fd, v);
    } else {
      Json r = Json::object();
      if (!bad.empty()) r.set("bad", Json::string(bad));
      send_json(ctl_fd_, r);
      const Json v = recv_json(ctl_fd_);
      if (v.has("bad")) bad = v.get("bad").as_string();
    }
    if (!bad.empty()) throw Error("pipeline IPC self-test failed: " + bad);
  }

  // ---- tensor parallel (one process per GPU, every rank 1/W of every layer)
  void ar_sum() {
    k_check(cake_ar_sum(partial_, resid_, lc_.H, 1, ch_sum_.peers.data(), ch_sum_.inbox, ar_seq_,
                        ar_err_, tp_rank_, tp_, hop_timeout_, st_), "ar_sum");
  }

  // this rank's lm_head rows -> the global token on every rank (greedy: shard argmax key,
  // max over ranks; sampled: the full logits gathered, the single-GPU draw on each rank)
  void head_tp(const float* row, const Mode& m) {
    const Cfg& c = lc_;
    k_check(cake_gemv_norm_f32(dt_, row, norm_, (float)c.eps, lm_head_, c.H, c.V, logits_, st_),
            "lm_head");
    if (m.greedy) {
      k_check(cake_select_shard(logits_, c.V, voff_, hist_, hist_len_, m.last_n, m.penalty, 0.f,
                                0, slot_, st_), "select_shard");
      k_check(cake_ar_max_key(slot_, ch_key_.peers.data(), ch_key_.inbox, ar_seq_ + 2,
                              ar_err_ + 1, tp_rank_, tp_, hop_timeout_, st_), "ar_max_key");
    } else {
      const int V = cfg_.V;
      k_check(cake_ar_gather(logits_, voff_, c.V, full_logits_, V, ch_gat_.peers.data(),
                             ch_gat_.inbox, ar_seq_ + 4, ar_err_ + 2, tp_rank_, tp_,
                             hop_timeout_, st_), "ar_gather");
      if (m.penalty != 1.f)
        k_check(cake_repeat_penalty(full_logits_, hist_, hist_len_, m.last_n, m.penalty, st_),
                "penalty");
      const bool restrict = m.top_k > 0 || m.top_p > 0.f;
      if (restrict)
        k_check(cake_sample_threshold(full_logits_, V, m.temperature, m.top_k, m.top_p, thr_, st_),
                "sample_threshold");
      k_check(cake_gumbel_argmax(full_logits_, V, m.temperature, m.seed, hist_len_,
                                 restrict ? thr_ : nullptr, slot_, st_), "gumbel_argmax");
    }
    k_check(cake_finalize_token(slot_, tok_, hist_, hist_len_, pos_, S_, st_), "finalize");
  }

  // prefill: partial rows ppart_ [T, H] summed over the ranks into hidden_ — every rank
  // copies its rows into slot `rank` of every rank's slab (uncached device memory,
  // IPC-mapped), a barrier, then each sums the W slots; two slab banks, alternating, so
  // the next all-reduce never overwrites rows a slower rank still sums
  void dense_allreduce(int T) {
    const int R = slab_rows();
    const size_t SH = (size_t)R * cfg_.H;
    // rounds of R rows; the two banks alternate, so a peer's copies of round k + 1 never
    // land in the bank its sum of round k reads (each rank syncs its stream, sum
    // included, before the barrier that releases the next round's copies)
    for (int c0 = 0; c0 < T; c0 += R) {
      const int rows = std::min(R, T - c0);
      const size_t off = (size_t)c0 * cfg_.H, bytes = sizeof(float) * (size_t)rows * cfg_.H;
      const int bank = slab_bank_;
      slab_bank_ ^= 1;
      for (int p = 0; p < tp_; ++p) {
        float* base = p == tp_rank_ ? slab_ : static_cast<float*>(peer_slab_[p]);
        hip_check(hipMemcpyAsync(base + ((size_t)bank * tp_ + tp_rank_) * SH, ppart_ + off, bytes,
                                 hipMemcpyDeviceToDevice, st_), "slab copy");
      }
      hip_check(hipStreamSynchronize(st_), "sync");
      tp_barrier();
      k_check(cake_sum_slices(hidden_ + off, slab_ + (size_t)bank * tp_ * SH, tp_, (long long)SH,
                              (long long)rows * cfg_.H, 1, st_), "sum_slices");
    }
  }

  int slab_rows() const { return std::min(S_, kSlabRows); }

  // host barrier of the tensor-parallel ranks over the control sockets (star on rank 0)
  void tp_barrier() {
    if (tp_rank_ == 0) {
      for (int fd : peers_) {
        const Json j = recv_json(fd);
        if (!j.has("cmd") || j.get("cmd").as_string() != "barrier") throw Error("TP barrier: bad message");
      }
      for (int fd : peers_) send_json(fd, msg("barrier"));
    } else {
      send_json(ctl_fd_, msg("barrier"));
      const Json j = recv_json(ctl_fd_);
      if (!j.has("cmd") || j.get("cmd").as_string() != "barrier") throw Error("TP barrier: bad message");
    }
  }

  void sync_tp_workers() {
    std::string err;
    for (size_t i = 0; i < peers_.size(); ++i) {
      try {
        send_json(peers_[i], msg("sync"));
        const Json r = recv_json(peers_[i]);
        if (r.has("ar_err") && r.get("ar_err").as_int() != 0)
          err = "tensor-parallel rank " + std::to_string(i + 1) + ": all-reduce timed out";
        if (r.has("error")) err = r.get("error").as_string();
      } catch (const std::exception& e) {
        err = e.what();
      }
    }
    int own[3] = {0, 0, 0};
    hip_check(hipMemcpy(own, ar_err_, sizeof(own), hipMemcpyDeviceToHost), "ar_err");
    if (own[0] | own[1] | own[2]) {
      (void)hipMemset(ar_err_, 0, sizeof(own));
      err = "tensor-parallel rank 0: all-reduce timed out";
    }
    if (!err.empty()) throw Error(err);
  }

  static std::vector<int32_t> eos_of(const Json& m) {
    std::vector<int32_t> v;
    if (m.has("eos"))
      for (const auto& x : m.get("eos").items()) v.push_back((int32_t)x.as_int());
    return v;
  }

  // worker rank: run the generations rank 0 announces, in lock step
  void serve_tp() {
    for (;;) {
      const Json m = recv_json(ctl_fd_);
      const std::string cmd = m.get("cmd").as_string();
      if (cmd == "exit") break;
      if (cmd == "generate") {
        std::vector<int32_t> prompt;
        for (const auto& x : m.get("prompt").items()) prompt.push_back((int32_t)x.as_int());
        CakeEngineSampling smp{};
        smp.temperature = (float)m.get("temperature").as_double();
        smp.top_k = (int32_t)m.get("top_k").as_int();
        smp.top_p = (float)m.get("top_p").as_double();
        smp.seed = std::strtoull(m.get("seed").as_string().c_str(), nullptr, 10);
        smp.repeat_penalty = (float)m.get("penalty").as_double();
        smp.repeat_last_n = (int32_t)m.get("last_n").as_int();
        const int max_new = (int)m.get("max_new").as_int();
        const std::vector<int32_t> eos = eos_of(m);
        run_generation(prompt.data(), (int)prompt.size(), max_new, smp, eos.data(),
                       (int)eos.size(), nullptr, nullptr, nullptr, 0, nullptr, false);
      } else if (cmd == "forced") {
        std::vector<int32_t> prompt, forced;
        for (const auto& x : m.get("prompt").items()) prompt.push_back((int32_t)x.as_int());
        for (const auto& x : m.get("forced").items()) forced.push_back((int32_t)x.as_int());
        forced_run(prompt.data(), (int)prompt.size(), forced.data(), (int)forced.size(), nullptr);
      } else if (cmd == "continue") {
        const std::vector<int32_t> eos = eos_of(m);
        const int L = read_i32(hist_len_);
        decode_tokens(L, (int)m.get("max_new").as_int(), eos.data(), (int)eos.size(), nullptr,
                      nullptr, nullptr, 0, false, nullptr);
      } else if (cmd == "sync") {
        Json r = Json::object();
        const hipError_t e = hipStreamSynchronize(st_);
        int errs[3] = {0, 0, 0};
        (void)hipMemcpy(errs, ar_err_, sizeof(errs), hipMemcpyDeviceToHost);
        if (errs[0] | errs[1] | errs[2]) (void)hipMemset(ar_err_, 0, sizeof(errs));
        r.set("ok", Json::boolean(e == hipSuccess));
        r.set("ar_err", Json::integer(errs[0] | errs[1] | errs[2]));
        if (e != hipSuccess) r.set("error", Json::string(hipGetErrorString(e)));
        try {
          check_attn_error("tensor-parallel rank " + std::to_string(tp_rank_));
        } catch (const std::exception& x) {
          r.set("error", Json::string(x.what()));
        }
        send_json(ctl_fd_, r);
      } else {
        throw Error("unknown control message " + cmd);
      }
    }
  }

  // Start-up self-test of every tensor-parallel channel (before any graph exists): a
  // sum all-reduce of a rank-scaled pattern, the argmax-key max, the vocabulary gather
  // and the prefill slab all-reduce, each checked word for word; verdicts to rank 0.
  void selftest_tp() {
    const int H = cfg_.H, W = tp_;
    std::string bad;
    auto fail = [&](const std::string& what) {
      if (bad.empty()) bad = "tensor-parallel rank " + std::to_string(tp_rank_) + ": " + what;
    };
    std::vector<float> pat(H);
    for (int i = 0; i < H; ++i) pat[i] = (float)(tp_rank_ + 1) * (float)((i % 17) - 8);
    const float tri = (float)(W * (W + 1) / 2);
    // (1) decode sum channel
    hip_check(hipMemcpyAsync(partial_, pat.data(), sizeof(float) * H, hipMemcpyHostToDevice, st_),
              "selftest H2D");
    k_check(cake_ar_sum(partial_, scratch_resid_, H, 0, ch_sum_.peers.data(), ch_sum_.inbox,
                        ar_seq_, ar_err_, tp_rank_, tp_, hop_timeout_, st_), "selftest ar_sum");
    std::vector<float> got(H);
    hip_check(hipMemcpyAsync(got.data(), scratch_resid_, sizeof(float) * H, hipMemcpyDeviceToHost,
                             st_), "selftest D2H");
    hip_check(hipStreamSynchronize(st_), "sync");
    trace(rank(), "self-test: sum channel done");
    for (int i = 0; i < H; ++i)
      if (got[i] != tri * (float)((i % 17) - 8)) { fail("sum all-reduce delivered wrong words"); break; }
    // (2) argmax-key max channel
    const unsigned long long key = ((unsigned long long)(100 + tp_rank_) << 32) | (unsigned)tp_rank_;
    hip_check(hipMemcpyAsync(slot_, &key, sizeof(key), hipMemcpyHostToDevice, st_), "H2D");
    k_check(cake_ar_max_key(slot_, ch_key_.peers.data(), ch_key_.inbox, ar_seq_ + 2, ar_err_ + 1,
                            tp_rank_, tp_, hop_timeout_, st_), "selftest ar_max_key");
    unsigned long long mx = 0;
    hip_check(hipMemcpyAsync(&mx, slot_, sizeof(mx), hipMemcpyDeviceToHost, st_), "D2H");
    hip_check(hipStreamSynchronize(st_), "sync");
    if (mx != (((unsigned long long)(100 + W - 1) << 32) | (unsigned)(W - 1)))
      fail("argmax-key all-reduce returned a wrong key");
    trace(rank(), "self-test: key channel done");
    hip_check(hipMemsetAsync(slot_, 0, sizeof(unsigned long long), st_), "memset");
    // (3) vocabulary gather channel
    std::vector<float> shard(lc_.V);
    for (int j = 0; j < lc_.V; ++j) shard[j] = (float)(voff_ + j);
    hip_check(hipMemcpyAsync(logits_, shard.data(), sizeof(float) * lc_.V, hipMemcpyHostToDevice,
                             st_), "H2D");
    k_check(cake_ar_gather(logits_, voff_, lc_.V, full_logits_, cfg_.V, ch_gat_.peers.data(),
                           ch_gat_.inbox, ar_seq_ + 4, ar_err_ + 2, tp_rank_, tp_, hop_timeout_,
                           st_), "selftest ar_gather");
    std::vector<float> full(cfg_.V);
    hip_check(hipMemcpyAsync(full.data(), full_logits_, sizeof(float) * cfg_.V,
                             hipMemcpyDeviceToHost, st_), "D2H");
    hip_check(hipStreamSynchronize(st_), "sync");
    for (int j = 0; j < cfg_.V; ++j)
      if (full[j] != (float)j) { fail("vocabulary gather delivered wrong words"); break; }
    trace(rank(), "self-test: gather channel done");
    // (4) prefill slab all-reduce (one row)
    hip_check(hipMemcpyAsync(ppart_, pat.data(), sizeof(float) * H, hipMemcpyHostToDevice, st_),
              "H2D");
    hip_check(hipMemsetAsync(hidden_, 0, sizeof(float) * H, st_), "memset");
    dense_allreduce(1);
    hip_check(hipMemcpyAsync(got.data(), hidden_, sizeof(float) * H, hipMemcpyDeviceToHost, st_),
              "D2H");
    int errs[3] = {0, 0, 0};
    hip_check(hipMemcpyAsync(errs, ar_err_, sizeof(errs), hipMemcpyDeviceToHost, st_), "D2H");
    hip_check(hipStreamSynchronize(st_), "sync");
    for (int i = 0; i < H; ++i)
      if (got[i] != tri * (float)((i % 17) - 8)) { fail("prefill slab all-reduce delivered wrong words"); break; }
    // (5) two more rounds with new values (the banks alternate, so the second one
    // rewrites the bank of (4)): every rank has already read that bank's contents, so a
    // stale cached copy of a peer's slot fails here
    for (int round = 1; round <= 2; ++round) {  // collective: every rank runs both
      const float sc = -2.f - (float)round;
      for (int i = 0; i < H; ++i) pat[i] = sc * (float)(tp_rank_ + 1) * (float)((i % 13) - 6);
      hip_check(hipMemcpyAsync(ppart_, pat.data(), sizeof(float) * H, hipMemcpyHostToDevice,
                               st_), "H2D");
      hip_check(hipMemsetAsync(hidden_, 0, sizeof(float) * H, st_), "memset");
      dense_allreduce(1);
      hip_check(hipMemcpyAsync(got.data(), hidden_, sizeof(float) * H, hipMemcpyDeviceToHost,
                               st_), "D2H");
      hip_check(hipStreamSynchronize(st_), "sync");
      for (int i = 0; i < H; ++i)
        if (got[i] != sc * tri * (float)((i % 13) - 6)) {
          fail("prefill slab all-reduce (round " + std::to_string(round + 1) +
               ") delivered wrong words");
          break;
        }
    }
    hip_check(hipMemcpyAsync(errs, ar_err_, sizeof(errs), hipMemcpyDeviceToHost, st_), "D2H");
    hip_check(hipStreamSynchronize(st_), "sync");
    if (errs[0] | errs[1] | errs[2]) {
      fail("an all-reduce channel timed out");
      hip_check(hipMemset(ar_err_, 0, sizeof(errs)), "memset");
    }
    if (selftest_forced_fail()) fail("failure forced by CAKE_IPC_SELFTEST_FAIL=1");
    if (tp_rank_ == 0) {
      for (int fd : peers_) {
        const Json r = recv_json(fd);
        if (r.has("bad") && bad.empty()) bad = r.get("bad").as_string();
      }
      Json v = Json::object();
      if (!bad.empty()) v.set("bad", Json::string(bad));
      for (int fd : peers_) send_json(fd, v);
    } else {
      Json r = Json::object();
      if (!bad.empty()) r.set("bad", Json::string(bad));
      send_json(ctl_fd_, r);
      const Json v = recv_json(ctl_fd_);
      if (v.has("bad")) bad = v.get("bad").as_string();
    }
    if (!bad.empty()) throw Error("tensor-parallel IPC self-test failed: " + bad);
  }

  // channel inboxes (uncached, hop.hip granules) and the prefill slab, exchanged as IPC
  // handles through rank 0 (full mesh)
  void connect_tp(const std::string& addr, double timeout_s) {
    std::string host;
    int port = 0;
    split_host_port(addr, &host, &port);
    auto alloc = [&](size_t words) {
      void* p = nullptr;
      k_check(cake_hop_alloc(words * 8, &p), "hop_alloc");
      tp_owned_.push_back(p);
      return p;
    };
    ch_sum_.inbox = alloc((size_t)cake_ar_inbox_words(tp_, cfg_.H));
    ch_key_.inbox = alloc((size_t)cake_ar_inbox_words(tp_, 2));
    ch_gat_.inbox = alloc(2 * (size_t)cfg_.V);
    const size_t slab_bytes = sizeof(float) * 2 * (size_t)tp_ * slab_rows() * cfg_.H;
    void* sp = nullptr;
    hip_check(hipExtMallocWithFlags(&sp, slab_bytes, hipDeviceMallocUncached), "slab alloc");
    tp_owned_.push_back(sp);
    slab_ = static_cast<float*>(sp);
    trace(rank(), "tensor-parallel inboxes + slab allocated (" +
                      std::to_string(slab_bytes >> 20) + " MiB slab)");
    void* mine[4] = {ch_sum_.inbox, ch_key_.inbox, ch_gat_.inbox, slab_};
    Json me = Json::array();
    for (void* p : mine) {
      hipIpcMemHandle_t h;
      hip_check(hipIpcGetMemHandle(&h, p), "IpcGetMemHandle");
      me.push(Json::string(hex_of(&h, sizeof(h))));
    }
    std::vector<Json> table(tp_);
    if (tp_rank_ == 0) {
      table[0] = me;
      const int lfd = tcp_listen(host, port);
      peers_.assign(tp_ - 1, -1);
      try {
        for (int i = 1; i < tp_; ++i) {
          std::string peer;
          const int fd = tcp_accept(lfd, &peer);
          tcp_set_timeout(fd, 0);
          const Json j = recv_json(fd);
          const int r = (int)j.get("rank").as_int();
          if (r < 1 || r >= tp_ || peers_[r - 1] >= 0) throw Error("bad TP rank hello");
          peers_[r - 1] = fd;
          table[r] = j.get("h");
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
      for (int fd : peers_) send_json(fd, m);
    } else {
      const auto deadline =
          std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
      for (;;) {
        try {
          ctl_fd_ = tcp_connect(host, port, 2.0);
          break;
        } catch (const std::exception&) {
          if (std::chrono::steady_clock::now() > deadline) throw;
          usleep(200000);
        }
      }
      tcp_set_timeout(ctl_fd_, 0);
      Json hello = Json::object();
      hello.set("rank", Json::integer(tp_rank_));
      hello.set("h", me);
      send_json(ctl_fd_, hello);
      const Json m = recv_json(ctl_fd_);
      for (int r = 0; r < tp_; ++r) table[r] = m.get("table").at(r);
    }
    trace(rank(), "tensor-parallel handle table exchanged");
    ArChan* chans[3] = {&ch_sum_, &ch_key_, &ch_gat_};
    for (auto* ch : chans) ch->peers.assign(tp_, nullptr);
    peer_slab_.assign(tp_, nullptr);
    for (int r = 0; r < tp_; ++r) {
      if (r == tp_rank_) continue;
      for (int k = 0; k < 4; ++k) {
        hipIpcMemHandle_t h;
        unhex(table[r].at(k).as_string(), &h, sizeof(h));
        void* p = nullptr;
        hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "IpcOpen");
        tp_mapped_.push_back(p);
        if (k < 3) chans[k]->peers[r] = p;
        else peer_slab_[r] = p;
      }
    }
  }

  void drop_graphs() {
    for (auto e : execs_) (void)hipGraphExecDestroy(e);
    for (auto g : graphs_) (void)hipGraphDestroy(g);
    execs_.clear();
    graphs_.clear();
    have_graphs_ = false;
  }

  // one graph per attention split cap (DeviceDecoder.capture position buckets)
  void ensure_graphs(const Mode& m) {
    if (have_graphs_ && graph_mode_ == m) return;
    trace(rank(), "capturing decode graphs");
    drop_graphs();
    if (!head_) {  // pipeline worker: its layers once, eagerly, at position 0 (the row is
                   // rewritten by every prefill), so no kernel's first launch is captured
      hip_check(hipMemsetAsync(resid_, 0, sizeof(float) * (cfg_.H + 1), st_), "memset");
      step_layers();
      hip_check(hipStreamSynchronize(st_), "sync");
    }
    if (world_ == 1) warm_step(m);
    capture_buckets(m);
  }

  // warm every kernel once outside capture on the live state, then restore it (the
  // K/V row this writes is the next step's, which that step rewrites)
  void warm_step(const Mode& m) {
    hip_check(hipMemcpyAsync(scratch_i32_, tok_, sizeof(int), hipMemcpyDeviceToDevice, st_), "snap");
    hip_check(hipMemcpyAsync(scratch_i32_ + 1, pos_, sizeof(int), hipMemcpyDeviceToDevice, st_), "snap");
    hip_check(hipMemcpyAsync(scratch_i32_ + 2, hist_len_, sizeof(int), hipMemcpyDeviceToDevice, st_), "snap");
    hip_check(hipMemcpyAsync(scratch_resid_, resid_, sizeof(float) * cfg_.H, hipMemcpyDeviceToDevice, st_), "snap");
    step_body(m);
    hip_check(hipMemcpyAsync(tok_, scratch_i32_, sizeof(int), hipMemcpyDeviceToDevice, st_), "restore");
    hip_check(hipMemcpyAsync(pos_, scratch_i32_ + 1, sizeof(int), hipMemcpyDeviceToDevice, st_), "restore");
    hip_check(hipMemcpyAsync(hist_len_, scratch_i32_ + 2, sizeof(int), hipMemcpyDeviceToDevice, st_), "restore");
    hip_check(hipMemcpyAsync(resid_, scratch_resid_, sizeof(float) * cfg_.H, hipMemcpyDeviceToDevice, st_), "restore");
    hip_check(hipMemsetAsync(slot_, 0, sizeof(unsigned long long), st_), "slot");
    hip_check(hipStreamSynchronize(st_), "sync");
  }

  void capture_buckets(const Mode& m) {
    // caps: 8 / 16 / 32 / 64 (clamped to the max_seq grid) up to the first covering
    // every live length (ops.hip.attn_split_caps)
    const int full = cake_attn_max_split(S_);
    int need = 1;
    for (int t = 1; t <= S_; ++t) need = std::max(need, cake_attn_splits(t));
    std::vector<int> caps;
    for (int cap : {8, 16, 32, 64}) {
      const int cc = std::min(cap, full);
      if (std::find(caps.begin(), caps.end(), cc) == caps.end()) caps.push_back(cc);
      if (cap >= need) break;
    }
    // cap 1: the one-split lengths with attention + o_proj fused (attn_oproj.hip), or the
    // short lengths on the head-parallel attention
    if (ao_ok_ || heads_max_ > 0) caps.push_back(1);
    std::sort(caps.begin(), caps.end());
    try {
      for (int cap : caps) {
        k_check(cake_attn_set_split_cap(cap == 1 ? full : cap), "attn_set_split_cap");
        hipGraph_t g = nullptr;
        short_step_ = cap == 1;
        hip_check(hipStreamBeginCapture(st_, hipStreamCaptureModeGlobal), "BeginCapture");
        try {
          for (int i = 0; i < k_; ++i) step_body(m);
        } catch (...) {
          short_step_ = false;
          (void)hipStreamEndCapture(st_, &g);
          if (g) (void)hipGraphDestroy(g);
          throw;
        }
        short_step_ = false;
        hip_check(hipStreamEndCapture(st_, &g), "EndCapture");
        graphs_.push_back(g);
        hipGraphExec_t e = nullptr;
        hip_check(hipGraphInstantiate(&e, g, nullptr, nullptr, 0), "GraphInstantiate");
        execs_.push_back(e);
      }
    } catch (...) {
      (void)cake_attn_set_split_cap(0);
      drop_graphs();
      throw;
    }
    k_check(cake_attn_set_split_cap(0), "attn_set_split_cap");
    bucket_of_.assign(S_ + 1, (int32_t)caps.size() - 1);
    for (int t = 0; t <= S_; ++t) {
      const int nd = cake_attn_splits(t);
      const bool sh = short_len(t);
      for (size_t i = 0; i < caps.size(); ++i)
        if ((caps[i] == 1) == sh && caps[i] >= nd) { bucket_of_[t] = (int32_t)i; break; }
    }
    graph_mode_ = m;
    have_graphs_ = true;
  }
};

void put_err(char* err, int errlen, const std::string& msg) {
  if (err && errlen > 0) {
    std::snprintf(err, (size_t)errlen, "%s", msg.c_str());
  }
}

}  // namespace
}  // namespace cake

using cake::Llama;

CAKE_API void* cake_engine_open(const char* model_dir, const CakeEngineOpts* opts, char* err,
                                int32_t errlen) {
  try {
    if (!model_dir || !opts) throw cake::Error("null argument");
    return new Llama(model_dir, *opts);
  } catch (const std::exception& e) {
    cake::put_err(err, errlen, e.what());
    return nullptr;
  }
}

CAKE_API void* cake_engine_open_pp(const char* model_dir, const CakeEngineOpts* opts,
                                   const CakePipeOpts* pipe, char* err, int32_t errlen) {
  try {
    if (!model_dir || !opts || !pipe) throw cake::Error("null argument");
    return new Llama(model_dir, *opts, pipe);
  } catch (const std::exception& e) {
    cake::put_err(err, errlen, e.what());
    return nullptr;
  }
}

CAKE_API void* cake_engine_open_remote(const char* model_dir, const CakeEngineOpts* opts,
                                       const CakeRemoteOpts* remote, char* err, int32_t errlen) {
  try {
    if (!model_dir || !opts || !remote) throw cake::Error("null argument");
    return new Llama(model_dir, *opts, nullptr, nullptr, nullptr, remote);
  } catch (const std::exception& e) {
    cake::put_err(err, errlen, e.what());
    return nullptr;
  }
}

CAKE_API void* cake_engine_open_layers(const char* model_dir, const CakeEngineOpts* opts,
                                       const int32_t* layers, int32_t n_layers, char* err,
                                       int32_t errlen) {
  try {
    if (!model_dir || !opts || !layers || n_layers <= 0) throw cake::Error("bad arguments");
    const std::vector<int> ls(layers, layers + n_layers);
    return new Llama(model_dir, *opts, nullptr, &ls);
  } catch (const std::exception& e) {
    cake::put_err(err, errlen, e.what());
    return nullptr;
  }
}

CAKE_API int32_t cake_engine_forward(void* h, uint64_t session, const int32_t* layers,
                                     int32_t n_layers, int32_t pos0, float* hidden, int32_t T,
                                     char* err, int32_t errlen) {
  try {
    if (!h || !layers || !hidden) throw cake::Error("null argument");
    static_cast<Llama*>(h)->forward_host(session, std::vector<int>(layers, layers + n_layers),
                                         pos0, hidden, T);
    return 0;
  } catch (const std::exception& e) {
    cake::put_err(err, errlen, e.what());
    return 1;
  }
}

CAKE_API void cake_engine_drop_session(void* h, uint64_t session) {
  try {
    if (h) static_cast<Llama*>(h)->drop_session(session);
  } catch (const std::exception&) {
  }
}

CAKE_API void* cake_engine_open_tp(const char* model_dir, const CakeEngineOpts* opts,
                                   const CakeTPOpts* tp, char* err, int32_t errlen) {
  try {
    if (!model_dir || !opts || !tp) throw cake::Error("null argument");
    return new Llama(model_dir, *opts, nullptr, nullptr, tp);
  } catch (const std::exception& e) {
    cake::put_err(err, errlen, e.what());
    return nullptr;
  }
}

CAKE_API int32_t cake_engine_serve(void* h, char* err, int32_t errlen) {
  try {
    if (!h) throw cake::Error("null engine");
    static_cast<Llama*>(h)->serve();
    return 0;
  } catch (const std::exception& e) {
    cake::put_err(err, errlen, e.what());
    return 1;
  }
}

CAKE_API int32_t cake_engine_rank_info(void* h, int32_t* o) {
  if (!h || !o) return (int32_t)hipErrorInvalidValue;
  const Llama* m = static_cast<Llama*>(h);
  const auto lr = m->layer_range();
  o[0] = m->rank();
  o[1] = m->world();
  o[2] = lr.first;
  o[3] = lr.second;
  return 0;
}

CAKE_API int32_t cake_engine_info(void* h, int32_t* o) {
  if (!h || !o) return (int32_t)hipErrorInvalidValue;
  const Llama* m = static_cast<Llama*>(h);
  const auto& c = m->cfg();
  const int32_t v[8] = {c.V, c.H, c.L, c.nh, c.nkv, c.hd, c.I, m->max_seq()};
  std::memcpy(o, v, sizeof(v));
  return 0;
}

CAKE_API int32_t cake_engine_eos(void* h, int32_t* out, int32_t cap) {
  if (!h) return 0;
  const auto& e = static_cast<Llama*>(h)->cfg().eos;
  for (int32_t i = 0; i < cap && i < (int32_t)e.size(); ++i) out[i] = e[i];
  return (int32_t)e.size();
}

CAKE_API int32_t cake_engine_generate(void* h, const int32_t* prompt, int32_t n_prompt,
                                      int32_t max_new, const CakeEngineSampling* sampling,
                                      const int32_t* eos, int32_t n_eos,
                                      cake_engine_token_cb cb, void* ctx, int32_t* out,
                                      int32_t out_cap, CakeEngineStats* stats, char* err,
                                      int32_t errlen) {
  try {
    if (!h || !prompt || !sampling || (!out && max_new > 0)) throw cake::Error("null argument");
    static_cast<Llama*>(h)->generate(prompt, n_prompt, max_new, *sampling, eos, n_eos, cb, ctx,
                                     out, out_cap, stats);
    return 0;
  } catch (const std::exception& e) {
    cake::put_err(err, errlen, e.what());
    return 1;
  }
}

CAKE_API int32_t cake_engine_continue(void* h, int32_t max_new, const int32_t* eos, int32_t n_eos,
                                      cake_engine_token_cb cb, void* ctx, int32_t* out,
                                      int32_t out_cap, CakeEngineStats* stats, char* err,
                                      int32_t errlen) {
  try {
    if (!h || (!out && max_new > 0)) throw cake::Error("null argument");
    static_cast<Llama*>(h)->continue_gen(max_new, eos, n_eos, cb, ctx, out, out_cap, stats);
    return 0;
  } catch (const std::exception& e) {
    cake::put_err(err, errlen, e.what());
    return 1;
  }
}

CAKE_API int32_t cake_engine_forced_logits(void* h, const int32_t* prompt, int32_t n_prompt,
                                           const int32_t* forced, int32_t n_forced, float* out,
                                           char* err, int32_t errlen) {
  try {
    if (!h || !prompt || (!forced && n_forced > 0) || !out) throw cake::Error("null argument");
    static_cast<Llama*>(h)->forced_logits(prompt, n_prompt, forced, n_forced, out);
    return 0;
  } catch (const std::exception& e) {
    cake::put_err(err, errlen, e.what());
    return 1;
  }
}

// "rank:first-last,..." runs of the token's walk (placement check), n = bytes written
CAKE_API int32_t cake_engine_walk(void* h, char* out, int32_t cap) {
  if (!h || !out || cap <= 0) return 0;
  const std::string s = static_cast<Llama*>(h)->walk_str();
  const int32_t n = (int32_t)std::min<size_t>(s.size(), (size_t)cap - 1);
  std::memcpy(out, s.data(), (size_t)n);
  out[n] = 0;
  return n;
}

CAKE_API int32_t cake_engine_prefill_logits(void* h, const int32_t* prompt, int32_t n_prompt,
                                            float* out, char* err, int32_t errlen) {
  try {
    if (!h || !prompt || !out) throw cake::Error("null argument");
    static_cast<Llama*>(h)->prefill_logits(prompt, n_prompt, out);
    return 0;
  } catch (const std::exception& e) {
    cake::put_err(err, errlen, e.what());
    return 1;
  }
}

CAKE_API void cake_engine_close(void* h) { delete static_cast<Llama*>(h); }
