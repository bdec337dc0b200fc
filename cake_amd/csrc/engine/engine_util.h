// Host helpers shared by the native engines (llama_engine.cpp, sd_engine.cpp): HIP error
// checks, the package directory, file reads and the GEMM tile planner (ops/gemm.py plan()).
#pragma once

#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../runtime/json.h"
#include "../runtime/net.h"

namespace cake {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error(std::string(what) + ": " + hipGetErrorString(e));
}
inline void k_check(int rc, const char* what) {
  if (rc == 0) return;
  if (rc >= 1000)  // driver/blaslt.cpp: 1000 + hipblasStatus_t
    throw Error(std::string(what) + ": hipBLASLt status " + std::to_string(rc - 1000));
  throw Error(std::string(what) + ": " + hipGetErrorString((hipError_t)rc));
}

// ---------------------------------------------------------------------------
// control plane of the multi-rank engines: IPC handles as hex, JSON frames over TCP
// ---------------------------------------------------------------------------
inline std::string hex_of(const void* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  const uint8_t* b = static_cast<const uint8_t*>(p);
  for (size_t i = 0; i < n; ++i) {
    s.push_back(d[b[i] >> 4]);
    s.push_back(d[b[i] & 15]);
  }
  return s;
}

inline void unhex(const std::string& s, void* out, size_t n) {
  if (s.size() != 2 * n) throw Error("bad IPC handle");
  auto v = [](char c) { return c <= '9' ? c - '0' : c - 'a' + 10; };
  uint8_t* b = static_cast<uint8_t*>(out);
  for (size_t i = 0; i < n; ++i) b[i] = (uint8_t)(v(s[2 * i]) << 4 | v(s[2 * i + 1]));
}

inline void send_json(int fd, const Json& j) {
  const std::string t = j.dump();
  send_frame(fd, reinterpret_cast<const uint8_t*>(t.data()), (uint32_t)t.size());
}
inline Json recv_json(int fd) { return Json::parse(recv_frame(fd)); }

// <root>/cake_amd/lib/libcake_engine.so -> <root>/cake_amd
inline std::string pkg_dir() {
  Dl_info info{};
  if (dladdr(reinterpret_cast<void*>(&pkg_dir), &info) && info.dli_fname) {
    char buf[4096];
    const char* p = realpath(info.dli_fname, buf);
    std::string s = p ? p : info.dli_fname;
    for (int i = 0; i < 2; ++i) {
      const auto cut = s.find_last_of('/');
      if (cut == std::string::npos) return ".";
      s = s.substr(0, cut);
    }
    return s;
  }
  return ".";
}

inline std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw Error("cannot read " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// ---------------------------------------------------------------------------
// GEMM tile plan (ops/gemm.py plan(): measured table, else the cost model)
// ---------------------------------------------------------------------------
// plan cfg naming the library GEMM (hipBLASLt, driver/blaslt.cpp; ops/gemm.py LIB).
// Off the default path: table entries naming it are read only under CAKE_GEMM_LIB=1
// (the A/B arm of scripts/bench_gemm_lib.py); otherwise every shape runs an MFMA plan.
constexpr int kGemmLib = -1;
inline bool gemm_lib_enabled() {
  const char* e = std::getenv("CAKE_GEMM_LIB");
  return e && *e == '1';
}

struct GemmPlanner {
  struct Tuned { long long M, Nv, K; std::string epi; int cfg, splits; };
  std::vector<Tuned> tuned;

  void load(std::string path) {  // CAKE_GEMM_TABLE overrides (A/B of plan tables)
    if (const char* e = std::getenv("CAKE_GEMM_TABLE"); e && *e) path = e;
    std::ifstream f(path);
    if (!f) return;
    const bool lib_ok = gemm_lib_enabled();
    try {
      const Json j = Json::parse(read_file(path));
      static const int known[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27};
      for (const auto& e : j.get("entries").items()) {
        const int cfg = (int)e.get("cfg").as_int();
        const std::string ep = e.get("epi").as_string();
        const bool lib = lib_ok && cfg == kGemmLib && (ep == "store" || ep == "resid32" || ep == "store32" ||
                                             ep == "swiglu");
        if (!lib && std::find(std::begin(known), std::end(known), cfg) == std::end(known)) continue;
        tuned.push_back({e.get("M").as_int(), e.get("Nv").as_int(), e.get("K").as_int(),
                         e.get("epi").as_string(), cfg, (int)e.get("splits").as_int()});
      }
    } catch (const std::exception&) {
      tuned.clear();  // a malformed table only loses the measured overrides
    }
  }

  bool has_lib() const {
    for (const auto& e : tuned)
      if (e.cfg == kGemmLib) return true;
    return false;
  }

  // the MFMA kernel's plan: the measured entries other than the library GEMM's
  std::pair<int, int> plan_mfma(long long M, long long Nv, long long K,
                                const std::string& epi) const {
    return plan(M, Nv, K, epi, true);
  }

  std::pair<int, int> plan(long long M, long long Nv, long long K, const std::string& epi,
                           bool mfma_only = false) const {
    const Tuned* near = nullptr;
    double near_r = 0;
    for (const auto& e : tuned) {
      if (e.Nv != Nv || e.K != K || e.epi != epi) continue;
      if (mfma_only && e.cfg == kGemmLib) continue;
      if (e.M == M) return {e.cfg, e.splits};
      const double r = (double)std::max(M, e.M) / (double)std::min(M, e.M);
      if (r <= 2 && (!near || r < near_r)) { near = &e; near_r = r; }
    }
    if (near) {  // split-K scaled to this M (ops/gemm.py _near_splits)
      if (near->cfg == kGemmLib) return {kGemmLib, 1};
      long long sc = (long long)near->splits * near->M / std::max(M, 1LL);
      int p = 1;
      while ((long long)p * 2 <= sc) p *= 2;
      return {near->cfg, p};
    }
    struct T { int cfg, bm, bn, slots; double eff; };
    static const T tiles[] = {{0, 128, 128, 2, 1.0}, {1, 64, 128, 2, 0.8}, {4, 64, 64, 4, 0.7},
                              {5, 256, 256, 1, 1.2}, {22, 256, 256, 1, 1.3}};
    static const int small_c[] = {1, 4, 0}, big_c[] = {0, 1, 4, 5, 22};
    const int* cands = M <= 64 ? small_c : big_c;
    // the four-wave 256x256 tile (cfg 22) where it can run: whole 64-element k steps,
    // operands under 2 GB (ops/gemm.py _cost_plan); unsplit
    const bool four = M > 64 && K % 64 == 0 && M * K * 2 < (1LL << 31) && Nv * K * 2 < (1LL << 31);
    const int nc = M <= 64 ? 3 : (four ? 5 : 4);
    const long long ksteps = (K + 63) / 64;
    double best = -1;
    std::pair<int, int> out{0, 1};
    for (int c = 0; c < nc; ++c) {
      const T* t = nullptr;
      for (const auto& x : tiles)
        if (x.cfg == cands[c]) t = &x;
      const long long tiles_n = ((M + t->bm - 1) / t->bm) * ((Nv + t->bn - 1) / t->bn);
      for (int splits : {1, 2, 4, 8, 16}) {
        if (splits > 1 && (t->cfg == 22 || ksteps / splits < 4 ||
                           tiles_n * splits > 2LL * 256 * t->slots))
          continue;
        const long long waves = (tiles_n * splits + 256LL * t->slots - 1) / (256LL * t->slots);
        double cost = (double)waves * t->slots * t->bm * t->bn * (double)((ksteps + splits - 1) / splits) / t->eff;
        if (splits > 1) cost += (double)M * Nv * splits * 0.1;
        if (best < 0 || cost < best) { best = cost; out = {t->cfg, splits}; }
      }
    }
    return out;
  }
};

}  // namespace cake
