// Plain library GEMMs through hipBLASLt.
//
//   C[M, N] (row-major, ldc) = A[M, K] . W[N, K]^T            out 0: bf16/f16 store
//                                                           out 1: fp32 store
//   C[M, N] += A . W^T    (C fp32, beta = 1)                 out 2: fp32 accumulate
//
// The hand-written MFMA GEMM (kernels/gemm.hip) keeps every fused epilogue
// (swiglu / geglu / add16 / partial) and the shapes where it measured faster; the
// native engine's planner sends a plain prefill GEMM here only where the library
// measured faster on this chip (profiles/r5_gemm_vs_hipblaslt.jsonl: the 8B / 70B
// prefill projections at M >= 512).  Row-major C = A W^T is the column-major
// product C^T = W^T' A': W is the K x N column-major matrix (op T), A the K x M one
// (op N) -- the "TN" layout the library's kernels are tuned for.
//
// One handle per device; one (desc, layouts, heuristic algo) plan per shape, built on
// first use (outside any graph capture: the engine's prefill runs eagerly).
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdint>
#include <map>
#include <mutex>
#include <tuple>

#define CAKE_API extern "C" __attribute__((visibility("default")))

namespace {

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
  int status = 0;  // 0 usable; else the failing hipblasStatus_t (kept: no retry per call)
};

using Key = std::tuple<int, int, int, int, int, long long, long long, long long, size_t>;

std::mutex g_mu;
std::map<int, hipblasLtHandle_t> g_handles;  // device -> handle
std::map<std::pair<int, Key>, Plan> g_plans;

constexpr size_t kMaxPlans = 4096;

void destroy(Plan& p) {
  if (p.la) hipblasLtMatrixLayoutDestroy(p.la);
  if (p.lb) hipblasLtMatrixLayoutDestroy(p.lb);
  if (p.lc) hipblasLtMatrixLayoutDestroy(p.lc);
  if (p.desc) hipblasLtMatmulDescDestroy(p.desc);
  p = Plan{};
}

hipDataType in_type(int dt) { return dt == 1 ? HIP_R_16F : HIP_R_16BF; }

int build(hipblasLtHandle_t h, const Key& k, Plan& p) {
  const auto [dt, out, M, N, K, lda, ldw, ldc, ws_cap] = k;
  const hipDataType ti = in_type(dt), to = out == 0 ? ti : HIP_R_32F;
  hipblasStatus_t s = hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F);
  if (s) return s;
  const int32_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
  if ((s = hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof opT)))
    return s;
  if ((s = hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof opN)))
    return s;
  if ((s = hipblasLtMatrixLayoutCreate(&p.la, ti, K, N, ldw))) return s;
  if ((s = hipblasLtMatrixLayoutCreate(&p.lb, ti, K, M, lda))) return s;
  if ((s = hipblasLtMatrixLayoutCreate(&p.lc, to, N, M, ldc))) return s;
  hipblasLtMatmulPreference_t pref = nullptr;
  if ((s = hipblasLtMatmulPreferenceCreate(&pref))) return s;
  const uint64_t cap = ws_cap;
  s = hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &cap,
                                            sizeof cap);
  hipblasLtMatmulHeuristicResult_t res[8];
  int n = 0;
  if (!s)
    s = hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.la, p.lb, p.lc, p.lc, pref, 8, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (s) return s;
  for (int i = 0; i < n; ++i)
    if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= ws_cap) {
      p.algo = res[i].algo;
      p.ws = res[i].workspaceSize;
      return 0;
    }
  return HIPBLAS_STATUS_NOT_SUPPORTED;
}

}  // namespace

// 0 on success, else a hipblasStatus_t (+1000 so it cannot read as a hipError_t 0..999)
CAKE_API int cake_blaslt_gemm(int dt, int out, const void* a, long long lda, const void* w,
                              long long ldw, void* c, long long ldc, int M, int N, int K,
                              void* ws, size_t ws_bytes, hipStream_t st) {
  if (out < 0 || out > 2 || M <= 0 || N <= 0 || K <= 0 || lda < K || ldw < K || ldc < N)
    return 1000 + HIPBLAS_STATUS_INVALID_VALUE;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 1000 + HIPBLAS_STATUS_INTERNAL_ERROR;
  const Key key{dt, out, M, N, K, lda, ldw, ldc, ws_bytes};
  // one lock over lookup and launch (an asynchronous enqueue): the cache may be emptied
  // by another thread's call once it holds kMaxPlans shapes (a server seeing every prompt
  // length), so no plan pointer outlives the lock
  std::lock_guard<std::mutex> g(g_mu);
  auto hit = g_handles.find(dev);
  if (hit == g_handles.end()) {
    hipblasLtHandle_t nh = nullptr;
    const hipblasStatus_t s = hipblasLtCreate(&nh);
    if (s) return 1000 + s;
    hit = g_handles.emplace(dev, nh).first;
  }
  hipblasLtHandle_t h = hit->second;
  auto it = g_plans.find({dev, key});
  if (it == g_plans.end()) {
    if (g_plans.size() >= kMaxPlans) {
      for (auto& kv : g_plans) destroy(kv.second);
      g_plans.clear();
    }
    it = g_plans.emplace(std::make_pair(dev, key), Plan{}).first;
    it->second.status = build(h, key, it->second);
  }
  const Plan& p = it->second;
  if (p.status) return 1000 + p.status;
  const float alpha = 1.f, beta = out == 2 ? 1.f : 0.f;
  const hipblasStatus_t s = hipblasLtMatmul(h, p.desc, &alpha, w, p.la, a, p.lb, &beta, c, p.lc, c,
                                            p.lc, &p.algo, p.ws ? ws : nullptr, p.ws, st);
  return s ? 1000 + s : 0;
}

