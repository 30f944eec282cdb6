// hipBLASLt fp16 x fp16 -> fp32 GEMM for the large-M prefill path (gemm.hip gemm_lib).
//
// Why a library GEMM here: at M >= a few hundred prompt tokens the prefill projections are compute
// bound, and hipBLASLt's gfx950 MFMA kernels run 0.85-1.2 PFLOP/s on the Llama-2-7B shapes at
// M = 2048 (profiles/r3_gemm/blas_probe.log) against 0.33 for the fused dequant GEMM, whose
// in-loop dequantisation is VALU/LDS-bound. The weight is dequantised once per call into an fp16
// scratch (dequant.hip, memory-bound: ~2 bytes written per weight), so the quantised weights stay the
// only resident copy. Plain library GEMM, nothing fused: the epilogue runs afterwards.
//
// Layout: hipBLASLt is column-major. Row-major D[M][N] is column-major N x M (ld N); row-major
// W[N][K] is column-major K x N (ld K) used transposed; row-major X[M][K] is column-major K x M.
// So D = op_T(W) * X, a "TN" GEMM. Plans (descriptors + algorithm) are cached per shape and device;
// the heuristic runs once per power-of-two M bucket (blas_prepare at model load) and its algorithm is
// reused for the other M of the bucket.
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <map>
#include <mutex>
#include <set>
#include <tuple>

#include "kernels/ops.h"

namespace omx {

namespace {

struct Plan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
  bool ok = false;
  int m_run = 0;  // rows the plan's layouts describe (M, or the bucket's rows when padded)
};

std::mutex g_mu;
std::map<int, hipblasLtHandle_t> g_handles;
// exact-shape plans (layouts + algorithm); the algorithm comes from a heuristic query at the
// power-of-two M bucket (>= 128) and is reused for every M in the bucket once
// hipblaslt_ext::matmulIsAlgoSupported accepts it -- a heuristic query costs tens of ms, so one per
// prompt length would land in the TTFT
std::map<std::tuple<int, int, int, int, size_t>, Plan> g_plans;
std::map<std::tuple<int, int, int, int, size_t>, Plan> g_bucket;
// exact M whose bucket algorithm matmulIsAlgoSupported rejected: asked once, never again (the padded
// bucket plan serves them when the caller's buffers hold the bucket's rows)
std::set<std::tuple<int, int, int, int, size_t>> g_rejected;

void destroy(Plan& p) {
  if (p.a) hipblasLtMatrixLayoutDestroy(p.a);
  if (p.b) hipblasLtMatrixLayoutDestroy(p.b);
  if (p.d) hipblasLtMatrixLayoutDestroy(p.d);
  if (p.op) hipblasLtMatmulDescDestroy(p.op);
  p = Plan{};
}

// M buckets: 128, 256, then every multiple of 256. A prompt of M rows runs its bucket's plan over
// padded rows whenever the caller's buffers hold them (no exact-M query: hipBLASLt's algorithm check
// cost ~0.3 s on its first call per shape, which landed in the first TTFT of every new burst size --
// the 4-client bench's ~0.4 s stall); at most 255 padded rows past 256.
int bucket_of(int M) {
  if (M <= 128) return 128;
  if (M <= 256) return 256;
  return (M + 255) / 256 * 256;
}

int next_bucket(int b) { return b < 256 ? b * 2 : b + 256; }

bool layouts(Plan& p, int M, int N, int K) {
  if (hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return false;
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  return hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16F, K, N, K) == HIPBLAS_STATUS_SUCCESS &&
         hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16F, K, M, K) == HIPBLAS_STATUS_SUCCESS &&
         hipblasLtMatrixLayoutCreate(&p.d, HIP_R_32F, N, M, N) == HIPBLAS_STATUS_SUCCESS;
}

hipblasLtHandle_t handle(int dev) {
  auto it = g_handles.find(dev);
  if (it != g_handles.end()) return it->second;
  hipblasLtHandle_t h = nullptr;
  if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) h = nullptr;
  g_handles[dev] = h;
  return h;
}

Plan heuristic_plan(hipblasLtHandle_t h, int M, int N, int K, size_t ws_bytes) {
  Plan p;
  if (!layouts(p, M, N, K)) {
    destroy(p);
    return p;
  }
  hipblasLtMatmulPreference_t pref = nullptr;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) {
    destroy(p);
    return p;
  }
  const uint64_t wsb = ws_bytes;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
  hipblasLtMatmulHeuristicResult_t res[8];
  int n = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, p.op, p.a, p.b, p.d, p.d, pref, 8, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  for (int i = 0; st == HIPBLAS_STATUS_SUCCESS && i < n && !p.ok; ++i) {
    if (res[i].state != HIPBLAS_STATUS_SUCCESS || res[i].workspaceSize > ws_bytes) continue;
    p.algo = res[i].algo;
    p.ws = res[i].workspaceSize;
    p.ok = true;
  }
  if (!p.ok) {
    fprintf(stderr, "[omx] hipBLASLt: no algorithm for M=%d N=%d K=%d (status %d, %d candidates, %zu B workspace); "
            "fused dequant GEMM used\n", M, N, K, (int)st, n, ws_bytes);
    destroy(p);  // a failed plan is cached as "no plan": it owns no descriptors
  }
  return p;
}

// caller holds g_mu; m_cap: rows the caller's buffers hold (0 = exactly M). Order: exact-M plan
// cached; the bucket's algorithm accepted for M; running the bucket's rows when they fit m_cap; a
// heuristic query at exactly M (slow: tens of ms) as the last resort
Plan plan_for(hipblasLtHandle_t h, int dev, int M, int N, int K, size_t ws_bytes, int m_cap) {
  const auto key = std::make_tuple(dev, M, N, K, ws_bytes);
  auto it = g_plans.find(key);
  if (it != g_plans.end()) return it->second;
  const int Mb = bucket_of(M);
  const auto bkey = std::make_tuple(dev, Mb, N, K, ws_bytes);
  auto bt = g_bucket.find(bkey);
  if (bt == g_bucket.end()) bt = g_bucket.emplace(bkey, heuristic_plan(h, Mb, N, K, ws_bytes)).first;
  Plan p;
  if (M == Mb) {
    p = bt->second;
    p.m_run = Mb;
  } else if (bt->second.ok && m_cap >= Mb) {  // padded rows: the bucket's plan as is (not cached: m_cap)
    Plan q = bt->second;
    q.m_run = Mb;
    return q;
  } else if (bt->second.ok && !g_rejected.count(key) && layouts(p, M, N, K)) {
    hipblasLtMatmulAlgo_t algo = bt->second.algo;
    size_t need = 0;
    const float alpha = 1.f, beta = 0.f;
    if (hipblaslt_ext::matmulIsAlgoSupported(h, p.op, &alpha, p.a, p.b, &beta, p.d, p.d, algo, need) ==
            HIPBLAS_STATUS_SUCCESS &&
        need <= ws_bytes) {
      p.algo = algo;
      p.ws = need;
      p.ok = true;
      p.m_run = M;
    } else {
      destroy(p);  // the descriptors of a rejected exact-M plan are not kept
      g_rejected.insert(key);
    }
  }
  if (!p.ok && bt->second.ok && m_cap >= Mb) {  // padded rows: not cached (m_cap may differ per call)
    Plan q = bt->second;
    q.m_run = Mb;
    return q;
  }
  if (!p.ok) {
    p = heuristic_plan(h, M, N, K, ws_bytes);
    p.m_run = M;
  }
  g_plans.emplace(key, p);
  return p;
}

}  // namespace

bool blas_gemm_tn(const void* w16, const void* x16, float* d, int M, int N, int K, void* ws, size_t ws_bytes,
                  hipStream_t s, int m_cap) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  Plan p;
  hipblasLtHandle_t h;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    h = handle(dev);
    if (!h) return false;
    p = plan_for(h, dev, M, N, K, ws_bytes, m_cap);
  }
  if (!p.ok) return false;
  const float alpha = 1.f, beta = 0.f;
  const hipblasStatus_t st = hipblasLtMatmul(h, p.op, &alpha, w16, p.a, x16, p.b, &beta, d, p.d, d, p.d, &p.algo,
                                             p.ws ? ws : nullptr, p.ws, s);
  if (st != HIPBLAS_STATUS_SUCCESS) {
    static bool warned = false;
    if (!warned) fprintf(stderr, "[omx] hipBLASLt matmul failed (status %d, M=%d N=%d K=%d)\n", (int)st, M, N, K);
    warned = true;
    return false;
  }
  return true;
}

bool blas_plan_ok(int M, int N, int K, size_t ws_bytes, int m_cap) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  std::lock_guard<std::mutex> lk(g_mu);
  hipblasLtHandle_t h = handle(dev);
  return h && plan_for(h, dev, M, N, K, ws_bytes, m_cap).ok;
}

void blas_prepare(int N, int K, int min_M, int max_M, size_t ws_bytes) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return;
  std::lock_guard<std::mutex> lk(g_mu);
  hipblasLtHandle_t h = handle(dev);
  if (!h) return;
  for (int Mb = bucket_of(min_M); Mb <= bucket_of(max_M); Mb = next_bucket(Mb)) (void)plan_for(h, dev, Mb, N, K, ws_bytes, 0);
}

}  // namespace omx
