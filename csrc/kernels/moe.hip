// MoE routing: softmax over the router logits, top-k experts, renormalised
// weights. The expert GEMVs themselves are the fused GEMV with blockIdx.z = selected expert, which
// offsets into the [X][N][K/..] expert streams on device -- no host round trip, graph-capturable.
#include "common.h"
#include "ops.h"

namespace omx {

__global__ void moe_route_kernel(const float* logits, int B, int X, int k, int* ids, float* w) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* l = logits + (long long)b * X;
  float mx = -INFINITY;
  for (int e = 0; e < X; ++e) mx = fmaxf(mx, l[e]);
  unsigned long long used = 0;
  float tot = 0.f;
  for (int j = 0; j < k; ++j) {
    int best = -1;
    float bv = -INFINITY;
    for (int e = 0; e < X; ++e)
      if (!((used >> e) & 1ull) && l[e] > bv) { bv = l[e]; best = e; }
    used |= 1ull << best;
    const float p = __expf(bv - mx);
    ids[b * k + j] = best;
    w[b * k + j] = p;
    tot += p;
  }
  for (int j = 0; j < k; ++j) w[b * k + j] /= tot;
}

void moe_route(const float* logits, int B, int X, int k, int* ids, float* w, hipStream_t s) {
  hipLaunchKernelGGL(moe_route_kernel, dim3((B + 63) / 64), dim3(64), 0, s, logits, B, X, k, ids, w);
}

__global__ void gather_rows_kernel(const float* x, int ld, const int* idx, int n, float* out) {
  const long long r = blockIdx.x;
  const float* src = x + (long long)idx[r] * ld;
  for (int i = threadIdx.x; i < n; i += blockDim.x) out[r * n + i] = src[i];
}

void gather_rows(const float* x, int ld, const int* idx, int rows, int n, float* out, hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(rows), dim3(256), 0, s, x, ld, idx, n, out);
}

}  // namespace omx
