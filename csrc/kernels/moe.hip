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

// Fused router (decode and prefill): RMSNorm + router logits + softmax top-k + renormalised weights in
// ONE launch, one 256-thread block per token. Replaces the router GEMV + moe_route pair (two launches,
// the logits' round trip through memory: 5.5 + 4.8 us per layer on Mixtral, profiles/r2_models). The
// X <= 64 logits are exact fp32 dots of the dequantised router rows with the fp32 normalised token
// (dequant_piece), the experts one wave each in turn; wave 0 then holds logit e in lane e and draws the
// k largest by wave argmax (lowest index among equals, as moe_route_kernel).
constexpr int ROUTER_NT = 256;
__global__ __launch_bounds__(ROUTER_NT) void moe_router_kernel(GemvParams P, int k, int* ids, float* wout) {
  __shared__ float red[ROUTER_NT / 64];
  __shared__ float lg[64];
  const int b = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const QMat& W = P.w;
  const int K = W.K, X = W.N, SB = n_sb(K);
  const float* x = P.x + (long long)b * P.ldx;
  float ss = 0.f;
  for (int i = tid; i < K / 4; i += ROUTER_NT) {
    const f32x4 v = *(const f32x4*)(x + 4 * i);
    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  ss = block_sum<ROUTER_NT>(ss, red);
  const float rstd = P.norm == NORM_RMS ? rsqrtf(ss / K + P.eps) : 1.f;
  const int n_pieces = SB * 8;  // 32-weight pieces per row (K padded to whole super-blocks)
  for (int e = wave; e < X; e += ROUTER_NT / 64) {
    float acc = 0.f;
    for (int p = lane; p < n_pieces; p += 64) {
      float lo[16], hi[16];
      int olo, ohi;
      dequant_piece(W, e, p, lo, hi, olo, ohi);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (olo + i < K) acc += lo[i] * x[olo + i] * (P.norm_w ? P.norm_w[olo + i] : 1.f);
        if (ohi + i < K) acc += hi[i] * x[ohi + i] * (P.norm_w ? P.norm_w[ohi + i] : 1.f);
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) lg[e] = acc * rstd;
  }
  __syncthreads();
  if (wave != 0) return;
  float v = lane < X ? lg[lane] : -INFINITY;
  const float mx = wave_max(v);
  float tot = 0.f, mine = 0.f;
  int rank = -1;
  for (int j = 0; j < k; ++j) {
    const float bv = wave_max(v);
    const unsigned long long hit = __ballot(v == bv && lane < X);
    const int best = hit ? __ffsll((long long)hit) - 1 : 0;
    const float pr = __expf(bv - mx);
    tot += pr;
    if (lane == best) {
      rank = j;
      mine = pr;
      v = -INFINITY;  // drawn
    }
  }
  if (rank >= 0) {
    ids[b * k + rank] = lane;
    wout[b * k + rank] = mine / tot;
  }
}

void moe_router(const GemvParams& P, int k, int* ids, float* w, hipStream_t s) {
  hipLaunchKernelGGL(moe_router_kernel, dim3(P.B), dim3(ROUTER_NT), 0, s, P, k, ids, w);
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

namespace omx {

// ---------------------------------------------------------------------------------------------
// Prefill grouping for the MFMA grouped GEMM (gemm.hip GROUPED): sort the B*k (token, expert)
// pairs by expert -- deterministic positions (pairs keep their original order inside an expert,
// via wave ballots + a block scan, no atomics) -- and cut each expert's rows into tiles of <= 128
// rows: tiles[t] = {expert, first sorted row, rows}. One block; B*k <= 1024 * MOE_SORT_PAIRS.
constexpr int MOE_SORT_NT = 1024;

__global__ __launch_bounds__(MOE_SORT_NT) void moe_sort_kernel(const int* eids, int n_pairs, int X, int* rows,
                                                               int* tiles, int* n_tiles, int tile_m) {
  __shared__ int wave_cnt[MOE_SORT_NT / 64];
  __shared__ int base_s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) base_s = 0;
  int n_t = 0;  // thread 0: tiles emitted
  __syncthreads();
  for (int e = 0; e < X; ++e) {
    const int base = base_s;
    int run = 0;  // pairs of expert e in earlier chunks
    for (int c0 = 0; c0 < n_pairs; c0 += MOE_SORT_NT) {
      const int i = c0 + tid;
      const bool mine = i < n_pairs && eids[i] == e;
      const unsigned long long m = __ballot(mine);
      const int before = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) wave_cnt[wave] = __popcll(m);
      __syncthreads();
      int woff = 0, tot = 0;
      for (int w = 0; w < MOE_SORT_NT / 64; ++w) {
        if (w < wave) woff += wave_cnt[w];
        tot += wave_cnt[w];
      }
      if (mine) rows[base + run + woff + before] = i;
      run += tot;
      __syncthreads();
    }
    if (tid == 0) {
      for (int r0 = 0; r0 < run; r0 += tile_m) {
        tiles[3 * n_t] = e;
        tiles[3 * n_t + 1] = base + r0;
        tiles[3 * n_t + 2] = min(tile_m, run - r0);
        ++n_t;
      }
      base_s = base + run;
    }
    __syncthreads();
  }
  if (tid == 0) *n_tiles = n_t;
}

void moe_sort(const int* eids, int n_pairs, int X, int* rows, int* tiles, int* n_tiles, int tile_m, hipStream_t s) {
  hipLaunchKernelGGL(moe_sort_kernel, dim3(1), dim3(MOE_SORT_NT), 0, s, eids, n_pairs, X, rows, tiles, n_tiles,
                     tile_m);
}

}  // namespace omx
