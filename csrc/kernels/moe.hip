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
constexpr int ROUTER_NT = 1024;
constexpr int ROUTER_KMAX = 16384;  // normalised token staged in LDS (72 KiB with the padding below)
// LDS index of token element o: 4 pad floats after every 32 so that lanes reading consecutive pieces
// (32 floats apart) spread over the banks instead of all hitting one (a 64-way conflict per ds_read)
__device__ __forceinline__ int rpad(int o) { return o + (o >> 5) * 4; }
constexpr int ROUTER_PPT = 2;       // 32-weight pieces per thread: X * K / 32 <= 2048 (X = 8 at K <= 8192)
// one 1024-thread block per token; thread t owns pieces t, t + 1024 of the flattened (expert, piece)
// list. A single block is latency-bound, so everything it reads from memory is requested up front:
// Q8 (the loader's requantised F32 router, Mixtral): the raw piece bytes go to registers before the
// token is read and are converted only after the statistics (one round trip for everything); other
// types dequantise through the generic dequant_piece. Measured phases (scripts/bench_router.py)
// before this: statistics 2.6 us, dots 2.7 us (piece loads serialised behind a per-type branch
// loop), top-k 1.6 us (a 16-deep dependent LDS sum per expert); after: 1.9 / 0.8 / 0.9 us, 4.9 us
// per launch (profiles/r3_moe/bench_router_after.log). Variants measured and dropped: v_readlane
// selection, group_max over the first 8 lanes, lane-0 serial top-k, DPP wave totals -- none faster
// in the engine (5.9-6.6 us); what remains in each phase is latency (cold instruction fetch of a
// once-per-layer kernel, HBM round trip of the token), not instruction count.
template <bool Q8>
__global__ __launch_bounds__(ROUTER_NT) void moe_router_kernel(GemvParams P, int k, int* ids, float* wout) {
  extern __shared__ __attribute__((aligned(16))) float xs[];  // [K padded to whole super-blocks]
  __shared__ float red[ROUTER_NT / 64];
  const int b = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const QMat& W = P.w;
  const int K = W.K, X = W.N, SB = n_sb(K), np = SB * 8, total = X * np;
  const float* x = P.x + (long long)b * P.ldx;
  // timeline probe (scripts/bench_router.py): 5 x s_memrealtime per block (entry, statistics reduced,
  // token staged, dots reduced, done); null in production
  auto stamp = [&](int k) {
    if (P.dbg_ts && tid == 0) P.dbg_ts[8 * b + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // 1. router pieces, then this thread's token slice, all in flight together
  int olo[ROUTER_PPT], ohi[ROUTER_PPT];
  u32x4 qa[Q8 ? ROUTER_PPT : 1][2];
  unsigned qd[Q8 ? ROUTER_PPT : 1];
  float lo[Q8 ? 1 : ROUTER_PPT][16], hi[Q8 ? 1 : ROUTER_PPT][16];
#pragma unroll
  for (int j = 0; j < ROUTER_PPT; ++j) {
    if (j > 0 && ROUTER_NT * j >= total) break;  // block-uniform: X * np <= 1024 needs one piece each
    const int i = min(tid + j * ROUTER_NT, total - 1);
    const int e = i / np, p = i - e * np;
    if constexpr (Q8) {
      const int sb = p >> 3, t = p & 7;
      const long long pi = (long long)t * SB + sb;
      const uint8_t* q = W.s0 + (long long)e * SB * 256 + 32 * pi;
      qa[j][0] = *(const u32x4*)q;
      qa[j][1] = *(const u32x4*)(q + 16);
      qd[j] = *(const uint16_t*)(W.s1 + (long long)e * SB * 16 + 16LL * sb + 2 * t);
      olo[j] = 256 * sb + 32 * t;
      ohi[j] = olo[j] + 16;
    } else {
      dequant_piece(W, e, p, lo[j], hi[j], olo[j], ohi[j]);
    }
  }
  f32x4 xv = {0.f, 0.f, 0.f, 0.f};
  f32x4 nv = {1.f, 1.f, 1.f, 1.f};
  if (4 * tid < K) {
    xv = *(const f32x4*)(x + 4 * tid);
    if (P.norm_w) nv = *(const f32x4*)(P.norm_w + 4 * tid);
  }
  // 2. RMS statistics (K <= 4 * ROUTER_NT in one pass; larger K: strided remainder), normalised copy
  float ss = xv.x * xv.x + xv.y * xv.y + xv.z * xv.z + xv.w * xv.w;
  for (int i = tid + ROUTER_NT; i < K / 4; i += ROUTER_NT) {
    const f32x4 v = *(const f32x4*)(x + 4 * i);
    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  ss = block_sum<ROUTER_NT>(ss, red);
  stamp(1);
  const float rstd = P.norm == NORM_RMS ? rsqrtf(ss / K + P.eps) : 1.f;
  for (int i = tid; i < SB * 64; i += ROUTER_NT) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (4 * i < K) {
      if (i == tid) {
        v = xv * rstd * nv;
      } else {
        v = *(const f32x4*)(x + 4 * i) * rstd;
        if (P.norm_w) v *= *(const f32x4*)(P.norm_w + 4 * i);
      }
    }
    *(f32x4*)(xs + rpad(4 * i)) = v;
  }
  __syncthreads();
  stamp(2);
  // 3. piece dots, summed per expert (pieces of one expert are consecutive in the flat list)
  float part[ROUTER_PPT];
#pragma unroll
  for (int j = 0; j < ROUTER_PPT; ++j) {
    part[j] = 0.f;
    if (j > 0 && ROUTER_NT * j >= total) continue;
    float acc = 0.f;
    if constexpr (Q8) {
      const unsigned qq[8] = {qa[j][0].x, qa[j][0].y, qa[j][0].z, qa[j][0].w,
                              qa[j][1].x, qa[j][1].y, qa[j][1].z, qa[j][1].w};
#pragma unroll
      for (int c = 0; c < 8; ++c) {  // 4 weights per dword; dwords 0-3 at olo, 4-7 at ohi
        const f32x4 a = *(const f32x4*)(xs + rpad(c < 4 ? olo[j] : ohi[j]) + 4 * (c & 3));
        const int w = (int)qq[c];
        acc += (float)((w << 24) >> 24) * a.x + (float)((w << 16) >> 24) * a.y + (float)((w << 8) >> 24) * a.z +
               (float)(w >> 24) * a.w;
      }
      acc *= h2f((uint16_t)qd[j]);
    } else {
#pragma unroll
      for (int i = 0; i < 16; i += 4) {
        const f32x4 a = *(const f32x4*)(xs + rpad(olo[j]) + i), c = *(const f32x4*)(xs + rpad(ohi[j]) + i);
        acc += lo[j][i] * a.x + lo[j][i + 1] * a.y + lo[j][i + 2] * a.z + lo[j][i + 3] * a.w;
        acc += hi[j][i] * c.x + hi[j][i + 1] * c.y + hi[j][i + 2] * c.z + hi[j][i + 3] * c.w;
      }
    }
    part[j] = tid + j * ROUTER_NT < total ? acc : 0.f;
  }
  // np is a multiple of 8: an expert's pieces span whole 8-lane groups; reduce within groups of 8,
  // one LDS slot per group; wave 0 adds an expert's SB slots in fixed order (deterministic logits:
  // TP ranks must route identically)
  __shared__ float gsum[ROUTER_PPT * ROUTER_NT / 8];
#pragma unroll
  for (int j = 0; j < ROUTER_PPT; ++j) {
    if (j > 0 && ROUTER_NT * j >= total) break;
    float v = group_sum<8>(part[j]);
    if ((lane & 7) == 0) gsum[(tid + j * ROUTER_NT) / 8] = v;
  }
  __syncthreads();
  stamp(3);
  if (wave != 0) return;
  // 4. wave 0: logit of expert e (lane e) = sum of its SB group sums (reads issued 16 at a time), top-k
  float v = -INFINITY;
  if (lane < X) {
    float t = 0.f;
    const float* g = gsum + lane * SB;
#pragma unroll 16
    for (int m = 0; m < SB; ++m) t += g[m];
    v = t;
  }
  const float mx = wave_max(v);
  float tot = 0.f, mine = 0.f;
  int rank = -1;
  for (int j = 0; j < k; ++j) {
    const float bv = j == 0 ? mx : wave_max(v);
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
  stamp(4);
}

bool moe_router(const GemvParams& P, int k, int* ids, float* w, hipStream_t s) {
  const int np = (P.w.K + 255) / 256 * 8;
  if (P.w.N > 64 || P.w.K > ROUTER_KMAX || P.w.K % 4 || P.w.N * np > ROUTER_PPT * ROUTER_NT) return false;
  static bool attr = false;  // dynamic LDS above 64 KiB: one attribute call, before any graph capture
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)moe_router_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              ROUTER_KMAX * 9 / 8 * (int)sizeof(float));
    (void)hipFuncSetAttribute((const void*)moe_router_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              ROUTER_KMAX * 9 / 8 * (int)sizeof(float));
    attr = true;
  }
  const size_t lds = (size_t)((P.w.K + 255) / 256) * 288 * sizeof(float);
  if (P.w.qtype == QT_Q8_0)
    hipLaunchKernelGGL(moe_router_kernel<true>, dim3(P.B), dim3(ROUTER_NT), lds, s, P, k, ids, w);
  else
    hipLaunchKernelGGL(moe_router_kernel<false>, dim3(P.B), dim3(ROUTER_NT), lds, s, P, k, ids, w);
  return true;
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
