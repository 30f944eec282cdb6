// Small-batch quantised GEMV for continuous-batching decode steps (2 <= B < GEMM_MIN_B).
// Shares the layout-v2 register tiles, activation prologue and epilogues with gemv.hip (gemv_core.h).
#include "gemv_core.h"

namespace omx {

// M block-wide sums in one pair of barriers (red: M * NT / 64 floats)
template <int NT, int M>
__device__ __forceinline__ void block_sums(float (&v)[M], float* red) {
  constexpr int NWV = NT / 64;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int m = 0; m < M; ++m) v[m] = wave_sum(v[m]);
  __syncthreads();
  if (l == 0) {
#pragma unroll
    for (int m = 0; m < M; ++m) red[m * NWV + w] = v[m];
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < M; ++m) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NWV; ++i) t += red[m * NWV + i];
    v[m] = t;
  }
}

// int8-quantise one normalised 16-element activation group into its LDS slot
__device__ __forceinline__ void quant_group(float (&v)[16], i32x4* lq, f32x2* lf, int slot) {
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) amax = fmaxf(amax, fabsf(v[j]));
  const float d = amax / 127.f;
  const float id = amax > 0.f ? 127.f / amax : 0.f;
  int qsum = 0;
  i32x4 pk;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int word = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int q = (int)rintf(v[4 * j + k] * id);
      qsum += q;
      word |= (q & 0xFF) << (8 * k);
    }
    pk[j] = word;
  }
  lq[slot] = pk;
  lf[slot] = (f32x2){d, d * (float)qsum};
}

// ---------------------------------------------------------------------------------------------
// Small-batch decode kernel (continuous batching, 2 <= B < GEMM_MIN_B): the all-in-flight design of
// flight_body for BT activation rows per block. Each piece's codes are unpacked once and dotted
// against BT rows (compute_wtile<.., BT>), so the weights stream once per BT rows. Before this kernel
// B = 4 ran the persistent qgemv_kernel whose activation prologue queued behind the first weight
// tile (rocprofv3, profiles/r2_batch: Q4_K gate_up 36.7 us at B = 4 vs 13 us at B = 1).
//  MODE 0/1 (BT * NSB <= 4, no norm / RMS norm): every row's activations (and the norm weights) are requested into registers
//    ahead of the weights, normalised / quantised while the weights stream.
//  MODE 2 (larger tiles, LayerNorm): x-first -- the BT rows are staged into LDS (stage_x) before any weight is requested; the
//    activation round trip is paid once, the weight stream then runs uninterrupted.
template <int QT, int NSB, int BT, int J, int MODE>
__global__ __launch_bounds__(GEMV_NT) void qgemv_batch_kernel(GemvParams P) {
  constexpr int ROWS_B = GEMV_NW * 4, NT = GEMV_NT;
  constexpr bool REG = MODE < 2;  // MODE 0: no norm, 1: RMS norm (registers); 2: x-first LDS staging
  static_assert(!REG || BT * NSB <= 4, "register prologue holds BT * NSB activation groups");
  constexpr bool nrm = MODE == 1, lnb = false;
  constexpr int NRM = nrm ? 1 : 0;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const QMat& w = P.w;
  const int K = w.K, N = w.N, SB = n_sb(K);
  const int XS = SB * XPAD;
  i32x4* lq = (i32x4*)smem;                                // [BT][XS] + dummy slot
  f32x2* lf = (f32x2*)(smem + (size_t)(BT * XS + 1) * 16);  // [BT][XS] + dummy slot
  float* red = (float*)(lf + BT * XS + 1);                  // [2 * BT][NT / 64]
  const int b0 = blockIdx.y * BT;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, s = lane & 15;
  const int n_tiles = (N + ROWS_B - 1) / ROWS_B;
  const int rbase = wave * 4 + g;
  const int bx = blockIdx.x, gxn = gridDim.x;

  if constexpr (!REG) {
#pragma unroll
    for (int b = 0; b < BT; ++b) {
      if (b0 + b < P.B) {
        stage_x<NT>(P, P.x + (long long)(b0 + b) * P.ldx, K, SB, lq + b * XS, lf + b * XS, red);
      } else {
        for (int i = tid; i < XS; i += NT) {
          lq[b * XS + i] = (i32x4){0, 0, 0, 0};
          lf[b * XS + i] = (f32x2){0.f, 0.f};
        }
      }
    }
  }
  constexpr int XB = REG ? BT : 1, XN = REG ? NSB : 1;
  f32x4 xv[XB][XN][4], nw[XN][4], nb[XN][4];
  if constexpr (REG) {
#pragma unroll
    for (int i = 0; i < NSB; ++i) {
      const int gi = min(tid + NT * i, K / 16 - 1);
#pragma unroll
      for (int b = 0; b < BT; ++b) {
        const float* xr = P.x + (long long)min(b0 + b, P.B - 1) * P.ldx;
#pragma unroll
        for (int j = 0; j < 4; ++j) xv[b][i][j] = *(const f32x4*)(xr + 16 * gi + 4 * j);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (nrm) nw[i][j] = *(const f32x4*)(P.norm_w + 16 * gi + 4 * j);
        if constexpr (lnb) nb[i][j] = *(const f32x4*)(P.norm_b + 16 * gi + 4 * j);
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);  // activations ahead of the weights
  WTile<QT, NSB, 1> T[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int t = min(bx + j * gxn, n_tiles - 1);
    load_wtile<QT, NSB, 1>(w, 0, t * ROWS_B + rbase, N, SB, 0, s, T[j]);
  }
  __builtin_amdgcn_sched_barrier(0);  // every load issued before the prologue's first wait
  if constexpr (REG) {
#pragma unroll
    for (int i = 0; i < NSB; ++i) {
      const bool ok = 16 * (tid + NT * i) < K;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int b = 0; b < BT; ++b)
          if (!ok) xv[b][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        if constexpr (!nrm) nw[i][j] = (f32x4){1.f, 1.f, 1.f, 1.f};
        if constexpr (!lnb) nb[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    }
    float mean[BT], rstd[BT];
#pragma unroll
    for (int b = 0; b < BT; ++b) { mean[b] = 0.f; rstd[b] = 1.f; }
    if constexpr (nrm) {
      float st[2 * BT];
#pragma unroll
      for (int b = 0; b < BT; ++b) {
        float sm = 0.f, ss = 0.f;
#pragma unroll
        for (int i = 0; i < NSB; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 v = xv[b][i][j];
            sm += v.x + v.y + v.z + v.w;
            ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
          }
        st[2 * b] = sm;
        st[2 * b + 1] = ss;
      }
      block_sums<NT, 2 * BT>(st, red);
#pragma unroll
      for (int b = 0; b < BT; ++b) {
        rstd[b] = rsqrtf(st[2 * b + 1] / K + P.eps);  // MODE 1 = RMS norm
      }
    }
#pragma unroll
    for (int i = 0; i < NSB; ++i) {
      const int gi = tid + NT * i;
#pragma unroll
      for (int b = 0; b < BT; ++b) {
        const int slot = gi < SB * 16 ? b * XS + (gi >> 4) * XPAD + (gi & 15) : BT * XS;  // dummy slot
        float v[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x4 t = xv[b][i][j];
          if (nrm) t = (t - mean[b]) * rstd[b] * nw[i][j] + nb[i][j];
          v[4 * j] = t.x; v[4 * j + 1] = t.y; v[4 * j + 2] = t.z; v[4 * j + 3] = t.w;
        }
        if (16 * gi >= K || b0 + b >= P.B) {
#pragma unroll
          for (int j = 0; j < 16; ++j) v[j] = 0.f;
        }
        quant_group(v, lq, lf, slot);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int t = bx + j * gxn;
    if (t >= n_tiles) break;  // block-uniform
    float acc[1][BT];
#pragma unroll
    for (int b = 0; b < BT; ++b) acc[0][b] = 0.f;
    compute_wtile<QT, NSB, 1, BT, false>(T[j], SB, 0, s, lq, lf, XS, acc);
    finish_rows<1, BT>(P, acc, t * ROWS_B + rbase, N, b0, s);
  }
}


template <int QT, int NSB, int BT, int J>
static void launch_batch_j(const GemvParams& P, int gx, int by, int mode, size_t lds, hipStream_t s) {
  const dim3 grid(gx, by, 1), blk(GEMV_NT);
  if constexpr (BT * NSB <= 4) {
    if (mode == 0) { hipLaunchKernelGGL((qgemv_batch_kernel<QT, NSB, BT, J, 0>), grid, blk, lds, s, P); return; }
    if (mode == 1) { hipLaunchKernelGGL((qgemv_batch_kernel<QT, NSB, BT, J, 1>), grid, blk, lds, s, P); return; }
  }
  hipLaunchKernelGGL((qgemv_batch_kernel<QT, NSB, BT, J, 2>), grid, blk, lds, s, P);
}

template <int QT, int NSB, int BT>
static void launch_batch_n(const GemvParams& P, size_t lds, hipStream_t s) {
  constexpr int PB = (QT == QT_Q8_0 || QT == QT_Q6_K8) ? 8 : QT == QT_Q6_K ? 6 : QT == QT_Q5_K ? 5 : 4;
  constexpr int regs = NSB * (8 * PB + 5);                       // one weight tile per lane
  constexpr int XR = BT * NSB <= 4 ? (BT + 1) * NSB * 16 : 0;     // register prologue
  constexpr int XF = 12 * BT;                                     // activation fragments per piece
  constexpr int JM = 3 * regs + XR + XF <= 224 ? 3 : 2 * regs + XR + XF <= 224 ? 2 : 1;
  const int tiles = (P.w.N + 4 * GEMV_NW - 1) / (4 * GEMV_NW);
  const int by = (P.B + BT - 1) / BT;
  const int want = (256 * g_tune.blocks_per_cu + by - 1) / by;
  int J = (tiles + want - 1) / want;
  J = J < 1 ? 1 : J > JM ? JM : J;
  const int gx = (tiles + J - 1) / J;
  int mode = P.norm == NORM_NONE ? 0 : P.norm == NORM_RMS ? 1 : 2;
  if (BT * NSB > 4) mode = 2;
  if (J == 1) launch_batch_j<QT, NSB, BT, 1>(P, gx, by, mode, lds, s);
  else launch_batch_j<QT, NSB, BT, JM>(P, gx, by, mode, lds, s);
}

template <int QT, int BT>
static void launch_batch_bt(const GemvParams& P, int need, size_t lds, hipStream_t s) {
  switch (need) {
    case 1: launch_batch_n<QT, 1, BT>(P, lds, s); return;
    case 2: launch_batch_n<QT, 2, BT>(P, lds, s); return;
    default: launch_batch_n<QT, 3, BT>(P, lds, s); return;
  }
}

template <int QT>
static void launch_batch_q(const GemvParams& P, int BT, int need, size_t lds, hipStream_t s) {
  if (BT == 2) launch_batch_bt<QT, 2>(P, need, lds, s);
  else if (BT == 4) launch_batch_bt<QT, 4>(P, need, lds, s);
  else launch_batch_bt<QT, 8>(P, need, lds, s);
}

static size_t batch_lds(int K, int BT) {
  const int SB = (K + 255) / 256;
  return (size_t)(BT * SB * XPAD + 1) * 24 + sizeof(float) * 2 * BT * GEMV_NW;
}

bool gemv_batch(const GemvParams& P, hipStream_t s) {
  if (P.B < 2 || P.B >= GEMM_MIN_B || P.expert_ids || P.merge_S || g_tune.debug) return false;
  const int need = ((P.w.K + 255) / 256 + 15) / 16;  // 16-super-block chunks: one chunk per lane group
  if (need > 3) return false;
  int BT = P.B <= 2 ? 2 : P.B <= 4 ? 4 : 8;
  while (BT > 2 && batch_lds(P.w.K, BT) > 80 * 1024) BT /= 2;
  const size_t lds = batch_lds(P.w.K, BT);
  if (lds > 80 * 1024) return false;
  switch (P.w.qtype) {
    case QT_Q4_K: launch_batch_q<QT_Q4_K>(P, BT, need, lds, s); return true;
    case QT_Q6_K: launch_batch_q<QT_Q6_K>(P, BT, need, lds, s); return true;
    case QT_Q5_K: launch_batch_q<QT_Q5_K>(P, BT, need, lds, s); return true;
    case QT_Q4_0: launch_batch_q<QT_Q4_0>(P, BT, need, lds, s); return true;
    case QT_Q8_0: launch_batch_q<QT_Q8_0>(P, BT, need, lds, s); return true;
    default: return false;
  }
}

}  // namespace omx
