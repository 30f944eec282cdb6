// Prefill dequant GEMM on the matrix cores: Y[M][N] = epi(X[M][K] . W[N][K]^T)
// for M = prompt tokens (or a large decode batch), W in the repacked quant layout v2.
//
// MI355X-first design:
//  * Block tile 128 (tokens) x 128 (weight rows), K step 128 = half a super-block = 4 pieces per
//    weight row for EVERY quant type (Q4_K: two sub-block pairs, Q6_K: one 128-weight half, Q4_0 /
//    Q8_0: four 32-blocks), so the dequant unit is uniform. 4 waves, each a 64 x 64 sub-tile of
//    2 x 2 `v_mfma_f32_32x32x16_f16` accumulators (64 fp32 acc registers per lane).
//  * Dequant is fused into the LDS staging: the raw quant bytes (+ scales) and fp16 activation tile
//    of the step two ahead are loaded into one of two register stages right after the barrier and
//    stay in flight through the MFMA work of two steps (register-staged pipeline); the
//    weights cross HBM once per 128 prompt tokens instead of once per 4 (batched GEMV).
//  * Both operands use the same "8 consecutive K of one row" fragment (A = X rows, B = W rows, see
//    the gfx950 32x32x16 lane map), so X and dequantised W share one padded row-major LDS format:
//    272-B rows keep the 16-B fragment reads of 32 rows on distinct banks.
//  * Dequant runs in packed fp16: `(q & 0x000F000F) | 0x64006400` is two exact halves 1024 + n in
//    one VALU op, then v_pk_add / v_pk_fma apply zero point and scale (~2 ops per weight; the scalar
//    byte -> fp32 -> fp16 path measured ~420 VALU per K step per wave, VALU-bound next to 32 MFMAs:
//    profiles/r1_gemm). The pair extraction yields K in the order (0, 2, 1, 3) within every 4
//    weights; `prep_x16` writes the activations in that same order (free there), and a dot product
//    is invariant to a common permutation of K.
//  * The activation input is converted once per GEMM to fp16 by `prep_x16` (RMSNorm / LayerNorm
//    fused there, the same norms the GEMV prologue applies), into the executor's x16 workspace.
//  * Small M (a short prompt) leaves the chip idle -- N = 4096 at M = 128 is 32 tiles for 256 CUs --
//    so K is split over blockIdx.z: each split writes an fp32 partial slab, and a finalize kernel sums
//    the slabs in fixed order (deterministic, no atomics) and applies the fused epilogue.
//  * Epilogue through LDS: the fp32 tile is staged so each output has its row-pair partner (SiLU-GLU
//    gate/up, RoPE pairs) and stores are coalesced; the element epilogue is the GEMV's (epilogue.h).
#include <stdexcept>

#include "common.h"
#include "epilogue.h"
#include "ops.h"

namespace omx {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GM_BM = 128, GM_BN = 128, GM_BK = 128, GM_NT = 256;
constexpr int GM_LD = GM_BK + 8;   // f16 LDS row stride (272 B)
constexpr int GM_LDC = GM_BN + 4;  // fp32 epilogue tile stride
constexpr size_t GM_LDS = (size_t)2 * GM_BM * GM_LD * sizeof(f16);

static_assert((size_t)GM_BM * GM_LDC * sizeof(float) <= GM_LDS, "epilogue tile must fit the operand LDS");

// ------------------------------------------------------------------------------------------------
// activation prep: x fp32 [B][ldx] -> (norm) -> fp16 [B][K]; one block per row
__global__ __launch_bounds__(256) void prep_x16_kernel(GemvParams P, f16* out) {
  __shared__ float red[4];
  const int b = blockIdx.x, K = P.w.K;
  // MoE grouped GEMM: sorted row b reads the token of its (token, expert) pair
  const int src = P.moe_gather ? P.moe_rows[b] / P.n_sel : b;
  const float* x = P.x + (long long)src * P.ldx;
  float mean = 0.f, rstd = 1.f;
  if (P.norm != NORM_NONE) {
    float s = 0.f, ss = 0.f;
    for (int i = threadIdx.x; i < K / 4; i += 256) {
      const f32x4 v = *(const f32x4*)(x + 4 * i);
      s += v.x + v.y + v.z + v.w;
      ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    ss = block_sum<256>(ss, red);
    if (P.norm == NORM_LAYER) {
      s = block_sum<256>(s, red);
      mean = s / K;
      rstd = rsqrtf(fmaxf(ss / K - mean * mean, 0.f) + P.eps);
    } else {
      rstd = rsqrtf(ss / K + P.eps);
    }
  }
  f16* o = out + (long long)b * K;
  for (int i = threadIdx.x; i < K / 4; i += 256) {
    f32x4 v = *(const f32x4*)(x + 4 * i);
    if (P.norm != NORM_NONE) {
      const f32x4 w = *(const f32x4*)(P.norm_w + 4 * i);
      v = (v - mean) * rstd * w;
      if (P.norm == NORM_LAYER && P.norm_b) v += *(const f32x4*)(P.norm_b + 4 * i);
    }
    // K order (0, 2, 1, 3) inside each 4 -- the order the packed dequant produces for the weights
    *(f16x4*)(o + 4 * i) = (f16x4){(f16)v.x, (f16)v.z, (f16)v.y, (f16)v.w};
  }
}

// ------------------------------------------------------------------------------------------------
// raw quant bytes of this thread's two pieces of one weight row for one K step
template <int QT>
struct WRaw {
  u32x4 a[2];
  u32x4 b[QT == QT_Q8_0 ? 2 : 1];
  u32x2 h[QT == QT_Q6_K ? 2 : 1];
  unsigned q5h[QT == QT_Q5_K ? 2 : 1];
  u32x4 m;
  unsigned d;
};

template <int QT>
__device__ __forceinline__ void load_wraw(const QMat& w, long long row, int SB, int ks, int pp, WRaw<QT>& R) {
  const long long sb = ks >> 1;
  const int t0 = 4 * (ks & 1) + pp;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long long pi = (long long)(t0 + i) * SB + sb;
    if constexpr (QT == QT_Q8_0) {
      const uint8_t* q = w.s0 + row * SB * 256 + 32 * pi;
      R.a[i] = __builtin_nontemporal_load((const u32x4*)q);
      R.b[i] = __builtin_nontemporal_load((const u32x4*)(q + 16));
    } else {
      R.a[i] = __builtin_nontemporal_load((const u32x4*)(w.s0 + row * SB * 128 + 16 * pi));
      if constexpr (QT == QT_Q6_K) R.h[i] = __builtin_nontemporal_load((const u32x2*)(w.s1 + row * SB * 64 + 8 * pi));
      if constexpr (QT == QT_Q5_K) R.q5h[i] = __builtin_nontemporal_load((const unsigned*)(w.s2 + row * SB * 32 + 4 * pi));
    }
  }
  if constexpr (QT == QT_Q6_K) {
    R.m = *(const u32x4*)(w.s2 + row * SB * 16 + 16 * sb);
    R.d = *(const uint16_t*)(w.s3 + row * SB * 2 + 2 * sb);
  } else {
    R.m = *(const u32x4*)(w.s1 + row * SB * 16 + 16 * sb);
  }
}

__device__ __forceinline__ unsigned sel4(const u32x4& v, int i) {
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h2 as_h2(unsigned v) { return __builtin_bit_cast(h2, v); }
__device__ __forceinline__ unsigned as_u(h2 v) { return __builtin_bit_cast(unsigned, v); }
__device__ __forceinline__ h2 hsplat(float f) { return (h2){(f16)f, (f16)f}; }

constexpr unsigned MAGIC = 0x64006400u;  // fp16 1024.0 in both halves

// 4-bit codes of one dword -> 4 packed pairs: lo (e0,e2),(e1,e3) and hi likewise, each (n + 1024)
__device__ __forceinline__ void nib_pairs(unsigned q, unsigned& l0, unsigned& l1, unsigned& h0, unsigned& h1) {
  l0 = (q & 0x000F000Fu) | MAGIC;
  l1 = ((q >> 8) & 0x000F000Fu) | MAGIC;
  h0 = ((q >> 4) & 0x000F000Fu) | MAGIC;
  h1 = ((q >> 12) & 0x000F000Fu) | MAGIC;
}

// (n + 1024) pairs -> (n - z) * s + c, 2 packed ops
__device__ __forceinline__ unsigned dq(unsigned p, h2 off, h2 sc, h2 c) {
  return as_u((as_h2(p) - off) * sc + c);
}

// store one half-piece (16 weights as 8 pairs in (0,2,1,3) order) -> two 16-B LDS stores
__device__ __forceinline__ void st8(f16* dst, const unsigned (&w)[8]) {
  *(u32x4*)dst = (u32x4){w[0], w[1], w[2], w[3]};
  *(u32x4*)(dst + 8) = (u32x4){w[4], w[5], w[6], w[7]};
}

template <int QT>
__device__ __forceinline__ void dequant_store(const WRaw<QT>& R, int ks, int pp, f16* wrow) {
  const int half = ks & 1;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = pp + i;        // piece within this K step (0..3)
    const int t = 4 * half + p;  // piece within the super-block
    unsigned lo[8], hi[8];
    int olo, ohi;
    if constexpr (QT == QT_Q5_K) {
      const int c = t >> 1, h = t & 1;
      const u32x4 q = R.a[i];  // unsigned nibbles; 5th bits from q5h (quant.py _q5k_qh_split)
      const unsigned H = R.q5h[i];
      const float d = h2f(R.m.x & 0xFFFF), dmin = h2f(R.m.x >> 16);
      float sc[2], mn[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int j = 2 * c + k, sh = 8 * (j & 3);
        const unsigned a = (R.m.y >> sh) & 0xFF, b = (R.m.z >> sh) & 0xFF, e = (R.m.w >> sh) & 0xFF;
        const unsigned s = j < 4 ? (a & 63) : ((e & 0xF) | ((a >> 6) << 4));
        const unsigned mm = j < 4 ? (b & 63) : ((e >> 4) | ((b >> 6) << 4));
        sc[k] = d * (float)s;
        mn[k] = -dmin * (float)mm;
      }
      const h2 off = hsplat(1024.f), s0 = hsplat(sc[0]), s1 = hsplat(sc[1]), c0 = hsplat(mn[0]), c1 = hsplat(mn[1]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        unsigned l0, l1, g0, g1;
        nib_pairs(sel4(q, e), l0, l1, g0, g1);
        // 5th bit of weights 4e + j: H byte j, bit e (lo) / 4 + e (hi) -> bit 4 of each fp16 half
        lo[2 * e] = dq(l0 | ((H << (4 - e)) & 0x00100010u), off, s0, c0);
        lo[2 * e + 1] = dq(l1 | ((H >> (4 + e)) & 0x00100010u), off, s0, c0);
        hi[2 * e] = dq(g0 | ((H >> e) & 0x00100010u), off, s1, c1);
        hi[2 * e + 1] = dq(g1 | ((H >> (8 + e)) & 0x00100010u), off, s1, c1);
      }
      olo = 64 * (c - 2 * half) + 16 * h;
      ohi = olo + 32;
    } else if constexpr (QT == QT_Q4_K) {
      const int c = t >> 1, h = t & 1;
      const u32x4 q = R.a[i] ^ 0x80808080u;  // undo the signed-high-nibble repack
      const float d = h2f(R.m.x & 0xFFFF), dmin = h2f(R.m.x >> 16);
      float sc[2], mn[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int j = 2 * c + k, sh = 8 * (j & 3);
        const unsigned a = (R.m.y >> sh) & 0xFF, b = (R.m.z >> sh) & 0xFF, e = (R.m.w >> sh) & 0xFF;
        const unsigned s = j < 4 ? (a & 63) : ((e & 0xF) | ((a >> 6) << 4));
        const unsigned mm = j < 4 ? (b & 63) : ((e >> 4) | ((b >> 6) << 4));
        sc[k] = d * (float)s;
        mn[k] = -dmin * (float)mm;
      }
      const h2 off = hsplat(1024.f), s0 = hsplat(sc[0]), s1 = hsplat(sc[1]), c0 = hsplat(mn[0]), c1 = hsplat(mn[1]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        unsigned l0, l1, g0, g1;
        nib_pairs(sel4(q, e), l0, l1, g0, g1);
        lo[2 * e] = dq(l0, off, s0, c0);
        lo[2 * e + 1] = dq(l1, off, s0, c0);
        hi[2 * e] = dq(g0, off, s1, c1);
        hi[2 * e + 1] = dq(g1, off, s1, c1);
      }
      olo = 64 * (c - 2 * half) + 16 * h;
      ohi = olo + 32;
    } else if constexpr (QT == QT_Q6_K) {
      const int sub = p;  // n == half
      const float d = h2f((uint16_t)R.d);
      const int il = 8 * half + sub, ih = il + 4;
      const float slo = d * (float)(int8_t)((sel4(R.m, il >> 2) >> (8 * (il & 3))) & 0xFF);
      const float shi = d * (float)(int8_t)((sel4(R.m, ih >> 2) >> (8 * (ih & 3))) & 0xFF);
      const h2 off = hsplat(1056.f), s0 = hsplat(slo), s1 = hsplat(shi), z = hsplat(0.f);  // 1024 + 32
      const unsigned H0 = R.h[i].x, H1 = R.h[i].y;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const unsigned q = sel4(R.a[i], e);
        // high 2 bits of weights 4e + j live in byte j, bits 2e..2e+1, of H0 (lo) / H1 (hi)
        const int sl = 4 - 2 * e;  // move bits 2e.. of bytes 0/2 to 4..5
        const unsigned hl0 = (sl >= 0 ? (H0 << sl) : (H0 >> -sl)) & 0x00300030u;
        const unsigned hl1 = (H0 >> (4 + 2 * e)) & 0x00300030u;  // bytes 1/3
        const unsigned hh0 = (sl >= 0 ? (H1 << sl) : (H1 >> -sl)) & 0x00300030u;
        const unsigned hh1 = (H1 >> (4 + 2 * e)) & 0x00300030u;
        lo[2 * e] = dq((q & 0x000F000Fu) | hl0 | MAGIC, off, s0, z);
        lo[2 * e + 1] = dq(((q >> 8) & 0x000F000Fu) | hl1 | MAGIC, off, s0, z);
        hi[2 * e] = dq(((q >> 4) & 0x000F000Fu) | hh0 | MAGIC, off, s1, z);
        hi[2 * e + 1] = dq(((q >> 12) & 0x000F000Fu) | hh1 | MAGIC, off, s1, z);
      }
      olo = 16 * sub;
      ohi = olo + 64;
    } else {
      const unsigned dw = sel4(R.m, t >> 1);
      const h2 sd = hsplat(h2f((t & 1) ? (dw >> 16) : (dw & 0xFFFF))), z = hsplat(0.f);
      if constexpr (QT == QT_Q4_0) {
        const u32x4 q = R.a[i] ^ 0x80808080u;
        const h2 off = hsplat(1032.f);  // 1024 + 8
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          unsigned l0, l1, g0, g1;
          nib_pairs(sel4(q, e), l0, l1, g0, g1);
          lo[2 * e] = dq(l0, off, sd, z);
          lo[2 * e + 1] = dq(l1, off, sd, z);
          hi[2 * e] = dq(g0, off, sd, z);
          hi[2 * e + 1] = dq(g1, off, sd, z);
        }
      } else {
        const h2 off = hsplat(1152.f);  // 1024 + 128: bytes are offset-binary after ^ 0x80
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned qa = sel4(R.a[i], e), qb = sel4(R.b[i], e);
          lo[2 * e] = dq(((qa & 0x00FF00FFu) | MAGIC) ^ 0x00800080u, off, sd, z);
          lo[2 * e + 1] = dq((((qa >> 8) & 0x00FF00FFu) | MAGIC) ^ 0x00800080u, off, sd, z);
          hi[2 * e] = dq(((qb & 0x00FF00FFu) | MAGIC) ^ 0x00800080u, off, sd, z);
          hi[2 * e + 1] = dq((((qb >> 8) & 0x00FF00FFu) | MAGIC) ^ 0x00800080u, off, sd, z);
        }
      }
      olo = 32 * p;
      ohi = olo + 16;
    }
    st8(wrow + olo, lo);
    st8(wrow + ohi, hi);
  }
}

template <int QT, bool GROUPED = false>
__global__ __launch_bounds__(GM_NT, 2) void qgemm_kernel(GemvParams P, const f16* __restrict__ X) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f16* Xs = (f16*)smem;             // [BM][LD]
  f16* Ws = Xs + GM_BM * GM_LD;     // [BN][LD]
  const QMat& w = P.w;
  int M = P.B;
  const int N = w.N, K = w.K, SB = n_sb(K);
  const int nks = (K + GM_BK - 1) / GM_BK;  // K steps (last may be zero-padded: Q4_0 / Q8_0 only)
  const int sk = gridDim.z, z = blockIdx.z;  // split-K: this block's K-step range
  const int ks0 = (int)((long long)z * nks / sk), ks1 = (int)((long long)(z + 1) * nks / sk);
  int m0 = blockIdx.y * GM_BM;
  long long row_base = 0;
  if constexpr (GROUPED) {  // one expert-homogeneous tile of sorted rows per blockIdx.y
    if ((int)blockIdx.y >= *P.moe_ntiles) return;  // block-uniform
    const int* tt = P.moe_tiles + 3 * blockIdx.y;
    row_base = (long long)tt[0] * N;
    m0 = tt[1];
    M = tt[1] + tt[2];  // rows of this tile: [m0, M)
  }
  const int n0 = blockIdx.x * GM_BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int srow = tid >> 1, spart = tid & 1;  // staging: row of the tile, which half of it
  const long long wrow = row_base + min(n0 + srow, N - 1);
  const f16* xrow = X + (long long)min(m0 + srow, M - 1) * K;

  // quant bytes in two register stages (A, B): the weights of K step ks + 2 (HBM) are requested while
  // ks + 1's wait in the other stage, so two steps of MFMA work cover their latency; the fp16
  // activation tile (L2-resident, shared by every N tile) keeps one stage, issued one step ahead.
  // One stage for both left the MFMA pipe mostly idle at the barrier (313 TFLOP/s at M = 2048,
  // profiles/r1_gemm); both in two stages needs > 256 VGPRs (1 wave per SIMD)
  WRaw<QT> wrA, wrB;
  f16x8 xr[8];
  auto issue_w = [&](int ks, WRaw<QT>& wr) { load_wraw<QT>(w, wrow, SB, ks, 2 * spart, wr); };
  auto issue_x = [&](int ks) {
    const int k0 = ks * GM_BK + 64 * spart;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + 8 * j;
      xr[j] = k < K ? *(const f16x8*)(xrow + k) : (f16x8){0, 0, 0, 0, 0, 0, 0, 0};
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 31, fk = 8 * (lane >> 5);
  auto step = [&](int ks, WRaw<QT>& wr) {
    __syncthreads();  // the previous step's fragment reads are done
#pragma unroll
    for (int j = 0; j < 8; ++j) *(f16x8*)(Xs + srow * GM_LD + 64 * spart + 8 * j) = xr[j];
    dequant_store<QT>(wr, ks, 2 * spart, Ws + srow * GM_LD);
    __syncthreads();
    if (ks + 1 < ks1) issue_x(ks + 1);      // in flight during this step's MFMAs
    if (ks + 2 < ks1) issue_w(ks + 2, wr);  // this stage is free again: two steps ahead
#pragma unroll
    for (int kk = 0; kk < GM_BK / 16; ++kk) {
      f16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = *(const f16x8*)(Xs + (wm * 64 + i * 32 + fr) * GM_LD + kk * 16 + fk);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = *(const f16x8*)(Ws + (wn * 64 + j * 32 + fr) * GM_LD + kk * 16 + fk);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };
  issue_w(ks0, wrA);
  issue_x(ks0);
  if (ks0 + 1 < ks1) issue_w(ks0 + 1, wrB);
  for (int ks = ks0; ks < ks1; ks += 2) {
    step(ks, wrA);
    if (ks + 1 >= ks1) break;
    step(ks + 1, wrB);
  }

  // C map: row = (r&3) + 8(r>>2) + 4(lane>>5), col = lane&31
  if (sk > 1) {  // partial slab z; gemm_finalize_kernel sums the slabs and applies the epilogue
    float* slab = P.gws + (long long)z * M * N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int gm = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const int gn = n0 + wn * 64 + j * 32 + (lane & 31);
          if (gm < M && gn < N) __builtin_nontemporal_store(acc[i][j][r], slab + (long long)gm * N + gn);
        }
    return;
  }
  // epilogue: fp32 tile through LDS
  __syncthreads();
  float* Cs = (float*)smem;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = wn * 64 + j * 32 + (lane & 31);
        Cs[row * GM_LDC + col] = acc[i][j][r];
      }
  __syncthreads();
  for (int e = tid; e < GM_BM * GM_BN; e += GM_NT) {
    const int m = e / GM_BN, n = e % GM_BN;
    const int gm = m0 + m, gn = n0 + n;
    if (gm >= M || gn >= N) continue;
    int bb = gm, zsel = 0;
    if (GROUPED && P.moe_scatter) {  // back to the token; routing weight + atomics in epi_apply
      const int pair = P.moe_rows[gm];
      bb = pair / P.n_sel;
      zsel = pair % P.n_sel;
    }
    epi_apply(P, bb, gn + P.row_offset, Cs[m * GM_LDC + n], Cs[m * GM_LDC + (n ^ 1)], zsel);
  }
}

// sums the split-K slabs in fixed order; each thread owns output pairs (n, n ^ 1), two per step
// (16-byte slab loads). scatter_rows (MoE down on the library path): output row m is the token of
// sorted pair scatter_rows[m]. 32-bit index math: the 64-bit division per element made this pass a
// third of the library GEMM's time at M = 2048 (profiles/r3_gemm PMC)
__global__ __launch_bounds__(256) void gemm_finalize_kernel(GemvParams P, int sk, const int* scatter_rows) {
  const int N = P.w.N, M = P.B;
  const int half = (N + 1) / 2, quads = (half + 1) / 2;  // pair pairs per row
  const long long slab = (long long)M * N;
  const unsigned total = (unsigned)M * (unsigned)quads;
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const int m = (int)(i / (unsigned)quads), q = (int)(i - (unsigned)m * (unsigned)quads);
    int bb = m, zsel = 0;
    if (scatter_rows) {
      const int pair = scatter_rows[m];
      bb = pair / P.n_sel;
      zsel = pair % P.n_sel;
    }
    const float* row = P.gws + (long long)m * N;
    const int n0 = 4 * q;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if ((N & 3) == 0) {  // n0 + 3 < N, 16-byte aligned
      for (int z = 0; z < sk; ++z) {
        const f32x4 t = *(const f32x4*)(row + z * slab + n0);
        v[0] += t.x;
        v[1] += t.y;
        v[2] += t.z;
        v[3] += t.w;
      }
    } else {
      for (int z = 0; z < sk; ++z)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (n0 + c < N) v[c] += row[z * slab + n0 + c];
    }
#pragma unroll
    for (int c = 0; c < 4; c += 2) {
      const int n = n0 + c;
      if (n >= N) break;
      epi_apply(P, bb, n + P.row_offset, v[c], v[c + 1], zsel);
      if (n + 1 < N) epi_apply(P, bb, n + 1 + P.row_offset, v[c + 1], v[c], zsel);
    }
  }
}

static dim3 finalize_grid(long long M, long long N) {
  const long long quads = ((N + 1) / 2 + 1) / 2;
  const long long b = (M * quads + 255) / 256;
  return dim3((unsigned)(b < 4096 ? (b > 0 ? b : 1) : 4096));
}

// split-K factor: fill ~2 blocks per CU when the (M, N) tile grid alone cannot, keeping >= 4 K
// steps per split and the slabs inside the workspace
static int split_k(const GemvParams& P, int tiles, int nks) {
  if (!P.gws || P.gws_elems <= 0) return 1;
  int sk = 1;
  while (sk < 8 && tiles * sk < 512 && nks / (2 * sk) >= 4 &&
         (long long)(2 * sk) * P.B * P.w.N <= P.gws_elems)
    sk *= 2;
  return sk;
}

void gemm_finalize(const GemvParams& P, int sk, hipStream_t s) {
  hipLaunchKernelGGL(gemm_finalize_kernel, finalize_grid(P.B, P.w.N), dim3(256), 0, s, P, sk, (const int*)nullptr);
}

template <int QT>
static void launch_gemm(const GemvParams& P, const f16* x16, hipStream_t s) {
  const int nt = (P.w.N + GM_BN - 1) / GM_BN, mt = (P.B + GM_BM - 1) / GM_BM;
  const int sk = split_k(P, nt * mt, (P.w.K + GM_BK - 1) / GM_BK);
  hipLaunchKernelGGL(qgemm_kernel<QT>, dim3(nt, mt, sk), dim3(GM_NT), GM_LDS, s, P, x16);
  if (sk > 1) {
    hipLaunchKernelGGL(gemm_finalize_kernel, finalize_grid(P.B, P.w.N), dim3(256), 0, s, P, sk, (const int*)nullptr);
  }
}

template <int QT>
static void launch_moe(const GemvParams& P, const f16* x16, hipStream_t s) {
  const int nt = (P.w.N + GM_BN - 1) / GM_BN;
  hipLaunchKernelGGL((qgemm_kernel<QT, true>), dim3(nt, P.moe_max_tiles, 1), dim3(GM_NT), GM_LDS, s, P, x16);
}

void moe_gemm(const GemvParams& P, hipStream_t s) {
  f16* x16 = (f16*)P.xws;
  hipLaunchKernelGGL(prep_x16_kernel, dim3(P.B), dim3(256), 0, s, P, x16);
  switch (P.w.qtype) {
    case QT_Q4_K: launch_moe<QT_Q4_K>(P, x16, s); break;
    case QT_Q6_K: launch_moe<QT_Q6_K>(P, x16, s); break;
    case QT_Q5_K: launch_moe<QT_Q5_K>(P, x16, s); break;
    case QT_Q4_0: launch_moe<QT_Q4_0>(P, x16, s); break;
    case QT_Q8_0: launch_moe<QT_Q8_0>(P, x16, s); break;
    default: break;
  }
}

bool moe_gemm_lib(const GemvParams& P, const int* counts, int X, hipStream_t s) {
  const int lm = moe_lib_min_m();
  const long long N = P.w.N, K = P.w.K;  // per-expert rows
  int maxc = 0, total = 0;
  for (int e = 0; e < X; ++e) {
    maxc = counts[e] > maxc ? counts[e] : maxc;
    total += counts[e];
  }
  if (lm <= 0 || P.B < lm || total != P.B || !P.w16ws || !P.yws || N * K > P.w16_elems || (long long)maxc * N > P.yws_elems)
    return false;
  const size_t wsb = P.gws ? (size_t)P.gws_elems * 4 : 0;
  const long long xrows = P.xws_elems ? P.xws_elems / K : P.B, yrows = P.yws_elems / N;
  auto cap_at = [&](int off) {  // rows readable from x16 row `off` on and writable in the slab
    const long long c = xrows - off < yrows ? xrows - off : yrows;
    return (int)(c > 0 ? c : 0);
  };
  for (int e = 0, o = 0; e < X; o += counts[e], ++e)  // every plan before any launch: no partial output
    if (counts[e] > 0 && !blas_plan_ok(counts[e], (int)N, (int)K, wsb, cap_at(o))) return false;
  f16* x16 = (f16*)P.xws;
  hipLaunchKernelGGL(prep_x16_kernel, dim3(P.B), dim3(256), 0, s, P, x16);  // all pairs (gathered when moe_gather)
  int off = 0;
  for (int e = 0; e < X; ++e) {
    const int cnt = counts[e];
    if (cnt > 0) {
      dequant_f16(P.w, P.w16ws, s, 1, (long long)e * N);
      if (!blas_gemm_tn(P.w16ws, x16 + (long long)off * K, P.yws, cnt, (int)N, (int)K, P.gws, wsb, s, cap_at(off)))
        throw std::runtime_error("moe_gemm_lib: hipBLASLt matmul failed after its plan was accepted");
      GemvParams F = P;
      F.gws = P.yws;
      F.B = cnt;
      const int* scatter = nullptr;
      if (P.moe_scatter) scatter = P.moe_rows + off;
      else F.y = P.y + (long long)off * P.ldy;  // GLU output in sorted order
      hipLaunchKernelGGL(gemm_finalize_kernel, finalize_grid(cnt, N), dim3(256), 0, s, F, 1, scatter);
    }
    off += cnt;
  }
  return true;
}

bool gemm_eligible(const GemvParams& P) {
  return P.xws != nullptr && P.B >= GEMM_MIN_B && P.expert_ids == nullptr && (P.w.K % 32) == 0;
}

// Large-M library path (blas.cpp): dequantise W once into fp16 (in prep_x16's K order), one hipBLASLt
// GEMM into the fp32 slab yws, then the fused epilogue as for split-K (finalize, one slab)
// -1: OMX_GEMM_LIB_MIN_M, read once. Default 0: prefill GEMMs never take the library. Round 6 made the
// hand-written dequant GEMM (gemm_dq.hip, register-ring edition) the only default path: the resident fp16
// weight copies that made hipBLASLt worth it (12.95 GB for 7B, 3.2x the model) are gone, and the per-call
// library path (dequantise W into fp16 scratch, GEMM, finalize) loses or ties at 2048 rows
// (profiles/r6_gemm). OMX_GEMM_LIB_MIN_M=<rows> keeps it reachable for A/B runs and the test oracle.
static int g_lib_min_m = -1;
// OMX_GEMM_LIB_GLU (default 1): 0 keeps the gate_up GEMMs on the dq kernel when the library path is on
static int g_lib_glu = -1;

int gemm_lib_min_m() {
  if (g_lib_min_m < 0) {
    const char* e = getenv("OMX_GEMM_LIB_MIN_M");
    g_lib_min_m = e ? atoi(e) : 0;
  }
  return g_lib_min_m;
}

// rows from which this matrix's prefill GEMM takes hipBLASLt (0 = never)
static int lib_min_for(const QMat&) { return gemm_lib_min_m(); }

static bool lib_glu() {
  if (g_lib_glu < 0) {
    const char* e = getenv("OMX_GEMM_LIB_GLU");
    g_lib_glu = e ? atoi(e) : 1;
  }
  return g_lib_glu != 0;
}

void set_gemm_lib_min_m(int m) { g_lib_min_m = m; }

// MoE prefill (default 256 pairs = 128 tokens at top-2): the per-expert GEMMs are plain dense GEMMs over
// contiguous sorted rows, and the grouped tile kernel (moe_gemm) they replace has no register-ring
// edition -- Mixtral's 2048-token TTFT is 196 ms on it vs 116 ms per expert on hipBLASLt (profiles/r6_models)
static int g_moe_lib_min_m = -1;
int moe_lib_min_m() {
  if (g_moe_lib_min_m < 0) {
    const char* e = getenv("OMX_MOE_LIB_MIN_M");
    g_moe_lib_min_m = e ? atoi(e) : 256;
  }
  return g_moe_lib_min_m;
}
void set_moe_lib_min_m(int m) { g_moe_lib_min_m = m; }

static bool gemm_lib(const GemvParams& P, const f16* x16, hipStream_t s) {
  const int lm = lib_min_for(P.w);
  const long long M = P.B, N = P.w.N, K = P.w.K;
  if (lm <= 0 || M < lm || !P.yws || M * N > P.yws_elems) return false;
  if (!P.w16ws || N * K > P.w16_elems) return false;
  const long long xcap = P.xws_elems ? P.xws_elems / K : M, ycap = P.yws_elems / N;
  const int m_cap = (int)(xcap < ycap ? xcap : ycap);
  if (!blas_plan_ok((int)M, (int)N, (int)K, P.gws ? (size_t)P.gws_elems * 4 : 0, m_cap)) return false;
  dequant_f16(P.w, P.w16ws, s, 1);
  if (!blas_gemm_tn(P.w16ws, x16, P.yws, (int)M, (int)N, (int)K, P.gws, P.gws ? (size_t)P.gws_elems * 4 : 0, s,
                    m_cap))
    throw std::runtime_error("gemm_lib: hipBLASLt matmul failed after its plan was accepted");
  GemvParams F = P;
  F.gws = P.yws;
  hipLaunchKernelGGL(gemm_finalize_kernel, finalize_grid(M, N), dim3(256), 0, s, F, 1, (const int*)nullptr);
  return true;
}

void gemm(const GemvParams& P, hipStream_t s) {
  f16* x16 = (f16*)P.xws;
  // hipBLASLt from gemm_lib_min_m() rows (the GLU matrices unless OMX_GEMM_LIB_GLU=0; always when the
  // threshold is forced below 128: the test oracle); from 128 rows the stream-order kernel
  // (gemm_dq.hip), below that the 128 x 128 tile here
  const int lm = lib_min_for(P.w);
  const bool glu = P.epi == EPI_GLU || P.epi == EPI_GEGLU;
  const bool lib = lm > 0 && P.B >= lm && (!glu || lib_glu() || lm < 128);
  if (lib) {
    hipLaunchKernelGGL(prep_x16_kernel, dim3(P.B), dim3(256), 0, s, P, x16);
    if (gemm_lib(P, x16, s)) {
      count_launch(LC_GEMM_LIB);
      return;
    }
  }
  if (dq_gemm(P, s)) return;
  count_launch(LC_GEMM_TILE);
  if (!lib) hipLaunchKernelGGL(prep_x16_kernel, dim3(P.B), dim3(256), 0, s, P, x16);
  switch (P.w.qtype) {
    case QT_Q4_K: launch_gemm<QT_Q4_K>(P, x16, s); break;
    case QT_Q6_K: launch_gemm<QT_Q6_K>(P, x16, s); break;
    case QT_Q5_K: launch_gemm<QT_Q5_K>(P, x16, s); break;
    case QT_Q4_0: launch_gemm<QT_Q4_0>(P, x16, s); break;
    case QT_Q8_0: launch_gemm<QT_Q8_0>(P, x16, s); break;
    default: break;
  }
}

}  // namespace omx
