// Stream-order dequant prefill GEMM: kernels, launch geometry and the tile x split-K chooser as
// templates. One translation unit per weight type instantiates them (gemm_dq_<type>.hip), so the six
// heavy instantiations compile in parallel; gemm_dq.hip holds the dispatcher and the knobs.
//
// Prefill dequant GEMM, stream-order edition: Y[M][N] = epi(X[M][K] . W[N][K]^T)
// for M = prompt tokens, W in the resident layout v2 (no second weight copy, no fp16 weight scratch).
//
// MI355X-first design:
//  * K in STORAGE order. Layout v2 keeps each row's codes piece-major (piece t of super-block sb at
//    byte (t * SB + sb) * piece_bytes), so the row's code stream is one contiguous run. A dot product
//    is invariant under a common permutation of K, so this kernel walks K in exactly that stream
//    order: K step ks is the 32 (64 for Q8_0) contiguous code bytes of pieces 2 ks, 2 ks + 1 of every
//    weight row -- no gather, each 128-B line is consumed over 4 consecutive K steps from L2. The
//    activations are written once per GEMM in the same order by `prep_xp_kernel` (RMSNorm / LayerNorm
//    fused there), so the X tile is a plain row-major [M][Kp] fp16 slab.
//  * Inside a piece the packed-fp16 dequant produces weights in the order lo(0,2,1,3, 4,6,5,7, ...),
//    hi(same): `(q >> {0,8,4,12}) & 0x000F000F | 0x64006400` is two exact halves 1024 + n per VALU op,
//    then one v_pk_add (remove 1024) + one v_pk_fma (scale, zero point) -- ~2.5 VALU per 2 weights,
//    paid once per weight per 256-token M tile (the decode GEMVs pay it once per token).
//  * Block tile BM (tokens) x BN (weight rows) x 64 K, 8 waves (WM x WN), each a (BM/WM) x (BN/WN)
//    sub-tile of `v_mfma_f32_32x32x16_f16` accumulators (128 fp32 per lane at 256 x 256; the 32-row
//    shape needs half the fragment registers per MFMA batch of the 16 x 16 one at the same rate). Both
//    operands are staged in LDS as [rows][64 + 8] fp16: 144-B rows put the 16-B fragment reads of 16
//    consecutive rows on distinct bank groups (conflict-free), and both A (X rows) and B (W rows) read
//    "8 consecutive K of one row" per lane, so one image format serves both.
//  * Software pipeline, one register stage (the guide's T14 form): after the barrier that publishes
//    K step ks, every thread dequantises step ks + 1 (loaded a whole step ago) into the other LDS
//    buffer, issues the loads of step ks + 2, then runs the MFMAs of step ks -- one barrier per K step,
//    HBM/L2 latency covered by a full step of matrix work, VALU dequant of one wave overlapping the
//    MFMAs of the other wave on its SIMD.
//  * Grid: XCD-aware bijective remap, M-major: the blocks that share an XCD (and its 4 MB L2) work on
//    the same activation tile and different weight tiles, so X lines come from L2 (each weight tile is
//    read once per M tile, from HBM / the Infinity Cache). Grids that cannot fill 256 CUs split K
//    (fp32 slabs + the deterministic finalize of gemm.hip).
//  * Epilogue straight from the accumulators: the C fragment holds weight rows n on lanes 16 apart
//    and the row pair (n, n ^ 1) on adjacent lanes (one DPP swap), so SiLU-GLU / RoPE + KV scatter /
//    residual add / bias run through the shared epi_apply (epilogue.h) with no LDS round trip.
// Parity: replaces llama.cpp's prefill matmul inside `ollama/ollama` (reference pkg/model/pod.go:10-12);
// numerics vs fp32 torch on the dequantised weights in tests/test_gemm_gpu.py (dq cases).
#pragma once
#include <stdexcept>

#include "common.h"
#include "epilogue.h"
#include "ops.h"

namespace omx {

namespace {

constexpr int DQ_NT = 512;        // 8 waves
constexpr int DQ_BK = 64;         // K per step (two 32-code pieces per weight row)
// LDS operand image: [rows][64] fp16 (128-B rows), 16-B chunk c of row r at physical chunk
// c ^ ((r >> 1) & 7): the fragment reads of 16 consecutive rows at one chunk then cover 16 distinct
// bank slots (rows 2p, 2p + 1 share a chunk in opposite 128-B halves), and each wave's X DMA writes
// whole rows lane-linearly (the swizzle is applied to the global source address instead)
__device__ __forceinline__ int swz(int r, int c) { return r * 64 + 8 * (c ^ ((r >> 1) & 7)); }
// both kernels' W image: also flips chunk bit 1 on odd rows. Its dequantised-piece stores go out as
// ds_write_b128, banked per 8-lane group over 128 B (MI355X_MICROARCH.md §LDS): a group is rows 4g..4g+3
// x 2 half-pieces, and under swz() rows 4g / 4g+1 put their chunk pair on the same two 16-B slots (2-way
// conflicts on every W store). With the extra flip the group covers all 8 slots; the ds_read_b128 fragment
// reads (16-lane groups, 256-B banking) stay conflict-free (even and odd rows sit in opposite 128-B halves)
__device__ __forceinline__ int swzw(int r, int c) { return r * 64 + 8 * (c ^ ((r >> 1) & 7) ^ ((r & 1) << 1)); }
constexpr unsigned DQ_MAGIC = 0x64006400u;

typedef _Float16 dh2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ dh2 dq_h2(unsigned v) { return __builtin_bit_cast(dh2, v); }
__device__ __forceinline__ unsigned dq_u(dh2 v) { return __builtin_bit_cast(unsigned, v); }
__device__ __forceinline__ dh2 dq_splat(float f) { return (dh2){(f16)f, (f16)f}; }
// (n + 1024) pairs -> (n - off') * s + c  (off' = 1024 + zero point)
__device__ __forceinline__ unsigned dq2(unsigned p, dh2 off, dh2 sc, dh2 c) {
  return dq_u((dq_h2(p) - off) * sc + c);
}
__device__ __forceinline__ unsigned dsel(const u32x4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }

// weight offsets (natural K) of the lo / hi 16-weight halves of piece t of super-block sb
template <int QT>
__host__ __device__ __forceinline__ int piece_off(int t, int sb, int g) {
  static_assert(QT != QT_F16, "F16 rows are in natural order (prep_xp copies them straight)");
  if constexpr (QT == QT_Q4_K || QT == QT_Q5_K) return 256 * sb + 64 * (t >> 1) + 16 * (t & 1) + 32 * g;
  else if constexpr (QT == QT_Q6_K) return 256 * sb + 128 * (t >> 2) + 16 * (t & 3) + 64 * g;
  else return 256 * sb + 32 * t + 16 * g;  // Q4_0 / Q8_0
}

// ------------------------------------------------------------------------------------------------
// activations: x fp32 [B][ldx] -> (norm) -> fp16 [B][Kp] in storage order; one block per row.
// Stream position kp: piece P = kp / 32 (t = P / SB, sb = P % SB), slot p = kp % 32: half g = p / 16,
// byte i = 4 ((p & 15) / 4) + (0, 2, 1, 3)[p & 3] -> natural k = piece_off(t, sb, g) + i
template <int QT>
__global__ __launch_bounds__(256) void prep_xp_kernel(GemvParams P, f16* out, int Kp) {
  // K-quant / Q4_0 / Q8_0 rows: the normalised row is staged in LDS in natural order (coalesced global
  // reads of x and the norm weights), then every thread gathers its 8 stream positions from LDS and
  // writes them as one 16-B store. Gathering straight from global memory made every x read a scattered
  // 4-B load: 36 us per call at 2048 rows, 10 % of the 2048-token TTFT (profiles/r5_gemm prefill trace)
  extern __shared__ float xs[];  // [Kp] (quantized rows; F16 rows do not use it)
  __shared__ float red[4];
  const int b = blockIdx.x, K = P.w.K, SB = Kp >> 8;
  const float* x = P.x + (long long)b * P.ldx;
  float mean = 0.f, rstd = 1.f;
  constexpr bool STAGE = QT != QT_F16;
  if (P.norm != NORM_NONE || STAGE) {
    float s = 0.f, ss = 0.f;
    for (int i = threadIdx.x; i < K / 4; i += 256) {
      const f32x4 v = *(const f32x4*)(x + 4 * i);
      if constexpr (STAGE) *(f32x4*)(xs + 4 * i) = v;
      s += v.x + v.y + v.z + v.w;
      ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    for (int k = (K & ~3) + threadIdx.x; k < K; k += 256) {  // K % 4 tail
      const float v = x[k];
      if constexpr (STAGE) xs[k] = v;
      s += v;
      ss += v * v;
    }
    if (P.norm != NORM_NONE) {
      ss = block_sum<256>(ss, red);
      if (P.norm == NORM_LAYER) {
        s = block_sum<256>(s, red);
        mean = s / K;
        rstd = rsqrtf(fmaxf(ss / K - mean * mean, 0.f) + P.eps);
      } else {
        rstd = rsqrtf(ss / K + P.eps);
      }
    }
  }
  f16* o = out + (long long)b * Kp;
  if constexpr (QT == QT_F16) {  // natural order: the weight rows are plain fp16
    for (int c = threadIdx.x; c < Kp / 8; c += 256) {
      f16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * c + j;
        float e = 0.f;
        if (k < K) {
          e = x[k];
          if (P.norm != NORM_NONE) {
            e = (e - mean) * rstd * P.norm_w[k];
            if (P.norm == NORM_LAYER && P.norm_b) e += P.norm_b[k];
          }
        }
        v[j] = (f16)e;
      }
      *(f16x8*)(o + 8 * c) = v;
    }
  } else {
    // a 16-B output chunk is 8 CONSECUTIVE natural positions base .. base + 7 in the order
    // 0 2 1 3 4 6 5 7: two 16-B LDS reads (+ two of the norm weights), permuted in registers
    __syncthreads();  // the staged row (and block_sum's broadcast) are visible
    const bool nrm = P.norm != NORM_NONE, lnb = P.norm == NORM_LAYER && P.norm_b;
    for (int c = threadIdx.x; c < Kp / 8; c += 256) {
      const int kp = 8 * c, pc = kp >> 5, p0 = kp & 31;
      const int t = pc / SB, sb = pc - t * SB;
      const int base = piece_off<QT>(t, sb, p0 >> 4) + 4 * ((p0 & 15) >> 2);
      f16x8 v;
      if (base + 8 <= K) {
        f32x4 a = *(const f32x4*)(xs + base), b = *(const f32x4*)(xs + base + 4);
        if (nrm) {
          const f32x4 wa = *(const f32x4*)(P.norm_w + base), wb = *(const f32x4*)(P.norm_w + base + 4);
          a = (a - mean) * rstd * wa;
          b = (b - mean) * rstd * wb;
          if (lnb) {
            a += *(const f32x4*)(P.norm_b + base);
            b += *(const f32x4*)(P.norm_b + base + 4);
          }
        }
        v = (f16x8){(f16)a.x, (f16)a.z, (f16)a.y, (f16)a.w, (f16)b.x, (f16)b.z, (f16)b.y, (f16)b.w};
      } else {  // the row's K padding (Q4_0 / Q8_0 with K % 256 != 0)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int r = j & 3, k = base + 4 * (j >> 2) + (r == 1 ? 2 : r == 2 ? 1 : r);
          float e = 0.f;
          if (k < K) {
            e = xs[k];
            if (nrm) {
              e = (e - mean) * rstd * P.norm_w[k];
              if (lnb) e += P.norm_b[k];
            }
          }
          v[j] = (f16)e;
        }
      }
      *(f16x8*)(o + kp) = v;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// one weight-row piece (32 codes) in registers: codes + the scale bytes it needs
template <int QT>
struct Piece {
  u32x4 a;                                   // 16 code bytes (Q8_0: first 16)
  u32x4 b;                                   // Q8_0: last 16 code bytes
  u32x4 m;                                   // Q4_K / Q5_K meta (d, dmin, scales12); Q6_K int8 scales
  u32x2 h;                                   // Q6_K high-bit pairs
  unsigned e;                                // Q5_K 5th bits; Q6_K / Q4_0 / Q8_0: fp16 d (low half)
  u32x4 f[QT == QT_F16 ? 2 : 1];             // F16: halves 16..31 of the piece
};

template <int QT>
__device__ __forceinline__ void load_piece(const QMat& w, long long row, int SB, int pc, Piece<QT>& R) {
  if constexpr (QT == QT_F16) {  // natural order: piece pc = halves 32 pc .. + 31 of the row
    const uint8_t* q = w.s0 + row * SB * 512 + 64LL * pc;
    R.a = *(const u32x4*)q;
    R.b = *(const u32x4*)(q + 16);
    R.f[0] = *(const u32x4*)(q + 32);
    R.f[1] = *(const u32x4*)(q + 48);
    return;
  }
  const int t = pc / SB, sb = pc - t * SB;
  if constexpr (QT == QT_Q8_0) {
    const uint8_t* q = w.s0 + row * SB * 256 + 32LL * pc;
    R.a = *(const u32x4*)q;
    R.b = *(const u32x4*)(q + 16);
    R.e = *(const uint16_t*)(w.s1 + row * SB * 16 + 16LL * sb + 2 * t);
  } else {
    R.a = *(const u32x4*)(w.s0 + row * SB * 128 + 16LL * pc);
    if constexpr (QT == QT_Q4_K || QT == QT_Q5_K) R.m = *(const u32x4*)(w.s1 + row * SB * 16 + 16LL * sb);
    if constexpr (QT == QT_Q5_K) R.e = *(const unsigned*)(w.s2 + row * SB * 32 + 4LL * pc);
    if constexpr (QT == QT_Q6_K) {
      R.h = *(const u32x2*)(w.s1 + row * SB * 64 + 8LL * pc);
      R.m = *(const u32x4*)(w.s2 + row * SB * 16 + 16LL * sb);
      R.e = *(const uint16_t*)(w.s3 + row * SB * 2 + 2LL * sb);
    }
    if constexpr (QT == QT_Q4_0) R.e = *(const uint16_t*)(w.s1 + row * SB * 16 + 16LL * sb + 2 * t);
  }
}

// Q4_K / Q5_K 6-bit scale and min of sub-block j
__device__ __forceinline__ void k_scale(const u32x4& m, int j, float& sc, float& mn) {
  const float d = h2f(m.x & 0xFFFF), dmin = h2f(m.x >> 16);
  const int sh = 8 * (j & 3);
  const unsigned a = (m.y >> sh) & 0xFF, b = (m.z >> sh) & 0xFF, e = (m.w >> sh) & 0xFF;
  const unsigned s = j < 4 ? (a & 63) : ((e & 0xF) | ((a >> 6) << 4));
  const unsigned mm = j < 4 ? (b & 63) : ((e >> 4) | ((b >> 6) << 4));
  sc = d * (float)s;
  mn = -dmin * (float)mm;
}

// dequantise a piece to 32 fp16 in stream order: o[0..7] = lo half pairs, o[8..15] = hi half pairs
template <int QT>
__device__ __forceinline__ void dq_piece(const Piece<QT>& R, int t, unsigned (&o)[16]) {
  if constexpr (QT == QT_F16) {
    const u32x4 v[4] = {R.a, R.b, R.f[0], R.f[1]};
#pragma unroll
    for (int i = 0; i < 16; ++i) o[i] = dsel(v[i >> 2], i & 3);
  } else if constexpr (QT == QT_Q4_K || QT == QT_Q5_K) {
    const int c = t >> 1;
    float s0, c0, s1, c1;
    k_scale(R.m, 2 * c, s0, c0);
    k_scale(R.m, 2 * c + 1, s1, c1);
    const dh2 off = dq_splat(1024.f), S0 = dq_splat(s0), S1 = dq_splat(s1), C0 = dq_splat(c0), C1 = dq_splat(c1);
    const u32x4 q = QT == QT_Q4_K ? (R.a ^ 0x80808080u) : R.a;  // Q4_K: undo the signed-high-nibble repack
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const unsigned w = dsel(q, e);
      unsigned l0 = (w & 0x000F000Fu) | DQ_MAGIC, l1 = ((w >> 8) & 0x000F000Fu) | DQ_MAGIC;
      unsigned g0 = ((w >> 4) & 0x000F000Fu) | DQ_MAGIC, g1 = ((w >> 12) & 0x000F000Fu) | DQ_MAGIC;
      if constexpr (QT == QT_Q5_K) {  // 5th bit of weight 4e + j: byte j of H, bit e (lo) / 4 + e (hi)
        const unsigned H = R.e;
        l0 |= (H << (4 - e)) & 0x00100010u;
        l1 |= (H >> (4 + e)) & 0x00100010u;
        g0 |= (H >> e) & 0x00100010u;
        g1 |= (H >> (8 + e)) & 0x00100010u;
      }
      o[2 * e] = dq2(l0, off, S0, C0);
      o[2 * e + 1] = dq2(l1, off, S0, C0);
      o[8 + 2 * e] = dq2(g0, off, S1, C1);
      o[8 + 2 * e + 1] = dq2(g1, off, S1, C1);
    }
  } else if constexpr (QT == QT_Q6_K) {
    const int n = t >> 2, sub = t & 3;
    const float d = h2f((uint16_t)R.e);
    // int8 scales 8 n + sub (lo codes) and 8 n + sub + 4 (hi codes): dwords 2 n / 2 n + 1, byte sub
    const unsigned mlo = n ? R.m.z : R.m.x, mhi = n ? R.m.w : R.m.y;
    const float slo = d * (float)(int8_t)((mlo >> (8 * sub)) & 0xFF);
    const float shi = d * (float)(int8_t)((mhi >> (8 * sub)) & 0xFF);
    const dh2 off = dq_splat(1056.f), S0 = dq_splat(slo), S1 = dq_splat(shi), z = dq_splat(0.f);  // 1024 + 32
    const unsigned H0 = R.h.x, H1 = R.h.y;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const unsigned q = dsel(R.a, e);
      // high 2 bits of weight 4e + j: byte j, bits 2e..2e+1 of H0 (lo) / H1 (hi) -> bits 4..5
      const int sl = 4 - 2 * e;
      const unsigned hl0 = (sl >= 0 ? (H0 << sl) : (H0 >> -sl)) & 0x00300030u;
      const unsigned hl1 = (H0 >> (4 + 2 * e)) & 0x00300030u;
      const unsigned hh0 = (sl >= 0 ? (H1 << sl) : (H1 >> -sl)) & 0x00300030u;
      const unsigned hh1 = (H1 >> (4 + 2 * e)) & 0x00300030u;
      o[2 * e] = dq2((q & 0x000F000Fu) | hl0 | DQ_MAGIC, off, S0, z);
      o[2 * e + 1] = dq2(((q >> 8) & 0x000F000Fu) | hl1 | DQ_MAGIC, off, S0, z);
      o[8 + 2 * e] = dq2(((q >> 4) & 0x000F000Fu) | hh0 | DQ_MAGIC, off, S1, z);
      o[8 + 2 * e + 1] = dq2(((q >> 12) & 0x000F000Fu) | hh1 | DQ_MAGIC, off, S1, z);
    }
  } else if constexpr (QT == QT_Q4_0) {
    const dh2 sd = dq_splat(h2f((uint16_t)R.e)), z = dq_splat(0.f), off = dq_splat(1032.f);  // 1024 + 8
    const u32x4 q = R.a ^ 0x80808080u;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const unsigned w = dsel(q, e);
      o[2 * e] = dq2((w & 0x000F000Fu) | DQ_MAGIC, off, sd, z);
      o[2 * e + 1] = dq2(((w >> 8) & 0x000F000Fu) | DQ_MAGIC, off, sd, z);
      o[8 + 2 * e] = dq2(((w >> 4) & 0x000F000Fu) | DQ_MAGIC, off, sd, z);
      o[8 + 2 * e + 1] = dq2(((w >> 12) & 0x000F000Fu) | DQ_MAGIC, off, sd, z);
    }
  } else {  // Q8_0: bytes are offset-binary after ^ 0x80
    const dh2 sd = dq_splat(h2f((uint16_t)R.e)), z = dq_splat(0.f), off = dq_splat(1152.f);  // 1024 + 128
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const unsigned qa = dsel(R.a, e), qb = dsel(R.b, e);
      o[2 * e] = dq2(((qa & 0x00FF00FFu) | DQ_MAGIC) ^ 0x00800080u, off, sd, z);
      o[2 * e + 1] = dq2((((qa >> 8) & 0x00FF00FFu) | DQ_MAGIC) ^ 0x00800080u, off, sd, z);
      o[8 + 2 * e] = dq2(((qb & 0x00FF00FFu) | DQ_MAGIC) ^ 0x00800080u, off, sd, z);
      o[8 + 2 * e + 1] = dq2((((qb >> 8) & 0x00FF00FFu) | DQ_MAGIC) ^ 0x00800080u, off, sd, z);
    }
  }
}

// C fragment -> fused epilogue: weight row n = nb + 32 j, token row = mb + 32 i + (r & 3) + 8 (r >> 2);
// the row pair partner n ^ 1 sits on the adjacent lane
template <int E, int TM, int TN>
__device__ __forceinline__ void dq_out(const GemvParams& P, const f32x16 (&acc)[TM][TN], int mb, int nb, int M, int N) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = acc[i][j][r];
        const float pv = __shfl_xor(v, 1);
        const int gm = mb + 32 * i + (r & 3) + 8 * (r >> 2), gn = nb + 32 * j;
        if (gm < M && gn < N) epi_apply_t<E>(P, gm, gn + P.row_offset, v, pv, 0);
      }
}

// ------------------------------------------------------------------------------------------------
template <int QT, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(DQ_NT, 1) void dq_gemm_kernel(GemvParams P, const f16* __restrict__ X, int Kp, int sk,
                                                            int dbg) {
  static_assert(WM * WN == 8, "8 waves");
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;  // 32 x 32 accumulator tiles per wave
  constexpr int XS = BM * DQ_BK, WS = BN * DQ_BK;      // halves per LDS buffer (128-B rows, swizzled)
  constexpr int XL = BM / 64;                          // 16-B X chunks per thread per K step
  static_assert(TM >= 1 && TN >= 1 && BN * 2 <= DQ_NT && XL >= 1, "tile shape");
  constexpr int NXB = 2;  // X buffers
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f16* Xs = (f16*)smem;     // [NXB][BM][64] swizzled
  f16* Ws = Xs + NXB * XS;  // [2][BN][64] swizzled

  const QMat& w = P.w;
  const int M = P.B, N = w.N, SB = Kp >> 8, nks = SB * 4;
  // pc / SB = umulhi(pc, ceil(2^32 / SB)) for pc < 8 SB (SB = 1 would overflow: taken apart)
  const unsigned sbinv = (0xFFFFFFFFu / (unsigned)SB) + 1u;
  // XCD-aware bijective remap: the blocks one XCD runs are a contiguous range of (tile, split) ids
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int z = wg % sk, tile = wg / sk;
  // M-major: the blocks of one XCD share an activation tile (BM x K fp16, 2-6 MB) and walk the weight
  // tiles, advancing through K roughly together -- each X line is fetched into that XCD's L2 once and
  // hit by every block there (N-major order streamed X from the Infinity Cache at full latency)
  const int nt = (N + BN - 1) / BN;
  const int m0 = (tile / nt) * BM, n0 = (tile % nt) * BN;
  const int ks0 = (int)((long long)z * nks / sk), ks1 = (int)((long long)(z + 1) * nks / sk);

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // staging roles: X chunk (row xr + 64 i, 16 B at column xc), W piece (row wr, piece 2 ks + wh)
  const int wr = tid >> 1, wh = tid & 1;
  const bool wact = BN * 2 >= DQ_NT || wr < BN;  // compile-time true when every thread stages a piece
  const long long wrow = min(n0 + wr, N - 1);
  // X rows by LDS DMA: wave w's i-th global_load_lds fills rows 64 i + 8 w .. + 7 (1 KiB, lane-linear);
  // lane l lands in physical chunk l & 7 of its row, so it fetches the logical chunk that swizzles there
  const f16* xsrc[XL];
#pragma unroll
  for (int i = 0; i < XL; ++i) {
    const int r = 64 * i + 8 * wave + (lane >> 3);
    xsrc[i] = X + (long long)min(m0 + r, M - 1) * Kp + 8 * ((lane & 7) ^ ((r >> 1) & 7));
  }
  typedef __attribute__((address_space(3))) void lds_void;
  typedef __attribute__((address_space(1))) void glb_void;

  Piece<QT> wreg;
  // dbg (microbenchmark only, OMX_DQ_DBG=1): after the first step no operand is re-loaded -- the
  // pipeline's compute, LDS and barrier time alone (garbage results)
  auto issue_w = [&](int ks) {
    if (dbg && ks > ks0 + 1) return;
    if (wact) load_piece<QT>(w, wrow, SB, 2 * ks + wh, wreg);
  };
  auto issue_x = [&](int ks, int buf) {
    if (dbg && ks > ks0 + 1) return;
#pragma unroll
    for (int i = 0; i < XL; ++i)
      __builtin_amdgcn_global_load_lds((glb_void*)(xsrc[i] + ks * DQ_BK), (lds_void*)(Xs + buf * XS + (64 * i + 8 * wave) * DQ_BK),
                                       16, 0, 0);
  };
  auto stage_w = [&](int ks, int buf) {
    if (wact) {
      const int pc = 2 * ks + wh;
      unsigned o[16];
      dq_piece<QT>(wreg, SB == 1 ? pc : (int)__umulhi((unsigned)pc, sbinv), o);  // t = pc / SB
      f16* wd = Ws + buf * WS;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *(u32x4*)(wd + swzw(wr, 4 * wh + i)) = (u32x4){o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]};
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 31, fq = lane >> 5;
  auto compute_b = [&](int xbuf, int wbuf) {
    const f16* xb = Xs + xbuf * XS;
    const f16* wb = Ws + wbuf * WS;
#pragma unroll
    for (int kk = 0; kk < DQ_BK / 16; ++kk) {
      f16x8 a[TM], b[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = *(const f16x8*)(wb + swzw(wn * (BN / WN) + 32 * j + fr, 2 * kk + fq));
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = *(const f16x8*)(xb + swz(wm * (BM / WM) + 32 * i + fr, 2 * kk + fq));
      __builtin_amdgcn_s_setprio(1);  // T5: the MFMA cluster first while the other wave dequantises
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };
  auto compute = [&](int buf) { compute_b(buf, buf); };

  // Two K steps per trip with literal buffer indices and no branches in between: the compiler sees the
  // staging writes (other buffer) and the fragment reads (this buffer) as disjoint, so it can interleave
  // the dequant VALU / LDS writes of step ks + 1 with the MFMAs of step ks. Order inside a step: the
  // dequant consumes the weight registers BEFORE the X DMA is issued (hipcc would otherwise wait for
  // the DMA at the first use of an ordinary load), the weight loads of step ks + 2 follow, and the wait
  // hipcc places before the next barrier retires both. Steps past the end are clamped to the last one
  // (a redundant load / a write into the buffer nobody reads again).
  const int kl = ks1 - 1;
  issue_w(ks0);
  stage_w(ks0, 0);
  issue_x(ks0, 0);
  issue_w(min(ks0 + 1, kl));
  int ks = ks0;
  for (; ks + 1 < ks1; ks += 2) {
    __syncthreads();  // buffer 0 holds step ks; buffer 1's readers (step ks - 1) are done
    stage_w(ks + 1, 1);
    issue_x(ks + 1, 1);
    issue_w(min(ks + 2, kl));
    compute(0);
    __syncthreads();  // buffer 1 holds step ks + 1; buffer 0's readers are done
    stage_w(min(ks + 2, kl), 0);
    issue_x(min(ks + 2, kl), 0);
    issue_w(min(ks + 3, kl));
    compute(1);
  }
  if (ks < ks1) {  // odd step count: the last step sits in buffer 0
    __syncthreads();
    compute(0);
  }

  // C fragment (32 x 32): weight row n = lane & 31 (+ 32 j), token row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  const int nb = n0 + wn * (BN / WN) + fr;
  const int mb = m0 + wm * (BM / WM) + 4 * fq;
  if (sk > 1) {
    float* slab = P.gws + (long long)z * M * N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int gm = mb + 32 * i + (r & 3) + 8 * (r >> 2), gn = nb + 32 * j;
          if (gm < M && gn < N) __builtin_nontemporal_store(acc[i][j][r], slab + (long long)gm * N + gn);
        }
    return;
  }
  switch (P.epi) {  // one epilogue kind per unrolled body (the generic switch x 128 outputs spills)
    case EPI_STORE: dq_out<EPI_STORE, TM, TN>(P, acc, mb, nb, M, N); break;
    case EPI_ADD: dq_out<EPI_ADD, TM, TN>(P, acc, mb, nb, M, N); break;
    case EPI_GELU: dq_out<EPI_GELU, TM, TN>(P, acc, mb, nb, M, N); break;
    case EPI_GLU: dq_out<EPI_GLU, TM, TN>(P, acc, mb, nb, M, N); break;
    case EPI_GEGLU: dq_out<EPI_GEGLU, TM, TN>(P, acc, mb, nb, M, N); break;
    case EPI_GELU_ERF: dq_out<EPI_GELU_ERF, TM, TN>(P, acc, mb, nb, M, N); break;
    case EPI_QGELU: dq_out<EPI_QGELU, TM, TN>(P, acc, mb, nb, M, N); break;
    default: dq_out<EPI_QKV, TM, TN>(P, acc, mb, nb, M, N); break;
  }
}

// ------------------------------------------------------------------------------------------------
// Register-ring edition (round 6): both operands are staged through registers, two K steps deep, and
// written into the LDS double buffer after the barrier (the guide's T14 form). The glds edition above
// issues the X DMA one step ahead, and every `__syncthreads()` drains the vector-memory queue while a
// glds is in flight: each K step then waits for loads issued only one compute phase earlier (~0.9 us
// of MFMA work at 2 waves per SIMD against a 1-3 us loaded HBM round trip), which is what held the
// 256 x 256 tile at ~2.2 us per K step (profiles/r4_gemm). With plain loads the barrier is a bare
// s_barrier, the compiler's counted vmcnt waits only for the slot being written, and every load has
// two compute phases to land. Same LDS image, fragments, MFMA shape and epilogues as the glds kernel.
template <int QT, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(DQ_NT, 1) void dq_gemm_ring_kernel(GemvParams P, const f16* __restrict__ X, int Kp, int sk) {
  static_assert(WM * WN == 8, "8 waves");
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int XS = BM * DQ_BK, WS = BN * DQ_BK;
  constexpr int XL = BM / 64;  // 16-B X chunks per thread per K step (BM rows x 8 chunks / 512 threads)
  static_assert(TM >= 1 && TN >= 1 && BN * 2 <= DQ_NT && XL >= 1, "tile shape");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f16* Xs = (f16*)smem;     // [2][BM][64] swizzled
  f16* Ws = Xs + 2 * XS;    // [2][BN][64] swizzled

  const QMat& w = P.w;
  const int M = P.B, N = w.N, SB = Kp >> 8, nks = SB * 4;
  const unsigned sbinv = (0xFFFFFFFFu / (unsigned)SB) + 1u;
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int z = wg % sk, tile = wg / sk;
  const int nt = (N + BN - 1) / BN;
  const int m0 = (tile / nt) * BM, n0 = (tile % nt) * BN;
  const int ks0 = (int)((long long)z * nks / sk), ks1 = (int)((long long)(z + 1) * nks / sk);

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = tid >> 1, wh = tid & 1;
  const bool wact = BN * 2 >= DQ_NT || wr < BN;
  const long long wrow = min(n0 + wr, N - 1);
  // X chunk i of this thread: row xr + 64 i, 16-B column chunk xc (8 threads cover a 128-B row)
  const int xr = tid >> 3, xc = tid & 7;
  const f16* xsrc[XL];
#pragma unroll
  for (int i = 0; i < XL; ++i) xsrc[i] = X + (long long)min(m0 + xr + 64 * i, M - 1) * Kp + 8 * xc;

  u32x4 xa[XL], xb[XL];
  Piece<QT> wa, wb;
  auto load_x = [&](int ks, u32x4 (&xv)[XL]) {
#pragma unroll
    for (int i = 0; i < XL; ++i) xv[i] = *(const u32x4*)(xsrc[i] + ks * DQ_BK);
  };
  auto load_w = [&](int ks, Piece<QT>& wp) {
    if (wact) load_piece<QT>(w, wrow, SB, 2 * ks + wh, wp);
  };
  auto write = [&](int ks, const u32x4 (&xv)[XL], const Piece<QT>& wp, int buf) {
    f16* xd = Xs + buf * XS;
#pragma unroll
    for (int i = 0; i < XL; ++i) *(u32x4*)(xd + swz(xr + 64 * i, xc)) = xv[i];
    if (wact) {
      const int pc = 2 * ks + wh;
      unsigned o[16];
      dq_piece<QT>(wp, SB == 1 ? pc : (int)__umulhi((unsigned)pc, sbinv), o);
      f16* wd = Ws + buf * WS;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *(u32x4*)(wd + swzw(wr, 4 * wh + i)) = (u32x4){o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]};
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 31, fq = lane >> 5;
  auto compute = [&](int buf) {
    const f16* xbp = Xs + buf * XS;
    const f16* wbp = Ws + buf * WS;
#pragma unroll
    for (int kk = 0; kk < DQ_BK / 16; ++kk) {
      f16x8 a[TM], b[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = *(const f16x8*)(wbp + swzw(wn * (BN / WN) + 32 * j + fr, 2 * kk + fq));
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = *(const f16x8*)(xbp + swz(wm * (BM / WM) + 32 * i + fr, 2 * kk + fq));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };

  // ring: before the even half of a trip, LDS buffer 0 holds step ks, registers b hold step ks + 1 and
  // registers a hold step ks + 2; each half writes the next step from the registers that have waited
  // longest, reloads them with the step two ahead, then computes (steps past the end are clamped: a
  // redundant load, a write into a buffer nobody reads)
  const int kl = ks1 - 1;
  load_x(ks0, xa);
  load_w(ks0, wa);
  load_x(min(ks0 + 1, kl), xb);
  load_w(min(ks0 + 1, kl), wb);
  write(ks0, xa, wa, 0);
  load_x(min(ks0 + 2, kl), xa);
  load_w(min(ks0 + 2, kl), wa);
  // two steps per trip and no branch inside it: a mid-trip exit split the trip into blocks, and at that
  // join hipcc waited vmcnt(0) for the step that had just been issued
  int ks = ks0;
  for (; ks + 1 < ks1; ks += 2) {
    __syncthreads();  // buffer 0 holds step ks; buffer 1's readers (step ks - 1) are done
    write(ks + 1, xb, wb, 1);
    load_x(min(ks + 3, kl), xb);
    load_w(min(ks + 3, kl), wb);
    compute(0);
    __syncthreads();  // buffer 1 holds step ks + 1; buffer 0's readers are done
    write(min(ks + 2, kl), xa, wa, 0);
    load_x(min(ks + 4, kl), xa);
    load_w(min(ks + 4, kl), wa);
    compute(1);
  }
  if (ks < ks1) {  // odd step count: the last step sits in buffer 0
    __syncthreads();
    compute(0);
  }

  const int nb = n0 + wn * (BN / WN) + fr;
  const int mb = m0 + wm * (BM / WM) + 4 * fq;
  if (sk > 1) {
    float* slab = P.gws + (long long)z * M * N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int gm = mb + 32 * i + (r & 3) + 8 * (r >> 2), gn = nb + 32 * j;
          if (gm < M && gn < N) __builtin_nontemporal_store(acc[i][j][r], slab + (long long)gm * N + gn);
        }
    return;
  }
  switch (P.epi) {
    case EPI_STORE: dq_out<EPI_STORE, TM, TN>(P, acc, mb, nb, M, N); break;
    case EPI_ADD: dq_out<EPI_ADD, TM, TN>(P, acc, mb, nb, M, N); break;
    case EPI_GELU: dq_out<EPI_GELU, TM, TN>(P, acc, mb, nb, M, N); break;
    case EPI_GLU: dq_out<EPI_GLU, TM, TN>(P, acc, mb, nb, M, N); break;
    case EPI_GEGLU: dq_out<EPI_GEGLU, TM, TN>(P, acc, mb, nb, M, N); break;
    case EPI_GELU_ERF: dq_out<EPI_GELU_ERF, TM, TN>(P, acc, mb, nb, M, N); break;
    case EPI_QGELU: dq_out<EPI_QGELU, TM, TN>(P, acc, mb, nb, M, N); break;
    default: dq_out<EPI_QKV, TM, TN>(P, acc, mb, nb, M, N); break;
  }
}

template <int BM, int BN>
constexpr size_t dq_lds() { return (size_t)(2 * BM + 2 * BN) * DQ_BK * sizeof(f16); }

}  // namespace

extern int g_dq_cfg;  // gemm_dq.hip: forced tile config (microbenchmarks), -1 auto
extern int g_dq_dbg;  // gemm_dq.hip: OMX_DQ_DBG microbenchmark mode (no operand reloads), 0 in production
extern int g_dq_sk;   // gemm_dq.hip: forced split-K factor (microbenchmarks), 0 auto
extern int g_dq_ring;  // gemm_dq.hip: 1 = the register-ring kernel (OMX_DQ_RING), 0 = the glds kernel

namespace {

template <int QT, int BM, int BN, int WM, int WN>
void launch_dq(const GemvParams& P, const f16* xp, int Kp, int sk, hipStream_t s) {
  const int mt = (P.B + BM - 1) / BM, nt = (P.w.N + BN - 1) / BN;
  const size_t lds = dq_lds<BM, BN>();
  // the Q6_K piece (codes + high bits + scales + d) in a two-deep ring at 256 x 256 exceeds 256 VGPRs
  // (268 B/lane of scratch): that one tile stays on the glds kernel
  constexpr bool ring_ok = !(QT == QT_Q6_K && BM == 256 && BN == 256);
  if constexpr (ring_ok) {
    if (g_dq_ring && !g_dq_dbg) {
      hipLaunchKernelGGL((dq_gemm_ring_kernel<QT, BM, BN, WM, WN>), dim3(mt * nt * sk), dim3(DQ_NT), lds, s, P, xp, Kp,
                         sk);
      return;
    }
  }
  hipLaunchKernelGGL((dq_gemm_kernel<QT, BM, BN, WM, WN>), dim3(mt * nt * sk), dim3(DQ_NT), lds, s, P, xp, Kp, sk,
                     g_dq_dbg);
}

template <int QT>
void run_dq(const GemvParams& P, f16* xp, int Kp, hipStream_t s) {
  hipLaunchKernelGGL(prep_xp_kernel<QT>, dim3(P.B), dim3(256), QT == QT_F16 ? 0 : (size_t)P.w.K * sizeof(float), s, P, xp,
                     Kp);
  const int M = P.B, N = P.w.N, nks = Kp / DQ_BK;
  // tile x split-K from a wave model calibrated on MI355X (scripts/bench_dq_sweep.py, profiles/r4_gemm):
  // time = waves * (K steps per split) * c[cfg] + split-K slab traffic, waves = ceil(units / slots);
  // c = measured cost of one K step of a full wave of tiles (256x256 2.19 us, 256x128 1.32, 128x256 1.44,
  // 128x128 1.34 with two blocks per CU, i.e. 512 slots); slabs: sk * M * N fp32 written + read at ~5 TB/s
  const int bm[4] = {256, 256, 128, 128}, bn[4] = {256, 128, 256, 128};
  const double cst[4] = {2.19, 1.32, 1.44, 1.34};
  const int slots[4] = {256, 256, 256, 512};
  auto ntl = [&](int c) { return (long long)((M + bm[c] - 1) / bm[c]) * ((N + bn[c] - 1) / bn[c]); };
  int cfg = 3, sk = 1;
  double best = -1.0;
  for (int c = 0; c < 4; ++c) {
    if (g_dq_cfg >= 0 && g_dq_cfg <= 3 && c != g_dq_cfg) continue;  // microbenchmark override (OMX_DQ_CFG)
    for (int k = 1; k <= 4; ++k) {
      if (k > 1 && (!P.gws || (long long)k * M * N > P.gws_elems || nks / k < 8)) break;
      if (g_dq_sk > 0 && k != g_dq_sk) continue;  // microbenchmark override (set_dq_tuning)
      const long long units = ntl(c) * k;
      const double waves = (double)((units + slots[c] - 1) / slots[c]);
      const double t = waves * ((double)nks / k) * cst[c] + (k > 1 ? 2.0 * k * M * N * 4 / 5e6 : 0.0);
      if (best < 0.0 || t < best) best = t, cfg = c, sk = k;
    }
  }
  switch (cfg) {
    case 0: launch_dq<QT, 256, 256, 2, 4>(P, xp, Kp, sk, s); break;
    case 1: launch_dq<QT, 256, 128, 4, 2>(P, xp, Kp, sk, s); break;
    case 2: launch_dq<QT, 128, 256, 2, 4>(P, xp, Kp, sk, s); break;
    default: launch_dq<QT, 128, 128, 2, 4>(P, xp, Kp, sk, s); break;
  }
  if (sk > 1) gemm_finalize(P, sk, s);
}

}  // namespace

}  // namespace omx
