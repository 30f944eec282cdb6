// Batched decode GEMV on the matrix cores (continuous batching, 2 <= B <= 16 rows per step).
//
// y[b, n] = epilogue( sum_k W[n, k] * norm(x[b, :])[k] )    for b < B
//
// Why a second decode kernel: the int8-dot GEMV (gemv.hip / gemv_batch.hip) unpacks each weight once
// and then pays ~12 VALU per (weight piece, batch row) for the dot products and the per-group scale
// math, so its VALU work grows with B (rocprofv3, profiles/r3_batch: gate_up 13 us at B = 1, 25 us
// at B = 4, 96 us at B = 8). Here the per-row work is done by one `v_mfma_f32_16x16x32_f16` per
// 32 weights x 16 rows x 16 batch rows, and the VALU work -- dequantising 8 weights per lane to fp16
// -- is paid once per weight whatever B is (<= 16).
//
// MI355X-first design:
//  * Reads the RESIDENT layout v2 (no second weight copy; round 3 kept a lane-linear "layout M" copy of
//    every dense matrix, +100 % weight memory). One unit record = 16 rows x one super-block: lane
//    (row j = l % 16, q = l / 16) loads 8 code bytes of each of the super-block's 8 pieces (its half of
//    the piece's 16 lo or 16 hi codes: q < 2 lo, q >= 2 hi) with non-temporal 8-B loads, plus the row's
//    scale block. The MFMA's 32-K group of piece t is {16 lo codes, 16 hi codes} -- two natural runs of
//    16 K -- so every lane's 8 K are contiguous in the natural activation row: the A fragment stays one
//    16-B load / `ds_read_b128` at a per-lane offset (mb_qoff) + a per-piece constant (mb_aoff).
//  * Dequant in natural K order: `v_perm_b32` drops bytes (k, k + 1) under the fp16 exponent bytes
//    0x64, one AND keeps the nibbles (after a per-lane shift selecting lo / hi) -> (1024 + n) pairs,
//    then `v_pk_add_f16` (remove 1024 + zero point) + `v_pk_fma_f16` (scale, min). Q4_K / Q4_0 undo the
//    signed-high-nibble repack with one XOR; Q6_K's 2 high bits come from the lane's high-bit word via
//    another v_perm + shift; Q8_0 bytes go straight through v_perm.
//  * Block = 8 waves (2 per SIMD); each wave owns a fixed 1/8 of K for every row tile the block
//    processes, so its per-wave weight registers stay small (1-8 super-blocks) and the block's
//    8 partial tiles meet in LDS (double-buffered, one barrier per tile) before the fused epilogue
//    (residual add, SiLU/GELU-GLU, RoPE + paged KV scatter: epilogue.h, shared with the GEMV/GEMM).
//    Persistent over row tiles with a register ping-pong (next tile's loads in flight while the
//    current one computes) when the wave's K share is small.
//  * Activation prologue once per block: x (fp32) -> RMSNorm (fused) -> fp16 rows in LDS (only the
//    B live rows; A-operand lanes of rows >= B read nothing and feed zeros).
// Reference parity: the batched decode of llama.cpp's runner inside `ollama/ollama` (reference
// pkg/model/pod.go:10-12, OLLAMA_NUM_PARALLEL); numerics checked against an fp32 torch GEMV on the
// dequantised weights (tests/test_gemv_mfma_gpu.py).
#include <type_traits>

#include "common.h"
#include "epilogue.h"
#include "ops.h"

namespace omx {

typedef _Float16 mh2 __attribute__((ext_vector_type(2)));

constexpr int MB_NW = 8;         // waves per block
constexpr int MB_NT = 64 * MB_NW;
constexpr int MB_BMAX = 16;      // batch rows per MFMA (A-operand rows)
constexpr int MB_BMIN = 3;       // smallest batch taken (profiles/r3_batch)
constexpr unsigned MB_MAGIC = 0x64006400u;  // fp16 1024.0 in both halves
constexpr int MB_SPL = 12;       // RMS partials per lane: producers of up to 64 * 12 row tiles (E <= 12288)

static inline int n_sb_host(int K) { return (K + 255) >> 8; }

// bytes of one unit record (16 rows x one super-block) in the resident layout v2, for the QKV launch split
constexpr int mb_rec_bytes(int qt) {
  return qt == QT_Q8_0 ? 16 * 272 : qt == QT_Q6_K ? 16 * 210 : qt == QT_Q4_K ? 16 * 144 : qt == QT_Q4_0 ? 16 * 144 : 0;
}

__device__ __forceinline__ mh2 ash2(unsigned v) { return __builtin_bit_cast(mh2, v); }
__device__ __forceinline__ unsigned asu2(mh2 v) { return __builtin_bit_cast(unsigned, v); }

// MFMA K grouping of piece t (32 codes of one weight row): lanes q = 0, 1 take the piece's 16 lo codes
// (natural K offsets lo + 8 q), lanes q = 2, 3 its 16 hi codes (hi + 8 (q - 2)), so a lane's 8 K are
// contiguous in the natural activation row. lo / hi of piece t relative to its super-block:
//   Q4_K:  lo = 64 (t >> 1) + 16 (t & 1), hi = lo + 32       (sub-blocks 2c / 2c + 1)
//   Q6_K:  lo = 128 (t >> 2) + 16 (t & 3), hi = lo + 64       (int8-scale groups il / il + 4)
//   Q4_0 / Q8_0: lo = 32 t, hi = lo + 16                      (one 32-block)
// this lane's part of the offset: half g = q >> 1 (lo / hi) and 8 (q & 1)
template <int QT>
__device__ __forceinline__ int mb_qoff(int q) {
  return (QT == QT_Q4_K ? 32 : QT == QT_Q6_K ? 64 : 16) * (q >> 1) + 8 * (q & 1);
}

// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// ring unit: NR layout M records (this lane's codes + scales) and, when the activations are read
// from global memory per record (CA), the record's 8 A-operand fragments
// ring unit: CH super-blocks of this wave's piece t for the 16 rows of one tile
template <int QT, int CH, bool CA>
struct MUnit {
  u32x2 c[CH];                                   // 8 code bytes (the lane's half of the lo / hi codes)
  unsigned h[QT == QT_Q6_K ? CH : 1];            // Q6_K: high-bit word of the lane's half
  u32x4 m[QT == QT_Q4_K ? CH : 1];               // Q4_K: meta (d, dmin, scales12)
  unsigned sd[QT == QT_Q4_K ? 1 : CH];           // Q6_K: int8-scale dword | Q4_0 / Q8_0: fp16 d of block t
  unsigned d6[QT == QT_Q6_K ? CH : 1];           // Q6_K: fp16 d
  f16x8 a[CA ? CH : 1];
  float eo[4];  // this lane's epilogue operands for the unit's tile (mb_epi_load)
};

// Epilogue operands of this lane's output of `tile` (row j = lane % 16, batch row 4 q + (wave & 3): the
// accumulator layout of the MFMA, one register per epilogue wave), loaded with the tile's weights: a
// global load issued inside the stream would be queued behind every weight load in flight (vmcnt
// retires in order) and drain the ring. Unconditional loads from clamped addresses; an operand an
// epilogue does not use reads a harmless valid address (the matrix codes).
//   eo[0]: EPI_ADD old y | eo[1]: bias[vn] | eo[2]: EPI_QKV bias[vn ^ 1] |
//   eo[3]: emit_nw[vn] (residual emission) or inv_freq[d / 2] (EPI_QKV)
constexpr int MB_EO = 4;
__device__ __forceinline__ void mb_epi_load(const GemvParams& P, int tile, float (&eo)[MB_EO]) {
  const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4, wave = threadIdx.x >> 6;
  const int row = min(tile * 16 + j, P.w.N - 1), vn = row + P.row_offset;
  const int b = min(4 * q + (wave & 3), P.B - 1);
  const float* dummy = (const float*)P.w.s0;
  int d = 0;
  if (P.epi == EPI_QKV) {
    const int Eq = P.Eq, Ekv = P.Ekv;
    d = (vn < Eq ? vn : vn < Eq + Ekv ? vn - Eq : vn - Eq - Ekv) % P.D;
    d = min(d >> 1, max(P.n_rot / 2 - 1, 0));
  }
  eo[0] = *(P.epi == EPI_ADD ? P.y + (long long)b * P.ldy + vn : dummy);
  eo[1] = *(P.bias ? P.bias + vn : dummy);
  eo[2] = *((P.epi == EPI_QKV && P.bias) ? P.bias + (vn ^ 1) : dummy);
  eo[3] = *(P.emit16 ? P.emit_nw + vn : P.epi == EPI_QKV ? P.inv_freq + d : dummy);
}

// the fused epilogue of one output element with preloaded operands (mirrors epilogue.h epi_apply for
// the epilogues a dense decode GEMV uses; no global load). yo = old y (EPI_ADD), bias / pbias = bias of
// the row / its pair partner, f = inv_freq of the row's rotary pair (EPI_QKV)
__device__ __forceinline__ void mb_epi(const GemvParams& P, int bb, int vn, float v, float pv, float yo, float bias,
                                       float pbias, float f, int pos, int slot) {
  switch (P.epi) {
    case EPI_STORE:
      if (P.bias) v += bias;
      P.y[(long long)bb * P.ldy + vn] = v;
      break;
    case EPI_ADD:
      if (P.bias) v += bias;
      P.y[(long long)bb * P.ldy + vn] = yo + v;
      break;
    case EPI_GELU:
      if (P.bias) v += bias;
      P.y[(long long)bb * P.ldy + vn] = gelu_tanh(v);
      break;
    case EPI_GLU:
    case EPI_GEGLU:
      if ((vn & 1) == 0) {
        const float g = P.epi == EPI_GLU ? silu(v) : gelu_tanh(v);
        if (P.y16) ((f16*)P.y16)[(long long)bb * P.ld16y + vn / 2] = (f16)(g * pv);
        else P.y[(long long)bb * P.ldy + vn / 2] = g * pv;
      }
      break;
    case EPI_QKV: {
      const int Eq = P.Eq, Ekv = P.Ekv, D = P.D;
      int which, hh, d;
      if (vn < Eq) { which = 0; hh = vn / D; d = vn % D; }
      else if (vn < Eq + Ekv) { which = 1; hh = (vn - Eq) / D; d = (vn - Eq) % D; }
      else { which = 2; hh = (vn - Eq - Ekv) / D; d = (vn - Eq - Ekv) % D; }
      if (P.bias) v += bias;
      float out = v;
      if (which < 2 && d < P.n_rot) {
        if (P.bias) pv += pbias;
        const float ang = (float)pos * f;
        float sn, cs;
        sincosf(ang, &sn, &cs);
        out = (d & 1) ? (pv * sn + v * cs) : (v * cs - pv * sn);
      }
      if (which == 0) {
        P.y[(long long)bb * P.ldy + vn] = out;
      } else {
        const long long blk = slot / P.bs, off = slot % P.bs;
        const long long idx = ((blk * P.n_kv + hh) * P.bs + off) * (P.Dc > 0 ? P.Dc : D) + d;
        if (which == 1) ((f16*)P.kc)[idx] = (f16)out;
        else ((f16*)P.vc)[idx] = (f16)out;
      }
      break;
    }
    default:
      break;
  }
}

// one unit straight from the resident v2 streams: lane (row j, q) loads, for each of the unit's super-
// blocks, 8 code bytes of piece t (its half of the piece's lo or hi codes) and the scale words piece t
// needs. Pieces t of consecutive super-blocks are consecutive 16-B runs of a row (piece-major streams),
// so a wave walks its rows' lines front to back: every 128-B line is fetched once and consumed by the
// next 7 loads of the same wave from L1.
template <int QT, int CH, bool CA>
__device__ __forceinline__ void mb_load_unit(const QMat& w, int tile, int SB, int sbf, int t, int lane,
                                             MUnit<QT, CH, CA>& U) {
  const int j = lane & 15, q = lane >> 4, g = q >> 1;
  OMX_KASSERT(tile >= 0 && tile < (w.N + 15) / 16 && sbf >= 0 && sbf < SB);
  const long long row = min(tile * 16 + j, w.N - 1);  // rows past N: a valid row, outputs discarded
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int sb = min(sbf + i, SB - 1);
    const long long pc = (long long)t * SB + sb;
    if constexpr (QT == QT_Q8_0)
      U.c[i] = __builtin_nontemporal_load((const u32x2*)(w.s0 + row * SB * 256 + 32 * pc + 8 * q));
    else
      U.c[i] = __builtin_nontemporal_load((const u32x2*)(w.s0 + row * SB * 128 + 16 * pc + 8 * (q & 1)));
    if constexpr (QT == QT_Q4_K) {
      U.m[i] = *(const u32x4*)(w.s1 + row * SB * 16 + 16LL * sb);
    } else if constexpr (QT == QT_Q6_K) {
      U.h[i] = __builtin_nontemporal_load((const unsigned*)(w.s1 + row * SB * 64 + 8 * pc + 4 * g));
      // int8 scale il = 8 (t >> 2) + (t & 3) + 4 g: dword 2 (t >> 2) + g of the row's 16 scales
      U.sd[i] = *(const unsigned*)(w.s2 + row * SB * 16 + 16LL * sb + 4 * (2 * (t >> 2) + g));
      U.d6[i] = *(const uint16_t*)(w.s3 + row * SB * 2 + 2LL * sb);
    } else {
      U.sd[i] = *(const uint16_t*)(w.s1 + row * SB * 16 + 16LL * sb + 2 * t);
    }
  }
}

// offset of piece t's A fragment within a super-block (the lane's mb_qoff comes on top)
template <int QT>
__device__ __forceinline__ int mb_aoff_rt(int t) {
  return QT == QT_Q4_K ? 64 * (t >> 1) + 16 * (t & 1) : QT == QT_Q6_K ? 128 * (t >> 2) + 16 * (t & 3) : 32 * t;
}

// the unit's A-operand fragments from a global fp16 activation row (xg already offset by the lane's
// mb_qoff and the wave's piece; lanes of batch rows >= B read the all-zero row GemvParams::zrow16)
template <int QT, int CH, bool CA>
__device__ __forceinline__ void mb_load_a(const f16* xg, int SB, int sbf, MUnit<QT, CH, CA>& U) {
#pragma unroll
  for (int i = 0; i < CH; ++i) U.a[i] = *(const f16x8*)(xg + min(sbf + i, SB - 1) * 256);
}

// (a & m) | o in one VALU op (hipcc emits v_and + v_or for the C expression)
__device__ __forceinline__ unsigned and_or(unsigned a, unsigned m, unsigned o) {
  unsigned r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(m), "v"(o));
  return r;
}

// bytes (b, b + 1) of w -> fp16 pair (1024 + low nibble) in natural order: v_perm places them under
// the 0x64 exponent bytes, one AND keeps the nibbles (selector 0x04010400: bytes 0, 1; 0x04030402: 2, 3)
template <unsigned SEL>
__device__ __forceinline__ unsigned nib_pair(unsigned w) {
  return __builtin_amdgcn_perm(0x64646464u, w, SEL) & 0x640F640Fu;
}
// Q6_K high bits of codes (k, k + 1) from the lane's shifted high-bit word -> bits 4-5 of each half
template <unsigned SEL, int SH>
__device__ __forceinline__ unsigned q6_hi(unsigned hb) {
  return (__builtin_amdgcn_perm(0u, hb, SEL) << SH) & 0x00300030u;
}

// fp16 B-operand fragment of piece T: this lane's 8 codes (natural K order), dequantised
template <int QT, int T>
__device__ __forceinline__ f16x8 mb_deq(const u32x2 c, unsigned hw, int g, int u, mh2 sc, mh2 mn) {
  u32x4 r;
  if constexpr (QT == QT_Q8_0) {
    const unsigned f0 = c.x ^ 0x80808080u, f1 = c.y ^ 0x80808080u;  // offset-binary bytes
    const mh2 off = {(f16)1152.f, (f16)1152.f};
    r.x = asu2((ash2(__builtin_amdgcn_perm(0x64646464u, f0, 0x04010400u)) - off) * sc);
    r.y = asu2((ash2(__builtin_amdgcn_perm(0x64646464u, f0, 0x04030402u)) - off) * sc);
    r.z = asu2((ash2(__builtin_amdgcn_perm(0x64646464u, f1, 0x04010400u)) - off) * sc);
    r.w = asu2((ash2(__builtin_amdgcn_perm(0x64646464u, f1, 0x04030402u)) - off) * sc);
  } else {
    // Q4_K / Q4_0 store the hi nibble ^ 8 (quant.py signed-high-nibble repack): one XOR undoes it
    // for both halves (it leaves the lo nibble alone); then the lane's half moves to the low nibble
    const unsigned xm = QT == QT_Q6_K ? 0u : 0x80808080u;
    const unsigned w0 = (c.x ^ xm) >> (4 * g), w1 = (c.y ^ xm) >> (4 * g);
    unsigned u0 = nib_pair<0x04010400u>(w0), u1 = nib_pair<0x04030402u>(w0);
    unsigned u2 = nib_pair<0x04010400u>(w1), u3 = nib_pair<0x04030402u>(w1);
    if constexpr (QT == QT_Q6_K) {  // high 2 bits of code k at bits 8 (k & 3) + 2 (k >> 2) of hw >> 4u
      const unsigned hb = hw >> (4 * u);
      u0 |= q6_hi<0x0C010C00u, 4>(hb);
      u1 |= q6_hi<0x0C030C02u, 4>(hb);
      u2 |= q6_hi<0x0C010C00u, 2>(hb);
      u3 |= q6_hi<0x0C030C02u, 2>(hb);
      const mh2 off = {(f16)1056.f, (f16)1056.f};  // 1024 + 32 (Q6_K codes are q - 32)
      r.x = asu2((ash2(u0) - off) * sc);
      r.y = asu2((ash2(u1) - off) * sc);
      r.z = asu2((ash2(u2) - off) * sc);
      r.w = asu2((ash2(u3) - off) * sc);
    } else {
      const mh2 off = QT == QT_Q4_0 ? (mh2){(f16)1032.f, (f16)1032.f} : (mh2){(f16)1024.f, (f16)1024.f};
      r.x = asu2((ash2(u0) - off) * sc + mn);
      r.y = asu2((ash2(u1) - off) * sc + mn);
      r.z = asu2((ash2(u2) - off) * sc + mn);
      r.w = asu2((ash2(u3) - off) * sc + mn);
    }
  }
  return __builtin_bit_cast(f16x8, r);
}

// the unit's CH MFMAs (super-blocks past SB are skipped: a partial last unit). t = this wave's piece
// (wave-uniform), g / u = the lane's half and 8-code slice; xl = the LDS A row for AM_LDS
template <int QT, int CH, bool CA>
__device__ __forceinline__ void mb_unit(const MUnit<QT, CH, CA>& U, int SB, int sbf, int t, int g, int u,
                                        const f16* xl, bool av, f32x4& acc) {
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    if (sbf + i >= SB) break;  // wave-uniform
    float scf, mnf = 0.f;
    if constexpr (QT == QT_Q4_K) {
      // sub-block jb = 2 (t >> 1) + g: 6-bit scale / min (scales12 packing: j < 4 direct, else split)
      const u32x4 m = U.m[i];
      const float d = h2f(m.x & 0xFFFF), dm = h2f(m.x >> 16);
      const int jb = 2 * (t >> 1) + g, sh = 8 * (jb & 3);
      const unsigned a = (m.y >> sh) & 0xFF, b = (m.z >> sh) & 0xFF, e = (m.w >> sh) & 0xFF;
      const unsigned sc = jb < 4 ? (a & 63) : ((e & 0xF) | ((a >> 6) << 4));
      const unsigned mn = jb < 4 ? (b & 63) : ((e >> 4) | ((b >> 6) << 4));
      scf = d * (float)sc;
      mnf = -dm * (float)mn;
    } else if constexpr (QT == QT_Q6_K) {
      scf = h2f((uint16_t)U.d6[i]) * (float)(int8_t)((U.sd[i] >> (8 * (t & 3))) & 0xFF);
    } else {
      scf = h2f((uint16_t)U.sd[i]);
    }
    const f16 a = (f16)scf, b = (f16)mnf;
    const f16x8 bw = mb_deq<QT, 0>(U.c[i], QT == QT_Q6_K ? U.h[i] : 0u, g, u, (mh2){a, a}, (mh2){b, b});
    f16x8 av8;
    if constexpr (CA) {
      av8 = U.a[i];
    } else {
      av8 = (f16x8){};
      if (av) av8 = *(const f16x8*)(xl + (sbf + i) * 256);
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av8, bw, acc, 0, 0, 0);
  }
}

// sum over the 16 lanes of a DPP row; every lane of the row gets the total
__device__ __forceinline__ float mb_row16_sum(float v) {
  auto dpp = [](float x, auto ctrl) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), decltype(ctrl)::value, 0xF, 0xF, false));
  };
  v += dpp(v, std::integral_constant<int, 0xB1>{});   // quad_perm [1,0,3,2]
  v += dpp(v, std::integral_constant<int, 0x4E>{});   // quad_perm [2,3,0,1]
  v += dpp(v, std::integral_constant<int, 0x141>{});  // row_half_mirror
  v += dpp(v, std::integral_constant<int, 0x140>{});  // row_mirror
  return v;
}

enum { AM_LDS = 0, AM_G16 = 1 };

constexpr int MB_NSLOT = 2;  // partial-tile slots (double-buffered: one block barrier per tile)

// LDS: [x rows fp16 [B][XSTR] (AM_LDS)] | partial tiles f32x4 [MB_NSLOT][MB_NW][64] |
//      (pad) | norm partials [MB_NW][16] + rstd [16]
static size_t mb_lds_bytes(int B, int K, int am) {
  const size_t xs = am == AM_LDS ? ((size_t)B * ((size_t)n_sb_host(K) * 256 + 8) * 2 + 15) & ~(size_t)15 : 0;
  return xs + (size_t)MB_NSLOT * MB_NW * 64 * 16 + 2 * MB_NSLOT * 4 + (MB_NW * 16 + 16) * 4;
}

// Grid: persistent blocks over 16-row tiles (tile = blockIdx.x + k * gridDim.x). Wave w owns piece
// t = w of every super-block (1/8 of K, contiguous 16-B runs per row in the piece-major v2 streams),
// streamed as units of CH super-blocks through a register ring of RD units (with their activation
// fragments in AM_G16). Each wave drops its partial tile into an LDS slot, refills its ring first (the
// next units stream across the barrier), meets the block, and waves 0..3 sum the 8 partials in wave
// order (deterministic) and run the fused epilogue, one output per lane each.
template <int QT, int CH, int RD, int AM, int DBG = 0>
__device__ __forceinline__ void mb_body(const GemvParams& P, const int bx, const int gxn) {
  constexpr bool G16 = AM == AM_G16;
  constexpr bool CA = G16;  // activation fragments ride with each unit
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const QMat& w = P.w;
  const int K = w.K, N = w.N, SB = n_sb(K), B = P.B;
  const int XSTR = SB * 256 + 8;
  f16* xs = (f16*)smem;
  float* red = (float*)(smem + (G16 ? 0 : (((size_t)B * XSTR * 2 + 15) & ~(size_t)15)));
  float* stat = red + MB_NSLOT * MB_NW * 64 * 4 + 2 * MB_NSLOT;
  float* srstd = stat + MB_NW * 16;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, j = lane & 15, q = lane >> 4;
  const int t = __builtin_amdgcn_readfirstlane(wave);  // this wave's piece
  const int g = q >> 1, u = q & 1;
  const int n_tiles = (N + 15) >> 4;
  const int my_tiles = bx < n_tiles ? (n_tiles - 1 - bx) / gxn + 1 : 0;
  const int upt = (SB + CH - 1) / CH;  // units per tile
  const int n_units = my_tiles * upt;
  const bool av = j < B;         // A-operand lane: batch row j
  const bool rs = G16 && P.xstat != nullptr && !(DBG & 2);

  // per-row epilogue operands (EPI_QKV) of this lane's batch row 4 q + (wave & 3), first
  int e_pos = 0, e_slot = 0;
  if (P.epi == EPI_QKV) {  // block-uniform
    const int b = min(4 * q + (wave & 3), B - 1);
    e_pos = P.pos[b];
    e_slot = P.slot[b];
  }
  // 0. (AM_G16) RMS partials [16][xstat_n] of this wave's batch rows w, w + 8 (coalesced rows)
  float sp[2][MB_SPL];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < MB_SPL; ++k) sp[h][k] = 0.f;
  if (rs) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int b = wave + 8 * h;
      if (b < B) {  // wave-uniform
#pragma unroll
        for (int k = 0; k < MB_SPL; ++k) {
          const int p = lane + 64 * k;
          const float v = P.xstat[(long long)b * P.xstat_n + min(p, P.xstat_n - 1)];
          sp[h][k] = p < P.xstat_n ? v : 0.f;
        }
      }
    }
  }
  const int aoff = mb_qoff<QT>(q) + mb_aoff_rt<QT>(t);
  const f16* xg = G16 ? (const f16*)P.x16 + (long long)(av ? j : P.zrow16) * P.ld16 + aoff : nullptr;
  // 2. (AM_LDS) activations -> (RMSNorm) -> fp16 rows in LDS, before any weight request
  if constexpr (!G16) {
    if (P.norm == NORM_RMS) {
      for (int b = 0; b < B; ++b) {  // block-uniform
        const float* xr = P.x + (long long)b * P.ldx;
        float s = 0.f;
        for (int i = tid; i < K / 4; i += MB_NT) {
          const f32x4 v = *(const f32x4*)(xr + 4 * i);
          s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        }
        s = wave_sum(s);
        if (lane == 0) stat[wave * 16 + b] = s;
      }
      __syncthreads();
      if (tid < B) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < MB_NW; ++i) t += stat[i * 16 + tid];
        srstd[tid] = rsqrtf(t / K + P.eps);
      }
      __syncthreads();
    }
    const int C8 = SB * 32;  // 8-element chunks per LDS row (K padded to whole super-blocks)
    for (int idx = tid; idx < B * C8; idx += MB_NT) {
      const int b = idx / C8, k = 8 * (idx - b * C8);
      f16x8 h = {};
      if (k < K) {
        const float* xr = P.x + (long long)b * P.ldx + k;
        f32x4 v0 = *(const f32x4*)xr, v1 = *(const f32x4*)(xr + 4);
        if (P.norm == NORM_RMS) {
          const float r = srstd[b];
          v0 = v0 * r * *(const f32x4*)(P.norm_w + k);
          v1 = v1 * r * *(const f32x4*)(P.norm_w + k + 4);
        }
        h = (f16x8){(f16)v0.x, (f16)v0.y, (f16)v0.z, (f16)v0.w, (f16)v1.x, (f16)v1.y, (f16)v1.z, (f16)v1.w};
      }
      *(f16x8*)(xs + (long long)b * XSTR + k) = h;
    }
  }

  // 3. the first RD units in flight (epilogue operands first: they are needed only after the weights)
  auto unit_tile = [&](int uu) { return bx + (uu / upt) * gxn; };
  auto load_unit = [&](MUnit<QT, CH, CA>& U, int uu) {
    // surplus slots (past the wave's last unit) re-read one line of the last unit: every lane the same
    // address, so a surplus load instruction costs one cache line (never computed)
    const int ln = uu < n_units ? lane : 0;
    uu = min(uu, n_units - 1);
    const int tl = unit_tile(uu), sbf = (uu % upt) * CH;
    mb_epi_load(P, tl, U.eo);
    mb_load_unit<QT, CH, CA>(w, tl, SB, sbf, t, ln, U);
    if constexpr (CA) mb_load_a<QT, CH, CA>(xg, SB, sbf, U);
    __builtin_amdgcn_sched_barrier(0);  // issue order = consumption order (vmcnt retires in order)
  };
  MUnit<QT, CH, CA> U[RD];
  if (n_units > 0) {
#pragma unroll
    for (int r = 0; r < RD; ++r) load_unit(U[r], r);
  }
  // 4. per-row RMS scale from the producer's partials
  if (rs) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < MB_SPL; ++k) s += sp[h][k];
      s = wave_sum(s);
      if (lane == 0 && wave + 8 * h < B) srstd[wave + 8 * h] = rsqrtf(s / K + P.eps);
    }
  }
  // staged rows and srstd visible to every wave
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // one tile done by every wave: partials meet in LDS, waves 0..3 run the epilogue
  int it = 0;
  auto finish = [&](const f32x4& acc, int tile, const float (&eo)[MB_EO]) {
    float* rb = red + (it++ & 1) * MB_NW * 64 * 4;
    *(f32x4*)(rb + (wave * 64 + lane) * 4) = acc;
    // LDS-only exchange: wait for this wave's LDS writes and meet; no memory fence (a workgroup
    // release would wait for the epilogue stores, i.e. drain every weight load in flight)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (wave >= 4 || (DBG & 4)) return;  // wave-uniform
    const int r = wave, b = 4 * q + r;  // this lane's output: row j, batch row 4 q + r
    OMX_KASSERT(tile >= 0 && tile < n_tiles && B <= MB_BMAX);
    float x = 0.f;
#pragma unroll
    for (int i = 0; i < MB_NW; ++i) x += rb[(i * 64 + lane) * 4 + r];
    if (rs) x *= srstd[b < B ? b : 0];
    const float px = __shfl_xor(x, 1, OMX_WAVE);  // pair partner: row j ^ 1, same batch row
    const int row = tile * 16 + j, vn = row + P.row_offset;
    const bool ok = b < B && row < N;
    if (P.emit16) {  // residual add that also feeds the next RMSNorm'd GEMV (AM_G16 + xstat)
      float sq = 0.f;
      if (ok) {
        if (P.bias) x += eo[1];
        const float nv = eo[0] + x;
        P.y[(long long)b * P.ldy + vn] = nv;
        ((f16*)P.emit16)[(long long)b * P.ld_emit + vn] = (f16)(nv * eo[3]);
        sq = nv * nv;
      }
      sq = mb_row16_sum(sq);  // the 16 lanes of a DPP row hold the tile's 16 rows of batch row b
      if (j == 0 && b < B) P.emit_stat[(long long)b * ((N + 15) >> 4) + tile] = sq;
    } else if (ok) {
      mb_epi(P, b, vn, x, px, eo[0], eo[1], eo[2], eo[3], e_pos, e_slot);
    }
  };

  // 5. stream the units
  const f16* xl = xs + (long long)(av ? j : 0) * XSTR + aoff;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  // one unit: its MFMAs, the slot's refill RD units ahead, then the tile's epilogue hand-off when the
  // unit completes the wave's share (operands copied out of the unit before its refill)
  auto step = [&](MUnit<QT, CH, CA>& Ur, int uu) {
    const int sbf = (uu % upt) * CH;
    if constexpr ((DBG & 1) != 0) {  // memory path only: consume every loaded word
      unsigned v = 0;
#pragma unroll
      for (int i = 0; i < CH; ++i) v ^= Ur.c[i].x ^ Ur.c[i].y;
      acc.x += (float)(v & 1);
    } else {
      mb_unit<QT, CH, CA>(Ur, SB, sbf, t, g, u, xl, av, acc);
    }
    const bool last = uu % upt == upt - 1;
    float eo[MB_EO];
#pragma unroll
    for (int e = 0; e < MB_EO; ++e) eo[e] = Ur.eo[e];
    const int tile = unit_tile(uu);
    load_unit(Ur, uu + RD);
    if (last) {
      finish(acc, tile, eo);
      acc = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  };
  // whole ring rounds without conditions (exact vmcnt counting), then the tail
  const int n_full = n_units / RD * RD;
  int uu = 0;
  for (; uu < n_full; uu += RD) {
#pragma unroll
    for (int r = 0; r < RD; ++r) step(U[r], uu + r);
  }
#pragma unroll
  for (int r = 0; r < RD; ++r)
    if (uu + r < n_units) step(U[r], uu + r);  // wave-uniform
}

template <int QT, int CH, int RD, int AM, int DBG = 0>
__global__ __launch_bounds__(MB_NT) void gemv_mb_kernel(GemvParams P) {
  mb_body<QT, CH, RD, AM, DBG>(P, blockIdx.x, gridDim.x);
}

// two matrices over the same activations in ONE launch (the Q4_K_M QKV: q,k rows Q4_K + v rows
// Q6_K): blocks [0, ga) run A, the rest B -- one launch ramp / drain instead of two
template <int QA, int QB, int CH, int RD, int AM>
__global__ __launch_bounds__(MB_NT) void gemv_mb2_kernel(GemvParams PA, GemvParams PB, int ga) {
  if ((int)blockIdx.x < ga) mb_body<QA, CH, RD, AM>(PA, blockIdx.x, ga);
  else mb_body<QB, CH, RD, AM>(PB, (int)blockIdx.x - ga, (int)gridDim.x - ga);
}

static int mb_cu_count() {
  static int n = 0;
  if (n <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

int g_mb_enable = 1, g_mb_dbg = 0, g_mb_bpc = 1;
static long long g_mb_launches = 0;
long long mb_launches() { return g_mb_launches; }
void set_mb_enable(int on) { g_mb_enable = on ? 1 : 0; }
void set_mb_tuning(int dbg, int bpc) {
  if (dbg >= 0 && dbg < 8) g_mb_dbg = dbg;
  if (bpc == 1 || bpc == 2) g_mb_bpc = bpc;
}
bool mb_enabled() { return g_mb_enable != 0; }

template <int QT, int CH, int RD, int AM, int DBG = 0>
static void mb_launch_k(const GemvParams& P, size_t lds, hipStream_t s) {
  auto kern = gemv_mb_kernel<QT, CH, RD, AM, DBG>;
  static bool attr = false;  // > 64 KB dynamic LDS: one attribute call per instantiation, before capture
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int tiles = (P.w.N + 15) / 16;
  // persistent: one (or two) 8-wave block(s) per CU
  const int slots = mb_cu_count() * g_mb_bpc;
  const int gx = tiles < slots ? tiles : slots;
  hipLaunchKernelGGL(kern, dim3(gx), dim3(MB_NT), lds, s, P);
  ++g_mb_launches;
}

template <int QT, int CH, int RD, int AM>
static void mb_launch(const GemvParams& P, size_t lds, hipStream_t s) {
  if constexpr (AM == AM_G16 && (QT == QT_Q4_K || QT == QT_Q6_K)) {
    switch (g_mb_dbg) {  // microbenchmark-only variants
      case 1: mb_launch_k<QT, CH, RD, AM, 1>(P, lds, s); return;
      case 2: mb_launch_k<QT, CH, RD, AM, 2>(P, lds, s); return;
      default: break;
    }
  }
  mb_launch_k<QT, CH, RD, AM>(P, lds, s);
}

template <int QT, int AM>
static bool mb_q(const GemvParams& P, size_t lds, hipStream_t s) {
  // units of 4 super-blocks of the wave's piece, 3 units in flight per wave: 12 x 16 rows x 16 B of
  // codes (+ scales) per wave, ~50 KB per CU
  mb_launch<QT, 4, 3, AM>(P, lds, s);
  return true;
}

static int mb_am(const GemvParams& P) { return P.x16 ? AM_G16 : AM_LDS; }

bool gemv_mb_supported(const GemvParams& P) {
  // B = 2 stays on the int8 GEMV (gemv_batch.hip): measured 2.08 vs 2.15 ms per Llama-2-7B step
  if (!g_mb_enable || P.B < MB_BMIN || P.B > MB_BMAX || P.expert_ids || P.merge_S) return false;
  if (g_tune.debug) return false;
  const int q = P.w.qtype;
  if (q != QT_Q4_K && q != QT_Q6_K && q != QT_Q4_0 && q != QT_Q8_0) return false;
  if (P.emit16 && (P.epi != EPI_ADD || !P.emit_nw || !P.emit_stat)) return false;
  if (P.y16 && P.epi != EPI_GLU && P.epi != EPI_GEGLU) return false;
  const int am = mb_am(P);
  if (am == AM_G16) {  // activations already normalised (times norm_w) and fp16 in global memory
    if (P.norm == NORM_LAYER || (P.norm == NORM_RMS && !P.xstat) || P.xstat_n > 64 * MB_SPL) return false;
  } else if (P.norm == NORM_LAYER) {
    return false;
  }
  return mb_lds_bytes(P.B, P.w.K, am) <= 160 * 1024;
}

// the QKV pair of a K-quant mix in one launch (gemv2 at B > 1): blocks split in proportion to bytes
bool gemv_mb2(const GemvParams& A, const GemvParams& Bp, hipStream_t s) {
  if (!gemv_mb_supported(A) || !gemv_mb_supported(Bp) || A.w.K != Bp.w.K || A.B != Bp.B) return false;
  if (mb_am(A) != AM_G16 || mb_am(Bp) != AM_G16 || g_mb_dbg) return false;
  if (A.w.qtype != QT_Q4_K || Bp.w.qtype != QT_Q6_K) return false;
  const int ta = (A.w.N + 15) / 16, tb = (Bp.w.N + 15) / 16, ncu = mb_cu_count();
  const double ba = (double)ta * mb_rec_bytes(QT_Q4_K), bb = (double)tb * mb_rec_bytes(QT_Q6_K);
  int ga = (int)(ncu * ba / (ba + bb) + 0.5);
  ga = ga < 1 ? 1 : ga > ta ? ta : ga;
  int gb = ncu - ga;
  gb = gb < 1 ? 1 : gb > tb ? tb : gb;
  const size_t lds = mb_lds_bytes(A.B, A.w.K, AM_G16);
  auto go = [&](auto kern) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    hipLaunchKernelGGL(kern, dim3(ga + gb), dim3(MB_NT), lds, s, A, Bp, ga);
    ++g_mb_launches;
  };
  go(gemv_mb2_kernel<QT_Q4_K, QT_Q6_K, 4, 3, AM_G16>);
  return true;
}

bool gemv_mb(const GemvParams& P, hipStream_t s) {
  if (!gemv_mb_supported(P)) return false;
  const int am = mb_am(P);
  const size_t lds = mb_lds_bytes(P.B, P.w.K, am);
  auto go = [&](auto qt) {
    constexpr int QT = decltype(qt)::value;
    return am == AM_G16 ? mb_q<QT, AM_G16>(P, lds, s) : mb_q<QT, AM_LDS>(P, lds, s);
  };
  switch (P.w.qtype) {
    case QT_Q4_K: return go(std::integral_constant<int, QT_Q4_K>{});
    case QT_Q6_K: return go(std::integral_constant<int, QT_Q6_K>{});
    case QT_Q4_0: return go(std::integral_constant<int, QT_Q4_0>{});
    case QT_Q8_0: return go(std::integral_constant<int, QT_Q8_0>{});
    default: return false;
  }
}

}  // namespace omx
