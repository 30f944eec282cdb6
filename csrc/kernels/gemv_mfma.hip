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
//  * Layout M (dedicated device copy, built from layout v2 on the GPU by `repack_m`): one 16-row
//    tile x one 256-weight super-block is a contiguous record; its codes are lane-linear, so a wave
//    streams a record with 2-4 fully coalesced 1 KiB `global_load_dwordx4` (weights are read ONCE
//    per step by exactly one wave -- non-temporal loads). Lane l (row j = l % 16, K slice q = l / 16)
//    holds, per 32-weight span s, the 8 codes of K positions 32 s + 8 q .. + 7 of row j: exactly the
//    MFMA B-operand fragment. Scales follow the codes in the same record (raw, no extra bytes).
//  * 4-bit codes of a span sit in one dword ordered so that `(w >> {0,8,4,12}) & 0x000F000F | 0x6400`
//    yields the fp16 pairs (1024 + n) of K positions (0,1), (2,3), (4,5), (6,7) -- the activation
//    fragment is then plain row-major fp16 (one `ds_read_b128`). Dequant = 1 shift + 1 and-or +
//    1 `v_pk_add_f16` + 1 `v_pk_fma_f16` per 2 weights (exact 1024 removal before the scale).
//    Q6_K's 2 high bits per weight come from a per-lane dword laid out so one shift + mask places
//    them at bits 4-5 of both halves; Q8_0 bytes become fp16 pairs through `v_perm_b32`.
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

// layout M record geometry per quant type: code bytes (lane-linear, 1 KiB per wave load) + scales
static inline int n_sb_host(int K) { return (K + 255) >> 8; }

__host__ __device__ constexpr int mb_code_bytes(int qt) {
  return qt == QT_Q8_0 ? 4096 : qt == QT_Q6_K ? 3072 : (qt == QT_Q4_K || qt == QT_Q4_0) ? 2048 : 0;
}
__host__ __device__ constexpr int mb_rec_bytes(int qt) {
  return qt == QT_Q6_K ? 3072 + 256 + 32 : mb_code_bytes(qt) + (mb_code_bytes(qt) ? 256 : 0);
}

size_t mfma_layout_bytes(int qtype, int N, int K) {
  const int rec = mb_rec_bytes(qtype);
  if (!rec) return 0;
  return (size_t)((N + 15) / 16) * ((K + 255) / 256) * rec;
}

__device__ __forceinline__ mh2 ash2(unsigned v) { return __builtin_bit_cast(mh2, v); }
__device__ __forceinline__ unsigned asu2(mh2 v) { return __builtin_bit_cast(unsigned, v); }

// ------------------------------------------------------------------------------------------------
// layout v2 -> layout M (one thread per (tile, super-block, lane)); rows >= N are zero

// 4-bit / 6-bit / 8-bit code of element e (0..255) of super-block sb of `row`, from layout v2
template <int QT>
__device__ __forceinline__ int v2_code(const QMat& w, long long row, int SB, int sb, int e) {
  if constexpr (QT == QT_Q4_K) {  // sub-block s = e / 32: lo nibbles (s even) / hi nibbles ^ 8 (s odd)
    const int s = e >> 5, i = e & 31, t = 2 * (s >> 1) + (i >> 4);
    const unsigned byte = w.s0[row * SB * 128 + (long long)t * SB * 16 + sb * 16 + (i & 15)];
    return (s & 1) ? (int)(((byte >> 4) ^ 8) & 15) : (int)(byte & 15);
  } else if constexpr (QT == QT_Q4_0) {  // block t = e / 32: lo nibble = element i, hi (^8) = 16 + i
    const int t = e >> 5, i = e & 31;
    const unsigned byte = w.s0[row * SB * 128 + (long long)t * SB * 16 + sb * 16 + (i & 15)];
    return i < 16 ? (int)(byte & 15) : (int)(((byte >> 4) ^ 8) & 15);
  } else if constexpr (QT == QT_Q8_0) {
    const int t = e >> 5, i = e & 31;
    return (int)(int8_t)w.s0[row * SB * 256 + (long long)t * SB * 32 + sb * 32 + i];
  } else {  // Q6_K (quant.py repack / _q6k_qh_split): y = 128 n + 32 f + l
    const int n = e >> 7, f = (e >> 5) & 3, l = e & 31;
    const int b = 64 * n + l + 32 * (f & 1);
    const unsigned qb = w.s0[row * SB * 128 + (long long)(b >> 4) * SB * 16 + sb * 16 + (b & 15)];
    const unsigned nib = (f >> 1) ? (qb >> 4) : (qb & 15);
    const int sub = 2 * (f & 1) + (l >> 4), half = f >> 1, i = l & 15;
    const unsigned hb = w.s1[row * SB * 64 + (long long)(4 * n + sub) * SB * 8 + sb * 8 + half * 4 + (i & 3)];
    return (int)(nib | (((hb >> (2 * (i >> 2))) & 3) << 4));
  }
}

template <int QT>
__global__ __launch_bounds__(256) void repack_m_kernel(QMat w, uint8_t* out) {
  const int SB = n_sb(w.K), tiles = (w.N + 15) / 16;
  const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (long long)tiles * SB * 64) return;
  const int lane = (int)(gid & 63);
  const long long rec = gid >> 6;
  const int sb = (int)(rec % SB), tile = (int)(rec / SB);
  const int j = lane & 15, q = lane >> 4;
  const long long row = (long long)tile * 16 + j;
  const bool live = row < w.N;
  uint8_t* R = out + rec * mb_rec_bytes(QT);
  if constexpr (QT == QT_Q8_0) {
    unsigned dw[16];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        unsigned v = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int c = live ? v2_code<QT>(w, row, SB, sb, 32 * s + 8 * q + 4 * h + k) : 0;
          v |= (unsigned)(c & 0xFF) << (8 * k);
        }
        dw[2 * s + h] = v;
      }
#pragma unroll
    for (int h = 0; h < 4; ++h)  // [h][lane][16 B]: spans 2h, 2h+1
      *(u32x4*)(R + h * 1024 + lane * 16) = (u32x4){dw[4 * h], dw[4 * h + 1], dw[4 * h + 2], dw[4 * h + 3]};
  } else {
    unsigned lo[8], hi[4] = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      int e[8];
#pragma unroll
      for (int p = 0; p < 8; ++p) e[p] = live ? v2_code<QT>(w, row, SB, sb, 32 * s + 8 * q + p) : 0;
      // byte k: lo nibble a_k, hi nibble b_k with a = (e0, e2, e1, e3), b = (e4, e6, e5, e7)
      const int a[4] = {e[0], e[2], e[1], e[3]}, bb[4] = {e[4], e[6], e[5], e[7]};
      unsigned v = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) v |= (unsigned)((a[k] & 15) | ((bb[k] & 15) << 4)) << (8 * k);
      lo[s] = v;
      if constexpr (QT == QT_Q6_K) {  // pair k = (e_2k, e_2k+1): bits 2i / 16 + 2i, i = 4 (s & 1) + k
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int i = 4 * (s & 1) + k;
          hi[s >> 1] |= (unsigned)((e[2 * k] >> 4) & 3) << (2 * i);
          hi[s >> 1] |= (unsigned)((e[2 * k + 1] >> 4) & 3) << (16 + 2 * i);
        }
      }
    }
    *(u32x4*)(R + lane * 16) = (u32x4){lo[0], lo[1], lo[2], lo[3]};
    *(u32x4*)(R + 1024 + lane * 16) = (u32x4){lo[4], lo[5], lo[6], lo[7]};
    if constexpr (QT == QT_Q6_K) *(u32x4*)(R + 2048 + lane * 16) = (u32x4){hi[0], hi[1], hi[2], hi[3]};
  }
  // scales: one lane per row
  if (q == 0) {
    uint8_t* S = R + mb_code_bytes(QT);
    if constexpr (QT == QT_Q6_K) {  // [16 rows][even 8 sc | odd 8 sc] + [16 rows][fp16 d]
      uint8_t sc[16];
      uint16_t d = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) sc[i] = live ? w.s2[row * SB * 16 + sb * 16 + i] : 0;
      if (live) d = *(const uint16_t*)(w.s3 + row * SB * 2 + sb * 2);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        S[j * 16 + i] = sc[2 * i];
        S[j * 16 + 8 + i] = sc[2 * i + 1];
      }
      *(uint16_t*)(S + 256 + j * 2) = d;
    } else {  // Q4_K meta (d, dmin, 12 B scales) / Q4_0, Q8_0 8 x fp16 d: the v2 row slice
      u32x4 m = (u32x4){0, 0, 0, 0};
      if (live) m = *(const u32x4*)(w.s1 + row * SB * 16 + sb * 16);
      *(u32x4*)(S + j * 16) = m;
    }
  }
}

void repack_m(const QMat& w, void* out, hipStream_t s) {
  const long long n = (long long)((w.N + 15) / 16) * ((w.K + 255) / 256) * 64;
  const dim3 grid((unsigned)((n + 255) / 256));
  uint8_t* o = (uint8_t*)out;
  switch (w.qtype) {
    case QT_Q4_K: hipLaunchKernelGGL(repack_m_kernel<QT_Q4_K>, grid, dim3(256), 0, s, w, o); break;
    case QT_Q6_K: hipLaunchKernelGGL(repack_m_kernel<QT_Q6_K>, grid, dim3(256), 0, s, w, o); break;
    case QT_Q4_0: hipLaunchKernelGGL(repack_m_kernel<QT_Q4_0>, grid, dim3(256), 0, s, w, o); break;
    case QT_Q8_0: hipLaunchKernelGGL(repack_m_kernel<QT_Q8_0>, grid, dim3(256), 0, s, w, o); break;
    default: break;
  }
}

// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// ring unit: NR layout M records (this lane's codes + scales) and, when the activations are read
// from global memory per record (CA), the record's 8 A-operand fragments
template <int QT, int NR, bool CA>
struct MUnit {
  static constexpr int NC = mb_code_bytes(QT) / 1024;
  u32x4 c[NR][NC];
  u32x4 s[NR];  // scales (Q6_K: x, y = this lane's 8 int8 sc, z = fp16 d)
  f16x8 a[CA ? 8 : 1];
  float eo[4];  // this lane's epilogue operands for the unit's tile (mb_epi_load)
};

// Epilogue operands of this lane's output of `tile` (row j = lane % 16, batch row 4 q + (wave & 3): the
// accumulator layout of the MFMA, one register per epilogue wave), loaded with the tile's weights: a
// global load issued inside the stream would be queued behind every weight load in flight (vmcnt
// retires in order) and drain the ring. Unconditional loads from clamped addresses; an operand an
// epilogue does not use reads a harmless valid address (the layout M codes).
//   eo[0]: EPI_ADD old y | eo[1]: bias[vn] | eo[2]: EPI_QKV bias[vn ^ 1] |
//   eo[3]: emit_nw[vn] (residual emission) or inv_freq[d / 2] (EPI_QKV)
constexpr int MB_EO = 4;

// emission range exponent e of a residual row from its old mean square: the row is stored times 2^-e,
// e = floor(log2(rms)) - 2 clamped to [0, 30], so fp16 keeps values up to ~2^18 x the row RMS (a
// random-init 32-layer stack grows its residual past fp16's 65504; trained rows keep e = 0)
__device__ __forceinline__ int emit_range_exp(float ms) {
  const int k = (int)floorf(0.5f * __log2f(fminf(fmaxf(ms, 1e-30f), 1e30f)));
  return min(max(k - 2, 0), 30);
}
__device__ __forceinline__ void mb_epi_load(const GemvParams& P, int tile, float (&eo)[MB_EO]) {
  const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4, wave = threadIdx.x >> 6;
  const int row = min(tile * 16 + j, P.w.N - 1), vn = row + P.row_offset;
  const int b = min(4 * q + (wave & 3), P.B - 1);
  const float* dummy = (const float*)P.w.mt;
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
        if (which == 1) kv_store(P.kc, idx, out, P.kv8);
        else kv_store(P.vc, idx, out, P.kv8);
      }
      break;
    }
    default:
      break;
  }
}

template <int QT, int NR, bool CA>
__device__ __forceinline__ void mb_load_rec(const QMat& w, int tile, int SB, int sb, int r, int lane,
                                            MUnit<QT, NR, CA>& U) {
  constexpr int REC = mb_rec_bytes(QT), CODE = mb_code_bytes(QT);
  const int j = lane & 15, q = lane >> 4;
  OMX_KASSERT(tile >= 0 && tile < (w.N + 15) / 16 && sb >= 0 && sb < SB);
  const uint8_t* R = w.mt + ((long long)tile * SB + sb) * REC;
#pragma unroll
  for (int c = 0; c < MUnit<QT, NR, CA>::NC; ++c)
    U.c[r][c] = __builtin_nontemporal_load((const u32x4*)(R + c * 1024 + lane * 16));
  if constexpr (QT == QT_Q6_K) {
    const u32x2 v = *(const u32x2*)(R + CODE + j * 16 + 8 * (q >> 1));
    U.s[r] = (u32x4){v.x, v.y, *(const uint16_t*)(R + CODE + 256 + j * 2), 0u};
  } else {
    U.s[r] = *(const u32x4*)(R + CODE + j * 16);
  }
}

// the 8 A-operand fragments of super-block sb from a global fp16 activation row (lanes of batch rows
// >= B read the buffer's all-zero row GemvParams::zrow16: no branch around the loads)
__device__ __forceinline__ void mb_load_a(const f16* xg, int sb, f16x8 (&a)[8]) {
#pragma unroll
  for (int s = 0; s < 8; ++s) a[s] = *(const f16x8*)(xg + sb * 256 + 32 * s);
}

// (a & m) | o in one VALU op (hipcc emits v_and + v_or for the C expression)
__device__ __forceinline__ unsigned and_or(unsigned a, unsigned m, unsigned o) {
  unsigned r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(m), "v"(o));
  return r;
}

__device__ __forceinline__ unsigned sel4(const u32x4& v, int i) {
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}
template <int SH>
__device__ __forceinline__ unsigned shr(unsigned v) {
  if constexpr (SH >= 0) return v >> SH;
  else return v << (-SH);
}

// fp16 B-operand fragment of span S of record r (8 weights of this lane's row), compile-time indices
template <int QT, int S>
__device__ __forceinline__ f16x8 mb_deq(const u32x4* c, mh2 sc, mh2 mn) {
  u32x4 r;
  if constexpr (QT == QT_Q8_0) {
    const u32x4 cc = c[S >> 1];
    const unsigned f0 = sel4(cc, 2 * (S & 1)) ^ 0x80808080u, f1 = sel4(cc, 2 * (S & 1) + 1) ^ 0x80808080u;
    const mh2 off = {(f16)1152.f, (f16)1152.f};
    r.x = asu2((ash2(__builtin_amdgcn_perm(0x64646464u, f0, 0x04010400u)) - off) * sc);
    r.y = asu2((ash2(__builtin_amdgcn_perm(0x64646464u, f0, 0x04030402u)) - off) * sc);
    r.z = asu2((ash2(__builtin_amdgcn_perm(0x64646464u, f1, 0x04010400u)) - off) * sc);
    r.w = asu2((ash2(__builtin_amdgcn_perm(0x64646464u, f1, 0x04030402u)) - off) * sc);
  } else {
    const unsigned wd = sel4(c[S >> 2], S & 3);
    unsigned u0 = and_or(wd, 0x000F000Fu, MB_MAGIC);
    unsigned u1 = and_or(wd >> 8, 0x000F000Fu, MB_MAGIC);
    unsigned u2 = and_or(wd >> 4, 0x000F000Fu, MB_MAGIC);
    unsigned u3 = and_or(wd >> 12, 0x000F000Fu, MB_MAGIC);
    if constexpr (QT == QT_Q6_K) {  // high bits of pair k at bits 2i / 16 + 2i of H, i = 4 (S & 1) + k
      const unsigned H = sel4(c[2], S >> 1);
      constexpr int I = 4 * (S & 1);
      u0 = and_or(shr<2 * I - 4>(H), 0x00300030u, u0);
      u1 = and_or(shr<2 * I - 2>(H), 0x00300030u, u1);
      u2 = and_or(shr<2 * I>(H), 0x00300030u, u2);
      u3 = and_or(shr<2 * I + 2>(H), 0x00300030u, u3);
      const mh2 off = {(f16)1056.f, (f16)1056.f};  // 1024 + 32 (Q6_K codes are q - 32)
      r.x = asu2((ash2(u0) - off) * sc);
      r.y = asu2((ash2(u1) - off) * sc);
      r.z = asu2((ash2(u2) - off) * sc);
      r.w = asu2((ash2(u3) - off) * sc);
    } else {
      const mh2 off = {(f16)1024.f, (f16)1024.f};
      r.x = asu2((ash2(u0) - off) * sc + mn);
      r.y = asu2((ash2(u1) - off) * sc + mn);
      r.z = asu2((ash2(u2) - off) * sc + mn);
      r.w = asu2((ash2(u3) - off) * sc + mn);
    }
  }
  return __builtin_bit_cast(f16x8, r);
}

// A-operand sources: LDS rows (prologue-staged) or register fragments
struct ALds {
  const f16* xa;  // this lane's LDS row + 8 q + sb * 256
  bool av;
  __device__ __forceinline__ f16x8 get(int s) const {
    f16x8 a = {};
    if (av) a = *(const f16x8*)(xa + 32 * s);
    return a;
  }
};
struct AReg {
  const f16x8* a;
  __device__ __forceinline__ f16x8 get(int s) const { return a[s]; }
};

template <int QT, int S, class AS>
__device__ __forceinline__ void mb_span(const u32x4* c, float d, float dm, unsigned scw, unsigned mnw, const AS& A,
                                        f32x4& acc) {
  mh2 sc, mn = {(f16)0.f, (f16)0.f};
  if constexpr (QT == QT_Q4_K) {
    const f16 a = (f16)(d * (float)((scw >> (8 * (S & 3))) & 0xFF));
    const f16 b = (f16)(-dm * (float)((mnw >> (8 * (S & 3))) & 0xFF));
    sc = (mh2){a, a};
    mn = (mh2){b, b};
  } else if constexpr (QT == QT_Q6_K) {
    const f16 a = (f16)(d * (float)(int8_t)((scw >> (8 * (S & 3))) & 0xFF));
    sc = (mh2){a, a};
  } else {  // Q4_0 / Q8_0: fp16 d of block S (scw = the dword holding it)
    const f16 a = __builtin_bit_cast(f16, (uint16_t)((scw >> (16 * (S & 1))) & 0xFFFF));
    sc = (mh2){a, a};
    if constexpr (QT == QT_Q4_0) {
      const f16 z = (f16)(-8.f) * a;  // n - 8: exact (8 d is a power-of-two multiple of d)
      mn = (mh2){z, z};
    }
  }
  const f16x8 bw = mb_deq<QT, S>(c, sc, mn);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(A.get(S), bw, acc, 0, 0, 0);
}

// the 8 MFMAs of one record
template <int QT, class AS>
__device__ __forceinline__ void mb_rec(const u32x4* c, const u32x4 m, const AS& A, f32x4& acc) {
  if constexpr (QT == QT_Q4_K) {
    const float d = h2f(m.x & 0xFFFF), dm = h2f(m.x >> 16);
    const unsigned sl = m.y & 0x3F3F3F3Fu, ml = m.z & 0x3F3F3F3Fu;
    const unsigned sh = (m.w & 0x0F0F0F0Fu) | ((m.y >> 2) & 0x30303030u);
    const unsigned mh = ((m.w >> 4) & 0x0F0F0F0Fu) | ((m.z >> 2) & 0x30303030u);
    mb_span<QT, 0>(c, d, dm, sl, ml, A, acc);
    mb_span<QT, 1>(c, d, dm, sl, ml, A, acc);
    mb_span<QT, 2>(c, d, dm, sl, ml, A, acc);
    mb_span<QT, 3>(c, d, dm, sl, ml, A, acc);
    mb_span<QT, 4>(c, d, dm, sh, mh, A, acc);
    mb_span<QT, 5>(c, d, dm, sh, mh, A, acc);
    mb_span<QT, 6>(c, d, dm, sh, mh, A, acc);
    mb_span<QT, 7>(c, d, dm, sh, mh, A, acc);
  } else if constexpr (QT == QT_Q6_K) {
    const float d = h2f(m.z & 0xFFFF);
    mb_span<QT, 0>(c, d, 0.f, m.x, 0u, A, acc);
    mb_span<QT, 1>(c, d, 0.f, m.x, 0u, A, acc);
    mb_span<QT, 2>(c, d, 0.f, m.x, 0u, A, acc);
    mb_span<QT, 3>(c, d, 0.f, m.x, 0u, A, acc);
    mb_span<QT, 4>(c, d, 0.f, m.y, 0u, A, acc);
    mb_span<QT, 5>(c, d, 0.f, m.y, 0u, A, acc);
    mb_span<QT, 6>(c, d, 0.f, m.y, 0u, A, acc);
    mb_span<QT, 7>(c, d, 0.f, m.y, 0u, A, acc);
  } else {
    mb_span<QT, 0>(c, 0.f, 0.f, m.x, 0u, A, acc);
    mb_span<QT, 1>(c, 0.f, 0.f, m.x, 0u, A, acc);
    mb_span<QT, 2>(c, 0.f, 0.f, m.y, 0u, A, acc);
    mb_span<QT, 3>(c, 0.f, 0.f, m.y, 0u, A, acc);
    mb_span<QT, 4>(c, 0.f, 0.f, m.z, 0u, A, acc);
    mb_span<QT, 5>(c, 0.f, 0.f, m.z, 0u, A, acc);
    mb_span<QT, 6>(c, 0.f, 0.f, m.w, 0u, A, acc);
    mb_span<QT, 7>(c, 0.f, 0.f, m.w, 0u, A, acc);
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

// Grid: persistent blocks over 16-row tiles (tile = blockIdx.x + k * gridDim.x); wave w owns
// super-blocks [w SB / 8, (w + 1) SB / 8) of every tile. Work is streamed as units through a
// register ring of RD units: a unit is the wave's whole share of one tile when that share is <= 2
// super-blocks (TU, activations of that share held in registers for the launch), else one
// super-block (with its own activation fragments in AM_G16).
// Each wave drops its partial tile into an LDS slot, refills its ring first (the next units stream
// across the barrier), meets the block, and waves 0..3 sum the 8 partials in wave order (deterministic)
// and run the fused epilogue, one output per lane each.
template <int QT, int NSBW, int RD, int AM, int DBG = 0>
__device__ __forceinline__ void mb_body(const GemvParams& P, const int bx, const int gxn) {
  constexpr bool TU = NSBW <= 2;
  constexpr int NR = TU ? NSBW : 1;
  constexpr bool G16 = AM == AM_G16;
  constexpr bool CA = G16 && !TU;  // activation fragments ride with each record
  constexpr bool AC = G16 && TU;   // activation fragments of the wave's share held for the launch
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const QMat& w = P.w;
  const int K = w.K, N = w.N, SB = n_sb(K), B = P.B;
  const int XSTR = SB * 256 + 8;
  f16* xs = (f16*)smem;
  float* red = (float*)(smem + (G16 ? 0 : (((size_t)B * XSTR * 2 + 15) & ~(size_t)15)));
  float* stat = red + MB_NSLOT * MB_NW * 64 * 4 + 2 * MB_NSLOT;
  float* srstd = stat + MB_NW * 16;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, j = lane & 15, q = lane >> 4;
  const int sb0 = wave * SB / MB_NW, sb1 = (wave + 1) * SB / MB_NW, nsb = sb1 - sb0;
  const int last_sb = nsb > 0 ? sb1 - 1 : min(sb0, SB - 1);  // surplus loads re-read it (cache hits)
  const int n_tiles = (N + 15) >> 4;
  const int my_tiles = bx < n_tiles ? (n_tiles - 1 - bx) / gxn + 1 : 0;
  const int upt = TU ? 1 : nsb;  // units per tile
  const int n_units = my_tiles * upt;
  const bool av = j < B;         // A-operand lane: batch row j
  const bool rs = G16 && P.xstat != nullptr && !(DBG & 2);
  const bool es = P.emit16 != nullptr && P.emit_prev != nullptr;  // emission range scale (never with rs)
  const bool er = P.emit16 != nullptr && P.rexp_in != nullptr && !es;  // the same, exponents precomputed
  const float* sx = rs ? P.xstat : P.emit_prev;
  const int sxn = rs ? P.xstat_n : P.emit_prev_n;

  // per-row epilogue operands (EPI_QKV) of this lane's batch row 4 q + (wave & 3), first
  int e_pos = 0, e_slot = 0;
  if (P.epi == EPI_QKV) {  // block-uniform
    const int b = min(4 * q + (wave & 3), B - 1);
    e_pos = P.pos[b];
    e_slot = P.slot[b];
  }
  // 0. (AM_G16) RMS partials [16][xstat_n] of this wave's batch rows w, w + 8 (coalesced rows); for an
  // emitting producer with emit_prev, the partials of the residual before the add (the range scale)
  float sp[2][MB_SPL];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < MB_SPL; ++k) sp[h][k] = 0.f;
  if (rs || es) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int b = wave + 8 * h;
      if (b < B) {  // wave-uniform
#pragma unroll
        for (int k = 0; k < MB_SPL; ++k) {
          const int p = lane + 64 * k;
          const float v = sx[(long long)b * sxn + min(p, sxn - 1)];
          sp[h][k] = p < sxn ? v : 0.f;
        }
      }
    }
  }
  const f16* xg = G16 ? (const f16*)P.x16 + (long long)(av ? j : P.zrow16) * P.ld16 + 8 * q : nullptr;
  // 1. (AC) the A fragments of this wave's super-blocks, before any weight request
  f16x8 Ac[AC ? NSBW : 1][8];
  if constexpr (AC) {
#pragma unroll
    for (int i = 0; i < NSBW; ++i) {
      if constexpr ((DBG & 2) != 0) {
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2) Ac[i][s2] = (f16x8){};
      } else {
        mb_load_a(xg, min(sb0 + i, last_sb), Ac[i]);
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
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
        if (P.rexp_out && bx == 0) P.rexp_out[tid] = (float)emit_range_exp(t / K);
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
  auto unit_tile = [&](int u) { return bx + (TU ? u : u / (nsb > 0 ? nsb : 1)) * gxn; };
  auto load_unit = [&](MUnit<QT, NR, CA>& U, int u) {
    // surplus slots (past the wave's last unit) re-read one line of the last unit: every lane the same
    // address, so a surplus load instruction costs one cache line (never computed)
    const int ln = u < n_units ? lane : 0;
    u = min(u, n_units - 1);
    const int t = unit_tile(u);
    mb_epi_load(P, t, U.eo);
    if constexpr (TU) {
#pragma unroll
      for (int r = 0; r < NR; ++r) mb_load_rec<QT, NR, CA>(w, t, SB, min(sb0 + r, last_sb), r, ln, U);
    } else {
      const int sb = sb0 + u % nsb;
      mb_load_rec<QT, NR, CA>(w, t, SB, sb, 0, ln, U);
      if constexpr (CA) mb_load_a(xg, sb, U.a);
    }
    __builtin_amdgcn_sched_barrier(0);  // issue order = consumption order (vmcnt retires in order)
  };
  MUnit<QT, NR, CA> U[RD];
  if (n_units > 0) {
#pragma unroll
    for (int r = 0; r < RD; ++r) load_unit(U[r], r);
  }
  // 4. per-row RMS scale from the producer's partials (times the producer's range scale), or this
  // producer's own emission range scale 2^-e (srstd doubles as its LDS slot)
  if (rs || es) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < MB_SPL; ++k) s += sp[h][k];
      s = wave_sum(s);
      const int b = wave + 8 * h;
      if (lane == 0 && b < B) {
        if (rs) {
          srstd[b] = rsqrtf(s / K + P.eps) * (P.xscale ? P.xscale[b] : 1.f);
          if (P.rexp_out && bx == 0) P.rexp_out[b] = (float)emit_range_exp(s / K);
        } else {
          const int e = emit_range_exp(s / N);
          srstd[b] = __builtin_ldexpf(1.f, -e);
          if (bx == 0 && P.emit_scale) P.emit_scale[b] = __builtin_ldexpf(1.f, e);
        }
      }
    }
  }
  if (er && tid < B) {
    const int e = (int)P.rexp_in[tid];
    srstd[tid] = __builtin_ldexpf(1.f, -e);
    if (bx == 0 && P.emit_scale) P.emit_scale[tid] = __builtin_ldexpf(1.f, e);
  }
  if (!es && !er && P.emit16 && P.emit_scale && bx == 0 && tid < B) P.emit_scale[tid] = 1.f;
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
        const float c = es || er ? srstd[b] : 1.f;  // range scale 2^-e of the emitted row (exact)
        ((f16*)P.emit16)[(long long)b * P.ld_emit + vn] = (f16)(nv * eo[3] * c);
        sq = nv * nv;
      }
      sq = mb_row16_sum(sq);  // the 16 lanes of a DPP row hold the tile's 16 rows of batch row b
      if (j == 0 && b < B) P.emit_stat[(long long)b * ((N + 15) >> 4) + tile] = sq;
    } else if (ok) {
      mb_epi(P, b, vn, x, px, eo[0], eo[1], eo[2], eo[3], e_pos, e_slot);
    }
  };

  // 5. stream the units
  if (!TU && nsb == 0) {  // no super-blocks in this wave (K < 2048): zero partials
    for (int t = 0; t < my_tiles; ++t) {
      float eo[MB_EO];
      mb_epi_load(P, bx + t * gxn, eo);
      finish((f32x4){0.f, 0.f, 0.f, 0.f}, bx + t * gxn, eo);
    }
    return;
  }
  const f16* xl = xs + (long long)(av ? j : 0) * XSTR + 8 * q;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  // one unit: its MFMAs, the slot's refill RD units ahead, then the tile's epilogue hand-off when the
  // unit completes the wave's share (operands copied out of the unit before its refill)
  auto step = [&](MUnit<QT, NR, CA>& Ur, int u) {
    bool last = true;
    if constexpr ((DBG & 1) != 0) {  // memory path only: consume every loaded word
      unsigned v = 0;
#pragma unroll
      for (int i = 0; i < NR; ++i) {
#pragma unroll
        for (int c = 0; c < MUnit<QT, NR, CA>::NC; ++c) v ^= Ur.c[i][c].x ^ Ur.c[i][c].w;
        v ^= Ur.s[i].y;
      }
      acc.x += (float)(v & 1);
      if constexpr (!TU) last = u % nsb == nsb - 1;
    } else if constexpr (TU) {
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        if (i < nsb) {
          if constexpr (AC) mb_rec<QT>(Ur.c[i], Ur.s[i], AReg{Ac[i]}, acc);
          else mb_rec<QT>(Ur.c[i], Ur.s[i], ALds{xl + (sb0 + i) * 256, av}, acc);
        }
      }
    } else {
      const int i = u % nsb;
      if constexpr (CA) mb_rec<QT>(Ur.c[0], Ur.s[0], AReg{Ur.a}, acc);
      else mb_rec<QT>(Ur.c[0], Ur.s[0], ALds{xl + (sb0 + i) * 256, av}, acc);
      last = i == nsb - 1;
    }
    float eo[MB_EO];
#pragma unroll
    for (int e = 0; e < MB_EO; ++e) eo[e] = Ur.eo[e];
    const int tile = unit_tile(u);
    load_unit(Ur, u + RD);
    if (last) {
      finish(acc, tile, eo);
      acc = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  };
  // whole ring rounds without conditions (exact vmcnt counting), then the tail
  const int n_full = n_units / RD * RD;
  int u = 0;
  for (; u < n_full; u += RD) {
#pragma unroll
    for (int r = 0; r < RD; ++r) step(U[r], u + r);
  }
#pragma unroll
  for (int r = 0; r < RD; ++r)
    if (u + r < n_units) step(U[r], u + r);  // wave-uniform
}

template <int QT, int NSBW, int RD, int AM, int DBG = 0>
__global__ __launch_bounds__(MB_NT) void gemv_mb_kernel(GemvParams P) {
  mb_body<QT, NSBW, RD, AM, DBG>(P, blockIdx.x, gridDim.x);
}

// two matrices over the same activations in ONE launch (the Q4_K_M QKV: q,k rows Q4_K + v rows
// Q6_K): blocks [0, ga) run A, the rest B -- one launch ramp / drain instead of two
template <int QA, int QB, int NSBW, int RD, int AM>
__global__ __launch_bounds__(MB_NT) void gemv_mb2_kernel(GemvParams PA, GemvParams PB, int ga) {
  if ((int)blockIdx.x < ga) mb_body<QA, NSBW, RD, AM>(PA, blockIdx.x, ga);
  else mb_body<QB, NSBW, RD, AM>(PB, (int)blockIdx.x - ga, (int)gridDim.x - ga);
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
void set_mb_enable(int on) { g_mb_enable = on ? 1 : 0; }
void set_mb_tuning(int dbg, int bpc) {
  if (dbg >= 0 && dbg < 8) g_mb_dbg = dbg;
  if (bpc == 1 || bpc == 2) g_mb_bpc = bpc;
}
bool mb_enabled() { return g_mb_enable != 0; }

template <int QT, int NSBW, int RD, int AM, int DBG = 0>
static void mb_launch_k(const GemvParams& P, size_t lds, hipStream_t s) {
  auto kern = gemv_mb_kernel<QT, NSBW, RD, AM, DBG>;
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
}

template <int QT, int NSBW, int RD, int AM>
static void mb_launch(const GemvParams& P, size_t lds, hipStream_t s) {
  if constexpr (AM == AM_G16 && (QT == QT_Q4_K || QT == QT_Q6_K)) {
    switch (g_mb_dbg) {  // microbenchmark-only variants
      case 1: mb_launch_k<QT, NSBW, RD, AM, 1>(P, lds, s); return;
      case 2: mb_launch_k<QT, NSBW, RD, AM, 2>(P, lds, s); return;
      case 3: mb_launch_k<QT, NSBW, RD, AM, 3>(P, lds, s); return;
      case 7: mb_launch_k<QT, NSBW, RD, AM, 7>(P, lds, s); return;
      default: break;
    }
  }
  mb_launch_k<QT, NSBW, RD, AM>(P, lds, s);
}

template <int QT, int AM>
static bool mb_q(const GemvParams& P, size_t lds, hipStream_t s) {
  const int SB = n_sb_host(P.w.K), nsbw = (SB + MB_NW - 1) / MB_NW;
  switch (nsbw) {
    case 1: mb_launch<QT, 1, 4, AM>(P, lds, s); return true;
    // Q8_0 records are twice the Q4 size: a 3-deep ring spills at these widths, keep 2 units in flight
    case 2: mb_launch<QT, 2, QT == QT_Q8_0 ? 2 : 3, AM>(P, lds, s); return true;
    case 3: case 4: case 5: case 6: case 7: case 8: mb_launch<QT, 8, QT == QT_Q8_0 ? 2 : 3, AM>(P, lds, s); return true;
    default: return false;
  }
}

static int mb_am(const GemvParams& P) { return P.x16 ? AM_G16 : AM_LDS; }

bool gemv_mb_supported(const GemvParams& P) {
  // B = 2 stays on the int8 GEMV (gemv_batch.hip): measured 2.08 vs 2.15 ms per Llama-2-7B step
  if (!g_mb_enable || !P.w.mt || P.B < MB_BMIN || P.B > MB_BMAX || P.expert_ids || P.merge_S) return false;
  if (g_tune.debug) return false;
  const int q = P.w.qtype;
  if (q != QT_Q4_K && q != QT_Q6_K && q != QT_Q4_0 && q != QT_Q8_0) return false;
  if ((n_sb_host(P.w.K) + MB_NW - 1) / MB_NW > 8) return false;
  if (P.emit16 && (P.epi != EPI_ADD || !P.emit_nw || !P.emit_stat)) return false;
  if (P.emit_prev && (!P.emit16 || P.xstat || P.emit_prev_n < 1 || P.emit_prev_n > 64 * MB_SPL)) return false;
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
  const int SB = n_sb_host(A.w.K), nsbw = (SB + MB_NW - 1) / MB_NW;
  if (nsbw > 2) return false;
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
  };
  if (nsbw == 1) go(gemv_mb2_kernel<QT_Q4_K, QT_Q6_K, 1, 4, AM_G16>);
  else go(gemv_mb2_kernel<QT_Q4_K, QT_Q6_K, 2, 3, AM_G16>);
  count_launch(LC_GEMV_MB);
  return true;
}

bool gemv_mb(const GemvParams& P, hipStream_t s) {
  if (!gemv_mb_supported(P)) return false;
  const int am = mb_am(P);
  const size_t lds = mb_lds_bytes(P.B, P.w.K, am);
  auto go = [&](auto qt) {
    constexpr int QT = decltype(qt)::value;
    const bool ok = am == AM_G16 ? mb_q<QT, AM_G16>(P, lds, s) : mb_q<QT, AM_LDS>(P, lds, s);
    if (ok) count_launch(LC_GEMV_MB);
    return ok;
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
