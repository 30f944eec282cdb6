// Fused quantized GEMV for decode and small batches (M = B <= a few rows) on gfx950.
//
// y[b, n] = epilogue( sum_k W[n, k] * norm(x[b, :])[k] )
//
// Design (MI355X-first, see SURVEY.md §7.4 hard part 1 and docs/kernels.md):
//  * Weights use repack layout v2 (ollama_operator_amd/quant.py "device repack"): K padded to SB
//    super-blocks of 256, codes stored piece-major across super-blocks -- qs[row][t][sb][16 B].
//  * Lane mapping: a wave = 4 row groups of 16 lanes; lane s of a group owns super-blocks
//    s, s+16, ... (NSB of them per K chunk) of R rows and walks all 8 pieces t of each. One load
//    instruction for piece t therefore reads a contiguous 256 B run per row group, and t is a
//    compile-time constant: the K-quant scales / mins are decoded once per 256 weights, with
//    constant byte selects (v_cvt_f32_ubyteN), instead of once per 32-weight piece. The previous
//    lane-per-piece kernel spent ~95 VALU ops per piece-row (rocprofv3 PMC, profiles/r1_pmc):
//    VALU-bound next to an 8 us HBM floor. This one spends ~30.
//  * 4-bit codes keep the high nibble signed (byte ^ 0x80 at repack), so `q & 0xF0F0F0F0` feeds
//    v_dot4_i32_i8 directly (16 * (n - 8)): 2 VALU per dword to unpack both nibbles.
//  * Activation prologue once per block: x (fp32) optionally RMS/Layer-normalised (fused), int8-
//    quantised per 16-element group (fp32 scale + group sum for the K-quant mins / zero points),
//    staged in LDS with one pad slot per super-block (17 slots) so the 16 lanes of a group -- one
//    super-block apart -- hit distinct banks.
//  * Weight loads for the first tile are issued before the prologue; persistent blocks prefetch the
//    next (tile, K chunk) unit into a second register tile when the tile fits (DB), else rely on
//    other waves for latency hiding.
//  * Row sums: 16-lane DPP reduction (quad_perm / row_half_mirror / row_mirror), no LDS.
//  * Epilogues fused: residual add (+ MoE routing weight, atomics for top-k > 1), bias, SiLU-GLU
//    (gate/up rows interleaved at load), GELU, and QKV (RoPE on adjacent row pairs + fp16 paged KV
//    scatter). Pair partners come from the same lane (R = 2) or the neighbouring row group (R = 1).
// Reference parity: the reference delegates all of this to llama.cpp inside `ollama/ollama`
// (reference pkg/model/pod.go:10-12); numerics are checked against quant.py + an fp32 torch GEMV.
#include "common.h"
#include "epilogue.h"
#include "ops.h"

namespace omx {


constexpr int GEMV_NW = 4;  // waves per block (8-wave blocks measured slower: profiles/r1_pmc)
constexpr int GEMV_NT = 64 * GEMV_NW;
constexpr int XPAD = 17;      // LDS x slots per super-block: 16 groups + 1 pad

GemvTuning g_tune;
void set_gemv_tuning(int blocks_per_cu, int rows, int debug, int ks, int xfirst) {
  g_tune.debug = debug > 0 ? debug : 0;
  if (xfirst == 0 || xfirst == 1) g_tune.xfirst = xfirst;
  if (ks >= 0 && ks <= 4) g_tune.ks = ks;
  if (blocks_per_cu > 0) g_tune.blocks_per_cu = blocks_per_cu;
  if (rows == 1 || rows == 2) g_tune.rows = rows;
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// sum over the 16 lanes of a DPP row; every lane of the row gets the total
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}

__device__ __forceinline__ int dot16(u32x4 q, i32x4 x) {
  int s = sdot4((int)q.x, x.x, 0);
  s = sdot4((int)q.y, x.y, s);
  s = sdot4((int)q.z, x.z, s);
  return sdot4((int)q.w, x.w, s);
}

__device__ __forceinline__ float ubyte(unsigned v, int k) { return (float)((v >> (8 * k)) & 0xFF); }
__device__ __forceinline__ float sbyte(unsigned v, int k) { return (float)(int8_t)((v >> (8 * k)) & 0xFF); }
__device__ __forceinline__ float f16lo(unsigned v) { return h2f(v & 0xFFFF); }
__device__ __forceinline__ float f16hi(unsigned v) { return h2f(v >> 16); }

// ---------------------------------------------------------------------------------------------
// register tile: R rows x NSB super-blocks x 8 pieces of one lane
template <int QT, int NSB, int R>
struct WTile {
  static constexpr bool Q8 = QT == QT_Q8_0, Q6 = QT == QT_Q6_K;
  u32x4 a[R][NSB][8];                                  // qs / ql / Q8_0 first 16 B
  u32x4 b[Q8 ? R : 1][Q8 ? NSB : 1][8];                // Q8_0 second 16 B
  u32x2 h[Q6 ? R : 1][Q6 ? NSB : 1][8];                // Q6_K high bits (H0 | H1)
  u32x4 m[R][NSB];                                     // super-block scales
  unsigned d[Q6 ? R : 1][Q6 ? NSB : 1];                // Q6_K super-block scale (fp16)
};

// the machine scheduler otherwise permutes independent loads; vmcnt retires in issue order, so a
// permutation makes the first consumer wait for (nearly) the whole tile
#define OMX_LOAD_ORDER() __builtin_amdgcn_sched_barrier(0)
// pieces are consumed in load order: VALU may not cross (hoisting a later piece's unpack would put
// its vmcnt wait first); LDS reads (activation fragments) and SALU may
#define OMX_PIECE_ORDER() __builtin_amdgcn_sched_barrier(0x0104)

template <int QT, int NSB, int R>
__device__ __forceinline__ void load_wtile(const QMat& w, long long row_base, int row0, int N, int SB, int sb0,
                                           int s, WTile<QT, NSB, R>& T, int se = -1) {
  if (se < 0) se = SB;  // lanes own super-blocks [sb0, se): an in-block K split ends a group's range early
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const long long row = row_base + min(row0 + r, N - 1);
#pragma unroll
    for (int i = 0; i < NSB; ++i) {
      const long long sb = min(sb0 + s + 16 * i, se - 1);  // clamped: padding lanes re-read, never use
      // issue order = consumption order: vmcnt retires loads in order, so the super-block scales go
      // first and each piece's operands together; otherwise the first dot product waits for the
      // wave's last load and no compute overlaps the stream
      if constexpr (QT == QT_Q8_0) {
        const uint8_t* q = w.s0 + row * SB * 256 + 32 * sb;
        T.m[r][i] = *(const u32x4*)(w.s1 + row * SB * 16 + 16 * sb);
        OMX_LOAD_ORDER();
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          T.a[r][i][t] = __builtin_nontemporal_load((const u32x4*)(q + 32LL * t * SB));
          T.b[r][i][t] = __builtin_nontemporal_load((const u32x4*)(q + 32LL * t * SB + 16));
          OMX_LOAD_ORDER();
        }
      } else if constexpr (QT == QT_Q6_K) {
        const uint8_t* q = w.s0 + row * SB * 128 + 16 * sb;
        const uint8_t* hq = w.s1 + row * SB * 64 + 8 * sb;
        T.m[r][i] = *(const u32x4*)(w.s2 + row * SB * 16 + 16 * sb);
        OMX_LOAD_ORDER();
        T.d[r][i] = *(const uint16_t*)(w.s3 + row * SB * 2 + 2 * sb);
        OMX_LOAD_ORDER();
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          T.a[r][i][t] = __builtin_nontemporal_load((const u32x4*)(q + 16LL * t * SB));
          T.h[r][i][t] = __builtin_nontemporal_load((const u32x2*)(hq + 8LL * t * SB));
          OMX_LOAD_ORDER();
        }
      } else {
        const uint8_t* q = w.s0 + row * SB * 128 + 16 * sb;
        T.m[r][i] = *(const u32x4*)(w.s1 + row * SB * 16 + 16 * sb);
        OMX_LOAD_ORDER();
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          T.a[r][i][t] = __builtin_nontemporal_load((const u32x4*)(q + 16LL * t * SB));
          OMX_LOAD_ORDER();
        }
      }
    }
  }
}

// x fragments of one piece for BT batch rows: int8 codes (lo/hi 16 groups) + {scale, sum}
template <int BT>
struct XFr {
  i32x4 lo[BT], hi[BT];
  f32x2 fl[BT], fh[BT];
};

template <int BT>
__device__ __forceinline__ void load_x(const i32x4* xq, const f32x2* xf, int XS, int slot_lo, int slot_hi,
                                       XFr<BT>& x) {
#pragma unroll
  for (int b = 0; b < BT; ++b) {
    x.lo[b] = xq[b * XS + slot_lo];
    x.hi[b] = xq[b * XS + slot_hi];
    x.fl[b] = xf[b * XS + slot_lo];
    x.fh[b] = xf[b * XS + slot_hi];
  }
}

template <int QT, int NSB, int R, int BT>
__device__ __forceinline__ void compute_wtile(const WTile<QT, NSB, R>& T, int SB, int sb0, int s, const i32x4* xq,
                                              const f32x2* xf, int XS, float (&acc)[R][BT], int se = -1) {
  if (se < 0) se = SB;
#pragma unroll
  for (int i = 0; i < NSB; ++i) {
    const int sb = sb0 + s + 16 * i;
    if (sb >= se) continue;
    const int xs0 = sb * XPAD;
    if constexpr (QT == QT_Q4_K) {
      // w = d*sc*n - dmin*m per 32-weight sub-block; lo nibbles: sub-block 2c, hi: 2c+1 (signed n-8)
      float d[R], dm[R];
      unsigned sl[R], ml[R], sh[R], mh[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const u32x4 m = T.m[r][i];
        d[r] = f16lo(m.x);
        dm[r] = f16hi(m.x);
        sl[r] = m.y & 0x3F3F3F3Fu;                                  // scales 0..3
        ml[r] = m.z & 0x3F3F3F3Fu;                                  // mins 0..3
        sh[r] = (m.w & 0x0F0F0F0Fu) | ((m.y >> 2) & 0x30303030u);  // scales 4..7
        mh[r] = ((m.w >> 4) & 0x0F0F0F0Fu) | ((m.z >> 2) & 0x30303030u);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float fsl[R], fml[R], fsh[R], gh[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const unsigned S = c < 2 ? sl[r] : sh[r], M = c < 2 ? ml[r] : mh[r];
          const int k0 = (2 * c) & 3, k1 = (2 * c + 1) & 3;
          const float s1 = ubyte(S, k1);
          fsl[r] = d[r] * ubyte(S, k0);
          fml[r] = dm[r] * ubyte(M, k0);
          fsh[r] = (0.0625f * d[r]) * s1;
          gh[r] = 8.f * d[r] * s1 - dm[r] * ubyte(M, k1);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int t = 2 * c + h, gl = 4 * c + h;
          XFr<BT> x;
          load_x<BT>(xq, xf, XS, xs0 + gl, xs0 + gl + 2, x);
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const u32x4 a = T.a[r][i][t];
            const u32x4 lo = a & 0x0F0F0F0Fu, hi = a & 0xF0F0F0F0u;
#pragma unroll
            for (int b = 0; b < BT; ++b) {
              const float il = (float)dot16(lo, x.lo[b]), ih = (float)dot16(hi, x.hi[b]);
              acc[r][b] += fsl[r] * (x.fl[b].x * il) + fsh[r] * (x.fh[b].x * ih) - fml[r] * x.fl[b].y +
                           gh[r] * x.fh[b].y;
            }
          }
          OMX_PIECE_ORDER();
        }
      }
    } else if constexpr (QT == QT_Q6_K) {
      // w = d*sc*(q - 32); q = ql nibble | (2 high bits << 4)
      float dq[R];
#pragma unroll
      for (int r = 0; r < R; ++r) dq[r] = h2f((uint16_t)T.d[r][i]);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int n = t >> 2, sub = t & 3, il_ = 8 * n + sub, ih_ = il_ + 4;
        XFr<BT> x;
        load_x<BT>(xq, xf, XS, xs0 + il_, xs0 + ih_, x);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const u32x4 m = T.m[r][i];
          const float fl = dq[r] * sbyte(m[il_ >> 2], il_ & 3), fh = dq[r] * sbyte(m[ih_ >> 2], ih_ & 3);
          const u32x4 a = T.a[r][i][t];
          const u32x2 H = T.h[r][i][t];
          u32x4 lo, hi;
          lo.x = (a.x & 0x0F0F0F0Fu) | ((H.x << 4) & 0x30303030u);
          lo.y = (a.y & 0x0F0F0F0Fu) | ((H.x << 2) & 0x30303030u);
          lo.z = (a.z & 0x0F0F0F0Fu) | (H.x & 0x30303030u);
          lo.w = (a.w & 0x0F0F0F0Fu) | ((H.x >> 2) & 0x30303030u);
          hi.x = ((a.x >> 4) & 0x0F0F0F0Fu) | ((H.y << 4) & 0x30303030u);
          hi.y = ((a.y >> 4) & 0x0F0F0F0Fu) | ((H.y << 2) & 0x30303030u);
          hi.z = ((a.z >> 4) & 0x0F0F0F0Fu) | (H.y & 0x30303030u);
          hi.w = ((a.w >> 4) & 0x0F0F0F0Fu) | ((H.y >> 2) & 0x30303030u);
#pragma unroll
          for (int b = 0; b < BT; ++b) {
            const float il = (float)dot16(lo, x.lo[b]), ih = (float)dot16(hi, x.hi[b]);
            acc[r][b] += fl * (x.fl[b].x * il - 32.f * x.fl[b].y) + fh * (x.fh[b].x * ih - 32.f * x.fh[b].y);
          }
        }
        OMX_PIECE_ORDER();
      }
    } else {
      // Q4_0: w = d*(n - 8), lo nibble unsigned, hi nibble signed; Q8_0: w = d*q
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        XFr<BT> x;
        load_x<BT>(xq, xf, XS, xs0 + 2 * t, xs0 + 2 * t + 1, x);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const unsigned dw = T.m[r][i][t >> 1];
          const float d = (t & 1) ? f16hi(dw) : f16lo(dw);
          const u32x4 a = T.a[r][i][t];
#pragma unroll
          for (int b = 0; b < BT; ++b) {
            if constexpr (QT == QT_Q4_0) {
              const float il = (float)dot16(a & 0x0F0F0F0Fu, x.lo[b]);
              const float ih = (float)dot16(a & 0xF0F0F0F0u, x.hi[b]);
              acc[r][b] += d * (x.fl[b].x * il - 8.f * x.fl[b].y + 0.0625f * x.fh[b].x * ih);
            } else {
              const float il = (float)dot16(a, x.lo[b]), ih = (float)dot16(T.b[r][i][t], x.hi[b]);
              acc[r][b] += d * (x.fl[b].x * il + x.fh[b].x * ih);
            }
          }
        }
        OMX_PIECE_ORDER();
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// activation prologue: x[b] (fp32) -> (norm) -> int8 groups of 16 in LDS (padded slots)
template <int NT>
__device__ void stage_x(const GemvParams& P, const float* x, int K, int SB, i32x4* lq, f32x2* lf, float* red) {
  float mean = 0.f, rstd = 1.f;
  if (P.norm != NORM_NONE) {
    float s = 0.f, ss = 0.f;
    for (int i = threadIdx.x; i < K / 4; i += NT) {
      const f32x4 v = *(const f32x4*)(x + 4 * i);
      s += v.x + v.y + v.z + v.w;
      ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    ss = block_sum<NT>(ss, red);
    if (P.norm == NORM_LAYER) {
      s = block_sum<NT>(s, red);
      mean = s / K;
      rstd = rsqrtf(fmaxf(ss / K - mean * mean, 0.f) + P.eps);
    } else {
      rstd = rsqrtf(ss / K + P.eps);
    }
  }
  for (int g = threadIdx.x; g < SB * 16; g += NT) {
    const int slot = (g >> 4) * XPAD + (g & 15);
    if (16 * g >= K) {  // K padding
      lq[slot] = (i32x4){0, 0, 0, 0};
      lf[slot] = (f32x2){0.f, 0.f};
      continue;
    }
    float v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 t = *(const f32x4*)(x + 16 * g + 4 * j);
      v[4 * j] = t.x; v[4 * j + 1] = t.y; v[4 * j + 2] = t.z; v[4 * j + 3] = t.w;
    }
    if (P.norm != NORM_NONE) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 w = *(const f32x4*)(P.norm_w + 16 * g + 4 * j);
        v[4 * j] = (v[4 * j] - mean) * rstd * w.x;
        v[4 * j + 1] = (v[4 * j + 1] - mean) * rstd * w.y;
        v[4 * j + 2] = (v[4 * j + 2] - mean) * rstd * w.z;
        v[4 * j + 3] = (v[4 * j + 3] - mean) * rstd * w.w;
      }
      if (P.norm == NORM_LAYER && P.norm_b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 bb = *(const f32x4*)(P.norm_b + 16 * g + 4 * j);
          v[4 * j] += bb.x; v[4 * j + 1] += bb.y; v[4 * j + 2] += bb.z; v[4 * j + 3] += bb.w;
        }
      }
    }
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) amax = fmaxf(amax, fabsf(v[j]));
    const float d = amax / 127.f;
    const float id = amax > 0.f ? 127.f / amax : 0.f;
    int q[16];
    int qsum = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      q[j] = (int)rintf(v[j] * id);
      qsum += q[j];
    }
    i32x4 pk;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      pk[j] = (q[4 * j] & 0xFF) | ((q[4 * j + 1] & 0xFF) << 8) | ((q[4 * j + 2] & 0xFF) << 16) |
              ((q[4 * j + 3] & 0xFF) << 24);
    lq[slot] = pk;
    lf[slot] = (f32x2){d, d * (float)qsum};
  }
}

// ---------------------------------------------------------------------------------------------
// row-group epilogue: reduce the 16 lanes, then lane s == r * BT + b writes (row0 + r, batch b)
template <int R, int BT>
__device__ __forceinline__ void finish_rows(const GemvParams& P, float (&acc)[R][BT], int row0, int N, int b0,
                                            int s) {
  float part[R][BT];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int b = 0; b < BT; ++b) acc[r][b] = row16_sum(acc[r][b]);
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int b = 0; b < BT; ++b) part[r][b] = R > 1 ? acc[r ^ 1][b] : __shfl_xor(acc[r][b], 16, OMX_WAVE);
#pragma unroll
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int b = 0; b < BT; ++b) {
      if (s != r * BT + b) continue;
      const int n = row0 + r;
      const int bb = b0 + b;
      if (n >= N || bb >= P.B) continue;
      epi_apply(P, bb, n + P.row_offset, acc[r][b], part[r][b], blockIdx.z);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Block = GEMV_NW waves x 4 row groups x R rows per tile. Work unit = (tile, K chunk of
// 16*NSB super-blocks); blocks are persistent over units (tile += gridDim.x).
// DBG (microbenchmark only, scripts/bench_gemv.py): bit 0 = replace the dot products by an XOR of
// the loaded words (memory path alone), bit 1 = skip the activation prologue
template <int QT, int NSB, int R, int BT, int DBG = 0>
__global__ __launch_bounds__(GEMV_NT) void qgemv_kernel(GemvParams P) {
  constexpr int PB = QT == QT_Q8_0 ? 8 : QT == QT_Q6_K ? 6 : 4;  // VGPRs per piece
  constexpr bool DB = R * NSB * (8 * PB + 5) <= 80;               // room for a prefetch tile
  constexpr int ROWS_W = 4 * R, ROWS_B = GEMV_NW * ROWS_W;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const QMat& w = P.w;
  const int K = w.K, N = w.N, SB = n_sb(K);
  const int XS = SB * XPAD;
  i32x4* lq = (i32x4*)smem;                         // [BT][XS]
  f32x2* lf = (f32x2*)(smem + (size_t)BT * XS * 16);  // [BT][XS]
  float* red = (float*)(lf + BT * XS);              // [NT/64]
  const int b0 = blockIdx.y * BT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, s = lane & 15;
  const int nc = (SB + 16 * NSB - 1) / (16 * NSB);
  const int n_tiles = (N + ROWS_B - 1) / ROWS_B;
  const int rbase = wave * ROWS_W + g * R;

  long long row_base = 0;
  const float* x = P.x;
  if (P.expert_ids) {  // MoE: blockIdx.z = k-th selected expert of batch row b0
    const int e = P.expert_ids[b0 * P.n_sel + blockIdx.z];
    row_base = (long long)e * N;
    if (P.x_per_sel) x = P.x + (long long)blockIdx.z * P.x_sel_stride;
  }

  int tile = blockIdx.x, c = 0;
  WTile<QT, NSB, R> A;
  if (tile < n_tiles) load_wtile<QT, NSB, R>(w, row_base, tile * ROWS_B + rbase, N, SB, 0, s, A);

#pragma unroll
  for (int b = 0; b < BT; ++b) {
    if (DBG & 2) break;
    if (b0 + b < P.B) {
      stage_x<GEMV_NT>(P, x + (long long)(b0 + b) * P.ldx, K, SB, lq + b * XS, lf + b * XS, red);
    } else {
      for (int i = threadIdx.x; i < XS; i += GEMV_NT) {
        lq[b * XS + i] = (i32x4){0, 0, 0, 0};
        lf[b * XS + i] = (f32x2){0.f, 0.f};
      }
    }
  }
  __syncthreads();

  float acc[R][BT];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int b = 0; b < BT; ++b) acc[r][b] = 0.f;
  auto finish = [&](int t) {
    finish_rows<R, BT>(P, acc, t * ROWS_B + rbase, N, b0, s);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int b = 0; b < BT; ++b) acc[r][b] = 0.f;
  };

  if constexpr (DB) {
    // explicit ping-pong (a register copy would force a vmcnt(0) drain every unit)
    WTile<QT, NSB, R> Bt;
    auto step = [&](WTile<QT, NSB, R>& cur, WTile<QT, NSB, R>& nxt) {
      int nt = tile, ncc = c + 1;
      if (ncc == nc) { ncc = 0; nt += gridDim.x; }
      if (nt < n_tiles) load_wtile<QT, NSB, R>(w, row_base, nt * ROWS_B + rbase, N, SB, ncc * 16 * NSB, s, nxt);
      if constexpr (DBG & 1) {
        unsigned v = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) v ^= cur.a[0][0][t].x ^ cur.a[0][0][t].w;
        acc[0][0] += (float)(v & 1);
      } else {
        compute_wtile<QT, NSB, R, BT>(cur, SB, c * 16 * NSB, s, lq, lf, XS, acc);
      }
      if (c == nc - 1) finish(tile);
      tile = nt;
      c = ncc;
    };
    while (tile < n_tiles) {
      step(A, Bt);
      if (tile >= n_tiles) break;
      step(Bt, A);
    }
  } else {
    while (tile < n_tiles) {
      compute_wtile<QT, NSB, R, BT>(A, SB, c * 16 * NSB, s, lq, lf, XS, acc);
      if (c == nc - 1) finish(tile);
      if (++c == nc) { c = 0; tile += gridDim.x; }
      if (tile < n_tiles) load_wtile<QT, NSB, R>(w, row_base, tile * ROWS_B + rbase, N, SB, c * 16 * NSB, s, A);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Decode kernel, "all in flight" (B = 1, one K chunk). scripts/bench_gemv.py DBG variants showed the
// persistent kernel above streams at the HBM ceiling only without its prologue and its dot products
// (gate_up 9.0 us vs 15.1 us): vector loads return in issue order, so the prologue's activation
// loads -- issued after the weight tiles -- waited for every tile, and the 2-deep register ping-pong
// then left HBM idle while tiles computed. Here each thread first loads its activation groups (and
// norm weights) into registers, THEN issues the loads of all J weight tiles of its block, computes
// the norm + int8 quantisation from registers while the weights stream, and consumes the tiles in
// order with counted vmcnt waits (fully unrolled), so HBM sees the whole matrix requested up front.
// NRM: 0 = no norm (only x is loaded), 1 = RMSNorm (x, w), 2 = LayerNorm (x, w, b). Stand-in loads
// for absent norm operands would spend the wave's 63-deep vmcnt budget (NSB = 3: 69 loads per lane).
// KS > 1 (matrices with few row tiles, e.g. the K = 11008 down projection: 256 tiles = one 4-wave
// block per CU): the block has KS groups of GEMV_NW waves on the same rows, group kg owning the
// super-block range [kg*CH, (kg+1)*CH); partial sums meet in LDS before the epilogue. More waves per
// CU = more weight bytes in flight.
// MRG > 0 (B == 1 decode, O projection): x holds MRG unmerged flash-decode partial slabs
// (attention.hip `defer`); the prologue merges them per head in registers -- the merge rides on the
// activation round trip this kernel pays anyway, instead of an in-launch ticket + re-read (~2.5 us).
template <int QT, int NSB, int R, int J, int NRM, int DBG = 0, int KS = 1, int MRG = 0>
__device__ __forceinline__ void flight_body(const GemvParams& P, const int bx, const int gxn) {
  constexpr int ROWS_B = GEMV_NW * 4 * R, NT = GEMV_NT * KS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const QMat& w = P.w;
  auto stamp = [&](int k) {
    if (P.dbg_ts && threadIdx.x == 0)
      P.dbg_ts[4 * ((long long)blockIdx.z * gxn + bx) + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  const int K = w.K, N = w.N, SB = n_sb(K);
  const int XS = SB * XPAD;
  i32x4* lq = (i32x4*)smem;                           // [XS + 1]: slot XS is a dummy
  f32x2* lf = (f32x2*)(smem + (size_t)(XS + 1) * 16);  // [XS + 1]
  float* red = (float*)(lf + XS + 1);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, s = lane & 15;
  const int kg = KS > 1 ? wave / GEMV_NW : 0, gtid = tid - kg * GEMV_NT;
  const int CH = KS > 1 ? (SB + KS - 1) / KS : SB;
  const int sb0 = kg * CH, se = min(SB, sb0 + CH);
  const int n_tiles = (N + ROWS_B - 1) / ROWS_B;
  const int rbase = (wave - kg * GEMV_NW) * (4 * R) + g * R;

  long long row_base = 0;
  const float* x = P.x;
  if (P.expert_ids) {  // MoE: blockIdx.z = k-th selected expert
    const int e = P.expert_ids[blockIdx.z];
    row_base = (long long)e * N;
    if (P.x_per_sel) x = P.x + (long long)blockIdx.z * P.x_sel_stride;
  }

  // 1. this thread's activation groups g = tid + NT i (i < NSB) and norm weights -> registers
  constexpr bool nrm = NRM != 0, lnb = NRM == 2;
  f32x4 xv[NSB][4], nw[NSB][4], nb[NSB][4];
  constexpr int MS = MRG > 0 ? MRG : 1;
  f32x4 av[MS][NSB][4];
  f32x2 ml[MS][NSB];
  // unconditional loads from clamped addresses (a conditional load would make the compiler drain it
  // before the weight loads are issued); out-of-range values are masked at use
#pragma unroll
  for (int i = 0; i < NSB; ++i) {
    const int gi = min(tid + NT * i, K / 16 - 1);
    if constexpr (MRG > 0) {
      const int h = 16 * gi / P.merge_D, nh = K / P.merge_D;
#pragma unroll
      for (int sp = 0; sp < MRG; ++sp) {
        ml[sp][i] = *(const f32x2*)(P.merge_ml + 2 * (sp * nh + h));
#pragma unroll
        for (int j = 0; j < 4; ++j) av[sp][i][j] = *(const f32x4*)(x + (long long)sp * K + 16 * gi + 4 * j);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (MRG == 0) xv[i][j] = *(const f32x4*)(x + 16 * gi + 4 * j);
      if constexpr (nrm) nw[i][j] = *(const f32x4*)(P.norm_w + 16 * gi + 4 * j);
      if constexpr (lnb) nb[i][j] = *(const f32x4*)(P.norm_b + 16 * gi + 4 * j);
    }
  }
  __builtin_amdgcn_sched_barrier(0);  // activations ahead of the weights
  if constexpr ((DBG & 4) != 0) __builtin_amdgcn_s_barrier();  // every wave's x requests queued first
  // x-first (GemvTuning::xfirst): wait for the activations BEFORE requesting any weight. The x lines
  // were just written by the previous kernel and miss L2; issued behind the whole matrix's requests
  // they return only after most of the weight stream (profiles/r1_defer/gemv_timeline.log: prologue
  // p50 4.6-8.3 us on the down projections), so every tile waits on them.
  if (P.xfirst) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  // 2. every weight tile of this block in flight (surplus slots re-read the last tile, unused)
  WTile<QT, NSB, R> T[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int t = min(bx + j * gxn, n_tiles - 1);
    load_wtile<QT, NSB, R>(w, row_base, t * ROWS_B + rbase, N, SB, sb0, s, T[j], se);
  }
  __builtin_amdgcn_sched_barrier(0);  // every load issued before the prologue's first wait
  if constexpr (MRG > 0) {  // flash-decode merge: splits without keys carry m = -inf, l = 0
#pragma unroll
    for (int i = 0; i < NSB; ++i) {
      float M = -INFINITY;
#pragma unroll
      for (int sp = 0; sp < MRG; ++sp) M = fmaxf(M, ml[sp][i].x);
      float L = 0.f;
      f32x4 a[4] = {};
#pragma unroll
      for (int sp = 0; sp < MRG; ++sp) {
        const float c = ml[sp][i].x == -INFINITY ? 0.f : __expf(ml[sp][i].x - M);
        L += c * ml[sp][i].y;
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] += c * av[sp][i][j];
      }
      const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[i][j] = a[j] * inv;
    }
  }
  // 3. norm statistics + quantisation from registers while the weights stream
#pragma unroll
  for (int i = 0; i < NSB; ++i) {
    const bool ok = 16 * (tid + NT * i) < K;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!ok) xv[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if constexpr (!nrm) nw[i][j] = (f32x4){1.f, 1.f, 1.f, 1.f};
      if constexpr (!lnb) nb[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  }
  float mean = 0.f, rstd = 1.f;
  if (nrm && !(DBG & 2)) {
    float sm = 0.f, ss = 0.f;
#pragma unroll
    for (int i = 0; i < NSB; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 v = xv[i][j];
        sm += v.x + v.y + v.z + v.w;
        ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      }
    ss = block_sum<NT>(ss, red);
    if (NRM == 2 || P.norm == NORM_LAYER) {
      sm = block_sum<NT>(sm, red);
      mean = sm / K;
      rstd = rsqrtf(fmaxf(ss / K - mean * mean, 0.f) + P.eps);
    } else {
      rstd = rsqrtf(ss / K + P.eps);
    }
  }
#pragma unroll
  for (int i = 0; i < NSB; ++i) {
    if constexpr (DBG & 2) continue;
    const int gi = tid + NT * i;
    // branch-free: surplus threads store to the dummy slot (a guarded block lets the compiler sink
    // the activation loads behind the weight loads, then drain them all with vmcnt(0))
    const int slot = gi < SB * 16 ? (gi >> 4) * XPAD + (gi & 15) : XS;
    float v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 t = xv[i][j];
      if (nrm) t = (t - mean) * rstd * nw[i][j] + nb[i][j];
      v[4 * j] = t.x; v[4 * j + 1] = t.y; v[4 * j + 2] = t.z; v[4 * j + 3] = t.w;
    }
    if (16 * gi >= K) {
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = 0.f;
    }
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
  __syncthreads();
  stamp(1);
  if constexpr (KS > 1) {  // one tile per block: groups 1.. hand their partial sums to group 0
    static_assert(J == 1, "in-block K split is for single-tile blocks");
    float acc[R][1];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = 0.f;
    if constexpr (DBG & 1) {
      unsigned v = 0;
#pragma unroll
      for (int i = 0; i < NSB; ++i)
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) v ^= T[0].a[0][i][tt].x ^ T[0].a[0][i][tt].w ^ T[0].m[0][i].y;
      acc[0][0] = (float)(v & 1);
    } else {
      compute_wtile<QT, NSB, R, 1>(T[0], SB, sb0, s, lq, lf, XS, acc, se);
    }
    stamp(2);
    float* part = red + NT / 64;  // [KS-1][R][GEMV_NT]
    if (kg > 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) part[((kg - 1) * R + r) * GEMV_NT + gtid] = acc[r][0];
    }
    __syncthreads();
    if (kg == 0 && bx < n_tiles) {
#pragma unroll
      for (int k = 1; k < KS; ++k)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][0] += part[((k - 1) * R + r) * GEMV_NT + gtid];
      finish_rows<R, 1>(P, acc, bx * ROWS_B + rbase, N, 0, s);
    }
    stamp(3);
    return;
  }
  // 4. consume the tiles in issue order
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int t = bx + j * gxn;
    if (t >= n_tiles) break;  // block-uniform
    float acc[R][1];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = 0.f;
    if constexpr (DBG & 1) {  // memory path only: consume every loaded word, no dot products
      unsigned v = 0;
#pragma unroll
      for (int i = 0; i < NSB; ++i)
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) {
          v ^= T[j].a[0][i][tt].x ^ T[j].a[0][i][tt].w ^ T[j].m[0][i].y;
          if constexpr (QT == QT_Q6_K) v ^= T[j].h[0][i][tt].x;
        }
      acc[0][0] = (float)(v & 1);
    } else {
      compute_wtile<QT, NSB, R, 1>(T[j], SB, 0, s, lq, lf, XS, acc);
    }
    if (j == 0) stamp(2);
    finish_rows<R, 1>(P, acc, t * ROWS_B + rbase, N, 0, s);
  }
  stamp(3);
}

template <int QT, int NSB, int R, int J, int NRM, int DBG = 0, int KS = 1, int MRG = 0>
__global__ __launch_bounds__(GEMV_NT * KS) void qgemv_flight_kernel(GemvParams P) {
  flight_body<QT, NSB, R, J, NRM, DBG, KS, MRG>(P, blockIdx.x, gridDim.x);
}

// two matrices that read the same normalised x in ONE launch (Q4_K_M QKV: q,k rows Q4_K + v rows
// Q6_K): blocks [0, gxa) run A, the rest B -- one launch ramp / drain instead of two (v alone was
// 6.3 us for 13.8 MB, rocprofv3 profiles/r1_defer)
template <int QA, int QB, int NSB, int NRM>
__global__ __launch_bounds__(GEMV_NT) void qgemv_flight_dual_kernel(GemvParams PA, GemvParams PB, int gxa) {
  if ((int)blockIdx.x < gxa) flight_body<QA, NSB, 1, 1, NRM>(PA, blockIdx.x, gxa);
  else flight_body<QB, NSB, 1, 1, NRM>(PB, (int)blockIdx.x - gxa, (int)gridDim.x - gxa);
}

// register tiles a block keeps in flight: ~150 VGPRs of weight tiles per lane
template <int QT, int NSB, int R>
constexpr int flight_jmax() {
  constexpr int PB = QT == QT_Q8_0 ? 8 : QT == QT_Q6_K ? 6 : 4;
  constexpr int regs = R * NSB * (8 * PB + 5);
  return regs * 3 <= 150 ? 3 : regs * 2 <= 150 ? 2 : 1;
}

static size_t lds_bytes(int K, int BT) { return (size_t)BT * ((K + 255) / 256) * XPAD * 24 + 24 + 4 * GEMV_NW; }
// flight kernel with an in-block K split: activation slots + reduction slots + partial sums
static size_t lds_bytes_ks(int K, int KS, int R) {
  return (size_t)((K + 255) / 256) * XPAD * 24 + 24 + 4 * GEMV_NW * KS + (size_t)4 * (KS - 1) * R * GEMV_NT;
}

template <int QT, int NSB, int R, int BT, int DBG = 0>
static void launch_t(const GemvParams& P, hipStream_t s) {
  const int N = P.w.N;
  const int tiles = (N + 4 * GEMV_NW * R - 1) / (4 * GEMV_NW * R);
  const int by = (P.B + BT - 1) / BT;
  const int bz = P.expert_ids ? P.n_sel : 1;
  int gx = tiles;
  const int slots = 256 * g_tune.blocks_per_cu;
  const int cap = slots / (by * bz) > 0 ? slots / (by * bz) : 1;
  if (gx > cap) gx = cap;
  hipLaunchKernelGGL((qgemv_kernel<QT, NSB, R, BT, DBG>), dim3(gx, by, bz), dim3(GEMV_NT), lds_bytes(P.w.K, BT), s, P);
}

template <int QT, int NSB, int R, int J, int NRM>
static void launch_flight_n(const GemvParams& P, int gx, hipStream_t s) {
  const int bz = P.expert_ids ? P.n_sel : 1;
  const size_t lds = lds_bytes(P.w.K, 1);
  if constexpr (NSB == 1 && R == 1 && NRM == 0) {
    switch (P.merge_S) {  // deferred flash-decode merge in the prologue (O projection)
      case 0: break;
      case 2: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 0, 1, 2>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      case 4: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 0, 1, 4>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      case 8: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 0, 1, 8>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      default: return;  // rejected by gemv() before launch
    }
  }
  if constexpr (R == 1 && (QT == QT_Q4_K || QT == QT_Q6_K) && (NSB == 1 || NSB == 3) && NRM < 2) {
    switch (g_tune.debug) {  // microbenchmark-only variants (scripts/bench_gemv.py OMX_BENCH_DEBUG)
      case 1: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 1>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      case 2: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 2>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      case 3: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 3>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      case 4: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 4>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      default: break;
    }
  }
  hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P);
}

template <int QT, int NSB, int KS, int NRM>
static void launch_flight_ks_n(const GemvParams& P, int gx, hipStream_t s) {
  const int bz = P.expert_ids ? P.n_sel : 1;
  const size_t lds = lds_bytes_ks(P.w.K, KS, 1);
  if constexpr ((QT == QT_Q4_K || QT == QT_Q6_K) && NRM == 0) {
    switch (g_tune.debug) {  // microbenchmark-only variants, as launch_flight_n
      case 1: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, 1, 1, NRM, 1, KS>), dim3(gx, 1, bz), dim3(GEMV_NT * KS), lds, s, P); return;
      case 2: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, 1, 1, NRM, 2, KS>), dim3(gx, 1, bz), dim3(GEMV_NT * KS), lds, s, P); return;
      case 3: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, 1, 1, NRM, 3, KS>), dim3(gx, 1, bz), dim3(GEMV_NT * KS), lds, s, P); return;
      case 4: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, 1, 1, NRM, 4, KS>), dim3(gx, 1, bz), dim3(GEMV_NT * KS), lds, s, P); return;
      default: break;
    }
  }
  hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, 1, 1, NRM, 0, KS>), dim3(gx, 1, bz), dim3(GEMV_NT * KS), lds, s, P);
}

template <int QT, int NSB, int R, int J>
static void launch_flight_j(const GemvParams& P, int gx, hipStream_t s) {
  if (P.norm == NORM_NONE) launch_flight_n<QT, NSB, R, J, 0>(P, gx, s);
  else if (P.norm == NORM_LAYER && P.norm_b) launch_flight_n<QT, NSB, R, J, 2>(P, gx, s);
  else launch_flight_n<QT, NSB, R, J, 1>(P, gx, s);
}

// grid: at least one block per CU while the matrix has the tiles, then up to J tiles per block
// in-block K split for single-row-tile matrices: KS groups of 4 waves, each NSB' = ceil(need / KS)
static int flight_ks(int need, int tiles, int bz) {
  if (g_tune.ks > 0) return g_tune.ks;
  // K <= 4096 (need 1): a split leaves half of every row group's lanes idle and doubles the VALU
  // work (measured: O 4.4 -> 5.0 us, V Q6_K 5.0 -> 7.8 us); enough tiles fill the CUs anyway
  if (need < 2 || tiles * bz > 256 * 2) return 1;
  return need >= 3 ? 3 : 2;
}

// VGPRs a K-split flight instantiation needs (weight tile + activation / norm registers + ~24 of
// addressing and accumulators) against the 512 / KS per lane that KS waves per SIMD leave. Calibrated
// on the built code objects (tests/test_isa.py): the two Q8_0 LayerNorm variants above budget
// (KS = 4 NSB = 1, KS = 2 NSB = 2) were the only ones spilling to scratch.
template <int QT, int NSB, int KS, int NRM>
constexpr bool flight_ks_fits() {
  constexpr int PB = QT == QT_Q8_0 ? 8 : QT == QT_Q6_K ? 6 : QT == QT_Q5_K ? 5 : 4;
  return NSB * (8 * PB + 5) + NSB * 16 * (1 + (NRM != 0) + (NRM == 2)) + 24 <= 512 / KS;
}

template <int QT, int NSB, int KS>
static bool launch_flight_ks_fit(const GemvParams& P, int gx, hipStream_t s) {
  const int nrm = P.norm == NORM_NONE ? 0 : (P.norm == NORM_LAYER && P.norm_b) ? 2 : 1;
  if (nrm == 0) {
    if constexpr (flight_ks_fits<QT, NSB, KS, 0>()) { launch_flight_ks_n<QT, NSB, KS, 0>(P, gx, s); return true; }
  } else if (nrm == 1) {
    if constexpr (flight_ks_fits<QT, NSB, KS, 1>()) { launch_flight_ks_n<QT, NSB, KS, 1>(P, gx, s); return true; }
  } else {
    if constexpr (flight_ks_fits<QT, NSB, KS, 2>()) { launch_flight_ks_n<QT, NSB, KS, 2>(P, gx, s); return true; }
  }
  return false;  // the variant would spill: the caller takes the unsplit kernel
}

template <int QT>
static bool launch_flight_split(const GemvParams& P, int need, hipStream_t s) {
  const int tiles = (P.w.N + 4 * GEMV_NW - 1) / (4 * GEMV_NW);
  const int bz = P.expert_ids ? P.n_sel : 1;
  const int ks = flight_ks(need, tiles, bz);
  if (ks <= 1) return false;
  const int nsb = (need + ks - 1) / ks;  // 16 * nsb >= ceil(SB / ks)
  if (ks == 2 && nsb == 1) return launch_flight_ks_fit<QT, 1, 2>(P, tiles, s);
  if (ks == 2 && nsb == 2) return launch_flight_ks_fit<QT, 2, 2>(P, tiles, s);
  if (ks == 3 && nsb == 1) return launch_flight_ks_fit<QT, 1, 3>(P, tiles, s);
  if (ks == 4 && nsb == 1) return launch_flight_ks_fit<QT, 1, 4>(P, tiles, s);
  return false;
}

template <int QT, int NSB, int R>
static void launch_flight(const GemvParams& P, hipStream_t s) {
  constexpr int JM = flight_jmax<QT, NSB, R>();
  const int tiles = (P.w.N + 4 * GEMV_NW * R - 1) / (4 * GEMV_NW * R);
  const int bz = P.expert_ids ? P.n_sel : 1;
  const int want = (256 * g_tune.blocks_per_cu + bz - 1) / bz;  // blocks per (z) slice
  int J = (tiles + want - 1) / want;
  J = J < 1 ? 1 : J > JM ? JM : J;
  const int gx = (tiles + J - 1) / J;
  if (J == 1) launch_flight_j<QT, NSB, R, 1>(P, gx, s);
  else if (J == 2) launch_flight_j<QT, NSB, R, (JM >= 2 ? 2 : 1)>(P, gx, s);
  else launch_flight_j<QT, NSB, R, JM>(P, gx, s);
}

template <int QT, int R, int BT>
static void launch_nsb(const GemvParams& P, hipStream_t s) {
  const int SB = (P.w.K + 255) / 256;
  const int need = (SB + 15) / 16;
  if constexpr (R == 2) {  // two rows per group only while both register tiles stay resident
    if (need == 1) launch_t<QT, 1, 2, BT>(P, s);
    else if (need == 2) launch_t<QT, 2, 2, BT>(P, s);
    else launch_nsb<QT, 1, BT>(P, s);
    return;
  } else {
    switch (need) {
      case 1: launch_t<QT, 1, R, BT>(P, s); return;
      case 2: launch_t<QT, 2, R, BT>(P, s); return;
      case 3: launch_t<QT, 3, R, BT>(P, s); return;
      default: launch_t<QT, 4, R, BT>(P, s); return;  // K > 12288: chunks of 64 super-blocks
    }
  }
}

template <int QT>
static void launch_q(const GemvParams& P, hipStream_t s) {
  if (P.merge_S > 0) {  // only the single-chunk B == 1 flight kernel merges (merge_supported())
    launch_flight<QT, 1, 1>(P, s);
    return;
  }
  if (P.B == 1 || P.expert_ids != nullptr) {  // decode (and MoE: experts differ per batch row)
    const int need = ((P.w.K + 255) / 256 + 15) / 16;
    if (P.B == 1 && need <= 4) {  // whole K in one chunk: all-in-flight kernel
      if (g_tune.rows == 2 && need == 1) { launch_flight<QT, 1, 2>(P, s); return; }
      if (launch_flight_split<QT>(P, need, s)) return;
      switch (need) {
        case 1: launch_flight<QT, 1, 1>(P, s); return;
        case 2: launch_flight<QT, 2, 1>(P, s); return;
        case 3: launch_flight<QT, 3, 1>(P, s); return;
        default: launch_flight<QT, 4, 1>(P, s); return;
      }
    }
    if (g_tune.rows == 2) launch_nsb<QT, 2, 1>(P, s);
    else launch_nsb<QT, 1, 1>(P, s);
    return;
  }
  // batch tiles: the weights are unpacked once per piece and dotted against BT activation rows;
  // BT bounded by the LDS the staged activations take
  if (lds_bytes(P.w.K, 4) <= 96 * 1024) launch_nsb<QT, 1, 4>(P, s);
  else if (lds_bytes(P.w.K, 2) <= 120 * 1024) launch_nsb<QT, 1, 2>(P, s);
  else launch_nsb<QT, 1, 1>(P, s);
}

template <int QA, int QB, int NSB>
static void launch_dual_n(const GemvParams& A, const GemvParams& Bp, hipStream_t s) {
  const int ta = (A.w.N + 4 * GEMV_NW - 1) / (4 * GEMV_NW), tb = (Bp.w.N + 4 * GEMV_NW - 1) / (4 * GEMV_NW);
  hipLaunchKernelGGL((qgemv_flight_dual_kernel<QA, QB, NSB, 1>), dim3(ta + tb), dim3(GEMV_NT), lds_bytes(A.w.K, 1),
                     s, A, Bp, ta);
}

template <int QA, int QB>
static void launch_dual_q(const GemvParams& A, const GemvParams& Bp, int need, hipStream_t s) {
  if (need == 1) launch_dual_n<QA, QB, 1>(A, Bp, s);
  else launch_dual_n<QA, QB, 2>(A, Bp, s);
}

template <int QA>
static bool launch_dual_a(const GemvParams& A, const GemvParams& Bp, int need, hipStream_t s) {
  switch (Bp.w.qtype) {
    case QT_Q4_K: if (QA != QT_Q4_K) { launch_dual_q<QA, QT_Q4_K>(A, Bp, need, s); return true; } break;
    case QT_Q6_K: if (QA != QT_Q6_K) { launch_dual_q<QA, QT_Q6_K>(A, Bp, need, s); return true; } break;
    case QT_Q4_0: if (QA != QT_Q4_0) { launch_dual_q<QA, QT_Q4_0>(A, Bp, need, s); return true; } break;
    case QT_Q8_0: if (QA != QT_Q8_0) { launch_dual_q<QA, QT_Q8_0>(A, Bp, need, s); return true; } break;
    default: break;
  }
  return false;
}

void gemv2(const GemvParams& A0, const GemvParams& B0, hipStream_t s) {
  GemvParams A = A0, Bp = B0;
  A.xfirst = Bp.xfirst = g_tune.xfirst;
  const int need = ((A.w.K + 255) / 256 + 15) / 16;
  const bool ok = A.B == 1 && Bp.B == 1 && A.w.K == Bp.w.K && need <= 2 && A.norm == NORM_RMS &&
                  Bp.norm == NORM_RMS && !A.expert_ids && !Bp.expert_ids && !A.merge_S && !Bp.merge_S &&
                  A.x == Bp.x && g_tune.debug == 0;
  if (ok) {
    bool done = false;
    switch (A.w.qtype) {
      case QT_Q4_K: done = launch_dual_a<QT_Q4_K>(A, Bp, need, s); break;
      case QT_Q6_K: done = launch_dual_a<QT_Q6_K>(A, Bp, need, s); break;
      case QT_Q4_0: done = launch_dual_a<QT_Q4_0>(A, Bp, need, s); break;
      case QT_Q8_0: done = launch_dual_a<QT_Q8_0>(A, Bp, need, s); break;
      default: break;
    }
    if (done) return;
  }
  gemv(A, s);
  gemv(Bp, s);
}

bool gemv_merge_supported(int B, int K, int D, int S) {
  return B == 1 && K <= 4096 && D % 16 == 0 && K % D == 0 && (S == 2 || S == 4 || S == 8);
}

void gemv(const GemvParams& P0, hipStream_t s) {
  GemvParams P = P0;
  P.xfirst = g_tune.xfirst;
  if (P.merge_S > 0) {
    // flight grid for K <= 4096 is one chunk, R = 1, no K split: the merge variant covers exactly it
    if (!gemv_merge_supported(P.B, P.w.K, P.merge_D, P.merge_S) || P.norm != NORM_NONE || P.expert_ids) return;
  }
  if (gemm_eligible(P)) {
    gemm(P, s);
    return;
  }
  switch (P.w.qtype) {
    case QT_Q4_K: launch_q<QT_Q4_K>(P, s); break;
    case QT_Q6_K: launch_q<QT_Q6_K>(P, s); break;
    case QT_Q4_0: launch_q<QT_Q4_0>(P, s); break;
    case QT_Q8_0: launch_q<QT_Q8_0>(P, s); break;
    default: break;
  }
}

}  // namespace omx
