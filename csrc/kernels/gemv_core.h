// Device building blocks of the quantised GEMV kernels: weight register tiles (layout v2), the
// int8 activation prologue, per-piece dot products and the row-group epilogue. Shared by gemv.hip
// (B == 1 decode, persistent kernel) and gemv_batch.hip (continuous-batching rows).
#pragma once
#include "common.h"
#include "epilogue.h"
#include "ops.h"

namespace omx {

constexpr int GEMV_NW = 4;  // waves per block (8-wave blocks measured slower: profiles/r1_pmc)
constexpr int GEMV_NT = 64 * GEMV_NW;
constexpr int XPAD = 17;      // LDS x slots per super-block: 16 groups + 1 pad

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
  static constexpr bool Q8 = QT == QT_Q8_0 || QT == QT_Q6_K8, Q6 = QT == QT_Q6_K, Q5 = QT == QT_Q5_K;
  static constexpr bool Q6D = QT == QT_Q6_K || QT == QT_Q6_K8;  // fp16 super-block scale
  u32x4 a[R][NSB][8];                                  // qs / ql / Q8_0 first 16 B
  u32x4 b[Q8 ? R : 1][Q8 ? NSB : 1][8];                // Q8_0 second 16 B
  u32x2 h[Q6 ? R : 1][Q6 ? NSB : 1][8];                // Q6_K high bits (H0 | H1)
  unsigned q5h[Q5 ? R : 1][Q5 ? NSB : 1][8];           // Q5_K 5th bits (one dword per piece)
  u32x4 m[R][NSB];                                     // super-block scales
  unsigned d[Q6D ? R : 1][Q6D ? NSB : 1];              // Q6_K super-block scale (fp16)
};

// the machine scheduler otherwise permutes independent loads; vmcnt retires in issue order, so a
// permutation makes the first consumer wait for (nearly) the whole tile
#define OMX_LOAD_ORDER() __builtin_amdgcn_sched_barrier(0)
// pieces are consumed in load order: VALU may not cross (hoisting a later piece's unpack would put
// its vmcnt wait first); LDS reads (activation fragments) and SALU may
#define OMX_PIECE_ORDER() __builtin_amdgcn_sched_barrier(0x0104)

// A sched_barrier only binds the machine scheduler: the SelectionDAG scheduler that runs before it
// still hoists pure VALU across it, and did -- the disassembly of the K-split down GEMV showed every
// piece's nibble masks hoisted to the top of the tile, behind ONE s_waitcnt vmcnt(0), so no dot
// product started before the block's last weight byte had landed (Q6_K: vmcnt(3) after piece 0).
// pin() redefines a loaded register through an empty volatile asm at the point where its piece is
// consumed: volatile asm statements keep program order, nothing that reads the value can move above
// its pin, and the waitcnt pass places that load's (counted) vmcnt wait right there.
__device__ __forceinline__ void pin(u32x4& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(u32x2& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(unsigned& v) { asm volatile("" : "+v"(v)); }

template <int QT, int NSB, int R>
__device__ __forceinline__ void load_wtile(const QMat& w, long long row_base, int row0, int N, int SB, int sb0,
                                           int s, WTile<QT, NSB, R>& T, int se = -1) {
  if (se < 0) se = SB;  // lanes own super-blocks [sb0, se): an in-block K split ends a group's range early
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const long long row = row_base + min(row0 + r, N - 1);
    OMX_KASSERT(row >= 0 && sb0 + s < SB + 16 * NSB);
#pragma unroll
    for (int i = 0; i < NSB; ++i) {
      const long long sb = min(sb0 + s + 16 * i, se - 1);  // clamped: padding lanes re-read, never use
      // issue order = consumption order: vmcnt retires loads in order, so the super-block scales go
      // first and each piece's operands together; otherwise the first dot product waits for the
      // wave's last load and no compute overlaps the stream
      if constexpr (QT == QT_Q6_K8) {
        const uint8_t* q = w.s4 + row * SB * 256 + 32 * sb;
        T.m[r][i] = *(const u32x4*)(w.s2 + row * SB * 16 + 16 * sb);
        OMX_LOAD_ORDER();
        T.d[r][i] = *(const uint16_t*)(w.s3 + row * SB * 2 + 2 * sb);
        OMX_LOAD_ORDER();
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          T.a[r][i][t] = __builtin_nontemporal_load((const u32x4*)(q + 32LL * t * SB));
          T.b[r][i][t] = __builtin_nontemporal_load((const u32x4*)(q + 32LL * t * SB + 16));
          OMX_LOAD_ORDER();
        }
      } else if constexpr (QT == QT_Q8_0) {
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
      } else if constexpr (QT == QT_Q5_K) {
        const uint8_t* q = w.s0 + row * SB * 128 + 16 * sb;
        const uint8_t* hq = w.s2 + row * SB * 32 + 4 * sb;
        T.m[r][i] = *(const u32x4*)(w.s1 + row * SB * 16 + 16 * sb);
        OMX_LOAD_ORDER();
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          T.a[r][i][t] = __builtin_nontemporal_load((const u32x4*)(q + 16LL * t * SB));
          T.q5h[r][i][t] = __builtin_nontemporal_load((const unsigned*)(hq + 4LL * t * SB));
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

// PIN: pin each piece where it is consumed (see pin()); off for the register-heaviest instantiations
// (many batch rows x tiles in flight), where holding every piece until its turn spills
template <int QT, int NSB, int R, int BT, bool PIN = true>
__device__ __forceinline__ void compute_wtile(WTile<QT, NSB, R>& T, int SB, int sb0, int s, const i32x4* xq,
                                              const f32x2* xf, int XS, float (&acc)[R][BT], int se = -1) {
  if (se < 0) se = SB;
  // piece t of super-block i: its weight registers, pinned where the piece is consumed (see pin())
  auto pin_piece = [&](int i, int t) {
    if constexpr (!PIN) return;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      pin(T.a[r][i][t]);
      if constexpr (WTile<QT, NSB, R>::Q8) pin(T.b[r][i][t]);
      if constexpr (WTile<QT, NSB, R>::Q6) pin(T.h[r][i][t]);
      if constexpr (WTile<QT, NSB, R>::Q5) pin(T.q5h[r][i][t]);
    }
  };
#pragma unroll
  for (int i = 0; i < NSB; ++i) {
    const int sb = sb0 + s + 16 * i;
    if (sb >= se) continue;
    const int xs0 = sb * XPAD;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if constexpr (PIN) {
        pin(T.m[r][i]);
        if constexpr (WTile<QT, NSB, R>::Q6D) pin(T.d[r][i]);
      }
    }
    if constexpr (QT == QT_Q5_K) {
      // w = d*sc*q - dmin*m, q = nibble | (5th bit << 4) in 0..31 (unsigned int8 codes)
      float d[R], dm[R];
      unsigned sl[R], ml[R], sh[R], mh[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const u32x4 m = T.m[r][i];
        d[r] = f16lo(m.x);
        dm[r] = f16hi(m.x);
        sl[r] = m.y & 0x3F3F3F3Fu;
        ml[r] = m.z & 0x3F3F3F3Fu;
        sh[r] = (m.w & 0x0F0F0F0Fu) | ((m.y >> 2) & 0x30303030u);
        mh[r] = ((m.w >> 4) & 0x0F0F0F0Fu) | ((m.z >> 2) & 0x30303030u);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float fsl[R], fml[R], fsh[R], fmh[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const unsigned S = c < 2 ? sl[r] : sh[r], M = c < 2 ? ml[r] : mh[r];
          const int k0 = (2 * c) & 3, k1 = (2 * c + 1) & 3;
          fsl[r] = d[r] * ubyte(S, k0);
          fml[r] = dm[r] * ubyte(M, k0);
          fsh[r] = d[r] * ubyte(S, k1);
          fmh[r] = dm[r] * ubyte(M, k1);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int t = 2 * c + h, gl = 4 * c + h;
          pin_piece(i, t);
          XFr<BT> x;
          load_x<BT>(xq, xf, XS, xs0 + gl, xs0 + gl + 2, x);
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const u32x4 a = T.a[r][i][t];
            const unsigned H = T.q5h[r][i][t];
            u32x4 lo, hi;
            lo.x = (a.x & 0x0F0F0F0Fu) | ((H << 4) & 0x10101010u);
            lo.y = (a.y & 0x0F0F0F0Fu) | ((H << 3) & 0x10101010u);
            lo.z = (a.z & 0x0F0F0F0Fu) | ((H << 2) & 0x10101010u);
            lo.w = (a.w & 0x0F0F0F0Fu) | ((H << 1) & 0x10101010u);
            hi.x = ((a.x >> 4) & 0x0F0F0F0Fu) | (H & 0x10101010u);
            hi.y = ((a.y >> 4) & 0x0F0F0F0Fu) | ((H >> 1) & 0x10101010u);
            hi.z = ((a.z >> 4) & 0x0F0F0F0Fu) | ((H >> 2) & 0x10101010u);
            hi.w = ((a.w >> 4) & 0x0F0F0F0Fu) | ((H >> 3) & 0x10101010u);
#pragma unroll
            for (int b = 0; b < BT; ++b) {
              const float il = (float)dot16(lo, x.lo[b]), ih = (float)dot16(hi, x.hi[b]);
              acc[r][b] += fsl[r] * (x.fl[b].x * il) - fml[r] * x.fl[b].y + fsh[r] * (x.fh[b].x * ih) -
                           fmh[r] * x.fh[b].y;
            }
          }
          OMX_PIECE_ORDER();
        }
      }
    } else if constexpr (QT == QT_Q4_K) {
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
          pin_piece(i, t);
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
    } else if constexpr (QT == QT_Q6_K8) {
      // widened Q6_K: w = d*sc*c with c = q - 32 already signed int8 (lo | hi 16-weight halves)
      float dq[R];
#pragma unroll
      for (int r = 0; r < R; ++r) dq[r] = h2f((uint16_t)T.d[r][i]);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int n = t >> 2, sub = t & 3, il_ = 8 * n + sub, ih_ = il_ + 4;
        pin_piece(i, t);
        XFr<BT> x;
        load_x<BT>(xq, xf, XS, xs0 + il_, xs0 + ih_, x);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const u32x4 m = T.m[r][i];
          const float fl = dq[r] * sbyte(m[il_ >> 2], il_ & 3), fh = dq[r] * sbyte(m[ih_ >> 2], ih_ & 3);
#pragma unroll
          for (int b = 0; b < BT; ++b) {
            const float il = (float)dot16(T.a[r][i][t], x.lo[b]), ih = (float)dot16(T.b[r][i][t], x.hi[b]);
            acc[r][b] += fl * (x.fl[b].x * il) + fh * (x.fh[b].x * ih);
          }
        }
        OMX_PIECE_ORDER();
      }
    } else if constexpr (QT == QT_Q6_K) {
      // w = d*sc*(q - 32); q = ql nibble | (2 high bits << 4)
      float dq[R];
#pragma unroll
      for (int r = 0; r < R; ++r) dq[r] = h2f((uint16_t)T.d[r][i]);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int n = t >> 2, sub = t & 3, il_ = 8 * n + sub, ih_ = il_ + 4;
        pin_piece(i, t);
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
        pin_piece(i, t);
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

// small-batch decode (gemv_batch.hip): false = shape not covered, caller falls back
bool gemv_batch(const GemvParams& P, hipStream_t s);

}  // namespace omx
