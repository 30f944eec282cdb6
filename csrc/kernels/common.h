// Shared device helpers for the gfx950 (CDNA4) kernels. Wave = 64 lanes everywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "qmat.h"

#define OMX_WAVE 64

typedef _Float16 f16;
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));


__device__ __forceinline__ float h2f(uint16_t h) {
  f16 v = __builtin_bit_cast(f16, h);
  return (float)v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, OMX_WAVE);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, OMX_WAVE));
  return v;
}

template <int W>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int m = W / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, OMX_WAVE);
  return v;
}

template <int W>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int m = W / 2; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, OMX_WAVE));
  return v;
}

__device__ __forceinline__ int sdot4(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }

__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k = 0.7978845608028654f;  // sqrt(2/pi)
  return 0.5f * x * (1.0f + tanhf(k * (x + 0.044715f * x * x * x)));
}

// Block-wide sum for blockDim.x == NT (multiple of 64); `red` needs NT/64 floats of LDS.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  return t;
}

template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t = fmaxf(t, red[i]);
  return t;
}


// Row stream strides in bytes for a given K.
__device__ __forceinline__ long long qs_row_bytes(int qt, int K) { return qt == QT_Q8_0 ? K : K / 2; }

// Dequantize one 32-weight "piece" p of row `row` into two groups of 16 floats (lo, hi) and their
// offsets (in weights) within the row. Used by the embedding gather and the fp16 dequant kernels.
__device__ inline void dequant_piece(const QMat& w, long long row, int p, float* lo, float* hi,
                                     int& off_lo, int& off_hi) {
  const int K = w.K;
  if (w.qtype == QT_Q4_K) {
    const int sb = p >> 3, t = p & 7, c = t >> 1, h = t & 1;
    off_lo = 256 * sb + 64 * c + 16 * h;
    off_hi = off_lo + 32;
    const u32x4 q = *(const u32x4*)(w.s0 + row * (K / 2) + 16LL * p);
    const u32x4 m = *(const u32x4*)(w.s1 + row * (K / 16) + 16LL * sb);
    const float d = h2f(m.x & 0xFFFF), dmin = h2f(m.x >> 16);
    float sc[2], mn[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int j = 2 * c + k, sh = 8 * (j & 3);
      const unsigned a = (m.y >> sh) & 0xFF, b = (m.z >> sh) & 0xFF, e = (m.w >> sh) & 0xFF;
      const unsigned s = j < 4 ? (a & 63) : ((e & 0xF) | ((a >> 6) << 4));
      const unsigned mm = j < 4 ? (b & 63) : ((e >> 4) | ((b >> 6) << 4));
      sc[k] = d * (float)s;
      mn[k] = dmin * (float)mm;
    }
    const unsigned qq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const unsigned byte = (qq[i >> 2] >> (8 * (i & 3))) & 0xFF;
      lo[i] = sc[0] * (float)(byte & 0xF) - mn[0];
      hi[i] = sc[1] * (float)(byte >> 4) - mn[1];
    }
  } else if (w.qtype == QT_Q6_K) {
    const int sb = p >> 3, t = p & 7, n = t >> 2, sub = t & 3;
    off_lo = 256 * sb + 128 * n + 16 * sub;
    off_hi = off_lo + 64;
    const u32x4 ql = *(const u32x4*)(w.s0 + row * (K / 2) + 16LL * p);
    const u32x4 qh = *(const u32x4*)(w.s1 + row * (K / 4) + 64LL * sb + 32 * n + 16 * (sub & 1));
    const int8_t* sc = (const int8_t*)(w.s2 + row * (K / 16) + 16LL * sb + 8 * n);
    const float d = h2f(*(const uint16_t*)(w.s3 + row * (K / 128) + 2LL * sb));
    const float slo = d * (float)sc[sub], shi = d * (float)sc[4 + sub];
    const int shl = sub < 2 ? 0 : 2, shh = sub < 2 ? 4 : 6;
    const unsigned L[4] = {ql.x, ql.y, ql.z, ql.w}, H[4] = {qh.x, qh.y, qh.z, qh.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const unsigned lb = (L[i >> 2] >> (8 * (i & 3))) & 0xFF, hb = (H[i >> 2] >> (8 * (i & 3))) & 0xFF;
      lo[i] = slo * (float)((int)((lb & 0xF) | (((hb >> shl) & 3) << 4)) - 32);
      hi[i] = shi * (float)((int)((lb >> 4) | (((hb >> shh) & 3) << 4)) - 32);
    }
  } else if (w.qtype == QT_Q4_0) {
    off_lo = 32 * p;
    off_hi = off_lo + 16;
    const u32x4 q = *(const u32x4*)(w.s0 + row * (K / 2) + 16LL * p);
    const float d = h2f(*(const uint16_t*)(w.s1 + row * (K / 16) + 2LL * p));
    const unsigned qq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const unsigned byte = (qq[i >> 2] >> (8 * (i & 3))) & 0xFF;
      lo[i] = d * ((float)(byte & 0xF) - 8.f);
      hi[i] = d * ((float)(byte >> 4) - 8.f);
    }
  } else {  // Q8_0
    off_lo = 32 * p;
    off_hi = off_lo + 16;
    const int8_t* q = (const int8_t*)(w.s0 + row * (long long)K + 32LL * p);
    const float d = h2f(*(const uint16_t*)(w.s1 + row * (K / 16) + 2LL * p));
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      lo[i] = d * (float)q[i];
      hi[i] = d * (float)q[16 + i];
    }
  }
}
