// Shared device helpers for the gfx950 (CDNA4) kernels. Wave = 64 lanes everywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "qmat.h"

#define OMX_WAVE 64

// In-kernel bounds assertions: compiled in only by the debug build
// (`python build_native.py --debug`: -DOMX_DEBUG_KERNELS -O1 -g, a separate in-tree build directory);
// a failing check prints the condition with the block / thread and aborts the kernel (device assert).
#ifdef OMX_DEBUG_KERNELS
#include <cassert>
#define OMX_KASSERT(c) assert(c)
#else
#define OMX_KASSERT(c) ((void)0)
#endif

typedef _Float16 f16;
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));


__device__ __forceinline__ float h2f(uint16_t h) {
  f16 v = __builtin_bit_cast(f16, h);
  return (float)v;
}

// fp8 KV cache (OMX_KV_CACHE_TYPE=fp8): one OCP e4m3fn byte per element (gfx950 v_cvt_pk_fp8_f32),
// saturated to the format's +-448 (the conversion itself does not clamp)
__device__ __forceinline__ uint8_t f2e4m3(float v) {
  return (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v, -448.f), 448.f), 0.f, 0, false) & 0xFF);
}
// element idx of a K or V cache row: fp16 or fp8 by kv8
__device__ __forceinline__ void kv_store(void* base, long long idx, float v, int kv8) {
  if (kv8) ((uint8_t*)base)[idx] = f2e4m3(v);
  else ((f16*)base)[idx] = (f16)v;
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

// runtime block size variant: nw = blockDim.x / 64 waves
__device__ __forceinline__ float block_sum_rt(float v, float* red, int nw) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
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


// Layout v2 geometry (ollama_operator_amd/quant.py "device repack"): SB super-blocks of 256 per
// row (K padded), codes piece-major: piece t of super-block sb at byte (t * SB + sb) * piece_bytes.
__device__ __forceinline__ int n_sb(int K) { return (K + 255) >> 8; }

// super-blocks per group of an in-block K split over KS wave groups (<= 16 each). When a row's piece
// run is a whole number of 128-B lines (SB % 8 == 0) the groups start on 16-super-block boundaries, so
// each group's run starts on a line too (K = 10240 split 14 / 14 / 12: 3.3 TB/s memory path only,
// 4.5 at 16 / 16 / 16, profiles/r5_decode align probe). Otherwise every row starts off a line anyway
// and the split is balanced: Llama-2-13B's down (SB = 54) ran 16 / 16 / 16 / 6 aligned.
__device__ __forceinline__ int ks_chunk(int SB, int KS) {
  if (KS <= 1) return SB;
  const int c = (SB + KS - 1) / KS;
  return (SB & 7) ? c : (c + 15) & ~15;
}

// Dequantize piece p (= 8 * sb + t, natural order) of row `row` into two groups of 16 floats
// (lo, hi) and their offsets (in weights) within the row. Used by the embedding gather and the fp16
// dequant kernels (the GEMV decodes pieces itself, see gemv.hip).
__device__ inline void dequant_piece(const QMat& w, long long row, int p, float* lo, float* hi,
                                     int& off_lo, int& off_hi) {
  const int SB = n_sb(w.K);
  const int sb = p >> 3, t = p & 7;
  const long long pi = (long long)t * SB + sb;
  if (w.qtype == QT_Q4_K) {
    const int c = t >> 1, h = t & 1;
    off_lo = 256 * sb + 64 * c + 16 * h;
    off_hi = off_lo + 32;
    const u32x4 q = *(const u32x4*)(w.s0 + row * SB * 128 + 16 * pi) ^ 0x80808080u;
    const u32x4 m = *(const u32x4*)(w.s1 + row * SB * 16 + 16LL * sb);
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
  } else if (w.qtype == QT_Q5_K) {
    const int c = t >> 1, h = t & 1;
    off_lo = 256 * sb + 64 * c + 16 * h;
    off_hi = off_lo + 32;
    const u32x4 q = *(const u32x4*)(w.s0 + row * SB * 128 + 16 * pi);
    const unsigned H = *(const unsigned*)(w.s2 + row * SB * 32 + 4 * pi);
    const u32x4 m = *(const u32x4*)(w.s1 + row * SB * 16 + 16LL * sb);
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
      const unsigned hb = H >> (8 * (i & 3));  // byte i & 3: lo bit (i >> 2), hi bit 4 + (i >> 2)
      lo[i] = sc[0] * (float)((byte & 0xF) | (((hb >> (i >> 2)) & 1) << 4)) - mn[0];
      hi[i] = sc[1] * (float)((byte >> 4) | (((hb >> (4 + (i >> 2))) & 1) << 4)) - mn[1];
    }
  } else if (w.qtype == QT_Q6_K) {
    const int n = t >> 2, sub = t & 3;
    off_lo = 256 * sb + 128 * n + 16 * sub;
    off_hi = off_lo + 64;
    const u32x4 ql = *(const u32x4*)(w.s0 + row * SB * 128 + 16 * pi);
    const u32x2 qh = *(const u32x2*)(w.s1 + row * SB * 64 + 8 * pi);
    const int8_t* sc = (const int8_t*)(w.s2 + row * SB * 16 + 16LL * sb);
    const float d = h2f(*(const uint16_t*)(w.s3 + row * SB * 2 + 2LL * sb));
    const float slo = d * (float)sc[8 * n + sub], shi = d * (float)sc[8 * n + sub + 4];
    const unsigned L[4] = {ql.x, ql.y, ql.z, ql.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const unsigned lb = (L[i >> 2] >> (8 * (i & 3))) & 0xFF;
      const int sh = 8 * (i & 3) + 2 * (i >> 2);  // field (i >> 2) of byte (i & 3)
      lo[i] = slo * (float)((int)((lb & 0xF) | (((qh.x >> sh) & 3) << 4)) - 32);
      hi[i] = shi * (float)((int)((lb >> 4) | (((qh.y >> sh) & 3) << 4)) - 32);
    }
  } else if (w.qtype == QT_Q4_0) {
    off_lo = 256 * sb + 32 * t;
    off_hi = off_lo + 16;
    const u32x4 q = *(const u32x4*)(w.s0 + row * SB * 128 + 16 * pi) ^ 0x80808080u;
    const float d = h2f(*(const uint16_t*)(w.s1 + row * SB * 16 + 16LL * sb + 2 * t));
    const unsigned qq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const unsigned byte = (qq[i >> 2] >> (8 * (i & 3))) & 0xFF;
      lo[i] = d * ((float)(byte & 0xF) - 8.f);
      hi[i] = d * ((float)(byte >> 4) - 8.f);
    }
  } else {  // Q8_0
    off_lo = 256 * sb + 32 * t;
    off_hi = off_lo + 16;
    const int8_t* q = (const int8_t*)(w.s0 + row * SB * 256 + 32 * pi);
    const float d = h2f(*(const uint16_t*)(w.s1 + row * SB * 16 + 16LL * sb + 2 * t));
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      lo[i] = d * (float)q[i];
      hi[i] = d * (float)q[16 + i];
    }
  }
}
