// Shared device pieces of the batch-1 int8 activation chain (gemv8.hip, allreduce.hip): the image layout
// and the group quantisers.
#pragma once
#include "gemv_core.h"

namespace omx {

// IN_X8_LN: a LayerNorm'd image (x * ln_w) with sums and sums of squares (Phi-2, GemvParams::x8_sum)
enum { IN_X8 = 0, IN_X8_RMS = 1, IN_MERGE = 2, IN_X8_LN = 3 };
// EM_ACT: a plain activated output (EPI_GELU: Phi-2's FFN up), one group per 16-row tile, no partials
enum { EM_NONE = 0, EM_ADD = 1, EM_GLU = 2, EM_ACT = 3 };

__device__ __forceinline__ int x8_slots_dev(int K) { return ((n_sb(K) * XPAD + 1) + 1) & ~1; }

// batched rows (continuous batching, B = 2..X8_MAX_B): row b's image at b * x8_bytes(K), its RMS
// partials at b * x8_stat_ld(K) floats (ops.h; 16-B aligned rows)
constexpr int X8_MAX_B = 4;
__device__ __forceinline__ int x8_stat_ld_dev(int K) { return ((K >> 4) + 3) & ~3; }

constexpr int X8_NWI = 3;   // 16-byte image words per thread (K <= 7424 per 256 threads of the K split)
// two super-blocks per lane, unsplit K (4096 < K <= 8192: Llama-2-70B's QKV / gate_up / LM head at
// K = 8192 need 13104 image bytes > 256 x 3 x 16): one word more
constexpr int x8_nwi(int nsb, int ks) { return nsb == 2 && ks == 1 ? 4 : X8_NWI; }
constexpr int X8_NSTW = 2;  // f32x4 RMS partials per lane (K <= 8192)

// quantise the 16 staged values of group G into the consumer image (one lane)
__device__ __forceinline__ void emit_group(void* img, int Kc, int G, const float* v, const float* sq,
                                           float* stat) {
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) amax = fmaxf(amax, fabsf(v[i]));
  const float d = amax / 127.f, id = amax > 0.f ? 127.f / amax : 0.f;
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
  const int XSP = x8_slots_dev(Kc);
  const int slot = (G >> 4) * XPAD + (G & 15);
  ((i32x4*)img)[slot] = pk;
  ((f32x2*)((char*)img + (size_t)XSP * 16))[slot] = (f32x2){d, d * (float)qsum};
  if (stat) {
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) ss += sq[i];
    stat[G] = ss;
  }
}

// emit_group spread over the 16 lanes of a row group (lane i holds staged value i): max and code sum by
// 16-lane shuffles, one byte store per lane, lane 0 writes the scale pair and the RMS partial. The same
// codes and scales as emit_group (integer sum, exact max); the partial's float sum is a tree. The
// producers' tails ran the one-lane form: ~0.6 us of gate_up's 12 us (scripts/bench_gemv8.py NOEMIT)
// sx / ssum (optional): the group's plain sum as well (a LayerNorm'd consumer's mean)
__device__ __forceinline__ void emit_group16(void* img, int Kc, int G, float v, float sq, float* stat, int i,
                                             float sx = 0.f, float* ssum = nullptr) {
  float amax = fabsf(v);
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) amax = fmaxf(amax, __shfl_xor(amax, m, 16));
  const float d = amax / 127.f, id = amax > 0.f ? 127.f / amax : 0.f;
  const int q = (int)rintf(v * id);
  int qsum = q;
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) qsum += __shfl_xor(qsum, m, 16);
  const int XSP = x8_slots_dev(Kc);
  const int slot = (G >> 4) * XPAD + (G & 15);
  ((int8_t*)img)[16 * slot + i] = (int8_t)q;
  if (i == 0) ((f32x2*)((char*)img + (size_t)XSP * 16))[slot] = (f32x2){d, d * (float)qsum};
  if (stat) {
    float ss = sq;
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) ss += __shfl_xor(ss, m, 16);
    if (i == 0) stat[G] = ss;
  }
  if (ssum) {
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) sx += __shfl_xor(sx, m, 16);
    if (i == 0) ssum[G] = sx;
  }
}

}  // namespace omx
