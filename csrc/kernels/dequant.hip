// Row gather + dequantisation from the repacked quant streams (SURVEY.md §2.2 N15 embedding
// gather) and whole-matrix dequantisation to fp16 (resident fp16 copies for MFMA prefill GEMMs).
#include "common.h"
#include "gemv8_core.h"
#include "ops.h"

namespace omx {

// one block per gathered row; each thread dequantises 32-weight pieces. A negative row id -(j + 1)
// takes row j of `ext` ([*][K] fp32, unscaled) instead: multimodal inputs (projected image patches,
// models/clip.py) enter the sequence as such rows.
// stat (optional, the batched fp16 decode chain): per-16-element sum-of-squares partials [n][K / 16] of
// the gathered rows, the "residual before the add" of layer 0's O emission (gemv_mfma.hip range scale)
// one 16-element group of a gathered row into layer 0's int8 input image (img8 != null)
// (isum: the group's sum of the row too, for a LayerNorm'd consumer)
__device__ __forceinline__ void embed_emit(void* img8, const float* nw, float* ist, float* isum, int K, int G,
                                           const float* v) {
  float xv[16], sq[16], sx = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    xv[j] = v[j] * nw[16 * G + j];
    sq[j] = v[j] * v[j];
    sx += v[j];
  }
  emit_group(img8, K, G, xv, sq, ist);
  if (isum) isum[G] = sx;
}

__global__ __launch_bounds__(256) void embed_rows_kernel(QMat w, const int* rows, float* out, int ldo, float scale,
                                                         const float* ext, float* stat, void* img8, const float* img_nw,
                                                         float* img_stat, float* img_sum) {
  const int b = blockIdx.x;
  const long long row = rows[b];
  const int P = w.K / 32;
  float* o = out + (long long)b * ldo;
  float* st = stat ? stat + (long long)b * (w.K / 16) : nullptr;
  void* im = img8 ? (char*)img8 + (size_t)b * x8_slots_dev(w.K) * 24 : nullptr;
  float* ist = img8 ? img_stat + (size_t)b * x8_stat_ld_dev(w.K) : nullptr;
  float* isum = img8 && img_sum ? img_sum + (size_t)b * x8_stat_ld_dev(w.K) : nullptr;
  if (row < 0) {
    const float* src = ext + (-row - 1) * (long long)w.K;
    OMX_KASSERT(ext != nullptr);
    for (int i = threadIdx.x; i < w.K; i += blockDim.x) o[i] = ext ? src[i] : 0.f;
    for (int g = threadIdx.x; g < w.K / 16; g += blockDim.x) {
      float v[16];
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        v[i] = ext ? src[16 * g + i] : 0.f;
        s += v[i] * v[i];
      }
      if (st) st[g] = s;
      if (im) embed_emit(im, img_nw, ist, isum, w.K, g, v);
    }
    return;
  }
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    float lo[16], hi[16];
    int olo, ohi;
    dequant_piece(w, row, p, lo, hi, olo, ohi);
    float slo = 0.f, shi = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      lo[j] *= scale;
      hi[j] *= scale;
      slo += lo[j] * lo[j];
      shi += hi[j] * hi[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      *(f32x4*)(o + olo + 4 * j) = (f32x4){lo[4 * j], lo[4 * j + 1], lo[4 * j + 2], lo[4 * j + 3]};
      *(f32x4*)(o + ohi + 4 * j) = (f32x4){hi[4 * j], hi[4 * j + 1], hi[4 * j + 2], hi[4 * j + 3]};
    }
    if (st) {  // 16-element pieces: every group of the row written once (only the row total is used)
      st[olo >> 4] = slo;
      st[ohi >> 4] = shi;
    }
    if (im) {  // a piece's halves are whole 16-groups: each emitted by the thread that holds it
      embed_emit(im, img_nw, ist, isum, w.K, olo >> 4, lo);
      embed_emit(im, img_nw, ist, isum, w.K, ohi >> 4, hi);
    }
  }
}

void embed_rows(const QMat& w, const int* rows, int n, float* out, int ldo, hipStream_t s, float scale,
                const float* ext, float* stat, void* img8, const float* img_nw, float* img_stat, float* img_sum) {
  if (n <= 0) return;
  if (img8 && (!img_nw || !img_stat || w.K % 16)) img8 = nullptr;
  hipLaunchKernelGGL(embed_rows_kernel, dim3(n), dim3(256), 0, s, w, rows, out, ldo, scale, ext, stat, img8, img_nw,
                     img_stat, img_sum);
}

// rows on blockIdx.y (grid-stride), pieces of a row on x (no 64-bit index division per piece); PERM:
// K order (0, 2, 1, 3) inside every 4, the order prep_x16 writes the prefill activations in
// (gemm.hip), so the library GEMM can consume both as they are
template <bool PERM>
__global__ __launch_bounds__(256) void dequant_f16_kernel(QMat w, f16* out, long long row0) {
  const int P = w.K / 32;
  for (int row = blockIdx.y; row < w.N; row += gridDim.y) {
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
      float lo[16], hi[16];
      int olo, ohi;
      dequant_piece(w, row0 + row, p, lo, hi, olo, ohi);
      f16* o = out + (long long)row * w.K;
      f16x8 a, b, c, d;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = PERM ? (j & ~3) | ((j & 1) << 1) | ((j >> 1) & 1) : j;  // 0 2 1 3
        a[j] = (f16)lo[k]; b[j] = (f16)lo[8 + k];
        c[j] = (f16)hi[k]; d[j] = (f16)hi[8 + k];
      }
      *(f16x8*)(o + olo) = a;
      *(f16x8*)(o + olo + 8) = b;
      *(f16x8*)(o + ohi) = c;
      *(f16x8*)(o + ohi + 8) = d;
    }
  }
}

void dequant_f16(const QMat& w, void* out, hipStream_t s, int perm, long long row0) {
  const int P = w.K / 32;
  const int nt = P >= 256 ? 256 : (P + 63) / 64 * 64;  // K = 4096: 128 pieces, 128 threads per row
  const dim3 grid((P + nt - 1) / nt > 0 ? (P + nt - 1) / nt : 1, w.N < 65535 ? (w.N > 0 ? w.N : 1) : 65535);
  if (perm)
    hipLaunchKernelGGL(dequant_f16_kernel<true>, grid, dim3(nt > 0 ? nt : 64), 0, s, w, (f16*)out, row0);
  else
    hipLaunchKernelGGL(dequant_f16_kernel<false>, grid, dim3(nt > 0 ? nt : 64), 0, s, w, (f16*)out, row0);
}

// Q6_K -> QT_Q6_K8 widening at load (qmat.h): one thread per (row, super-block, piece) writes the
// piece's 32 signed codes q - 32 (lo 16 | hi 16 weights), in the Q6_K piece order the GEMV uses
__global__ void widen_q6k_kernel(QMat w, int8_t* out) {
  const int SB = n_sb(w.K);
  const long long total = (long long)w.N * SB * 8;
  for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < total;
       u += (long long)gridDim.x * blockDim.x) {
    const long long row = u / (SB * 8);
    const int rem = (int)(u % (SB * 8)), t = rem / SB, sb = rem % SB;
    const long long pi = (long long)t * SB + sb;
    const u32x4 ql = *(const u32x4*)(w.s0 + row * SB * 128 + 16 * pi);
    const u32x2 qh = *(const u32x2*)(w.s1 + row * SB * 64 + 8 * pi);
    const unsigned L[4] = {ql.x, ql.y, ql.z, ql.w};
    int8_t c[32];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const unsigned lb = (L[i >> 2] >> (8 * (i & 3))) & 0xFF;
      const int sh = 8 * (i & 3) + 2 * (i >> 2);  // field (i >> 2) of byte (i & 3)
      c[i] = (int8_t)((int)((lb & 0xF) | (((qh.x >> sh) & 3) << 4)) - 32);
      c[16 + i] = (int8_t)((int)((lb >> 4) | (((qh.y >> sh) & 3) << 4)) - 32);
    }
    int8_t* o = out + row * SB * 256 + 32 * pi;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      u32x4 v;
      unsigned wd[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        wd[j] = (unsigned)(uint8_t)c[16 * k + 4 * j] | ((unsigned)(uint8_t)c[16 * k + 4 * j + 1] << 8) |
                ((unsigned)(uint8_t)c[16 * k + 4 * j + 2] << 16) | ((unsigned)(uint8_t)c[16 * k + 4 * j + 3] << 24);
      v.x = wd[0]; v.y = wd[1]; v.z = wd[2]; v.w = wd[3];
      *(u32x4*)(o + 16 * k) = v;
    }
  }
}

void widen_q6k(const QMat& w, void* out, hipStream_t s) {
  const long long total = (long long)w.N * ((w.K + 255) / 256) * 8;
  const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  hipLaunchKernelGGL(widen_q6k_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, s, w, (int8_t*)out);
}

__global__ void add_inplace_kernel(float* y, const float* x, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] += x[i];
}

void add_inplace(float* y, const float* x, long long n, hipStream_t s) {
  const int blocks = (int)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
  hipLaunchKernelGGL(add_inplace_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, s, y, x, n);
}

__global__ __launch_bounds__(256) void rmsnorm_kernel(const float* x, const float* w, float eps, int n, float* out) {
  __shared__ float red[4];
  const float* xr = x + (long long)blockIdx.x * n;
  float ss = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) ss += xr[i] * xr[i];
  ss = block_sum<256>(ss, red);
  const float r = rsqrtf(ss / n + eps);
  for (int i = threadIdx.x; i < n; i += 256) out[(long long)blockIdx.x * n + i] = xr[i] * r * w[i];
}

void rmsnorm(const float* x, const float* w, float eps, int rows, int n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(rmsnorm_kernel, dim3(rows), dim3(256), 0, s, x, w, eps, n, out);
}

}  // namespace omx
