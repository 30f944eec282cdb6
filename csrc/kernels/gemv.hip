// Fused quantized GEMV for decode (M = batch <= a few rows) on gfx950.
//
// y[b, n] = epilogue( sum_k W[n, k] * norm(x[b, :])[k] )
//
// Design (MI355X-first, see SURVEY.md §7.4 hard part 1 and docs/kernels.md):
//  * Weights are repacked at load into 16-byte-aligned streams (quant.py `repack`), so one lane's
//    16-B load is always one "piece" = 32 weights (two groups of 16) and a wave's loads coalesce
//    into whole 1 KiB lines. Register-streamed, never through LDS (cdna_hip_programming.md §5 GEMV
//    row): every lane issues all its R x NPC loads up front.
//  * The activation prologue runs once per 256-thread block: x (fp32) is optionally RMS/Layer-
//    normalised (the norm is FUSED here -- no separate launch), quantised to int8 per 16-element
//    group with an fp32 scale and group sum, and staged in LDS. Every wave then reads its x
//    fragments from LDS: x crosses L2 once per block, not once per wave.
//  * Inner product: v_dot4c_i32_i8 on 4-bit/6-bit/8-bit codes against int8 x; K-quant mins and the
//    Q4_0/Q6_K zero points are applied with the precomputed group sums.
//  * Epilogues are fused: residual add, bias, SiLU-GLU (gate/up rows interleaved at load), GELU,
//    and QKV (RoPE on adjacent row pairs + K/V scatter into the paged fp16 cache).
// Reference parity: the reference delegates all of this to llama.cpp inside `ollama/ollama`
// (reference pkg/model/pod.go:10-12); numerics are checked against quant.py + an fp32 torch GEMV.
#include "common.h"
#include "ops.h"

namespace omx {

// per-type piece geometry --------------------------------------------------------------------
__device__ __forceinline__ int pieces_per_row(int qt, int K) { return K / 32; }

// 16-group indices (in x) of the lo/hi halves of piece p
__device__ __forceinline__ void piece_groups(int qt, int p, int& glo, int& ghi) {
  if (qt == QT_Q4_K) {
    const int sb = p >> 3, t = p & 7, c = t >> 1, h = t & 1;
    glo = 16 * sb + 4 * c + h;
    ghi = glo + 2;
  } else if (qt == QT_Q6_K) {
    const int sb = p >> 3, t = p & 7, n = t >> 2, sub = t & 3;
    glo = 16 * sb + 8 * n + sub;
    ghi = glo + 4;
  } else {
    glo = 2 * p;
    ghi = 2 * p + 1;
  }
}

struct WFrag {
  u32x4 a;  // qs / ql / q0
  u32x4 b;  // meta / qh / q1
  u32x2 c;  // Q6_K: 8 scale bytes of this half
  unsigned d;  // fp16 scale bits (Q6_K / Q4_0 / Q8_0)
};

template <int QT>
__device__ __forceinline__ void load_wfrag(const QMat& w, long long row, int p, WFrag& f) {
  const int K = w.K;
  if constexpr (QT == QT_Q4_K) {
    f.a = __builtin_nontemporal_load((const u32x4*)(w.s0 + row * (K / 2) + 16LL * p));
    f.b = *(const u32x4*)(w.s1 + row * (K / 16) + 16LL * (p >> 3));
  } else if constexpr (QT == QT_Q6_K) {
    const int sb = p >> 3, t = p & 7, n = t >> 2, sub = t & 3;
    f.a = __builtin_nontemporal_load((const u32x4*)(w.s0 + row * (K / 2) + 16LL * p));
    f.b = *(const u32x4*)(w.s1 + row * (K / 4) + 64LL * sb + 32 * n + 16 * (sub & 1));
    f.c = *(const u32x2*)(w.s2 + row * (K / 16) + 16LL * sb + 8 * n);
    f.d = *(const uint16_t*)(w.s3 + row * (K / 128) + 2LL * sb);
  } else if constexpr (QT == QT_Q4_0) {
    f.a = __builtin_nontemporal_load((const u32x4*)(w.s0 + row * (K / 2) + 16LL * p));
    f.d = *(const uint16_t*)(w.s1 + row * (K / 16) + 2LL * p);
  } else {  // Q8_0
    const u32x4* q = (const u32x4*)(w.s0 + row * (long long)K + 32LL * p);
    f.a = __builtin_nontemporal_load(q);
    f.b = __builtin_nontemporal_load(q + 1);
    f.d = *(const uint16_t*)(w.s1 + row * (K / 16) + 2LL * p);
  }
}

struct XFrag {
  i32x4 lo, hi;
  float dlo, dhi, slo, shi;
};

__device__ __forceinline__ int dot16(u32x4 q, i32x4 x) {
  int s = sdot4((int)q.x, x.x, 0);
  s = sdot4((int)q.y, x.y, s);
  s = sdot4((int)q.z, x.z, s);
  return sdot4((int)q.w, x.w, s);
}

template <int QT>
__device__ __forceinline__ float piece_dot(const WFrag& f, const XFrag& x, int p) {
  if constexpr (QT == QT_Q4_K) {
    const u32x4 lo = f.a & 0x0F0F0F0Fu;
    const u32x4 hi = (f.a >> 4) & 0x0F0F0F0Fu;
    const float dl = (float)dot16(lo, x.lo), dh = (float)dot16(hi, x.hi);
    const float d = h2f(f.b.x & 0xFFFF), dmin = h2f(f.b.x >> 16);
    const int c = (p & 7) >> 1;
    const int sh = 8 * ((2 * c) & 3);  // j = 2c (lo) and 2c+1 (hi): shifts sh and sh+8
    const unsigned a0 = (f.b.y >> sh) & 0xFF, b0 = (f.b.z >> sh) & 0xFF, e0 = (f.b.w >> sh) & 0xFF;
    const unsigned a1 = (f.b.y >> (sh + 8)) & 0xFF, b1 = (f.b.z >> (sh + 8)) & 0xFF,
                   e1 = (f.b.w >> (sh + 8)) & 0xFF;
    const bool low = c < 2;
    const float s0 = (float)(low ? (a0 & 63) : ((e0 & 0xF) | ((a0 >> 6) << 4)));
    const float m0 = (float)(low ? (b0 & 63) : ((e0 >> 4) | ((b0 >> 6) << 4)));
    const float s1 = (float)(low ? (a1 & 63) : ((e1 & 0xF) | ((a1 >> 6) << 4)));
    const float m1 = (float)(low ? (b1 & 63) : ((e1 >> 4) | ((b1 >> 6) << 4)));
    return d * (s0 * x.dlo * dl + s1 * x.dhi * dh) - dmin * (m0 * x.slo + m1 * x.shi);
  } else if constexpr (QT == QT_Q6_K) {
    const int sub = p & 3;
    const int shl = sub < 2 ? 0 : 2;
    const u32x4 lo = (f.a & 0x0F0F0F0Fu) | (((f.b >> shl) & 0x03030303u) << 4);
    const u32x4 hi = ((f.a >> 4) & 0x0F0F0F0Fu) | (((f.b >> (shl + 4)) & 0x03030303u) << 4);
    const float dl = (float)dot16(lo, x.lo), dh = (float)dot16(hi, x.hi);
    const unsigned wlo = f.c.x, whi = f.c.y;  // bytes 0..3 and 4..7 of this half's scales
    const float sl = (float)(int8_t)((wlo >> (8 * sub)) & 0xFF);
    const float shh = (float)(int8_t)((whi >> (8 * sub)) & 0xFF);
    const float d = h2f(f.d);
    return d * (sl * (x.dlo * dl - 32.f * x.slo) + shh * (x.dhi * dh - 32.f * x.shi));
  } else if constexpr (QT == QT_Q4_0) {
    const u32x4 lo = f.a & 0x0F0F0F0Fu;
    const u32x4 hi = (f.a >> 4) & 0x0F0F0F0Fu;
    const float dl = (float)dot16(lo, x.lo), dh = (float)dot16(hi, x.hi);
    return h2f(f.d) * (x.dlo * dl + x.dhi * dh - 8.f * (x.slo + x.shi));
  } else {
    const float dl = (float)dot16(f.a, x.lo), dh = (float)dot16(f.b, x.hi);
    return h2f(f.d) * (x.dlo * dl + x.dhi * dh);
  }
}

// --------------------------------------------------------------------------------------------
// activation prologue: x[b] (fp32) -> (norm) -> int8 groups of 16 in LDS
// LDS layout per batch slot: i32x4 q[G] | float d[G] | float s[G]   (G = K/16)
template <int NT>
__device__ void stage_activation(const GemvParams& P, int b, int K, i32x4* lq, float* ld, float* ls,
                                 float* red) {
  const int G = K / 16;
  const float* x = P.x + (long long)b * P.ldx;
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
  for (int g = threadIdx.x; g < G; g += NT) {
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
    lq[g] = pk;
    ld[g] = d;
    ls[g] = d * (float)qsum;
  }
}

// --------------------------------------------------------------------------------------------
// Kernel structure (per 256-thread block = 4 waves, each wave owns R = 2 rows of a row tile):
//   1. issue the first tile's weight loads (they do not depend on x)
//   2. activation prologue into LDS (overlaps the weight fetch)
//   3. persistent loop over row tiles (tile += gridDim.x): prefetch the next tile's weights into
//      a second register set while the current tile is computed (MODE 0), or reload (MODE 1/2).
// MODE 0: one K round, double-buffered; MODE 1: one K round, single buffer; MODE 2: K split in
// rounds of 64*NPC pieces (K > 16384).
constexpr int GEMV_NW = 4;
constexpr int GEMV_R = 2;

GemvTuning g_tune;
void set_gemv_tuning(int blocks_per_cu, int rows_per_wave, int r1) {
  if (blocks_per_cu > 0) g_tune.blocks_per_cu = blocks_per_cu;
  if (rows_per_wave == 2 || rows_per_wave == 4) g_tune.rows_per_wave = rows_per_wave;
  if (r1 >= 0) g_tune.r1 = r1;
}

template <int QT, int NPC, int R>
__device__ __forceinline__ void load_tile(const QMat& w, long long row_base, int row0, int N, int base, int Pc,
                                          int lane, WFrag (&wf)[R][NPC]) {
#pragma unroll
  for (int i = 0; i < NPC; ++i) {
    const int p = min(base + 64 * i + lane, Pc - 1);
#pragma unroll
    for (int r = 0; r < R; ++r) load_wfrag<QT>(w, row_base + min(row0 + r, N - 1), p, wf[r][i]);
  }
}

template <int QT, int NPC, int BT, int R>
__device__ __forceinline__ void compute_tile(const WFrag (&wf)[R][NPC], int base, int Pc, int lane, int G,
                                             const i32x4* lq, const float* ld, const float* ls,
                                             float (&acc)[R][BT]) {
#pragma unroll
  for (int i = 0; i < NPC; ++i) {
    const int p = base + 64 * i + lane;
    if (p < Pc) {
      int glo, ghi;
      piece_groups(QT, p, glo, ghi);
#pragma unroll
      for (int b = 0; b < BT; ++b) {
        XFrag xf;
        xf.lo = lq[b * G + glo];
        xf.hi = lq[b * G + ghi];
        xf.dlo = ld[b * G + glo];
        xf.dhi = ld[b * G + ghi];
        xf.slo = ls[b * G + glo];
        xf.shi = ls[b * G + ghi];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][b] += piece_dot<QT>(wf[r][i], xf, p);
      }
    }
  }
}

template <int BT, int R>
__device__ __forceinline__ void epilogue(const GemvParams& P, float (&acc)[R][BT], int row0, int N, int b0,
                                         int lane) {
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int b = 0; b < BT; ++b) acc[r][b] = wave_sum(acc[r][b]);
#pragma unroll
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int b = 0; b < BT; ++b) {
      if (lane != r * BT + b) continue;
      const int n = row0 + r;
      const int bb = b0 + b;
      if (n >= N || bb >= P.B) continue;
      float v = acc[r][b];
      const int vn = n + P.row_offset;  // row index in the virtual (concatenated) matrix
      switch (P.epi) {
        case EPI_STORE:
          if (P.bias) v += P.bias[vn];
          P.y[(long long)bb * P.ldy + vn] = v;
          break;
        case EPI_ADD: {
          if (P.bias) v += P.bias[vn];
          if (P.expert_w) v *= P.expert_w[bb * P.n_sel + blockIdx.z];
          float* dst = P.y + (long long)bb * P.ldy + vn;
          if (P.expert_ids && P.n_sel > 1) atomicAdd(dst, v);
          else *dst += v;
          break;
        }
        case EPI_GELU:
          if (P.bias) v += P.bias[vn];
          P.y[(long long)bb * P.ldy + vn] = gelu_tanh(v);
          break;
        case EPI_GLU:
          if ((r & 1) == 0) {  // even row = gate, odd row = up
            const float u = acc[(r + 1) % R][b];  // R == 1 never takes this path (dispatch)
            P.y[(long long)bb * P.ldy + (long long)blockIdx.z * P.y_sel_stride + vn / 2] = silu(v) * u;
          }
          break;
        case EPI_QKV: {
          const int Eq = P.Eq, Ekv = P.Ekv, D = P.D;
          int which, hh, d;
          if (vn < Eq) { which = 0; hh = vn / D; d = vn % D; }
          else if (vn < Eq + Ekv) { which = 1; hh = (vn - Eq) / D; d = (vn - Eq) % D; }
          else { which = 2; hh = (vn - Eq - Ekv) / D; d = (vn - Eq - Ekv) % D; }
          if (P.bias) v += P.bias[vn];
          float out = v;
          if (which < 2 && d < P.n_rot) {
            float pv = acc[(r ^ 1) % R][b];
            if (P.bias) pv += P.bias[vn ^ 1];
            const float ang = (float)P.pos[bb] * P.inv_freq[d >> 1];
            float sn, cs;
            sincosf(ang, &sn, &cs);
            out = (d & 1) ? (pv * sn + v * cs) : (v * cs - pv * sn);
          }
          if (which == 0) {
            P.y[(long long)bb * P.ldy + vn] = out;
          } else {
            const int slot = P.slot[bb];
            const long long blk = slot / P.bs, off = slot % P.bs;
            const long long idx = ((blk * P.n_kv + hh) * P.bs + off) * D + d;
            // two explicit stores: a pointer select here is lowered to an indexed scratch array
            if (which == 1) ((f16*)P.kc)[idx] = (f16)out;
            else ((f16*)P.vc)[idx] = (f16)out;
          }
          break;
        }
      }
    }
  }
}

template <int QT, int NPC, int BT, int MODE, int R>
__global__ __launch_bounds__(256) void gemv_kernel(GemvParams P) {
  constexpr int NT = 256, ROWS = GEMV_NW * R;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const QMat& w = P.w;
  const int K = w.K, N = w.N;
  const int G = K / 16;
  i32x4* lq = (i32x4*)smem;                               // [BT][G]
  float* ld = (float*)(smem + (size_t)BT * G * 16);       // [BT][G]
  float* ls = ld + BT * G;                                // [BT][G]
  float* red = ls + BT * G;                               // [NT/64]
  const int b0 = blockIdx.y * BT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int Pc = K / 32;
  const int n_tiles = (N + ROWS - 1) / ROWS;
  int tile = blockIdx.x;

  long long row_base = 0;
  GemvParams Q = P;
  if (P.expert_ids) {  // MoE: blockIdx.z = k-th selected expert of batch row b0
    const int e = P.expert_ids[b0 * P.n_sel + blockIdx.z];
    row_base = (long long)e * N;
    if (P.x_per_sel) Q.x = P.x + (long long)blockIdx.z * P.x_sel_stride;
  }

  WFrag wa[R][NPC];
  if (MODE != 2 && tile < n_tiles) load_tile<QT, NPC, R>(w, row_base, tile * ROWS + wave * R, N, 0, Pc, lane, wa);

#pragma unroll
  for (int b = 0; b < BT; ++b) {
    if (b0 + b < P.B) {
      stage_activation<NT>(Q, b0 + b, K, lq + b * G, ld + b * G, ls + b * G, red);
    } else {
      for (int g = threadIdx.x; g < G; g += NT) {
        lq[b * G + g] = (i32x4){0, 0, 0, 0};
        ld[b * G + g] = 0.f;
        ls[b * G + g] = 0.f;
      }
    }
  }
  __syncthreads();

  if constexpr (MODE == 0) {
    // explicit ping-pong (no register copy: a wa = wb copy would force a vmcnt(0) drain every
    // tile): while one register set is consumed, the other tile's loads are in flight
    WFrag wb[R][NPC];
    auto step = [&](WFrag (&cur)[R][NPC], WFrag (&nxt)[R][NPC], int t) {
      const int row0 = t * ROWS + wave * R;
      const int next = t + gridDim.x;
      if (next < n_tiles) load_tile<QT, NPC, R>(w, row_base, next * ROWS + wave * R, N, 0, Pc, lane, nxt);
      float acc[R][BT];
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int b = 0; b < BT; ++b) acc[r][b] = 0.f;
      compute_tile<QT, NPC, BT, R>(cur, 0, Pc, lane, G, lq, ld, ls, acc);
      if (row0 < N) epilogue<BT, R>(P, acc, row0, N, b0, lane);
    };
    while (tile < n_tiles) {
      step(wa, wb, tile);
      tile += gridDim.x;
      if (tile >= n_tiles) break;
      step(wb, wa, tile);
      tile += gridDim.x;
    }
    return;
  }
  for (; tile < n_tiles; tile += gridDim.x) {
    const int row0 = tile * ROWS + wave * R;
    const int next = tile + gridDim.x;
    float acc[R][BT];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int b = 0; b < BT; ++b) acc[r][b] = 0.f;
    if constexpr (MODE == 1) {
      compute_tile<QT, NPC, BT, R>(wa, 0, Pc, lane, G, lq, ld, ls, acc);
      if (next < n_tiles) load_tile<QT, NPC, R>(w, row_base, next * ROWS + wave * R, N, 0, Pc, lane, wa);
    } else {
      for (int base = 0; base < Pc; base += 64 * NPC) {
        load_tile<QT, NPC, R>(w, row_base, row0, N, base, Pc, lane, wa);
        compute_tile<QT, NPC, BT, R>(wa, base, Pc, lane, G, lq, ld, ls, acc);
      }
    }
    if (row0 < N) epilogue<BT, R>(P, acc, row0, N, b0, lane);
  }
}

template <int QT, int NPC, int BT, int MODE, int R = GEMV_R>
static void launch_t(const GemvParams& P, hipStream_t s) {
  const int N = P.w.N;
  const int rows_per_block = GEMV_NW * R;
  const int tiles = (N + rows_per_block - 1) / rows_per_block;
  const int by = (P.B + BT - 1) / BT;
  const int bz = P.expert_ids ? P.n_sel : 1;
  // persistent grid: ~2 blocks per CU over all (y, z) slices; each block walks its row tiles
  int gx = tiles;
  const int slots = 256 * g_tune.blocks_per_cu;
  const int cap = slots / (by * bz) > 0 ? slots / (by * bz) : 1;
  if (gx > cap) gx = cap;
  dim3 grid(gx, by, bz);
  const size_t lds = (size_t)BT * (P.w.K / 16) * 24 + 64;
  hipLaunchKernelGGL((gemv_kernel<QT, NPC, BT, MODE, R>), grid, dim3(256), lds, s, P);
}

template <int QT, int BT>
static void launch_b(const GemvParams& P, hipStream_t s) {
  const int Pc = P.w.K / 32;
  const int need = (Pc + 63) / 64;
  // one row per wave doubles the waves in flight and halves each wave's serial dot work; only
  // the epilogues that pair adjacent rows (GLU gate/up, QKV RoPE) need two rows per wave
  const bool r1 = BT == 1 && g_tune.r1 && P.epi != EPI_GLU && P.epi != EPI_QKV && need <= 8;
  if (r1) {
    switch (need) {
      case 1: launch_t<QT, 1, BT, 0, 1>(P, s); return;
      case 2: launch_t<QT, 2, BT, 0, 1>(P, s); return;
      case 3: launch_t<QT, 3, BT, 0, 1>(P, s); return;
      case 4: launch_t<QT, 4, BT, 0, 1>(P, s); return;
      case 5: launch_t<QT, 5, BT, 1, 1>(P, s); return;
      case 6: launch_t<QT, 6, BT, 1, 1>(P, s); return;
      case 7: launch_t<QT, 7, BT, 1, 1>(P, s); return;
      default: launch_t<QT, 8, BT, 1, 1>(P, s); return;
    }
  }
  switch (need) {
    case 1:
      if (BT == 1 && g_tune.rows_per_wave == 4) launch_t<QT, 1, BT, 0, 4>(P, s);
      else launch_t<QT, 1, BT, 0>(P, s);
      break;
    case 2:
      if (BT == 1 && g_tune.rows_per_wave == 4) launch_t<QT, 2, BT, 0, 4>(P, s);
      else launch_t<QT, 2, BT, 0>(P, s);
      break;
    case 3: launch_t<QT, 3, BT, 1>(P, s); break;
    case 4: launch_t<QT, 4, BT, 1>(P, s); break;
    case 5: launch_t<QT, 5, BT, 1>(P, s); break;
    case 6: launch_t<QT, 6, BT, 1>(P, s); break;
    case 7: launch_t<QT, 7, BT, 1>(P, s); break;
    case 8: launch_t<QT, 8, BT, 1>(P, s); break;
    default: launch_t<QT, 8, BT, 2>(P, s); break;
  }
}

template <int QT>
static void launch_q(const GemvParams& P, hipStream_t s) {
  if (P.B == 1 || P.expert_ids != nullptr) {  // decode (and MoE: experts differ per batch row)
    launch_b<QT, 1>(P, s);
    return;
  }
  // small-batch tiles of 4 rows (chunked prefill / batched decode): 2 pieces per lane per K
  // round keeps the 4 x-fragment sets + weights inside the register budget
  const int need = (P.w.K / 32 + 63) / 64;
  if (need == 1) launch_t<QT, 1, 4, 0>(P, s);
  else if (need == 2) launch_t<QT, 2, 4, 0>(P, s);
  else launch_t<QT, 2, 4, 2>(P, s);
}

void gemv(const GemvParams& P, hipStream_t s) {
  switch (P.w.qtype) {
    case QT_Q4_K: launch_q<QT_Q4_K>(P, s); break;
    case QT_Q6_K: launch_q<QT_Q6_K>(P, s); break;
    case QT_Q4_0: launch_q<QT_Q4_0>(P, s); break;
    case QT_Q8_0: launch_q<QT_Q8_0>(P, s); break;
    default: break;
  }
}

size_t gemv_lds_bytes(int K, int B) { return (size_t)(B == 1 ? 1 : 4) * (K / 16) * 24 + 64; }

}  // namespace omx
