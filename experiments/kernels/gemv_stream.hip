// Bounded-depth streaming decode GEMV (B == 1) -- the default decode projection kernel.
//
// Why not "everything in flight" (gemv.hip flight kernel): measured with scripts/gemv_timeline.py
// (profiles/r3_gemv), the flight kernel's activation loads -- issued FIRST by every wave -- still land
// only at the end of the weight stream (gate_up: prologue p50 6.3 us of a 12 us launch; down Q6_K
// 8.2 of 12.5 us), also with every wave draining them before any weight request (x-barrier variant,
// one block per CU). Without any weight traffic the same prologue takes 0.8-2.1 us. With every tile
// of every block requested up front, the chip holds ~the whole matrix (28-50 MB) of outstanding
// requests, and an activation line that misses L2 queues behind that backlog; all dot products then
// run after the stream (first tile +1 us, rest +1.2-1.9 us) instead of under it.
//
// Here each wave keeps at most two (tile, K-chunk) units of weights in registers -- one being
// computed, one landing (explicit register ping-pong) -- so a CU has ~40-80 KB outstanding and the
// chip-wide backlog stays ~10-20 MB (1.5-3 us at HBM rate): the activations are requested first and
// land after one unit, and from then on the dot products keep pace with the stream. One block of 4
// waves per CU (`GemvTuning::stream_bpc` blocks per CU), persistent over units in tile-major order:
// a wave accumulates a tile's K chunks (16 super-blocks = 4096 weights each) and runs the fused
// epilogue once per tile. Reference parity: the decode GEMV of llama.cpp's runner inside
// `ollama/ollama` (reference pkg/model/pod.go:10-12); numerics as gemv.hip (tests/test_kernels_gpu.py).
#include "gemv_core.h"

namespace omx {

// NXG: activation groups of 16 per thread (K <= 4096 * NXG); NRM 0 none / 1 RMS / 2 LayerNorm+bias;
// MRG > 0: deferred flash-decode merge of MRG partial slabs in the prologue (O projection, K <= 4096)
template <int QT, int NXG, int NRM, int MRG>
__device__ __forceinline__ void stream_body(const GemvParams& P, const int bx, const int G) {
  constexpr int NT = GEMV_NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const QMat& w = P.w;
  const int K = w.K, N = w.N, SB = n_sb(K);
  const int XS = SB * XPAD;
  i32x4* lq = (i32x4*)smem;                           // [XS + 1]: slot XS is a dummy
  f32x2* lf = (f32x2*)(smem + (size_t)(XS + 1) * 16);  // [XS + 1]
  float* red = (float*)(lf + XS + 1);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, s = lane & 15;
  const int rbase = wave * 4 + g;
  const int nc = (SB + 15) / 16;
  const int n_tiles = (N + 15) / 16;
  const float* x = P.x;

  // 1. activations (+ norm weights, + merge partials) of this thread's groups -> registers, FIRST
  constexpr bool nrm = NRM != 0, lnb = NRM == 2;
  constexpr int MS = MRG > 0 ? MRG : 1;
  f32x4 xv[NXG][4], nw[NXG][4], nb[NXG][4];
  f32x4 av[MS][NXG][4];
  f32x2 ml[MS][NXG];
#pragma unroll
  for (int i = 0; i < NXG; ++i) {
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
  __builtin_amdgcn_sched_barrier(0);  // activations ahead of every weight request

  // 2. the first unit only (tile bx, chunk 0): the backlog ahead of later activation loads on the
  //    chip stays one unit per wave
  int tile = bx, c = 0;
  WTile<QT, 1, 1> A, Bt;
  if (tile < n_tiles) load_wtile<QT, 1, 1>(w, 0, tile * 16 + rbase, N, SB, 0, s, A);
  __builtin_amdgcn_sched_barrier(0);

  // 3. merge / norm / int8 quantisation from registers into LDS (waits for the activations only)
  if constexpr (MRG > 0) {  // splits without keys carry m = -inf, l = 0
#pragma unroll
    for (int i = 0; i < NXG; ++i) {
      float M = -INFINITY;
#pragma unroll
      for (int sp = 0; sp < MRG; ++sp) M = fmaxf(M, ml[sp][i].x);
      float L = 0.f;
      f32x4 a[4] = {};
#pragma unroll
      for (int sp = 0; sp < MRG; ++sp) {
        const float cc = ml[sp][i].x == -INFINITY ? 0.f : __expf(ml[sp][i].x - M);
        L += cc * ml[sp][i].y;
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] += cc * av[sp][i][j];
      }
      const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[i][j] = a[j] * inv;
    }
  }
#pragma unroll
  for (int i = 0; i < NXG; ++i) {
    const bool ok = 16 * (tid + NT * i) < K;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!ok) xv[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if constexpr (!nrm) nw[i][j] = (f32x4){1.f, 1.f, 1.f, 1.f};
      if constexpr (!lnb) nb[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  }
  float mean = 0.f, rstd = 1.f;
  if constexpr (nrm) {
    float sm = 0.f, ss = 0.f;
#pragma unroll
    for (int i = 0; i < NXG; ++i)
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
  for (int i = 0; i < NXG; ++i) {
    const int gi = tid + NT * i;
    const int slot = gi < SB * 16 ? (gi >> 4) * XPAD + (gi & 15) : XS;  // surplus threads: dummy slot
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

  // 4. units in tile-major order, two in flight: compute `cur` while `nxt` lands
  float acc[1][1] = {{0.f}};
  auto step = [&](WTile<QT, 1, 1>& cur, WTile<QT, 1, 1>& nxt) {
    int nt = tile, ncc = c + 1;
    if (ncc == nc) { ncc = 0; nt += G; }
    if (nt < n_tiles) load_wtile<QT, 1, 1>(w, 0, nt * 16 + rbase, N, SB, ncc * 16, s, nxt);
    compute_wtile<QT, 1, 1, 1>(cur, SB, c * 16, s, lq, lf, XS, acc);
    if (c == nc - 1) {
      finish_rows<1, 1>(P, acc, tile * 16 + rbase, N, 0, s);
      acc[0][0] = 0.f;
    }
    tile = nt;
    c = ncc;
  };
  while (tile < n_tiles) {
    step(A, Bt);
    if (tile >= n_tiles) break;
    step(Bt, A);
  }
}

template <int QT, int NXG, int NRM, int MRG>
__global__ __launch_bounds__(GEMV_NT) void qgemv_stream_kernel(GemvParams P) {
  stream_body<QT, NXG, NRM, MRG>(P, blockIdx.x, gridDim.x);
}

// two matrices over the same normalised x (Q4_K_M QKV: q,k rows Q4_K + v rows Q6_K): blocks [0, ga)
// stream A, the rest B, split in proportion to their bytes
template <int QA, int QB, int NRM>
__global__ __launch_bounds__(GEMV_NT) void qgemv_stream_dual_kernel(GemvParams PA, GemvParams PB, int ga) {
  if ((int)blockIdx.x < ga) stream_body<QA, 1, NRM, 0>(PA, blockIdx.x, ga);
  else stream_body<QB, 1, NRM, 0>(PB, (int)blockIdx.x - ga, (int)gridDim.x - ga);
}

static int stream_cus() {
  static int n = 0;
  if (n <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

static size_t stream_lds(int K) { return (size_t)((K + 255) / 256 * XPAD + 1) * 24 + 4 * GEMV_NW + 16; }

template <int QT, int NXG, int NRM>
static bool launch_stream_n(const GemvParams& P, int gx, hipStream_t s) {
  const size_t lds = stream_lds(P.w.K);
  if constexpr (NXG == 1 && NRM == 0) {
    switch (P.merge_S) {
      case 0: break;
      case 2: hipLaunchKernelGGL((qgemv_stream_kernel<QT, 1, 0, 2>), dim3(gx), dim3(GEMV_NT), lds, s, P); return true;
      case 4: hipLaunchKernelGGL((qgemv_stream_kernel<QT, 1, 0, 4>), dim3(gx), dim3(GEMV_NT), lds, s, P); return true;
      case 8: hipLaunchKernelGGL((qgemv_stream_kernel<QT, 1, 0, 8>), dim3(gx), dim3(GEMV_NT), lds, s, P); return true;
      default: return false;
    }
  }
  if (P.merge_S) return false;
  hipLaunchKernelGGL((qgemv_stream_kernel<QT, NXG, NRM, 0>), dim3(gx), dim3(GEMV_NT), lds, s, P);
  return true;
}

template <int QT, int NXG>
static bool launch_stream_x(const GemvParams& P, int gx, hipStream_t s) {
  if (P.norm == NORM_NONE) return launch_stream_n<QT, NXG, 0>(P, gx, s);
  if (P.norm == NORM_LAYER && P.norm_b) return launch_stream_n<QT, NXG, 2>(P, gx, s);
  return launch_stream_n<QT, NXG, 1>(P, gx, s);
}

template <int QT>
static bool launch_stream_q(const GemvParams& P, hipStream_t s) {
  const int nxg = (P.w.K / 16 + GEMV_NT - 1) / GEMV_NT;
  const int tiles = (P.w.N + 15) / 16;
  int gx = stream_cus() * (g_tune.stream_bpc > 0 ? g_tune.stream_bpc : 1);
  if (gx > tiles) gx = tiles;
  switch (nxg) {
    case 1: return launch_stream_x<QT, 1>(P, gx, s);
    case 2: return P.merge_S ? false : launch_stream_x<QT, 2>(P, gx, s);
    case 3: return P.merge_S ? false : launch_stream_x<QT, 3>(P, gx, s);
    default: return false;
  }
}

bool gemv_stream(const GemvParams& P, hipStream_t s) {
  if (!g_tune.stream || P.B != 1 || P.expert_ids || g_tune.debug || P.w.s4) return false;
  switch (P.w.qtype) {
    case QT_Q4_K: return launch_stream_q<QT_Q4_K>(P, s);
    case QT_Q6_K: return launch_stream_q<QT_Q6_K>(P, s);
    case QT_Q5_K: return launch_stream_q<QT_Q5_K>(P, s);
    case QT_Q4_0: return launch_stream_q<QT_Q4_0>(P, s);
    case QT_Q8_0: return launch_stream_q<QT_Q8_0>(P, s);
    default: return false;
  }
}

template <int QA, int QB>
static bool launch_stream_dual(const GemvParams& A, const GemvParams& Bp, hipStream_t s) {
  const int ta = (A.w.N + 15) / 16, tb = (Bp.w.N + 15) / 16;
  const double ba = (double)A.w.N * A.w.K, bb = (double)Bp.w.N * Bp.w.K * (QB == QT_Q6_K ? 210.0 / 144.0 : 1.0);
  int G = stream_cus() * (g_tune.stream_bpc > 0 ? g_tune.stream_bpc : 1);
  if (G > ta + tb) G = ta + tb;
  int ga = (int)(G * ba / (ba + bb) + 0.5);
  ga = ga < 1 ? 1 : ga > G - 1 ? G - 1 : ga;
  if (ga > ta) ga = ta;
  if (G - ga > tb) G = ga + tb;
  const size_t lds = stream_lds(A.w.K);
  if (A.norm == NORM_LAYER && A.norm_b)
    hipLaunchKernelGGL((qgemv_stream_dual_kernel<QA, QB, 2>), dim3(G), dim3(GEMV_NT), lds, s, A, Bp, ga);
  else
    hipLaunchKernelGGL((qgemv_stream_dual_kernel<QA, QB, 1>), dim3(G), dim3(GEMV_NT), lds, s, A, Bp, ga);
  return true;
}

bool gemv_stream2(const GemvParams& A, const GemvParams& Bp, hipStream_t s) {
  if (!g_tune.stream || g_tune.debug || A.w.K > 4096 || A.w.s4 || Bp.w.s4) return false;
  if (A.w.qtype == QT_Q4_K && Bp.w.qtype == QT_Q6_K) return launch_stream_dual<QT_Q4_K, QT_Q6_K>(A, Bp, s);
  if (A.w.qtype == QT_Q5_K && Bp.w.qtype == QT_Q6_K) return launch_stream_dual<QT_Q5_K, QT_Q6_K>(A, Bp, s);
  return false;
}

}  // namespace omx
