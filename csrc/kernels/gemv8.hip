// Batch-1 decode GEMV on the int8 activation chain (Llama-family decode, tp == 1).
//
// Why: the gemv.hip flight kernel pays an activation prologue in every launch -- each block loads the
// fp32 input row (16-44 KB) plus the RMSNorm weights, reduces the sum of squares across the block and
// int8-quantises per 16-element group before its first dot product. Measured (profiles/r3_gemv
// timeline + dbg variants): that prologue ends only when most of the weight stream has landed (the
// block's waves sit behind their own weight-load issue, then meet at the norm barriers), and it costs
// 1-3 us per launch (gate_up: 11.9 us with the prologue and no dot products, 9.0 us without either).
//
// Here the PRODUCER of each GEMV input writes it already quantised, in the consumer's LDS image layout
// (ops.h x8_bytes): the residual-adding projections (O, down) emit int8(new_resid * next_norm_w) per
// 16-row group plus the group's sum of squares of new_resid; gate_up emits int8(silu(g) * u). The
// consumer copies the image (6.5 KB for K = 4096) into LDS -- loads issued before any weight load --
// and applies rsqrt(sum / K + eps) to its outputs (an RMSNorm is a per-row scalar of the input), so a
// launch has no norm reduction, no quantisation and no fp32 activation traffic. The weight tiles, lane
// mapping, dot products and epilogues are gemv.hip's (gemv_core.h): layout v2 pieces, 16 lanes per row
// group, one super-block per lane, v_dot4 int8 dots, fused RoPE/KV-scatter/GLU/residual epilogues.
//
// Emission: one quantisation group = 16 consecutive outputs = one 16-row tile (EPI_ADD) or two
// consecutive tiles of interleaved gate/up rows (EPI_GLU: 8 outputs each), so a block owns whole
// groups: its tiles are consecutive (tile0 = block * J). The 16 values meet in LDS; one lane quantises.
// The O projection keeps the deferred flash-decode merge input (IN_MERGE) and emits like down.
// Reference parity: the decode GEMVs of llama.cpp inside `ollama/ollama` (reference
// pkg/model/pod.go:10-12); numerics checked against an fp32 torch GEMV (tests/test_gemv8_gpu.py).
#include "gemv8_body.h"

namespace omx {

template <int QT, int NSB, int J, int KS, int IN, int MS, int EMIT, int BT>
__global__ __launch_bounds__(GEMV_NT * KS) void qgemv8_kernel(GemvParams P) {
  gemv8_body<QT, NSB, J, KS, IN, MS, EMIT, false, BT>(P, blockIdx.x);
}

// q,k rows + v rows of different quant types (Q4_K_M QKV) over the same image: one launch
template <int QA, int QB, int IN, int BT>
__global__ __launch_bounds__(GEMV_NT) void qgemv8_dual_kernel(GemvParams PA, GemvParams PB, int gxa) {
  if ((int)blockIdx.x < gxa) gemv8_body<QA, 1, 1, 1, IN, 0, EM_NONE, false, BT>(PA, blockIdx.x);
  else gemv8_body<QB, 1, 1, 1, IN, 0, EM_NONE, false, BT>(PB, (int)blockIdx.x - gxa);
}

// ------------------------------------------------------------------------------------------------
// gate_up -> down in ONE launch (batch-1 FFN). Phase A: every block computes its gate_up tile pair and
// emits its slice of down's int8 image with write-through (sc1) stores, then arrives on a counter.
// Phase B: the last N_down / 16 blocks of the grid also own one down tile each: they request that
// tile's weights right after their phase-A work -- BEFORE the hand-off -- so the down weight stream
// overlaps the gate_up tail, the launch boundary and the hand-off wait, then wait for every arrival
// and read the image with sc1 loads. Hand-off form: MI355X_MICROARCH.md "Valid forms" table row 1
// (every storing wave vmcnt(0) -> workgroup barrier -> one lane's agent-scope atomic add; the poller
// loads after its poll matched, the other waves after the barrier it joins; every byte stored and
// loaded sc1). Deadlock freedom: waiting blocks never exceed the grid's residency minus the other
// blocks' slots (host check), and a wait gives up after 2 ms (error word; the runner raises).
constexpr int FFN_IMG_DW = 20;  // image dwords per thread (K <= 13568 at 256 threads)

// phase B: one 16-row down tile, input image handed off in this launch, EPI_ADD + emission
template <int QT, int NSB>
__device__ __forceinline__ void gemv8_after(const GemvParams& P, const int tile, const Handoff& H) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const QMat& w = P.w;
  const int K = w.K, N = w.N, SB = n_sb(K), XS = SB * XPAD, XSP = x8_slots_dev(K);
  i32x4* lq = (i32x4*)smem;
  f32x2* lf = (f32x2*)(smem + (size_t)XSP * 16);
  float* stage = (float*)(lf + XSP);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, s = lane & 15;
  const int rbase = wave * 4 + g;
  WTile<QT, NSB, 1> T;
  load_wtile<QT, NSB, 1>(w, 0, tile * 16 + rbase, N, SB, 0, s, T, SB);  // ahead of the hand-off
  __builtin_amdgcn_sched_barrier(0);
  handoff_wait(H);
  const int nd = XSP * 6;  // image dwords
  const unsigned* src = (const unsigned*)P.x8;
  unsigned xd[FFN_IMG_DW];
#pragma unroll
  for (int i = 0; i < FFN_IMG_DW; ++i)
    xd[i] = __hip_atomic_load(src + min(tid + GEMV_NT * i, nd - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int i = 0; i < FFN_IMG_DW; ++i)
    if (tid + GEMV_NT * i < nd) ((unsigned*)smem)[tid + GEMV_NT * i] = xd[i];
  __syncthreads();
  float acc[1][1] = {{0.f}};
  compute_wtile<QT, NSB, 1, 1>(T, SB, 0, s, lq, lf, XS, acc, SB);
  const float v = row16_sum(acc[0][0]);
  const int n = tile * 16 + rbase;
  if (s == 0) {
    float nv = 0.f;
    if (n < N) {
      float* dst = P.y + n;
      nv = *dst + v + (P.bias ? P.bias[n] : 0.f);
      *dst = nv;
    }
    stage[rbase] = n < N ? nv * P.emit8_nw[n] : 0.f;
    stage[16 + rbase] = nv * nv;
  }
  __syncthreads();
  if (tid == 0) emit_group(P.emit8, N, tile, stage, stage + 16, P.emit8_stat);
}

template <int QA, int QB, int NSBB>
__global__ __launch_bounds__(GEMV_NT, 2) void ffn8_kernel(GemvParams PA, GemvParams PB, Handoff H) {
  const int bx = blockIdx.x;
  gemv8_body<QA, 1, 2, 1, IN_X8_RMS, 0, EM_GLU, true>(PA, bx);  // gate_up tile pair -> down's image
  handoff_arrive(H);
  const int tb = bx - ((int)gridDim.x - H.n_cons);  // this block's down tile (the grid's last blocks)
  if (tb < 0) return;
  __syncthreads();  // the LDS image of phase A is rewritten below
  gemv8_after<QB, NSBB>(PB, tb, H);
}

// ------------------------------------------------------------------------------------------------
// host side
namespace {

size_t lds8(int K, int KS, int BT = 1) { return BT * x8_bytes(K) + (size_t)BT * (32 + (KS - 1) * GEMV_NT) * 4; }

// batch rows per launch: exactly B (1-4)
int bt_of(int B) { return B; }

// 4 rows fit the register budget of 768 / 1024-thread blocks only without the RMS partials and the
// Q5_K high-bit planes (kernel-resource-usage: these would spill); such launches are not covered
constexpr bool bt4_ok(int qt, int ks, int in) { return ks <= 2 || (ks == 3 && in != IN_X8_RMS && qt != QT_Q5_K); }

// > 64 KB of LDS (batched rows of a long-K image): raised once per kernel instantiation
template <typename Kern>
void lds_attr(Kern k, size_t lds) {
  static bool done = false;
  if (lds > 64 * 1024 && !done) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    done = true;
  }
}

int emit_mode(const GemvParams& P) {
  if (!P.emit8) return EM_NONE;
  if (P.epi == EPI_ADD) return EM_ADD;
  if (P.epi == EPI_GLU || P.epi == EPI_GEGLU) return EM_GLU;
  return -1;
}

int in_mode(const GemvParams& P) {
  if (P.x8) return P.x8_stat ? IN_X8_RMS : IN_X8;
  if (P.norm != NORM_NONE) return -1;  // fp32 input with a norm: gemv.hip's prologue
  return IN_MERGE;                      // merge slabs (O) or a plain fp32 row
}

// launch geometry: (NSB, KS) from K; J tiles per block
struct Geo {
  int nsb = 0, ks = 0, J = 0, grid = 0;
};

bool geometry(const GemvParams& P, Geo& G) {
  const int SB = (P.w.K + 255) / 256, need = (SB + 15) / 16;
  const int tiles = (P.w.N + 15) / 16;
  if (need == 1) { G.nsb = 1; G.ks = 1; }
  else if (need == 2) { G.nsb = tiles > 512 ? 2 : 1; G.ks = tiles > 512 ? 1 : 2; }
  else if (need <= 4) { G.nsb = 1; G.ks = need; }
  else return false;
  if (G.ks > 1) {
    G.J = 1;
  } else {
    const int want = 256 * g_tune.blocks_per_cu;
    G.J = (tiles + want - 1) / want;
    G.J = G.J < 1 ? 1 : G.J > 2 ? 2 : G.J;
    if (emit_mode(P) == EM_GLU) G.J = 2;  // a block owns whole groups (two tiles each)
    // two super-blocks per lane and two tiles: the GLU producer at 4096 < K <= 8192 only (Llama-2-13B
    // gate_up, K = 5120), from the RMS image, at most 2 batch rows (launch_glu_nsb2)
    if (G.nsb == 2 && G.J > 1) {
      if (emit_mode(P) == EM_GLU) {
        if (in_mode(P) != IN_X8_RMS || P.B > 2) return false;
      } else {
        G.J = 1;  // > 512 tiles: one tile per block still fills the chip (QKV at K = 5120: 960 blocks)
      }
    }
  }
  G.grid = (tiles + G.J - 1) / G.J;
  return true;
}

bool covered(const GemvParams& P, Geo& G) {
  if (P.B < 1 || P.B > X8_MAX_B || P.expert_ids || P.w.s0 == nullptr || P.dbg_ts) return false;
  const int em = emit_mode(P), in = in_mode(P);
  if (em < 0 || in < 0) return false;
  if (P.B > 1 && in == IN_MERGE && P.merge_S > 0) return false;  // batched rows: plain fp32 attention rows
  if (!P.x8 && !P.emit8) return false;  // nothing for this path to do
  if (in == IN_MERGE && P.merge_S > 0 && !(P.merge_S == 2 || P.merge_S == 4 || P.merge_S == 8)) return false;
  if (in == IN_MERGE && P.w.K % 16) return false;
  if (in == IN_X8_RMS && (P.w.K > 8192 || P.w.K % 64)) return false;
  if (em == EM_ADD && (!P.emit8_nw || !P.emit8_stat || P.w.N % 16)) return false;
  if (em == EM_GLU && P.w.N % 32) return false;
  const int q = P.w.qtype;
  if (!(q == QT_Q4_K || q == QT_Q6_K || q == QT_Q4_0 || q == QT_Q8_0 || q == QT_Q5_K)) return false;
  if (!geometry(P, G)) return false;
  // merge prologue: one 16-element group per thread and group slot (NSB slots); the deferred merge
  // (merge_S > 1) exists for the unsplit geometry only
  if (in == IN_MERGE && (P.w.K > GEMV_NT * G.ks * G.nsb * 16 || (P.merge_S > 1 && G.ks > 1))) return false;
  if (em == EM_GLU && G.J != 2) return false;  // a block owns whole groups: two tiles, unsplit K
  if (in != IN_MERGE && (size_t)G.ks * GEMV_NT * X8_NWI * 16 < x8_bytes(P.w.K)) return false;
  if (bt_of(P.B) >= 3 && !bt4_ok(q, G.ks, in)) return false;
  return lds8(P.w.K, G.ks, bt_of(P.B)) <= (P.B > 1 ? 160 : 64) * 1024;
}

template <int QT, int NSB, int J, int KS, int IN, int MS, int EMIT, int BT>
void launch_k(const GemvParams& P, int grid, hipStream_t s) {
  const size_t lds = lds8(P.w.K, KS, BT);
  auto k = qgemv8_kernel<QT, NSB, J, KS, IN, MS, EMIT, BT>;
  lds_attr(k, lds);
  hipLaunchKernelGGL(k, dim3(grid), dim3(GEMV_NT * KS), lds, s, P);
}

template <int QT, int NSB, int J, int KS, int IN, int MS, int BT>
void launch_em_bt(const GemvParams& P, int em, int grid, hipStream_t s) {
  if (em == EM_ADD) launch_k<QT, NSB, J, KS, IN, MS, EM_ADD, BT>(P, grid, s);
  else if (em == EM_GLU) {
    if constexpr (J == 2) launch_k<QT, NSB, J, KS, IN, MS, EM_GLU, BT>(P, grid, s);
  } else launch_k<QT, NSB, J, KS, IN, MS, EM_NONE, BT>(P, grid, s);
}

template <int QT, int NSB, int J, int KS, int IN, int MS>
void launch_em(const GemvParams& P, int em, int grid, hipStream_t s) {
  if constexpr (MS > 1) {
    launch_em_bt<QT, NSB, J, KS, IN, MS, 1>(P, em, grid, s);
  } else {
    switch (bt_of(P.B)) {
      case 1: launch_em_bt<QT, NSB, J, KS, IN, MS, 1>(P, em, grid, s); break;
      case 2: launch_em_bt<QT, NSB, J, KS, IN, MS, 2>(P, em, grid, s); break;
      case 3:
        if constexpr (bt4_ok(QT, KS, IN)) launch_em_bt<QT, NSB, J, KS, IN, MS, 3>(P, em, grid, s);
        break;
      default:
        if constexpr (bt4_ok(QT, KS, IN)) launch_em_bt<QT, NSB, J, KS, IN, MS, 4>(P, em, grid, s);
        break;
    }
  }
}

template <int QT, int NSB, int J, int KS>
void launch_in(const GemvParams& P, const Geo& G, hipStream_t s) {
  const int em = emit_mode(P), in = in_mode(P);
  if (in == IN_X8) launch_em<QT, NSB, J, KS, IN_X8, 0>(P, em, G.grid, s);
  else if (in == IN_X8_RMS) launch_em<QT, NSB, J, KS, IN_X8_RMS, 0>(P, em, G.grid, s);
  else if constexpr (NSB == 1 && KS == 2 && J == 1) {  // O at 4096 < K <= 8192: plain fp32 rows
    launch_em<QT, 1, 1, 2, IN_MERGE, 1>(P, em, G.grid, s);
  } else if constexpr (NSB == 1 && KS == 1 && J == 1) {  // the O projection: merge slabs or plain fp32
    switch (P.merge_S) {
      case 2: launch_em<QT, 1, 1, 1, IN_MERGE, 2>(P, em, G.grid, s); break;
      case 4: launch_em<QT, 1, 1, 1, IN_MERGE, 4>(P, em, G.grid, s); break;
      case 8: launch_em<QT, 1, 1, 1, IN_MERGE, 8>(P, em, G.grid, s); break;
      default: launch_em<QT, 1, 1, 1, IN_MERGE, 1>(P, em, G.grid, s); break;
    }
  }
}

template <int QT>
void launch_glu_nsb2(const GemvParams& P, const Geo& G, hipStream_t s) {
  if (bt_of(P.B) == 1) launch_k<QT, 2, 2, 1, IN_X8_RMS, 0, EM_GLU, 1>(P, G.grid, s);
  else launch_k<QT, 2, 2, 1, IN_X8_RMS, 0, EM_GLU, 2>(P, G.grid, s);
}

template <int QT>
void launch_q(const GemvParams& P, const Geo& G, hipStream_t s) {
  if (G.ks == 1 && G.nsb == 2 && G.J == 2) launch_glu_nsb2<QT>(P, G, s);
  else if (G.ks == 1 && G.nsb == 1 && G.J == 1) launch_in<QT, 1, 1, 1>(P, G, s);
  else if (G.ks == 1 && G.nsb == 1) launch_in<QT, 1, 2, 1>(P, G, s);
  else if (G.ks == 1 && G.nsb == 2) launch_in<QT, 2, 1, 1>(P, G, s);
  else if (G.ks == 2) launch_in<QT, 1, 1, 2>(P, G, s);
  else if (G.ks == 3) launch_in<QT, 1, 1, 3>(P, G, s);
  else launch_in<QT, 1, 1, 4>(P, G, s);
}

bool launchable(const GemvParams& P, const Geo& G) {
  // the merge / plain-fp32 input exists for single-tile blocks, unsplit or split in 2 (K <= 8192)
  return in_mode(P) != IN_MERGE || (G.ks <= 2 && G.nsb == 1 && G.J == 1);
}

template <int QA, int QB, int IN, int BT>
void launch_dual_k(const GemvParams& A, const GemvParams& B, int gxa, int gxb, hipStream_t s) {
  const size_t lds = lds8(A.w.K, 1, BT);
  auto k = qgemv8_dual_kernel<QA, QB, IN, BT>;
  lds_attr(k, lds);
  hipLaunchKernelGGL(k, dim3(gxa + gxb), dim3(GEMV_NT), lds, s, A, B, gxa);
}

template <int QA, int QB, int IN>
void launch_dual_in(const GemvParams& A, const GemvParams& B, int gxa, int gxb, hipStream_t s) {
  switch (bt_of(A.B)) {
    case 1: launch_dual_k<QA, QB, IN, 1>(A, B, gxa, gxb, s); break;
    case 2: launch_dual_k<QA, QB, IN, 2>(A, B, gxa, gxb, s); break;
    case 3: launch_dual_k<QA, QB, IN, 3>(A, B, gxa, gxb, s); break;
    default: launch_dual_k<QA, QB, IN, 4>(A, B, gxa, gxb, s); break;
  }
}

template <int QA, int QB>
void launch_dual(const GemvParams& A, const GemvParams& B, int gxa, int gxb, hipStream_t s) {
  if (A.x8_stat) launch_dual_in<QA, QB, IN_X8_RMS>(A, B, gxa, gxb, s);
  else launch_dual_in<QA, QB, IN_X8>(A, B, gxa, gxb, s);
}

template <int QA>
bool dual_b(const GemvParams& A, const GemvParams& B, int gxa, int gxb, hipStream_t s) {
  switch (B.w.qtype) {
    case QT_Q6_K: launch_dual<QA, QT_Q6_K>(A, B, gxa, gxb, s); return true;
    case QT_Q4_K: launch_dual<QA, QT_Q4_K>(A, B, gxa, gxb, s); return true;
    case QT_Q8_0: launch_dual<QA, QT_Q8_0>(A, B, gxa, gxb, s); return true;
    default: return false;
  }
}

template <int QA, int QB, int NSBB>
bool launch_ffn(const GemvParams& G, const GemvParams& D, Handoff H, hipStream_t s) {
  const size_t lds = lds8(max(G.w.K, D.w.K), 1);
  const int nA = ((G.w.N + 15) / 16 + 1) / 2, nB = (D.w.N + 15) / 16;
  const int grid = max(nA, nB);
  static int cap_cache[8][2] = {};  // (blocks per CU, CUs) per device, for this instantiation
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 8) return false;
  int* cc = cap_cache[dev];
  if (cc[0] == 0) {
    int nb = 0, ncu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, ffn8_kernel<QA, QB, NSBB>, GEMV_NT, lds) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return false;
    cc[0] = nb > 0 ? nb : -1;
    cc[1] = ncu;
  }
  // the nB waiting blocks must leave at least as many slots to the rest of the grid (progress)
  if (cc[0] < 0 || (long long)cc[0] * cc[1] < 2LL * nB) return false;
  H.n_prod = grid;
  H.n_cons = nB;
  hipLaunchKernelGGL((ffn8_kernel<QA, QB, NSBB>), dim3(grid), dim3(GEMV_NT), lds, s, G, D, H);
  return true;
}

template <int QA, int QB>
bool ffn_nsb(const GemvParams& G, const GemvParams& D, const Handoff& H, hipStream_t s) {
  switch (((D.w.K + 255) / 256 + 15) / 16) {
    case 1: return launch_ffn<QA, QB, 1>(G, D, H, s);
    case 2: return launch_ffn<QA, QB, 2>(G, D, H, s);
    case 3: return launch_ffn<QA, QB, 3>(G, D, H, s);
    default: return false;
  }
}

template <int QA>
bool ffn_b(const GemvParams& G, const GemvParams& D, const Handoff& H, hipStream_t s) {
  switch (D.w.qtype) {
    case QT_Q4_K: return ffn_nsb<QA, QT_Q4_K>(G, D, H, s);
    case QT_Q6_K: return ffn_nsb<QA, QT_Q6_K>(G, D, H, s);
    case QT_Q4_0: return ffn_nsb<QA, QT_Q4_0>(G, D, H, s);
    case QT_Q8_0: return ffn_nsb<QA, QT_Q8_0>(G, D, H, s);
    default: return false;
  }
}

}  // namespace

bool gemv8_ffn(const GemvParams& G, const GemvParams& D, void* sync, hipStream_t s) {
  Geo GG, GD;
  if (!sync || G.B != 1 || !covered(G, GG) || !covered(D, GD)) return false;
  if (emit_mode(G) != EM_GLU || in_mode(G) != IN_X8_RMS || GG.nsb != 1 || GG.ks != 1 || GG.J != 2) return false;
  if (emit_mode(D) != EM_ADD || in_mode(D) != IN_X8 || D.x8 != G.emit8 || D.w.K != G.w.N / 2) return false;
  if ((size_t)FFN_IMG_DW * GEMV_NT * 4 < x8_bytes(D.w.K)) return false;
  Handoff H{};
  H.count = (unsigned*)sync;
  H.done = (unsigned*)sync + 1;
  H.err = (int*)sync + 2;
  switch (G.w.qtype) {
    case QT_Q4_K: return ffn_b<QT_Q4_K>(G, D, H, s);
    case QT_Q4_0: return ffn_b<QT_Q4_0>(G, D, H, s);
    case QT_Q8_0: return ffn_b<QT_Q8_0>(G, D, H, s);
    default: return false;
  }
}

bool gemv8_supported(const GemvParams& P) {
  Geo G;
  return covered(P, G) && launchable(P, G);
}

bool gemv8(const GemvParams& P, hipStream_t s) {
  Geo G;
  if (!covered(P, G) || !launchable(P, G)) return false;
  count_launch(P.B > 1 ? LC_GEMV8_ROWS : LC_GEMV8_ROW1);
  switch (P.w.qtype) {
    case QT_Q4_K: launch_q<QT_Q4_K>(P, G, s); return true;
    case QT_Q6_K: launch_q<QT_Q6_K>(P, G, s); return true;
    case QT_Q5_K: launch_q<QT_Q5_K>(P, G, s); return true;
    case QT_Q4_0: launch_q<QT_Q4_0>(P, G, s); return true;
    case QT_Q8_0: launch_q<QT_Q8_0>(P, G, s); return true;
    default: return false;
  }
}

bool gemv8_2(const GemvParams& A, const GemvParams& B, hipStream_t s) {
  Geo GA, GB;
  if (!A.x8 || !B.x8 || A.x8 != B.x8 || A.emit8 || B.emit8 || A.w.K != B.w.K || A.B != B.B) return false;
  if (!covered(A, GA) || !covered(B, GB) || GA.nsb != 1 || GA.ks != 1 || GB.nsb != 1 || GB.ks != 1) return false;
  const int gxa = (A.w.N + 15) / 16, gxb = (B.w.N + 15) / 16;  // one tile per block on both sides
  count_launch(LC_GEMV8_DUAL);
  switch (A.w.qtype) {
    case QT_Q4_K: return dual_b<QT_Q4_K>(A, B, gxa, gxb, s);
    case QT_Q5_K: return dual_b<QT_Q5_K>(A, B, gxa, gxb, s);
    case QT_Q4_0: return dual_b<QT_Q4_0>(A, B, gxa, gxb, s);
    default: return false;
  }
}

}  // namespace omx
