// The attention half of a batch-1 decode layer in ONE launch (Llama family, tp == 1, short context):
//
//   phase A  QKV GEMV (int8 image in, gemv8.hip) + RoPE + KV-cache scatter, stores write-through (sc1)
//   phase A2 per KV group: the LAST block to finish the group's q/k/v tiles runs that group's attention
//            (G query heads over the paged cache) and writes its slice of the O projection's int8
//            input image -- no block ever waits in this phase
//   phase B  O projection (+ residual, + gate_up's int8 image): every block requests its O tile's
//            weights right after phase A, then waits until every group's attention is published
//
// Why: as separate launches (QKV 7.7-9.0 us, attention 5.4-7.3 us, O 5.3-5.9 us; profiles/r4_*),
// each pays a launch boundary, a cold weight-stream ramp and a compute tail; attention is pure latency
// (q + block table -> K/V -> softmax -> merge) on a few dozen blocks while the chip idles. Here the O
// weights stream under the attention, and the q/k/v hand-off is a last-arriver ticket (no spin).
// Hand-offs follow MI355X_MICROARCH.md "Valid forms" table row 1 (sc1 stores, vmcnt(0) -> barrier ->
// one agent-scope atomic; sc1 loads after the poll / ticket). Residency: every block waits in phase B,
// so the grid (one block per CU) must be co-resident -- the host checks the occupancy; a wait gives
// up after 2 ms and raises the error word (the runner checks it). Long contexts (> 512 keys) keep the
// split flash-decode kernel (attention.hip): one block per KV group would be bandwidth-starved there.
// Reference parity: the attention + projections of llama.cpp's decode graph inside `ollama/ollama`
// (reference pkg/model/pod.go:10-12); numerics vs the fp32 torch twin (tests/test_attn8_gpu.py).
#include "attn8_core.h"

namespace omx {

template <int QA, int QB, int G, int JA, int JB, int JO, int NSB>
__global__ __launch_bounds__(GEMV_NT, 1) void attn8_kernel(Attn8Params P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bx = blockIdx.x, g = bx / P.bpg, j = bx % P.bpg;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, gq = lane >> 4, s = lane & 15;
  const int rbase = wave * 4 + gq;
  const GemvParams& A = P.A;
  const int Eq = A.Eq, Ekv = A.Ekv;
  constexpr bool FUSED = QB == 0;
  constexpr int NAT = (G + 1 + (FUSED ? 1 : 0)) * A8_TPH, NBT = FUSED ? 0 : A8_TPH;

  // ---- phase A: QKV rows of this block (image + RMS partials first, then every weight tile)
  const int K = A.w.K, SB = n_sb(K), XS = SB * XPAD, XSP = x8_slots_dev(K);
  i32x4* lq = (i32x4*)smem;
  f32x2* lf = (f32x2*)(smem + (size_t)XSP * 16);
  const int nwords = XSP * 3 / 2;
  u32x4 xw[X8_NWI];
  f32x4 stv[X8_NSTW];
#pragma unroll
  for (int i = 0; i < X8_NWI; ++i) xw[i] = ((const u32x4*)A.x8)[min(tid + GEMV_NT * i, nwords - 1)];
  const int n4 = K / 64;
#pragma unroll
  for (int i = 0; i < X8_NSTW; ++i) stv[i] = ((const f32x4*)A.x8_stat)[min(lane + 64 * i, n4 - 1)];
  __builtin_amdgcn_sched_barrier(0);
  WTile<QA, NSB, 1> TA[JA];
#pragma unroll
  for (int i = 0; i < JA; ++i) {
    const int idx = min(j + P.bpg * i, NAT - 1);
    load_wtile<QA, NSB, 1>(A.w, 0, a_row<G>(idx, g, Eq, Ekv) + rbase, A.w.N, SB, 0, s, TA[i]);
  }
  constexpr int QBT = FUSED ? QA : QB;
  WTile<QBT, NSB, 1> TB[JB > 0 ? JB : 1];
#pragma unroll
  for (int i = 0; i < JB; ++i) {
    const int idx = min(j + P.bpg * i, NBT - 1);
    load_wtile<QBT, NSB, 1>(P.B.w, 0, g * A8_D + 16 * idx + rbase, P.B.w.N, SB, 0, s, TB[i]);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < X8_NWI; ++i)
    if (tid + GEMV_NT * i < nwords) ((u32x4*)smem)[tid + GEMV_NT * i] = xw[i];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < X8_NSTW; ++i)
    if (lane + 64 * i < n4) ss += stv[i].x + stv[i].y + stv[i].z + stv[i].w;
  const float rstd = rsqrtf(wave_sum(ss) / K + A.eps);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < JA; ++i) {
    const int idx = j + P.bpg * i;
    if (idx >= NAT) break;  // block-uniform
    float acc[1][1] = {{0.f}};
    compute_wtile<QA, NSB, 1, 1>(TA[i], SB, 0, s, lq, lf, XS, acc);
    const float v = row16_sum(acc[0][0] * rstd), pv = __shfl_xor(v, 16, OMX_WAVE);
    if (s == 0) epi_qkv_wt(A, a_row<G>(idx, g, Eq, Ekv) + rbase, v, pv);
  }
#pragma unroll
  for (int i = 0; i < JB; ++i) {
    const int idx = j + P.bpg * i;
    if (idx >= NBT) break;
    float acc[1][1] = {{0.f}};
    compute_wtile<QBT, NSB, 1, 1>(TB[i], SB, 0, s, lq, lf, XS, acc);
    const float v = row16_sum(acc[0][0] * rstd), pv = __shfl_xor(v, 16, OMX_WAVE);
    if (s == 0) epi_qkv_wt(P.B, g * A8_D + 16 * idx + rbase + P.B.row_offset, v, pv);
  }
  // ---- group ticket: the last of the bpg blocks of group g runs its attention
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(P.sync + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == (unsigned)P.bpg - 1;
    if (s_last) __hip_atomic_store(P.sync + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  }
  __syncthreads();
  if (s_last) {
    attn_group<G>(P, g, smem);
    Handoff Hh{P.sync + 64, P.sync + 65, (int*)P.sync + 66, 0, 0};
    handoff_arrive(Hh);
    __syncthreads();  // smem is rewritten by phase B
  }

  // ---- phase B: O tiles (weights requested before the wait), input image handed off above
  const GemvParams& O = P.O;
  const int KO = O.w.K, SBO = n_sb(KO), XSO = SBO * XPAD, XSPO = x8_slots_dev(KO);
  const int nO = (O.w.N + 15) / 16;
  WTile<QA, NSB, 1> TO[JO];
#pragma unroll
  for (int i = 0; i < JO; ++i) {
    const int t = min(bx + (int)gridDim.x * i, nO - 1);
    load_wtile<QA, NSB, 1>(O.w, 0, t * 16 + rbase, O.w.N, SBO, 0, s, TO[i]);
  }
  __builtin_amdgcn_sched_barrier(0);
  Handoff H{P.sync + 64, P.sync + 65, (int*)P.sync + 66, P.Hkv, (int)gridDim.x};
  handoff_wait(H);
  {
    const int nd = XSPO * 6;
    const unsigned* src = (const unsigned*)O.x8;
    constexpr int NDW = 20;
    unsigned xd[NDW];
#pragma unroll
    for (int i = 0; i < NDW; ++i)
      xd[i] = __hip_atomic_load(src + min(tid + GEMV_NT * i, nd - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int i = 0; i < NDW; ++i)
      if (tid + GEMV_NT * i < nd) ((unsigned*)smem)[tid + GEMV_NT * i] = xd[i];
  }
  __syncthreads();
  i32x4* lqo = (i32x4*)smem;
  f32x2* lfo = (f32x2*)(smem + (size_t)XSPO * 16);
  float* stage = (float*)(lfo + XSPO);
#pragma unroll
  for (int i = 0; i < JO; ++i) {
    const int t = bx + (int)gridDim.x * i;
    if (t >= nO) break;  // block-uniform
    float acc[1][1] = {{0.f}};
    compute_wtile<QA, NSB, 1, 1>(TO[i], SBO, 0, s, lqo, lfo, XSO, acc);
    const float v = row16_sum(acc[0][0]);
    const int n = t * 16 + rbase;
    if (s == 0) {
      float nv = 0.f;
      if (n < O.w.N) {
        float* dst = O.y + n;
        nv = *dst + v + (O.bias ? O.bias[n] : 0.f);
        *dst = nv;
      }
      stage[rbase] = n < O.w.N ? nv * O.emit8_nw[n] : 0.f;
      stage[16 + rbase] = nv * nv;
    }
    __syncthreads();
    if (tid == 0) emit_group(O.emit8, O.w.N, t, stage, stage + 16, O.emit8_stat);
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
namespace {

template <int QA, int QB, int G, int JA, int JB, int JO, int NSB>
bool launch_a8(const Attn8Params& P, int grid, size_t lds, hipStream_t s) {
  static int occ[8] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 8) return false;
  if (occ[dev] == 0) {
    int nb = 0, ncu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, attn8_kernel<QA, QB, G, JA, JB, JO, NSB>, GEMV_NT, lds) !=
            hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return false;
    occ[dev] = nb * ncu > 0 ? nb * ncu : -1;
  }
  if (occ[dev] < grid) return false;  // every block waits in phase B: the grid must be co-resident
  hipLaunchKernelGGL((attn8_kernel<QA, QB, G, JA, JB, JO, NSB>), dim3(grid), dim3(GEMV_NT), lds, s, P);
  return true;
}

template <int QA, int QB, int G>
bool a8_shape(const Attn8Params& P, int grid, size_t lds, hipStream_t s) {
  constexpr bool FUSED = QB == 0;
  constexpr int NAT = (G + 1 + (FUSED ? 1 : 0)) * A8_TPH, NBT = FUSED ? 0 : A8_TPH;
  const int ja = (NAT + P.bpg - 1) / P.bpg, jb = FUSED ? 0 : (NBT + P.bpg - 1) / P.bpg;
  const int jo = ((P.O.w.N + 15) / 16 + grid - 1) / grid;
  const int need = ((P.A.w.K + 255) / 256 + 15) / 16;
  if (need != 1 || jo != 1) return false;
  constexpr int JB = FUSED ? 0 : 1;
  if (jb != JB) return false;
  switch (ja) {
    case 1: return launch_a8<QA, QB, G, 1, JB, 1, 1>(P, grid, lds, s);
    case 2: return launch_a8<QA, QB, G, 2, JB, 1, 1>(P, grid, lds, s);
    case 3: return launch_a8<QA, QB, G, 3, JB, 1, 1>(P, grid, lds, s);
    default: return false;
  }
}

template <int QA, int QB>
bool a8_g(const Attn8Params& P, int grid, size_t lds, hipStream_t s) {
  switch (P.H / P.Hkv) {
    case 1: return a8_shape<QA, QB, 1>(P, grid, lds, s);
    case 4: return a8_shape<QA, QB, 4>(P, grid, lds, s);
    default: return false;
  }
}

}  // namespace

bool attn8(const GemvParams& A, const GemvParams& B, const GemvParams& O, const AttnParams& At, void* sync,
           hipStream_t s) {
  if (!sync || At.kv8 || A.kv8 || A.B != 1 || !A.x8 || !A.x8_stat || A.epi != EPI_QKV || A.D != A8_D || At.D != A8_D || At.window > 0 ||
      At.NQ != 1 || O.B != 1 || !O.x8 || !O.emit8 || !O.emit8_nw || !O.emit8_stat || O.epi != EPI_ADD ||
      O.w.K != At.H * A8_D || A.w.K % 64 || A.w.K > 8192 || O.w.N % 16 || At.H % At.n_kv)
    return false;
  const bool fused = B.w.s0 == nullptr;
  if (fused && A.w.N != (At.H + 2 * At.n_kv) * A8_D) return false;
  if (!fused && (A.w.N != (At.H + At.n_kv) * A8_D || B.w.N != At.n_kv * A8_D || B.w.K != A.w.K)) return false;
  if (O.w.qtype != A.w.qtype) return false;  // the O tiles share phase A's register tile type
  int ncu = 0, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return false;
  Attn8Params P{};
  P.A = A;
  P.B = B;
  P.O = O;
  P.block_table = At.block_table;
  P.max_blocks = At.max_blocks;
  P.q_seq = At.q_seq;
  P.q_len = At.q_len;
  P.scale = At.scale;
  P.H = At.H;
  P.Hkv = At.n_kv;
  P.bpg = ncu / At.n_kv;
  if (P.bpg < 1 || At.n_kv > 64) return false;
  P.sync = (unsigned*)sync + 16;
  const int grid = P.bpg * At.n_kv;
  const int G = At.H / At.n_kv;
  const size_t img = x8_bytes(max(A.w.K, O.w.K)) + 32 * 4;
  const size_t att = (size_t)(4 * G * (A8_D + 2) + G * A8_D) * 4 + A8_MAXBT * 4;
  const size_t lds = img > att ? img : att;
  switch (A.w.qtype) {
    case QT_Q4_K:
      if (fused) return a8_g<QT_Q4_K, 0>(P, grid, lds, s);
      if (B.w.qtype == QT_Q6_K) return a8_g<QT_Q4_K, QT_Q6_K>(P, grid, lds, s);
      if (B.w.qtype == QT_Q4_K) return a8_g<QT_Q4_K, QT_Q4_K>(P, grid, lds, s);
      return false;
    case QT_Q4_0:
      if (fused) return a8_g<QT_Q4_0, 0>(P, grid, lds, s);
      return false;
    case QT_Q8_0:
      if (fused) return a8_g<QT_Q8_0, 0>(P, grid, lds, s);
      return false;
    default: return false;
  }
}

}  // namespace omx
