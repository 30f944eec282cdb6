// Batch-1 decode: paged attention and the O projection in ONE launch (Llama family).
//
//   blocks [0, n_att)   attention: KV group g, key split s (G query heads over keys [k0, k1)); split
//                       partials go to a workspace with write-through (sc1) stores and the LAST split
//                       of a group to finish (agent-scope ticket) merges them; the merged heads are
//                       quantised into the O projection's int8 image (sc1) and the merging block
//                       arrives on the hand-off counter. No attention block ever waits.
//   blocks [n_att, ..)  O projection: each block requests its 16-row O tile's weights and its epilogue
//                       operands FIRST, then waits until every group is published, reads the image
//                       (sc1 loads), computes, adds the residual and emits gate_up's int8 image.
//
// Why: the attention of a decode step is pure latency (q + block table -> K/V -> cross-wave merge ->
// split merge) on a few dozen blocks while the chip idles: 5.7 us per layer at ~150 keys, 14.6 us at
// 2,048 (profiles/r5_decode), and the O launch after it waits for it before it even requests its
// 9.4 MB of weights (4.9-5.2 us). Here the O weights stream while the attention runs, and the split
// merge moves into the attention launch (the O prologue reads a ready image, no merge slabs).
// Deadlock freedom: the O blocks wait, so the whole grid must be co-resident -- the host checks
// hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs >= grid (every block then holds its slot from the
// start; no dispatch order is assumed); a wait gives up after 2 ms and raises the error word
// (runner.x8_error). Hand-offs: MI355X_MICROARCH.md "Valid forms" table row 1 (every storing wave
// vmcnt(0) -> workgroup barrier -> one agent-scope atomic; readers use sc1 loads after the poll /
// ticket). attn8.hip (QKV + attention + O, one block per CU) measured slower because its QKV phase ran
// at one block per CU; here QKV stays its own launch at full occupancy.
// Reference parity: the attention + output projection of llama.cpp's decode graph inside
// `ollama/ollama` (reference pkg/model/pod.go:10-12); numerics vs the fp32 torch twin
// (tests/test_attn_o_gpu.py).
#include "attn8_core.h"
#include "gemv8_body.h"

namespace omx {

struct AttnOParams {
  Attn8Params P;       // P.A: q rows (y), kc, vc, bs, Dc; P.O: O projection (x8 = the image, EPI_ADD + emission)
  float* ws;           // [S][H][D + 2] split partials (write-through)
  unsigned* tickets;   // [n_kv] split tickets per group (self re-arming)
  Handoff H;           // merged groups -> O blocks
  int S, kps, n_att;   // split slots per group, target keys per split, attention blocks (n_kv * S)
};

template <int G>
__device__ void attn_o_attention(const AttnOParams& Q, int bx, char* smem) {
  constexpr int D = A8_D;
  const Attn8Params& P = Q.P;
  const int g = bx / Q.S, split = bx % Q.S;
  const int len = P.q_len[0];
  const int Se = max(1, min(Q.S, (len + Q.kps - 1) / Q.kps));  // same rule on every block
  if (split >= Se) return;  // surplus split of a short query: nothing to do, nothing to publish
  const int chunk = (len + Se - 1) / Se, k0 = split * chunk, k1 = min(len, k0 + chunk);
  float* sm = (float*)smem;          // [4][G][D + 2]
  float* ob = sm + 4 * G * (D + 2);  // [G][D]
  int* sbt = (int*)(ob + G * D);     // [A8_MAXBT]
  __shared__ int s_last;
  attn_core<G, false>(P, g, k0, k1, sm, sbt);
  const int tid = threadIdx.x;
  if (Se == 1) {
    for (int i = tid; i < G * D; i += GEMV_NT) {
      float M, L, Av;
      attn_merge4<G>(sm, i, M, L, Av);
      ob[i] = L > 0.f ? Av / L : 0.f;
    }
  } else {
    // this split's unnormalised partial of the G heads -> workspace (sc1), then the group ticket
    for (int i = tid; i < G * D; i += GEMV_NT) {
      float M, L, Av;
      attn_merge4<G>(sm, i, M, L, Av);
      const int h = g * G + i / D, d = i % D;
      float* w = Q.ws + ((long long)split * P.H + h) * (D + 2);
      st_wt(w + d, Av);
      if (d == 0) {
        st_wt(w + D, M);
        st_wt(w + D + 1, L);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(Q.tickets + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == (unsigned)Se - 1;
      if (s_last) __hip_atomic_store(Q.tickets + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
    __syncthreads();
    if (!s_last) return;
    // last split of the group: merge the Se partials (sc1 loads: other blocks of this launch wrote
    // them). Two round trips, not one per split: (1) lane sp of half-wave gg loads split sp's (m, l) of
    // head gg, the 32 lanes fold the merge weights; (2) every output loads all Se partial values at
    // once (a fully unrolled, predicated loop) and takes the weighted sum.
    float* sw = (float*)sbt;  // [G][32] merge weights (the staged block table is dead now)
    float* sL = sw + G * 32;  // [G]
    if (tid < 32 * G) {
      const int gg = tid >> 5, sp = tid & 31;
      const float* w = Q.ws + ((long long)min(sp, Se - 1) * P.H + g * G + gg) * (D + 2);
      const float m = sp < Se ? ld_wt(w + D) : -INFINITY, l = sp < Se ? ld_wt(w + D + 1) : 0.f;
      float M = m;
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) M = fmaxf(M, __shfl_xor(M, o, 32));
      const float c = m == -INFINITY ? 0.f : __expf(m - M);
      float L = c * l;
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) L += __shfl_xor(L, o, 32);
      sw[gg * 32 + sp] = c;
      if (sp == 0) sL[gg] = L;
    }
    __syncthreads();
    for (int i = tid; i < G * D; i += GEMV_NT) {
      const int gg = i / D, d = i % D;
      const float* w = Q.ws + ((long long)g * G + gg) * (D + 2) + d;
      float v[32];
#pragma unroll
      for (int sp = 0; sp < 32; ++sp) v[sp] = sp < Se ? ld_wt(w + (long long)sp * P.H * (D + 2)) : 0.f;
      float Av = 0.f;
#pragma unroll
      for (int sp = 0; sp < 32; ++sp) Av += sw[gg * 32 + sp] * v[sp];
      ob[i] = sL[gg] > 0.f ? Av / sL[gg] : 0.f;
    }
  }
  __syncthreads();
  // the G heads' 16-dim groups -> the O projection's image (write-through: the O blocks of this launch)
  const int g0 = g * G * D / 16;
  if (tid < G * D / 16) emit_group<true>(const_cast<void*>(P.O.x8), P.O.w.K, g0 + tid, ob + 16 * tid, nullptr, nullptr);
  handoff_arrive(Q.H);
}

// one 16-row O tile: weights + epilogue operands requested before the hand-off wait
template <int QT>
__device__ void attn_o_proj(const AttnOParams& Q, int tile, char* smem) {
  const GemvParams& O = Q.P.O;
  const QMat& w = O.w;
  const int K = w.K, N = w.N, SB = n_sb(K), XS = SB * XPAD, XSP = x8_slots_dev(K);
  i32x4* lq = (i32x4*)smem;
  f32x2* lf = (f32x2*)(smem + (size_t)XSP * 16);
  float* stage = (float*)(lf + XSP);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, s = lane & 15;
  const int rbase = wave * 4 + g;
  EpiPre<1, 1> pre;
  epi_prefetch<EM_ADD, 1, 1>(O, tile, rbase, s, pre);
  WTile<QT, 1, 1> T;
  load_wtile<QT, 1, 1>(w, 0, tile * 16 + rbase, N, SB, 0, s, T, SB);
  __builtin_amdgcn_sched_barrier(0);
  // wait for every group's image slice: one lane polls (sc1 loads), the block joins at the barrier
  const Handoff& H = Q.H;
  if (tid == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    while (__hip_atomic_load(H.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)H.n_prod) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000ull) {  // 2 ms: never in a healthy step
        __hip_atomic_store(H.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  const int nd = XSP * 6;  // image dwords
  constexpr int NDW = 8;   // K <= 4096: x8_bytes / 4 <= 1644 dwords = 7 per thread at 256 threads
  const unsigned* src = (const unsigned*)O.x8;
  unsigned xd[NDW];
#pragma unroll
  for (int i = 0; i < NDW; ++i)
    xd[i] = __hip_atomic_load(src + min(tid + GEMV_NT * i, nd - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // passes counted AFTER the image loads are issued: the add's round trip hides behind them (vmcnt
  // retires in order, so an add issued first would hold up the image); the last pass re-arms
  unsigned passed = 0;
  if (tid == 0) passed = __hip_atomic_fetch_add(H.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int i = 0; i < NDW; ++i)
    if (tid + GEMV_NT * i < nd) ((unsigned*)smem)[tid + GEMV_NT * i] = xd[i];
  __syncthreads();
  float acc[1][1] = {{0.f}};
  compute_wtile<QT, 1, 1, 1>(T, SB, 0, s, lq, lf, XS, acc, SB);
  const float v = row16_sum(acc[0][0]);
  const int n = tile * 16 + rbase;
  if (s == 0) {
    float nv = 0.f;
    if (n < N) {
      nv = pre.res[0][0] + v + pre.bias[0];
      O.y[n] = nv;
    }
    stage[rbase] = n < N ? nv * pre.nw[0] : 0.f;
    stage[16 + rbase] = nv * nv;
  }
  __syncthreads();
  if (tid == 0) {
    emit_group(O.emit8, N, tile, stage, stage + 16, O.emit8_stat);  // read by the next launch
    if (passed == (unsigned)H.n_cons - 1) {  // every O block has passed: re-arm for the next launch
      __hip_atomic_store(H.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(H.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int QT, int G>
__global__ __launch_bounds__(GEMV_NT) void attn_o_kernel(AttnOParams Q) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if ((int)blockIdx.x < Q.n_att) attn_o_attention<G>(Q, blockIdx.x, smem);
  else attn_o_proj<QT>(Q, (int)blockIdx.x - Q.n_att, smem);
}

namespace {

template <int QT, int G>
bool launch_ao(const AttnOParams& Q, int grid, size_t lds, hipStream_t s) {
  static int occ[8] = {};  // co-resident blocks per device for this instantiation (0 = not queried)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 8) return false;
  if (occ[dev] == 0) {
    int nb = 0, ncu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, attn_o_kernel<QT, G>, GEMV_NT, lds) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return false;
    occ[dev] = nb * ncu > 0 ? nb * ncu : -1;
  }
  if (occ[dev] < grid) return false;  // the O blocks wait: every block must hold its slot from the start
  count_launch(LC_ATTN_O);
  hipLaunchKernelGGL((attn_o_kernel<QT, G>), dim3(grid), dim3(GEMV_NT), lds, s, Q);
  return true;
}

template <int QT>
bool ao_g(const AttnOParams& Q, int G, int grid, size_t lds, hipStream_t s) {
  switch (G) {
    case 1: return launch_ao<QT, 1>(Q, grid, lds, s);
    case 4: return launch_ao<QT, 4>(Q, grid, lds, s);
    case 8: return launch_ao<QT, 8>(Q, grid, lds, s);
    default: return false;
  }
}

}  // namespace

bool attn_o(const GemvParams& O, const AttnParams& At, void* img, void* sync, hipStream_t s) {
  if (!img || !sync || At.kv8 || !At.ws || !At.counters || O.B != 1 || O.epi != EPI_ADD || !O.emit8 || !O.emit8_nw ||
      !O.emit8_stat || At.D != A8_D || (At.Dv != 0 && At.Dv != A8_D) || At.window > 0 || At.NQ != 1 ||
      At.H % At.n_kv || At.n_kv > 64 || O.w.K != At.H * A8_D || O.w.N % 16 || At.n_splits < 1 || At.n_splits > 32)
    return false;
  if (((O.w.K + 255) / 256 + 15) / 16 != 1) return false;  // one super-block per lane (K <= 4096)
  // a split never spans more than the A8_MAXBT block-table entries a block stages (attn8_core.h)
  if ((At.max_blocks + At.n_splits - 1) / At.n_splits > A8_MAXBT) return false;
  const int G = At.H / At.n_kv;
  const int q = O.w.qtype;
  AttnOParams Q{};
  Q.P.A.y = const_cast<float*>(At.q);
  Q.P.A.kc = const_cast<void*>(At.kc);
  Q.P.A.vc = const_cast<void*>(At.vc);
  Q.P.A.bs = At.bs;
  Q.P.A.Dc = At.D;
  Q.P.O = O;
  Q.P.O.x8 = img;
  Q.P.O.x8_stat = nullptr;
  Q.P.block_table = At.block_table;
  Q.P.max_blocks = At.max_blocks;
  Q.P.q_seq = At.q_seq;
  Q.P.q_len = At.q_len;
  Q.P.scale = At.scale;
  Q.P.H = At.H;
  Q.P.Hkv = At.n_kv;
  Q.P.sync = (unsigned*)sync + 16;  // error word at [66] (x8_error reads it)
  Q.ws = At.ws;
  Q.tickets = (unsigned*)At.counters;
  Q.S = At.n_splits;
  // keys per split: the block stages <= A8_MAXBT block-table entries, so a split never spans more
  Q.kps = At.kps > 0 ? At.kps : 128;
  Q.n_att = At.n_kv * Q.S;
  const int n_o = O.w.N / 16;
  Q.H.count = (unsigned*)sync + 96;
  Q.H.done = (unsigned*)sync + 97;
  Q.H.err = (int*)sync + 98;
  Q.H.n_prod = At.n_kv;
  Q.H.n_cons = n_o;
  const size_t img_lds = x8_bytes(O.w.K) + 32 * 4;
  const size_t att = (size_t)(4 * G * (A8_D + 2) + G * A8_D) * 4 + (size_t)(A8_MAXBT > 33 * G ? A8_MAXBT : 33 * G) * 4;
  const size_t lds = img_lds > att ? img_lds : att;
  const int grid = Q.n_att + n_o;
  switch (q) {
    case QT_Q4_K: return ao_g<QT_Q4_K>(Q, G, grid, lds, s);
    case QT_Q6_K: return ao_g<QT_Q6_K>(Q, G, grid, lds, s);
    case QT_Q5_K: return ao_g<QT_Q5_K>(Q, G, grid, lds, s);
    case QT_Q4_0: return ao_g<QT_Q4_0>(Q, G, grid, lds, s);
    case QT_Q8_0: return ao_g<QT_Q8_0>(Q, G, grid, lds, s);
    default: return false;
  }
}

}  // namespace omx
