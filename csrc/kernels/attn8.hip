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
#include "gemv8_core.h"

namespace omx {

struct Attn8Params {
  GemvParams A;            // q,k rows (q,k,v when B.w.s0 is null): x8 RMS image in, EPI_QKV fields
  GemvParams B;            // v rows of another quant type (Q4_K_M), or unused
  GemvParams O;            // O projection: x8 = the attention image (this launch), EPI_ADD + emission
  const int* block_table;  // [seqs][max_blocks]
  int max_blocks;
  const int* q_seq;        // [1] (null: row 0)
  const int* q_len;        // [1] visible keys = pos + 1
  float scale;
  int H, Hkv, bpg;         // query heads, KV heads, blocks per KV group
  unsigned* sync;          // [0, Hkv) group tickets, [64] heads published, [65] O passes, [66] error
};

constexpr int A8_D = 128, A8_TPH = A8_D / 16;  // head dim, 16-row tiles per head
constexpr int A8_U = 4;                         // keys per key group per pipeline step
constexpr int A8_MAXBT = 64;                    // block-table entries staged (<= 1024 keys at bs 16)

// EPI_QKV for batch row 0 with write-through stores: another block of this launch reads q / k / v
__device__ __forceinline__ void epi_qkv_wt(const GemvParams& P, int vn, float v, float pv) {
  const int Eq = P.Eq, Ekv = P.Ekv, D = P.D;
  int which, hh, d;
  if (vn < Eq) { which = 0; hh = vn / D; d = vn % D; }
  else if (vn < Eq + Ekv) { which = 1; hh = (vn - Eq) / D; d = (vn - Eq) % D; }
  else { which = 2; hh = (vn - Eq - Ekv) / D; d = (vn - Eq - Ekv) % D; }
  if (P.bias) v += P.bias[vn];
  float out = v;
  if (which < 2 && d < P.n_rot) {
    if (P.bias) pv += P.bias[vn ^ 1];
    const float ang = (float)P.pos[0] * P.inv_freq[d >> 1];
    float sn, cs;
    sincosf(ang, &sn, &cs);
    out = (d & 1) ? (pv * sn + v * cs) : (v * cs - pv * sn);
  }
  if (which == 0) {
    st_wt(P.y + vn, out);
  } else {
    const int slot = P.slot[0];
    const long long blk = slot / P.bs, off = slot % P.bs;
    const long long idx = ((blk * P.n_kv + hh) * P.bs + off) * (P.Dc > 0 ? P.Dc : D) + d;
    const unsigned short bits = __builtin_bit_cast(unsigned short, (f16)out);
    // two explicit stores: a pointer select here is lowered to an indexed scratch array
    if (which == 1) __hip_atomic_store((unsigned short*)P.kc + idx, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_store((unsigned short*)P.vc + idx, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// global row of tile `idx` of KV group g's A-side tile list: G q heads, then k (then v when fused)
template <int G>
__device__ __forceinline__ int a_row(int idx, int g, int Eq, int Ekv) {
  if (idx < G * A8_TPH) return ((g * G + idx / A8_TPH) * A8_D) + 16 * (idx % A8_TPH);
  idx -= G * A8_TPH;
  if (idx < A8_TPH) return Eq + g * A8_D + 16 * idx;
  return Eq + Ekv + g * A8_D + 16 * (idx - A8_TPH);
}

// 16 B of the paged cache: plain (written by an earlier launch) or write-through (this launch)
__device__ __forceinline__ f16x8 kv_load(const f16* p, bool fresh) {
  if (!fresh) return __builtin_nontemporal_load((const f16x8*)p);
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = __hip_atomic_load((const unsigned*)p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_bit_cast(f16x8, r);
}

// G query heads of KV group g over keys [0, len) by one 4-wave block: 16 key groups of 16 lanes (8
// dims each), U keys per group per step, two steps in flight; merged output quantised into the O
// projection's image (write-through)
template <int G>
__device__ void attn_group(const Attn8Params& P, int g, char* smem) {
  constexpr int D = A8_D, DPL = 8, NG = 16, U = A8_U, STEP = NG * U;
  const GemvParams& A = P.A;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, grp = wave * 4 + (lane >> 4), li = lane & 15;
  const int len = P.q_len[0];
  const int seq = P.q_seq ? P.q_seq[0] : 0;
  const int bs = A.bs, Dc = A.Dc > 0 ? A.Dc : D, Hkv = P.Hkv;
  float* sm = (float*)smem;                   // [4][G][D + 2]
  float* ob = sm + 4 * G * (D + 2);           // [G][D]
  int* sbt = (int*)(ob + G * D);              // [A8_MAXBT]
  const int nb = (len + bs - 1) / bs;
  for (int i = tid; i < nb; i += GEMV_NT) sbt[i] = P.block_table[(long long)seq * P.max_blocks + i];
  float q[G][DPL];
#pragma unroll
  for (int gg = 0; gg < G; ++gg)
#pragma unroll
    for (int jj = 0; jj < DPL; ++jj) q[gg][jj] = ld_wt(A.y + (g * G + gg) * D + li * DPL + jj) * P.scale;
  float m[G], l[G], acc[G][DPL];
#pragma unroll
  for (int gg = 0; gg < G; ++gg) {
    m[gg] = -INFINITY;
    l[gg] = 0.f;
#pragma unroll
    for (int jj = 0; jj < DPL; ++jj) acc[gg][jj] = 0.f;
  }
  __syncthreads();  // sbt
  const f16* kc = (const f16*)A.kc;
  const f16* vc = (const f16*)A.vc;
  struct Step {
    f16x8 k[U], v[U];
  };
  auto issue = [&](int t0, Step& st) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = min(t0 + u * NG + grp, len - 1);
      const long long base = (((long long)sbt[t / bs] * Hkv + g) * bs + (t % bs)) * Dc + li * DPL;
      const bool fresh = t == len - 1;  // the key this launch wrote
      st.k[u] = kv_load(kc + base, fresh);
      st.v[u] = kv_load(vc + base, fresh);
    }
  };
  auto consume = [&](int t0, const Step& st) {
    float sc[U][G];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = t0 + u * NG + grp < len;
#pragma unroll
      for (int gg = 0; gg < G; ++gg) {
        float s = 0.f;
#pragma unroll
        for (int jj = 0; jj < DPL; ++jj) s += q[gg][jj] * (float)st.k[u][jj];
        s = row16_sum(s);
        sc[u][gg] = ok ? s : -INFINITY;
      }
    }
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      float mn = m[gg];
#pragma unroll
      for (int u = 0; u < U; ++u) mn = fmaxf(mn, sc[u][gg]);
      if (mn == -INFINITY) continue;
      const float corr = __expf(m[gg] - mn);
      float p[U], ps = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        p[u] = __expf(sc[u][gg] - mn);
        ps += p[u];
      }
      l[gg] = l[gg] * corr + ps;
#pragma unroll
      for (int jj = 0; jj < DPL; ++jj) {
        float a = acc[gg][jj] * corr;
#pragma unroll
        for (int u = 0; u < U; ++u) a += p[u] * (float)st.v[u][jj];
        acc[gg][jj] = a;
      }
      m[gg] = mn;
    }
  };
  Step S0, S1;
  int t0 = 0;
  issue(t0, S0);
  while (true) {
    if (t0 + STEP < len) issue(t0 + STEP, S1);
    consume(t0, S0);
    t0 += STEP;
    if (t0 >= len) break;
    if (t0 + STEP < len) issue(t0 + STEP, S0);
    consume(t0, S1);
    t0 += STEP;
    if (t0 >= len) break;
  }
  // the 4 key groups of a wave, then the 4 waves (LDS)
#pragma unroll
  for (int sh = 16; sh <= 32; sh <<= 1) {
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      const float mo = __shfl_xor(m[gg], sh, 64), lo = __shfl_xor(l[gg], sh, 64);
      const float mn = fmaxf(m[gg], mo);
      const float c0 = mn == -INFINITY ? 0.f : __expf(m[gg] - mn);
      const float c1 = mn == -INFINITY ? 0.f : __expf(mo - mn);
      l[gg] = l[gg] * c0 + lo * c1;
#pragma unroll
      for (int jj = 0; jj < DPL; ++jj) acc[gg][jj] = acc[gg][jj] * c0 + __shfl_xor(acc[gg][jj], sh, 64) * c1;
      m[gg] = mn;
    }
  }
  if (lane < 16) {
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
#pragma unroll
      for (int jj = 0; jj < DPL; ++jj) sm[(wave * G + gg) * (D + 2) + li * DPL + jj] = acc[gg][jj];
      if (li == 0) {
        sm[(wave * G + gg) * (D + 2) + D] = m[gg];
        sm[(wave * G + gg) * (D + 2) + D + 1] = l[gg];
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < G * D; i += GEMV_NT) {
    const int gg = i / D, d = i % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, sm[(w * G + gg) * (D + 2) + D]);
    float L = 0.f, Av = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float c = __expf(sm[(w * G + gg) * (D + 2) + D] - M);
        L += sm[(w * G + gg) * (D + 2) + D + 1] * c;
        Av += sm[(w * G + gg) * (D + 2) + d] * c;
      }
    }
    ob[i] = L > 0.f ? Av / L : 0.f;
  }
  __syncthreads();
  // the G heads' 16-dim groups -> the O projection's image (write-through: phase B of other blocks)
  const int g0 = g * G * D / 16;
  if (tid < G * D / 16) emit_group<true>(const_cast<void*>(P.O.x8), P.O.w.K, g0 + tid, ob + 16 * tid, nullptr, nullptr);
}

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
  if (!sync || A.B != 1 || !A.x8 || !A.x8_stat || A.epi != EPI_QKV || A.D != A8_D || At.D != A8_D || At.window > 0 ||
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
