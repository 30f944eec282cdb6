// Shared pieces of the fused attention launches (attn8.hip, qkv_attn.hip): the parameter block, the
// write-through QKV epilogue and the per-KV-group decode attention run by a last-arriving block.
#pragma once
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

// G query heads of KV group g over keys [k0, k1) by one 4-wave block: 16 key groups of 16 lanes (8
// dims each), U keys per group per step, two steps in flight. Leaves the per-wave (m, l, acc) of each
// head in sm[4][G][D + 2] (block-synchronised); attn_merge4 folds the 4 waves. SAME: q / k / v of the
// current token were written by THIS launch (write-through stores): q and the newest key are read
// with sc1 loads; otherwise every load is plain (an earlier launch wrote them).
// Staged block-table entries: at most A8_MAXBT; a longer range raises the error word (sync[66]) and
// attends to none of the keys beyond it rather than writing past the LDS allocation (hosts never
// launch such a range).
template <int G, bool SAME>
__device__ void attn_core(const Attn8Params& P, int g, int k0, int k1, float* sm, int* sbt) {
  constexpr int D = A8_D, DPL = 8, NG = 16, U = A8_U, STEP = NG * U;
  const GemvParams& A = P.A;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, grp = wave * 4 + (lane >> 4), li = lane & 15;
  const int len_all = P.q_len[0];
  const int seq = P.q_seq ? P.q_seq[0] : 0;
  const int bs = A.bs, Dc = A.Dc > 0 ? A.Dc : D, Hkv = P.Hkv;
  const int b0 = k0 / bs, nb_all = k1 > k0 ? (k1 - 1) / bs - b0 + 1 : 0, nb = min(nb_all, A8_MAXBT);
  const int len = min(k1, (b0 + nb) * bs);
  if (nb_all > A8_MAXBT && tid == 0) __hip_atomic_store((int*)P.sync + 66, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int i = tid; i < nb; i += GEMV_NT) sbt[i] = P.block_table[(long long)seq * P.max_blocks + b0 + i];
  float q[G][DPL];
#pragma unroll
  for (int gg = 0; gg < G; ++gg) {
    const float* qp = A.y + (g * G + gg) * D + li * DPL;
    if constexpr (SAME) {
#pragma unroll
      for (int jj = 0; jj < DPL; ++jj) q[gg][jj] = ld_wt(qp + jj) * P.scale;
    } else {
      const f32x4 a = *(const f32x4*)qp, b = *(const f32x4*)(qp + 4);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        q[gg][jj] = a[jj] * P.scale;
        q[gg][4 + jj] = b[jj] * P.scale;
      }
    }
  }
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
      const long long base = (((long long)sbt[t / bs - b0] * Hkv + g) * bs + (t % bs)) * Dc + li * DPL;
      const bool fresh = SAME && t == len_all - 1;  // the key this launch wrote
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
  if (len > k0) {
    Step S0, S1;
    int t0 = k0;
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
  }
  // the 4 key groups of a wave, then (attn_merge4) the 4 waves through LDS
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
}

// output i = gg * D + d of the block: the 4 waves' partials folded -> (M, L, unnormalised A)
template <int G>
__device__ __forceinline__ void attn_merge4(const float* sm, int i, float& M, float& L, float& Av) {
  constexpr int D = A8_D;
  const int gg = i / D, d = i % D;
  M = -INFINITY;
#pragma unroll
  for (int w = 0; w < 4; ++w) M = fmaxf(M, sm[(w * G + gg) * (D + 2) + D]);
  L = 0.f;
  Av = 0.f;
  if (M != -INFINITY) {
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float c = __expf(sm[(w * G + gg) * (D + 2) + D] - M);
      L += sm[(w * G + gg) * (D + 2) + D + 1] * c;
      Av += sm[(w * G + gg) * (D + 2) + d] * c;
    }
  }
}

// G query heads of KV group g over ALL keys [0, len) (q / k / v written by this launch); merged output
// quantised into the O projection's image (write-through: later blocks of the launch read it)
template <int G>
__device__ void attn_group(const Attn8Params& P, int g, char* smem) {
  constexpr int D = A8_D;
  float* sm = (float*)smem;          // [4][G][D + 2]
  float* ob = sm + 4 * G * (D + 2);  // [G][D]
  int* sbt = (int*)(ob + G * D);     // [A8_MAXBT]
  attn_core<G, true>(P, g, 0, P.q_len[0], sm, sbt);
  for (int i = threadIdx.x; i < G * D; i += GEMV_NT) {
    float M, L, Av;
    attn_merge4<G>(sm, i, M, L, Av);
    ob[i] = L > 0.f ? Av / L : 0.f;
  }
  __syncthreads();
  // the G heads' 16-dim groups -> the O projection's image (write-through: phase B of other blocks)
  const int g0 = g * G * D / 16;
  if (threadIdx.x < G * D / 16)
    emit_group<true>(const_cast<void*>(P.O.x8), P.O.w.K, g0 + threadIdx.x, ob + 16 * threadIdx.x, nullptr, nullptr);
}

}  // namespace omx
