// Paged-KV grouped-query attention for decode and chunked prefill.
//
// Grid (query, kv_head x head_split, split); one 512-thread block (8 waves) serves G of the H/H_kv
// query heads that share a KV head, so each K/V row is read once per G heads (GQA reuse). Decode
// launches few blocks (70B: 8 KV heads), and each lane's per-key work grows with G, so for GQA the
// group is split over H/H_kv/G blocks (head_split, `hpb` knob): the K/V re-reads hit L2/MALL and
// the block count / per-lane chain shrink (scripts/bench_attn.py OMX_BENCH_HPB sweep). Design points (measured with
// scripts/bench_attn.py, profiles/r1_attn):
//  * 16 lanes cooperate on one key (D/16 dims each: one 16-B load for D = 128); a wave's 4 DPP rows
//    are 4 key groups, the block's 32 groups x U = 4 slots (2 when G = 8) stream 128 keys per step.
//  * Software pipeline: the next step's K/V loads are in flight while the current step computes
//    (explicit register ping-pong), so a long range costs one HBM round trip, not one per step.
//  * The page entries of a step are loaded into registers one step ahead of its K/V loads (the first
//    step's right at entry, ahead of q): no LDS staging or barrier sits in front of the first K/V load.
//  * q.k reductions are 16-lane DPP sums (no LDS permutes); the online softmax is batched per step
//    (one max/rescale per 4 keys).
//  * Flash-decode split count is decided ON DEVICE from the length: S_eff = min(n_splits,
//    ceil(keys / 256)). Short contexts (the common decode case) therefore run one block per head
//    with no cross-block merge at all; long ones split, and the last split block to arrive (agent-
//    scope ticket, sc1 write-through partials: MI355X_MICROARCH.md hand-off form, no fences) merges
//    in the same launch. The grid is fixed, so the launch is hipGraph-capturable for any length.
// Causal prefill uses the same kernel: each prompt token is a query with length pos + 1.
#include <stdexcept>
#include <type_traits>
#include <string>

#include "common.h"
#include "ops.h"

namespace omx {

constexpr int ATT_NW = 8;               // waves per block
constexpr int ATT_NT = 64 * ATT_NW;
constexpr int ATT_NG = 4 * ATT_NW;      // key groups (16 lanes each) per block
int g_attn_kps = 256;                   // target keys per split (runtime knob, set_attn_tuning)
int g_attn_hpb = 0;                     // query heads per decode block (0 = auto, see launch_d)
void set_attn_tuning(int kps, int hpb) {
  if (kps >= 16) g_attn_kps = kps;
  if (hpb >= 0) g_attn_hpb = hpb;
}

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum_a(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  v += dppf<0x140>(v);
  return v;
}
// sum over the LPK (16 or 8) lanes of one key: quad sums, then row_half_mirror (8), then row_mirror (16)
template <int LPK>
__device__ __forceinline__ float key_sum(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  if constexpr (LPK == 16) v += dppf<0x140>(v);
  return v;
}

// one key's D/16 fp16 values for this lane, loaded with the widest aligned vector
template <int DPL>
struct KRow {
  f16 v[DPL];
};
template <int DPL>
__device__ __forceinline__ void load_krow(const f16* p, KRow<DPL>& r) {
  if constexpr (DPL == 8) {
    const f16x8 t = __builtin_nontemporal_load((const f16x8*)p);
#pragma unroll
    for (int j = 0; j < 8; ++j) r.v[j] = t[j];
  } else if constexpr (DPL == 16) {  // head dim 256 (Gemma)
    const f16x8 t0 = __builtin_nontemporal_load((const f16x8*)p), t1 = __builtin_nontemporal_load((const f16x8*)p + 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      r.v[j] = t0[j];
      r.v[8 + j] = t1[j];
    }
  } else if constexpr (DPL == 4) {
    const f16x4 t = *(const f16x4*)p;
#pragma unroll
    for (int j = 0; j < 4; ++j) r.v[j] = t[j];
  } else if constexpr (DPL % 2 == 0) {
    // head dims 80 / 96 / 112 at 8 lanes per key (DPL 10 / 12 / 14): the lane's run is only 4-B aligned,
    // so whole 16-B / 8-B pieces go through 4-B-aligned vector copies (dwordx4 / dwordx2 loads on gfx950's
    // unaligned-access mode) instead of one 4-B load per pair
    constexpr int J8 = DPL / 8 * 8, J4 = J8 + (DPL - J8) / 4 * 4;
#pragma unroll
    for (int j = 0; j < J8; j += 8) {
      f16x8 t;
      __builtin_memcpy(&t, __builtin_assume_aligned(p + j, 4), 16);
#pragma unroll
      for (int i = 0; i < 8; ++i) r.v[j + i] = t[i];
    }
    if constexpr (J4 > J8) {
      f16x4 t;
      __builtin_memcpy(&t, __builtin_assume_aligned(p + J8, 4), 8);
#pragma unroll
      for (int i = 0; i < 4; ++i) r.v[J8 + i] = t[i];
    }
#pragma unroll
    for (int j = J4; j < DPL; j += 2) {
      const f16x2 t = *(const f16x2*)(p + j);
      r.v[j] = t[0];
      r.v[j + 1] = t[1];
    }
  } else {
#pragma unroll
    for (int j = 0; j < DPL; ++j) r.v[j] = p[j];
  }
}

// fp8 KV cache (OCP e4m3fn): four bytes -> four fp16
__device__ __forceinline__ void e4m3x4_to_f16(unsigned w, f16* o) {
  const auto a = __builtin_amdgcn_cvt_pk_f32_fp8(w, false), b = __builtin_amdgcn_cvt_pk_f32_fp8(w, true);
  o[0] = (f16)a[0];
  o[1] = (f16)a[1];
  o[2] = (f16)b[0];
  o[3] = (f16)b[1];
}
// one key's D/16 fp8 values for this lane (half the bytes of the fp16 row), widened to fp16
template <int DPL>
__device__ __forceinline__ void load_krow8(const uint8_t* p, KRow<DPL>& r) {
  if constexpr (DPL == 8) {
    const u32x2 t = __builtin_nontemporal_load((const u32x2*)p);
    e4m3x4_to_f16(t.x, r.v);
    e4m3x4_to_f16(t.y, r.v + 4);
  } else if constexpr (DPL == 16) {
    const u32x4 t = __builtin_nontemporal_load((const u32x4*)p);
    e4m3x4_to_f16(t.x, r.v);
    e4m3x4_to_f16(t.y, r.v + 4);
    e4m3x4_to_f16(t.z, r.v + 8);
    e4m3x4_to_f16(t.w, r.v + 12);
  } else if constexpr (DPL == 4) {
    e4m3x4_to_f16(*(const unsigned*)p, r.v);
  } else {  // 5 / 6 / 7 (head dims 80 / 96 / 112): byte loads
#pragma unroll
    for (int j = 0; j < DPL; ++j) r.v[j] = (f16)__builtin_amdgcn_cvt_f32_fp8((unsigned)p[j], 0);
  }
}

// fp8 rows whose lane width is a multiple of 4 stay raw in registers (DPL / 4 dwords, half the staging
// registers of the widened fp16 row) and are widened to fp32 where they are consumed
template <int DPL>
struct KRow8 {
  unsigned w[DPL / 4];
};
template <int DPL>
__device__ __forceinline__ void load_krow8_raw(const uint8_t* p, KRow8<DPL>& r) {
  if constexpr (DPL == 16) {
    const u32x4 t = __builtin_nontemporal_load((const u32x4*)p);
    r.w[0] = t.x, r.w[1] = t.y, r.w[2] = t.z, r.w[3] = t.w;
  } else if constexpr (DPL == 8) {
    const u32x2 t = __builtin_nontemporal_load((const u32x2*)p);
    r.w[0] = t.x, r.w[1] = t.y;
  } else {
#pragma unroll
    for (int i = 0; i < DPL / 4; ++i) r.w[i] = ((const unsigned*)p)[i];
  }
}
template <int DPL>
__device__ __forceinline__ void row_f32(const KRow<DPL>& r, float (&o)[DPL]) {
#pragma unroll
  for (int j = 0; j < DPL; ++j) o[j] = (float)r.v[j];
}
template <int DPL>
__device__ __forceinline__ void row_f32(const KRow8<DPL>& r, float (&o)[DPL]) {
#pragma unroll
  for (int i = 0; i < DPL / 4; ++i) {
    const auto a = __builtin_amdgcn_cvt_pk_f32_fp8(r.w[i], false), b = __builtin_amdgcn_cvt_pk_f32_fp8(r.w[i], true);
    o[4 * i] = a[0], o[4 * i + 1] = a[1], o[4 * i + 2] = b[0], o[4 * i + 3] = b[1];
  }
}

// RAW: fp8 rows kept as KRow8 (KV8 with DPL % 4 == 0), else fp16 KRow (fp8 rows widened at load)
template <int DPL, int U, bool RAW = false>
struct KVStep {
  typedef typename std::conditional<RAW, KRow8<DPL>, KRow<DPL>>::type Row;
  Row k[U], v[U];
};

// U key slots per lane group per step: 4, or 2 when 8 query heads share a KV head or the head dim is
// 256 (registers: 4 slots of D = 256 spilled 188 B per lane).
// LPK lanes per key: 16 (D / 16 dims per lane: one 16-B fp16 load at D = 128), or 8 for the fp8 cache at
// D = 128 (16 dims per lane: again one 16-B load, so a wave keeps the same bytes per load instruction in
// flight; 16 lanes per key would move 8 B per load and stay load-issue bound, profiles/r5_kv8)
template <int D, int G, bool KV8 = false, int LPK = 16, int U = (G >= 8 || D > 128 ? 2 : 4)>
__global__ __launch_bounds__(ATT_NT) void attn_decode_kernel(AttnParams P) {
  static_assert(LPK == 16 || (LPK == 8 && D % 8 == 0), "lanes per key");
  constexpr int DPL = D / LPK;
  constexpr int KPW = 64 / LPK;                 // keys (lane groups) per wave
  constexpr int NG = KPW * ATT_NW;              // lane groups per block
  constexpr int ATT_U = U, ATT_STEP = NG * U;
  constexpr bool RAW = KV8 && DPL % 4 == 0;
  __shared__ float sm[ATT_NW][G][D + 2];
  const int qi = blockIdx.x, split = blockIdx.z;
  const int kvh = blockIdx.y / (P.H / P.n_kv / G);  // KV head of this block's G query heads
  const int h0 = blockIdx.y * G;                    // first query head of the block
  const int seq = P.q_seq ? P.q_seq[qi] : qi;
  const int len = P.q_len[qi];
  const int kstart = P.window > 0 ? max(0, len - P.window) : 0;
  const int nk = len - kstart;
  // deferred merge: exactly gridDim.z splits (empty ones publish m = -inf, l = 0) and the consumer
  // (the O-projection GEMV prologue) merges them; otherwise the split count follows the length
  const int S = P.defer ? (int)gridDim.z : max(1, min((int)gridDim.z, (nk + P.kps - 1) / P.kps));
  if (split >= S) return;  // block-uniform: surplus splits of a short query leave immediately
  const int chunk = (nk + S - 1) / S;
  const int t0 = kstart + split * chunk;
  const int t1 = min(len, t0 + chunk);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, tg = lane / LPK, li = lane % LPK;
  const int grp = wave * KPW + tg;

  const int Dv = P.Dv > 0 ? P.Dv : D;  // valid dims: q / output head stride; dims >= Dv are padding
  float q[G][DPL];
  float m[G], l[G], acc[G][DPL];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < DPL; ++j) acc[g][j] = 0.f;
  }
  const int* bt = P.block_table + (long long)seq * P.max_blocks;
  const int bs = P.bs;
  // page arithmetic: shifts for the power-of-two page sizes the runner uses (a runtime division per
  // key slot sat in the dependent address chain), division otherwise (uniform branch)
  const bool p2 = (bs & (bs - 1)) == 0;
  const int bsh = __ffs(bs) - 1;

  auto load_q = [&]() {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float* qp = P.q + (long long)qi * P.ldq + (h0 + g) * Dv;
      if (Dv == D) {  // unpadded head: plain loads (a per-element select makes hipcc wait per load)
#pragma unroll
        for (int j = 0; j < DPL; ++j) q[g][j] = qp[li * DPL + j] * P.scale;
      } else {
#pragma unroll
        for (int j = 0; j < DPL; ++j) {
          const int d = li * DPL + j;  // clamped load, then zero: padded K dims never contribute
          q[g][j] = qp[min(d, Dv - 1)] * (d < Dv ? P.scale : 0.f);
        }
      }
    }
  };

  if (t0 < t1) {
    // The page of every key slot of a step is loaded straight into registers one step ahead (no LDS
    // staging and no barrier before the first K/V load), and q is requested behind the first K/V issue:
    // the probe (experiments/attn_probe, profiles/r6_attn) timed the old staged prologue at 1.0 us of
    // the 5.7 us of a 150-key launch
    // lane li < U of a key group loads the page of the group's slot li; issue() takes slot u's page from
    // lane (group base + u) -- one register per step instead of U (the fp8 / D = 112 / G >= 4 kernels
    // would spill U pages twice over)
    auto ldbt = [&](int s0) {
      const int t = min(s0 + (li & (ATT_U - 1)) * NG + grp, t1 - 1);
      return bt[p2 ? t >> bsh : t / bs];
    };
    auto issue = [&](int s0, int pl, KVStep<DPL, U, RAW>& st) {
#pragma unroll
      for (int u = 0; u < ATT_U; ++u) {
        const int t = min(s0 + u * NG + grp, t1 - 1);  // clamped; masked at use
        const long long blk = __shfl(pl, (lane & ~(LPK - 1)) + u, 64);
        OMX_KASSERT(t >= 0 && blk >= 0 && (p2 ? t >> bsh : t / bs) < P.max_blocks);
        const long long base = ((blk * P.n_kv + kvh) * bs + (p2 ? t & (bs - 1) : t % bs)) * D + li * DPL;
        if constexpr (RAW) {
          load_krow8_raw<DPL>((const uint8_t*)P.kc + base, st.k[u]);
          load_krow8_raw<DPL>((const uint8_t*)P.vc + base, st.v[u]);
        } else if constexpr (KV8) {
          load_krow8<DPL>((const uint8_t*)P.kc + base, st.k[u]);
          load_krow8<DPL>((const uint8_t*)P.vc + base, st.v[u]);
        } else {
          load_krow<DPL>((const f16*)P.kc + base, st.k[u]);
          load_krow<DPL>((const f16*)P.vc + base, st.v[u]);
        }
      }
    };
    auto consume = [&](int s0, const KVStep<DPL, U, RAW>& st) {
      float sc[ATT_U][G];
#pragma unroll
      for (int u = 0; u < ATT_U; ++u) {
        const bool ok = s0 + u * NG + grp < t1;  // uniform within the key's lane group
        float kf[DPL];
        row_f32(st.k[u], kf);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < DPL; ++j) s += q[g][j] * kf[j];
          s = key_sum<LPK>(s);
          sc[u][g] = ok ? s : -INFINITY;
        }
      }
      float p[ATT_U][G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float mn = m[g];
#pragma unroll
        for (int u = 0; u < ATT_U; ++u) mn = fmaxf(mn, sc[u][g]);
        if (mn == -INFINITY) {  // nothing visible yet in this group
#pragma unroll
          for (int u = 0; u < ATT_U; ++u) p[u][g] = 0.f;
          continue;
        }
        const float corr = __expf(m[g] - mn);
        float ps = 0.f;
#pragma unroll
        for (int u = 0; u < ATT_U; ++u) {
          p[u][g] = __expf(sc[u][g] - mn);
          ps += p[u][g];
        }
        l[g] = l[g] * corr + ps;
#pragma unroll
        for (int j = 0; j < DPL; ++j) acc[g][j] *= corr;
        m[g] = mn;
      }
      // P.V one key slot at a time: a row is widened once and feeds every head of the group
#pragma unroll
      for (int u = 0; u < ATT_U; ++u) {
        float vf[DPL];
        row_f32(st.v[u], vf);
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
          for (int j = 0; j < DPL; ++j) acc[g][j] += p[u][g] * vf[j];
      }
    };

    KVStep<DPL, U, RAW> A, B;
    int pA = ldbt(t0), pB = 0;
    issue(t0, pA, A);
    if (t0 + ATT_STEP < t1) pB = ldbt(t0 + ATT_STEP);
    load_q();
    int s0 = t0;
    while (true) {  // step s0 in A / B; the next step's K/V and the page entries of the one after in flight
      if (s0 + ATT_STEP < t1) {
        issue(s0 + ATT_STEP, pB, B);
        if (s0 + 2 * ATT_STEP < t1) pA = ldbt(s0 + 2 * ATT_STEP);
      }
      consume(s0, A);
      s0 += ATT_STEP;
      if (s0 >= t1) break;
      if (s0 + ATT_STEP < t1) {
        issue(s0 + ATT_STEP, pA, A);
        if (s0 + 2 * ATT_STEP < t1) pB = ldbt(s0 + 2 * ATT_STEP);
      }
      consume(s0, B);
      s0 += ATT_STEP;
      if (s0 >= t1) break;
    }
  }

  // merge the key groups of the wave (lanes li, li + LPK, ...)
#pragma unroll
  for (int sh = LPK; sh <= 32; sh <<= 1) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float mo = __shfl_xor(m[g], sh, 64), lo = __shfl_xor(l[g], sh, 64);
      const float mn = fmaxf(m[g], mo);
      const float c0 = mn == -INFINITY ? 0.f : __expf(m[g] - mn);
      const float c1 = mn == -INFINITY ? 0.f : __expf(mo - mn);
      l[g] = l[g] * c0 + lo * c1;
#pragma unroll
      for (int j = 0; j < DPL; ++j) acc[g][j] = acc[g][j] * c0 + __shfl_xor(acc[g][j], sh, 64) * c1;
      m[g] = mn;
    }
  }
  if (lane < LPK) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int j = 0; j < DPL; ++j) sm[wave][g][li * DPL + j] = acc[g][j];
      if (li == 0) {
        sm[wave][g][D] = m[g];
        sm[wave][g][D + 1] = l[g];
      }
    }
  }
  __syncthreads();
  // merge the waves: threads over the G*D outputs
  for (int i = threadIdx.x; i < G * D; i += ATT_NT) {
    const int g = i / D, d = i % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < ATT_NW; ++w) M = fmaxf(M, sm[w][g][D]);
    float L = 0.f, A = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < ATT_NW; ++w) {
        const float c = __expf(sm[w][g][D] - M);
        L += sm[w][g][D + 1] * c;
        A += sm[w][g][d] * c;
      }
    }
    const int h = h0 + g;
    if (d >= Dv) continue;  // padding dims of a padded head (never written)
    if (P.defer) {  // partial slabs [NQ][S][H*D] + [NQ][S][H]{m, l}; the kernel boundary publishes them
      const long long row = (long long)qi * S + split;
      P.ws[row * P.H * D + h * D + d] = A;
      if (d == 0) *(f32x2*)(P.ws + (long long)P.NQ * S * P.H * D + (row * P.H + h) * 2) = (f32x2){M, L};
    } else if (S == 1) {
      const float o = L > 0.f ? A / L : 0.f;
      P.out[(long long)qi * P.ldo + h * Dv + d] = o;
      if (P.out16) ((f16*)P.out16)[(long long)qi * P.ldo + h * Dv + d] = (f16)o;
    } else {  // write-through (sc1) stores: the hand-off below then needs no release fence
      float* ws = P.ws + (((long long)qi * P.H + h) * gridDim.z + split) * (D + 2);
      __hip_atomic_store(ws + d, A, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == 0) {
        __hip_atomic_store(ws + D, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ws + D + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (S == 1 || P.defer) return;
  // ---- in-launch split combine (cdna_hip_programming.md §6 Guideline 16 / MI355X_MICROARCH.md
  // "Valid forms" row 1): partials were stored sc1; every wave drains them (vmcnt(0)), the block
  // barriers, one lane takes an agent-scope ticket. The block drawing the last of S tickets reads
  // every partial with sc1 loads (no acquire needed) and merges its G heads.
  __shared__ int s_last;
  __shared__ float sw[G][64];
  __shared__ float sL[G];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int* cnt = P.counters + (long long)qi * gridDim.y + blockIdx.y;
    const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == S - 1;
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  auto ld1 = [](const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  if (threadIdx.x < 64) {
    const int s = threadIdx.x;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float* ws = P.ws + (((long long)qi * P.H + h0 + g) * gridDim.z + (s < S ? s : 0)) * (D + 2);
      const float lv = ld1(ws + D + 1);
      const bool live = s < S && lv > 0.f;
      const float mm = live ? ld1(ws + D) : -INFINITY;
      const float MM = wave_max(mm);
      const float w = live ? __expf(mm - MM) : 0.f;
      sw[g][s] = w;
      const float LL = wave_sum(live ? w * lv : 0.f);
      if (s == 0) sL[g] = LL;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += ATT_NT) {
    const int g = i / D, d = i % D;
    if (d >= Dv) continue;
    const float* ws = P.ws + ((long long)qi * P.H + h0 + g) * gridDim.z * (D + 2);
    float A = 0.f;
#pragma unroll 8
    for (int s = 0; s < S; ++s) A += sw[g][s] * ld1(ws + s * (D + 2) + d);
    const float L = sL[g];
    const float o = L > 0.f ? A / L : 0.f;
    P.out[(long long)qi * P.ldo + (h0 + g) * Dv + d] = o;
    if (P.out16) ((f16*)P.out16)[(long long)qi * P.ldo + (h0 + g) * Dv + d] = (f16)o;
  }
}

// ---------------------------------------------------------------------------------------------
// Causal prefill attention on the matrix cores: one sequence, NQ >= 16
// contiguous query positions (a prefill chunk), K/V already in the paged cache (the QKV epilogue
// wrote them). Block = 4 waves x 32 queries of one head; key tiles of 32 staged in LDS and shared
// by the waves. Per tile and wave:
//   S^T = K . Q^T   (v_mfma_f32_32x32x16_f16; keys on the accumulator rows, one query per lane, so
//                    the online softmax is lane-local + one exchange with lane ^ 32)
//   O^T += V^T . P^T (P^T used straight from the accumulator registers as the B operand in the
//                    permuted k order of cdna_hip_programming.md §3; V^T fragments come from
//                    ds_read_b64_tr_b16 hardware-transposed reads of the row-major V tile, stored
//                    with the XOR swizzle of §5.5 T10 (b) so both the row writes and the transposed
//                    reads are bank-conflict-free)
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16a __attribute__((ext_vector_type(16)));
constexpr int PF_BQ = 128, PF_BK = 32;

// T10 (b): byte offset of 16-B chunk ch of V row `row`; rows of VROW bytes (256, or 512 for D = 256:
// each 256-B half swizzled on its own)
template <int VROW>
__device__ __forceinline__ int vswz(int row, int ch) {
  return VROW * row + 256 * (ch >> 4) + 16 * ((ch & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

template <int D, bool KV8 = false>
__global__ __launch_bounds__(256) void attn_prefill_kernel(AttnParams P) {
  constexpr int NKS = D / 16;             // k-steps of S^T over the head dim
  constexpr int NDT = (D + 31) / 32;      // 32-row d tiles of O^T
  constexpr int LDK = D + 8;              // K tile row stride (f16): 16-B rows offset by 4 banks
  constexpr int KCH = D / 8;              // 16-B chunks per K/V row
  constexpr int VROW = D > 128 ? 2 * D : 256;
  __shared__ __attribute__((aligned(16))) f16 Ks[PF_BK * LDK];
  __shared__ __attribute__((aligned(16))) char Vs[PF_BK * VROW];  // [key][VROW B] swizzled, zero-padded
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h2 = lane >> 5, qc = lane & 31;
  const int head = blockIdx.y, G = P.H / P.n_kv, kvh = head / G;
  // causal load balance: block b and b + 256 share a CU in the first dispatch wave (2 blocks per CU), and
  // consecutive heads hold the same query-block index, so the CUs that drew the last query blocks got twice
  // the heaviest work. The upper half of the heads walks the query blocks in reverse: every CU pairs a
  // heavy block with a light one.
  const int qb = blockIdx.y >= gridDim.y / 2 ? (int)(gridDim.x - 1 - blockIdx.x) : (int)blockIdx.x;
  const int q0 = qb * PF_BQ;
  const int NQ = P.NQ;
  const int qi = min(q0 + wave * 32 + qc, NQ - 1);  // this lane's query (clamped; stores masked)
  const int len_q = P.q_len[qi];                    // visible keys = pos + 1
  const int kstart_q = P.window > 0 ? max(0, len_q - P.window) : 0;
  const int seq = P.q_seq ? P.q_seq[0] : 0;
  const int* bt = P.block_table + (long long)seq * P.max_blocks;
  const f16* kc = (const f16*)P.kc;
  const f16* vc = (const f16*)P.vc;
  const int bs = P.bs;
  // key range of the block: contiguous positions -> first query has the smallest window start,
  // the last query the largest length
  const int q_last = min(q0 + PF_BQ, NQ) - 1;
  const int len_max = P.q_len[q_last];
  const int k_lo = P.window > 0 ? max(0, P.q_len[q0] - P.window) / PF_BK * PF_BK : 0;

  // Q^T fragments (B operand of S^T): lane = query, 8 consecutive d per k-step, scaled by scale * log2(e):
  // the scores come out in the log2 domain, so the softmax takes v_exp_f32 directly (no multiply per score)
  f16x8 qf[NKS];
  const float qs = P.scale * 1.44269504f;
  const int Dv = P.Dv > 0 ? P.Dv : D;  // valid dims (multiple of 4): q / output head stride
  {
    const float* qp = P.q + (long long)qi * P.ldq + head * Dv;
    const f32x4 z4 = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < NKS; ++kk) {
      const int d0 = 16 * kk + 8 * h2;  // padded dims load nothing (next head's q / past the row)
      const f32x4 a = d0 + 4 <= Dv ? *(const f32x4*)(qp + min(d0, Dv - 4)) : z4;
      const f32x4 b = d0 + 8 <= Dv ? *(const f32x4*)(qp + min(d0 + 4, Dv - 4)) : z4;
      qf[kk] = (f16x8){(f16)(a.x * qs), (f16)(a.y * qs), (f16)(a.z * qs), (f16)(a.w * qs),
                       (f16)(b.x * qs), (f16)(b.y * qs), (f16)(b.z * qs), (f16)(b.w * qs)};
    }
  }
  f32x16a o[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m = -INFINITY, l = 0.f;

  // zero the V padding columns once (d in [D, 128)): they feed the last O^T tile when D % 32 != 0
  if (D < 128) {
    for (int i = tid; i < PF_BK * 16; i += 256) {
      const int row = i >> 4, ch = i & 15;
      if (ch >= KCH) *(u32x4*)(Vs + vswz<VROW>(row, ch)) = (u32x4){0u, 0u, 0u, 0u};
    }
  }
  // staging: each thread moves chunks of the K and V tiles (global paged cache -> registers -> LDS)
  constexpr int NCH = (PF_BK * KCH + 255) / 256;
  u32x4 kr[NCH], vr[NCH];
  auto issue = [&](int kt0) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int i = tid + 256 * c;
      const int row = min(i / KCH, PF_BK - 1), ch = i % KCH;
      const int t = min(kt0 + row, len_max - 1);
      const long long base = (((long long)bt[t / bs] * P.n_kv + kvh) * bs + (t % bs)) * D + 8 * ch;
      if constexpr (KV8) {  // 8 fp8 bytes in .x / .y, widened at the LDS write
        const u32x2 k8 = *(const u32x2*)((const uint8_t*)P.kc + base), v8 = *(const u32x2*)((const uint8_t*)P.vc + base);
        kr[c] = (u32x4){k8.x, k8.y, 0u, 0u};
        vr[c] = (u32x4){v8.x, v8.y, 0u, 0u};
      } else {
        kr[c] = *(const u32x4*)(kc + base);
        vr[c] = *(const u32x4*)(vc + base);
      }
    }
  };
  auto widen = [](const u32x4& r) -> u32x4 {  // KV8: 8 e4m3 bytes -> 8 fp16
    if constexpr (!KV8) return r;
    f16x8 h;
    f16 t[8];
    e4m3x4_to_f16(r.x, t);
    e4m3x4_to_f16(r.y, t + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) h[j] = t[j];
    return __builtin_bit_cast(u32x4, h);
  };
  issue(k_lo);
  for (int kt0 = k_lo; kt0 < len_max; kt0 += PF_BK) {
    __syncthreads();  // previous tile's LDS reads done
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int i = tid + 256 * c;
      if (i < PF_BK * KCH) {
        const int row = i / KCH, ch = i % KCH;
        *(u32x4*)(Ks + row * LDK + 8 * ch) = widen(kr[c]);
        *(u32x4*)(Vs + vswz<VROW>(row, ch)) = widen(vr[c]);
      }
    }
    __syncthreads();
    if (kt0 + PF_BK < len_max) issue(kt0 + PF_BK);  // next tile in flight during the MFMAs
    // S^T = K . Q^T : rows = keys kt0 + (r&3) + 8(r>>2) + 4*h2, column = this lane's query
    f32x16a sacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
#pragma unroll
    for (int kk = 0; kk < NKS; ++kk) {
      const f16x8 kf = *(const f16x8*)(Ks + qc * LDK + 16 * kk + 8 * h2);
      sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[kk], sacc, 0, 0, 0);
    }
    // causal / window / length mask + online softmax (per lane = per query; halves exchange). The VALU
    // work per tile is what bounds this kernel (~200 ops per lane vs 16 MFMAs per wave): tiles wholly
    // inside every query's window of this wave skip the mask, and the accumulator rescale is skipped
    // when no query's running max moved
    float tmax = -INFINITY;
    if (__all(kt0 + PF_BK <= len_q && kt0 >= kstart_q)) {
#pragma unroll
      for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, sacc[r]);
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int t = kt0 + (r & 3) + 8 * (r >> 2) + 4 * h2;
        const bool ok = t < len_q && t >= kstart_q;
        sacc[r] = ok ? sacc[r] : -INFINITY;
        tmax = fmaxf(tmax, sacc[r]);
      }
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax);
    const float corr = mn == -INFINITY ? 1.f : __builtin_amdgcn_exp2f(m - mn);
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sacc[r] = mn == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(sacc[r] - mn);
      ps += sacc[r];
    }
    ps += __shfl_xor(ps, 32, 64);
    l = l * corr + ps;
    m = mn;
    if (__any(corr != 1.f)) {
#pragma unroll
      for (int i = 0; i < NDT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] *= corr;
    }
    // O^T += V^T . P^T : two k-steps of 16 keys; P^T fragment s = registers 8s..8s+7
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      f16x8 pf;
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[j] = (f16)sacc[8 * s2 + j];
      const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
      for (int i = 0; i < NDT; ++i) {
        const int c0 = (32 * i + 16 * (g & 1)) / 8;  // first 16-B chunk of this group's 16 d columns
        const int r0 = 16 * s2 + 4 * h2;             // element j < 4: keys r0 + 0..3; j >= 4: + 8
        const int a0 = vswz<VROW>(r0 + qq, c0 + (pp >> 1)) + 8 * (pp & 1);
        const int a1 = vswz<VROW>(r0 + 8 + qq, c0 + (pp >> 1)) + 8 * (pp & 1);
        typedef __attribute__((address_space(3))) s16x4 lds_s4;
        // whole-vector bit casts: element-wise extraction from the v4i16 result miscompiled
        // (duplicated pairs), caught by scripts/dbg_prefill_attn.py + scripts/probes/tr16_probe.hip
        const f16x4 lo = __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(Vs + a0)));
        const f16x4 hi = __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(Vs + a1)));
        const f16x8 vf = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        o[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pf, o[i], 0, 0, 0);
      }
    }
  }
  // O = O^T / l : lane = query, rows = d (r&3) + 8(r>>2) + 4*h2 of d tile i
  const int qo = q0 + wave * 32 + qc;
  if (qo < NQ) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    float* out = P.out + (long long)qo * P.ldo + head * Dv;
#pragma unroll
    for (int i = 0; i < NDT; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int d = 32 * i + 8 * k + 4 * h2;
        if (d < Dv)
          *(f32x4*)(out + d) = (f32x4){o[i][4 * k] * inv, o[i][4 * k + 1] * inv, o[i][4 * k + 2] * inv,
                                       o[i][4 * k + 3] * inv};
      }
  }
}

// query heads per block: the whole GQA group (one K/V read) unless the launch would be too narrow to
// fill the chip; then one head per block (K/V re-reads hit L2/MALL). Measured (profiles/r2_attn,
// scripts/bench_attn.py OMX_BENCH_HPB): H 64 / 8 KV heads, 560 keys: 9.4 us at 1 head per block vs
// 23.5 us with the whole group of 8 (Llama-2-70B decode); H 32 / 8, 560 keys: 8.5 vs 14.6 us
static int heads_per_block(const AttnParams& P) {
  const int G = P.H / P.n_kv;
  int hpb = g_attn_hpb > 0 ? g_attn_hpb : (P.NQ * P.n_kv < 64 ? 1 : G);
  if (P.D > 128 && hpb > 2) hpb = 2;  // head dim 256: the per-wave merge tile [8][G][D + 2] fits LDS for G <= 2
  // head dims 80 / 96 / 112 (an fp8 row of 5-7 bytes per lane is widened at load): at 4+ heads per block
  // the kernel spills, so those dims take at most 2 (K/V re-reads of a wider group hit L2)
  if (P.D % 64 && hpb > 2) hpb = 2;
  while (hpb > 1 && (G % hpb || (hpb != 1 && hpb != 2 && hpb != 4 && hpb != 8))) --hpb;
  return hpb < 1 ? 1 : hpb;
}

template <int D, bool KV8>
static void launch_dk(const AttnParams& P, hipStream_t s) {
  const int G = heads_per_block(P);
  dim3 grid(P.NQ, P.H / G, P.n_splits);
  // 8 lanes per key: fp8 rows at D = 128 (8 lanes x 16 B), and fp16 rows of head dims 80 / 96 / 112 (20-28 B
  // per lane in 2-3 vector loads; at 16 lanes a lane's 10-14 B are 2-B aligned: one load per element)
  constexpr int LPK8 = (KV8 && D == 128) || (!KV8 && (D == 80 || D == 96 || D == 112)) ? 8 : 16;
  switch (G) {
    case 1: hipLaunchKernelGGL((attn_decode_kernel<D, 1, KV8, LPK8>), grid, dim3(ATT_NT), 0, s, P); break;
    case 2: hipLaunchKernelGGL((attn_decode_kernel<D, 2, KV8, LPK8>), grid, dim3(ATT_NT), 0, s, P); break;
    case 4: if constexpr (D <= 128 && D % 64 == 0) hipLaunchKernelGGL((attn_decode_kernel<D, 4, KV8>), grid, dim3(ATT_NT), 0, s, P); break;
    case 8: if constexpr (D <= 128 && D % 64 == 0) hipLaunchKernelGGL((attn_decode_kernel<D, 8, KV8>), grid, dim3(ATT_NT), 0, s, P); break;
    default: break;
  }
}
template <int D>
static void launch_d(const AttnParams& P, hipStream_t s) {
  if (P.kv8) launch_dk<D, true>(P, s);
  else launch_dk<D, false>(P, s);
}
template <int D>
static void launch_pf(const AttnParams& P, dim3 grid, hipStream_t s) {
  if (P.kv8) hipLaunchKernelGGL((attn_prefill_kernel<D, true>), grid, dim3(256), 0, s, P);
  else hipLaunchKernelGGL((attn_prefill_kernel<D, false>), grid, dim3(256), 0, s, P);
}

void attention_decode(const AttnParams& P0, hipStream_t s) {
  if (P0.NQ <= 0) return;
  AttnParams P = P0;
  if (P.kps <= 0) P.kps = g_attn_kps;
  if (P.prefill && P.NQ >= 16 && P.D % 16 == 0) {  // one sequence, contiguous positions: MFMA flash
    dim3 grid((P.NQ + PF_BQ - 1) / PF_BQ, P.H);
    count_launch(LC_ATTN_PREFILL);
    switch (P.D) {
      case 64: launch_pf<64>(P, grid, s); return;
      case 80: launch_pf<80>(P, grid, s); return;
      case 96: launch_pf<96>(P, grid, s); return;
      case 112: launch_pf<112>(P, grid, s); return;  // Orca (100)
      case 128: launch_pf<128>(P, grid, s); return;
      case 256: launch_pf<256>(P, grid, s); return;  // Gemma
      default: break;
    }
  }
  count_launch(LC_ATTN_DECODE);
  switch (P.D) {
    case 64: launch_d<64>(P, s); break;
    case 80: launch_d<80>(P, s); break;
    case 96: launch_d<96>(P, s); break;
    case 112: launch_d<112>(P, s); break;  // Orca Mini (head dim 100 in a 112-wide cache row)
    case 128: launch_d<128>(P, s); break;
    case 256: launch_d<256>(P, s); break;  // Gemma
    default:  // models/config.py rejects any other head dim at load; a direct caller must not no-op
      throw std::runtime_error("attention: unsupported head dim " + std::to_string(P.D));
  }
}

size_t attention_ws_floats(int NQ, int H, int D, int n_splits) {
  return n_splits > 1 ? (size_t)NQ * H * n_splits * (D + 2) : 0;
}

}  // namespace omx
