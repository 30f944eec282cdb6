// Paged-KV grouped-query attention for decode and chunked prefill.
//
// Grid (query, kv_head, split). One 256-thread block serves the G = H/H_kv query heads that share a
// KV head, so each K/V row is read from HBM once per group (GQA reuse). 16 lanes cooperate on one
// key (D/16 dims each, one 16-B load for D = 128), so a wave streams 4 keys per load instruction
// and the 4 waves 16 keys per step; scores reduce inside the 16-lane group with xor-shuffles.
// Online softmax per lane group, merged across groups/waves at the end. The key range of a query
// is cut into `n_splits` equal chunks computed ON DEVICE from its length (flash-decode), so the
// grid is fixed and the launch is hipGraph-capturable for any context length; the last split
// block to arrive (agent-scope release/acquire ticket) merges the partials in the same launch.
// Causal prefill uses the same kernel: each prompt token is a query with length pos + 1.
#include "common.h"
#include "ops.h"

namespace omx {

template <int DPL>
__device__ __forceinline__ void load_row(const f16* p, float* v) {
  if constexpr (DPL == 8) {
    const f16x8 t = *(const f16x8*)p;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)t[j];
  } else if constexpr (DPL == 4) {
    const f16x4 t = *(const f16x4*)p;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (float)t[j];
  } else {
#pragma unroll
    for (int j = 0; j < DPL; ++j) v[j] = (float)p[j];
  }
}

template <int D, int G>
__global__ __launch_bounds__(256) void attn_partial_kernel(AttnParams P) {
  constexpr int DPL = D / 16;
  __shared__ float sm[4][G][D + 2];
  const int qi = blockIdx.x, kvh = blockIdx.y, split = blockIdx.z, S = gridDim.z;
  const int seq = P.q_seq ? P.q_seq[qi] : qi;
  const int len = P.q_len[qi];
  const int kstart = P.window > 0 ? max(0, len - P.window) : 0;
  const int nk = len - kstart;
  const int chunk = (nk + S - 1) / S;
  const int t0 = kstart + split * chunk;
  const int t1 = min(len, t0 + chunk);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, tg = lane >> 4, li = lane & 15;

  float q[G][DPL];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float* qp = P.q + (long long)qi * P.ldq + (kvh * G + g) * D + li * DPL;
#pragma unroll
    for (int j = 0; j < DPL; ++j) q[g][j] = qp[j] * P.scale;
  }
  float m[G], l[G], acc[G][DPL];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < DPL; ++j) acc[g][j] = 0.f;
  }
  const int* bt = P.block_table + (long long)seq * P.max_blocks;
  const f16* kc = (const f16*)P.kc;
  const f16* vc = (const f16*)P.vc;
  // 4 key slots per lane group per step (64 keys per block-step): all K/V loads of a step are
  // issued before any is consumed, so one HBM round trip covers 64 keys
  constexpr int U = 4;
  for (int ts = t0; ts < t1; ts += 16 * U) {
    float k[U][DPL], v[U][DPL];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = ts + u * 16 + wave * 4 + tg;
      ok[u] = t < t1;
      const int tt = ok[u] ? t : t0;
      const long long blk = bt[tt / P.bs];
      const long long base = ((blk * P.n_kv + kvh) * P.bs + (tt % P.bs)) * D + li * DPL;
      load_row<DPL>(kc + base, k[u]);
      load_row<DPL>(vc + base, v[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;  // uniform within the 16-lane group
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float sc = 0.f;
#pragma unroll
        for (int j = 0; j < DPL; ++j) sc += q[g][j] * k[u][j];
        sc = group_sum<16>(sc);
        const float mn = fmaxf(m[g], sc);
        const float corr = __expf(m[g] - mn);
        const float p = __expf(sc - mn);
        l[g] = l[g] * corr + p;
#pragma unroll
        for (int j = 0; j < DPL; ++j) acc[g][j] = acc[g][j] * corr + p * v[u][j];
        m[g] = mn;
      }
    }
  }
  // merge the 4 token groups of the wave (lanes li, li+16, li+32, li+48)
#pragma unroll
  for (int sh = 16; sh <= 32; sh <<= 1) {
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
  if (lane < 16) {
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
  // 4 waves merge: threads (g, d) over G*D outputs
  for (int i = threadIdx.x; i < G * D; i += 256) {
    const int g = i / D, d = i % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, sm[w][g][D]);
    float L = 0.f, A = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float c = __expf(sm[w][g][D] - M);
        L += sm[w][g][D + 1] * c;
        A += sm[w][g][d] * c;
      }
    }
    const int h = kvh * G + g;
    if (S == 1) {
      P.out[(long long)qi * P.ldo + h * D + d] = L > 0.f ? A / L : 0.f;
    } else {  // write-through (sc1) stores: the hand-off below then needs no release fence
      float* ws = P.ws + (((long long)qi * P.H + h) * S + split) * (D + 2);
      __hip_atomic_store(ws + d, A, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == 0) {
        __hip_atomic_store(ws + D, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ws + D + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (S == 1) return;
  // ---- in-launch split combine (cdna_hip_programming.md §6 Guideline 16 / MI355X_MICROARCH.md
  // "Valid forms" row 1): partials were stored sc1; every wave drains them (vmcnt(0)), the block
  // barriers, one lane takes an agent-scope ticket. The block drawing the last ticket reads every
  // partial with sc1 loads (no acquire needed) and merges its G heads. Saves the separate
  // combine launch (~4.5 us per layer at batch 1).
  __shared__ int s_last;
  __shared__ float sw[G][64];
  __shared__ float sL[G];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int* cnt = P.counters + (long long)qi * P.n_kv + kvh;
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
      const float* ws = P.ws + (((long long)qi * P.H + kvh * G + g) * S + (s < S ? s : 0)) * (D + 2);
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
  for (int i = threadIdx.x; i < G * D; i += 256) {
    const int g = i / D, d = i % D;
    const float* ws = P.ws + ((long long)qi * P.H + kvh * G + g) * S * (D + 2);
    float A = 0.f;
#pragma unroll 8
    for (int s = 0; s < S; ++s) A += sw[g][s] * ld1(ws + s * (D + 2) + d);
    const float L = sL[g];
    P.out[(long long)qi * P.ldo + (kvh * G + g) * D + d] = L > 0.f ? A / L : 0.f;
  }
}

template <int D>
static void launch_d(const AttnParams& P, hipStream_t s) {
  const int G = P.H / P.n_kv;
  dim3 grid(P.NQ, P.n_kv, P.n_splits);
  switch (G) {
    case 1: hipLaunchKernelGGL((attn_partial_kernel<D, 1>), grid, dim3(256), 0, s, P); break;
    case 2: hipLaunchKernelGGL((attn_partial_kernel<D, 2>), grid, dim3(256), 0, s, P); break;
    case 4: hipLaunchKernelGGL((attn_partial_kernel<D, 4>), grid, dim3(256), 0, s, P); break;
    case 8: hipLaunchKernelGGL((attn_partial_kernel<D, 8>), grid, dim3(256), 0, s, P); break;
    default: break;
  }
}

void attention_decode(const AttnParams& P, hipStream_t s) {
  if (P.NQ <= 0) return;
  switch (P.D) {
    case 64: launch_d<64>(P, s); break;
    case 80: launch_d<80>(P, s); break;
    case 96: launch_d<96>(P, s); break;
    case 128: launch_d<128>(P, s); break;
    default: break;
  }
  // split partials are merged in-launch by the last-arriving block (see attn_partial_kernel)
}

size_t attention_ws_floats(int NQ, int H, int D, int n_splits) {
  return n_splits > 1 ? (size_t)NQ * H * n_splits * (D + 2) : 0;
}

}  // namespace omx
