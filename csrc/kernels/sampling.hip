// On-device token sampling, one 1024-thread block per sequence, so the whole
// decode step -- forward + sampling + history update -- stays inside one hipGraph replay.
// Order follows Ollama's (llama.cpp) default chain: repeat/presence/frequency penalties over the
// last `repeat_last_n` tokens -> top-k -> top-p -> min-p (on T = 1 probabilities) -> temperature
// -> categorical draw. temperature <= 0 is greedy argmax. Top-k: a histogram of (max - logit) in
// fine bins locates the k-th largest, the survivors are bitonic-sorted in LDS; an exact 4-pass
// radix select over order-preserving float keys is the fallback when too many logits tie.
#include "common.h"
#include "feedback.h"
#include "ops.h"
#include "wave_shuffle.h"

namespace omx {

constexpr int SAMPLE_NT = 1024;
constexpr int SAMPLE_CAP = 1024;
constexpr int SAMPLE_BINS = 2 * SAMPLE_NT;  // 2048 bins of 1/32 logit unit = 64 units below max
constexpr float SAMPLE_BIN_SCALE = 32.f;

__device__ __forceinline__ unsigned fkey(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ void block_argmax(const float* lg, int V, float* sv, int* si, float& best, int& bi) {
  float bv = -INFINITY;
  int bidx = 0x7FFFFFFF;
  for (int i = threadIdx.x; i < V; i += SAMPLE_NT) {
    const float v = lg[i];
    if (v > bv) { bv = v; bidx = i; }
  }
  for (int m = 32; m >= 1; m >>= 1) {
    const float ov = __shfl_xor(bv, m, 64);
    const int oi = __shfl_xor(bidx, m, 64);
    if (ov > bv || (ov == bv && oi < bidx)) { bv = ov; bidx = oi; }
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) { sv[w] = bv; si[w] = bidx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < SAMPLE_NT / 64; ++k)
      if (sv[k] > sv[0] || (sv[k] == sv[0] && si[k] < si[0])) { sv[0] = sv[k]; si[0] = si[k]; }
  }
  __syncthreads();
  best = sv[0];
  bi = si[0];
}

// repeat / presence / frequency penalties over the recent-token window, in place (each distinct
// token once, with its count); block-wide
__device__ void apply_penalties_inplace(const SampleParams& P, int b, float* lg, int V) {
  const int seen = P.hist_count[b];
  int win = min(seen, P.repeat_last_n[b]);
  win = min(win, P.hist_cap);
  const float rp = P.repeat_penalty[b], pp = P.presence_penalty[b], fp = P.frequency_penalty[b];
  if (win > 0 && (rp != 1.f || pp != 0.f || fp != 0.f)) {
    const int* h = P.history + (long long)b * P.hist_cap;
    for (int i = threadIdx.x; i < win; i += blockDim.x) {
      const int tok = h[(seen - 1 - i) % P.hist_cap];
      bool first = true;
      int cnt = 1;
      for (int j = 0; j < win; ++j) {
        if (j == i) continue;
        const int o = h[(seen - 1 - j) % P.hist_cap];
        if (o == tok) {
          ++cnt;
          if (j < i) first = false;
        }
      }
      if (first && tok >= 0 && tok < V) {
        float v = lg[tok];
        if (rp != 1.f) v = v > 0.f ? v / rp : v * rp;
        v -= (float)cnt * fp + pp;
        lg[tok] = v;
      }
    }
    __syncthreads();
  }
}

// single-block selection over the whole (penalised) row: greedy, or top-k (any k <= SAMPLE_CAP)
// -> top-p -> min-p -> temperature -> draw. Needs blockDim.x == SAMPLE_NT.
__device__ void legacy_select(const SampleParams& P, int b, float* lg, int V, int& chosen, float& chosen_lp) {

  __shared__ float cval[SAMPLE_CAP];
  __shared__ int cidx[SAMPLE_CAP];
  __shared__ unsigned hist[256];
  __shared__ float redv[SAMPLE_NT / 64];
  __shared__ int redi[SAMPLE_NT / 64];
  __shared__ unsigned s_prefix, s_mask, s_remaining;
  __shared__ int s_count, s_bstar;
  __shared__ unsigned bins[SAMPLE_BINS];
  __shared__ unsigned wsum[SAMPLE_NT / 64];

  const float temp = P.temperature[b];
  chosen = 0;
  chosen_lp = 0.f;
  if (temp <= 0.f) {
    float best;
    block_argmax(lg, V, redv, redi, best, chosen);
  } else {
    int k = P.top_k[b];
    if (k <= 0 || k > SAMPLE_CAP) k = SAMPLE_CAP;
    if (k > V) k = V;
    // ---- fast path: histogram of (max - x) in 1/32-wide bins. Logits spread over the bins, so
    // the LDS atomics rarely collide (a radix pass on raw float keys puts nearly every logit in
    // 2-3 exponent bins and serialises). Everything in bins <= b* (the bin holding the k-th
    // largest) is collected and sorted exactly; the radix select below remains the fallback.
    float mx;
    {
      float lm = -INFINITY;
      for (int i = threadIdx.x; i < V; i += SAMPLE_NT) lm = fmaxf(lm, lg[i]);
      mx = block_max<SAMPLE_NT>(lm, redv);
    }
    for (int i = threadIdx.x; i < SAMPLE_BINS; i += SAMPLE_NT) bins[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < V; i += SAMPLE_NT) {
      const float d = (mx - lg[i]) * SAMPLE_BIN_SCALE;
      if (d < (float)(SAMPLE_BINS - 1)) atomicAdd(&bins[(int)d], 1u);
    }
    if (threadIdx.x == 0) { s_bstar = SAMPLE_BINS - 1; s_count = 0; }
    __syncthreads();
    {  // block-wide exclusive scan over bins (2 per thread) -> first bin where cum >= k
      const unsigned a0 = bins[2 * threadIdx.x], a1 = bins[2 * threadIdx.x + 1];
      unsigned v = a0 + a1, incl = v;
      const int ln = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(incl, o, 64);
        if (ln >= o) incl += t;
      }
      if (ln == 63) wsum[wv] = incl;
      __syncthreads();
      unsigned pre = 0;
      for (int w = 0; w < wv; ++w) pre += wsum[w];
      const unsigned ex = pre + incl - v;
      if (ex < (unsigned)k && ex + a0 >= (unsigned)k) s_bstar = 2 * threadIdx.x;
      else if (ex + a0 < (unsigned)k && ex + v >= (unsigned)k) s_bstar = 2 * threadIdx.x + 1;
    }
    __syncthreads();
    const int bstar = s_bstar;
    for (int i = threadIdx.x; i < V; i += SAMPLE_NT) {
      const float v = lg[i];
      const float d = (mx - v) * SAMPLE_BIN_SCALE;
      if (d < (float)(bstar + 1)) {
        const int slot = atomicAdd(&s_count, 1);
        if (slot < SAMPLE_CAP) { cval[slot] = v; cidx[slot] = i; }
      }
    }
    __syncthreads();
    if (s_count > SAMPLE_CAP) {
    // ---- radix select fallback: key of the k-th largest logit
    if (threadIdx.x == 0) { s_prefix = 0; s_mask = 0; s_remaining = k; }
    __syncthreads();
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
      for (int i = threadIdx.x; i < 256; i += SAMPLE_NT) hist[i] = 0;
      __syncthreads();
      const unsigned prefix = s_prefix, mask = s_mask;
      for (int i = threadIdx.x; i < V; i += SAMPLE_NT) {
        const unsigned key = fkey(lg[i]);
        if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 0xFF], 1u);
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        unsigned rem = s_remaining, cum = 0;
        int bin = 255;
        for (; bin > 0; --bin) {
          if (cum + hist[bin] >= rem) break;
          cum += hist[bin];
        }
        s_prefix = prefix | ((unsigned)bin << shift);
        s_mask = mask | (0xFFu << shift);
        s_remaining = rem - cum;
      }
      __syncthreads();
    }
    const unsigned thr = s_prefix;
    if (threadIdx.x == 0) s_count = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < V; i += SAMPLE_NT) {  // strictly above the k-th key: < k of them
      const float v = lg[i];
      if (fkey(v) > thr) {
        const int slot = atomicAdd(&s_count, 1);
        cval[slot] = v;
        cidx[slot] = i;
      }
    }
    __syncthreads();
    // ties with the k-th key fill the rest lowest index first (the host's stable order; atomic
    // arrival order would make the kept set depend on scheduling when > SAMPLE_CAP logits tie)
    int have = s_count;
    const int ln = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int base = 0; base < V && have < k; base += SAMPLE_NT) {
      const int i = base + threadIdx.x;
      const bool tie = i < V && fkey(lg[i]) == thr;
      const unsigned long long m = __ballot(tie);
      if (ln == 0) wsum[wv] = (unsigned)__popcll(m);
      __syncthreads();
      unsigned pre = 0, tot = 0;
      for (int w = 0; w < SAMPLE_NT / 64; ++w) {
        if (w < wv) pre += wsum[w];
        tot += wsum[w];
      }
      const int pos = have + (int)pre + __popcll(m & ((1ull << ln) - 1));
      if (tie && pos < k) { cval[pos] = lg[i]; cidx[pos] = i; }
      have = min(k, have + (int)tot);
      __syncthreads();  // wsum reuse
    }
    if (threadIdx.x == 0) s_count = have;
    __syncthreads();
    }
    const int cnt = min(s_count, SAMPLE_CAP);
    int n2 = 1;
    while (n2 < cnt) n2 <<= 1;
    for (int i = cnt + threadIdx.x; i < n2; i += SAMPLE_NT) { cval[i] = -INFINITY; cidx[i] = 0x7FFFFFFF; }
    __syncthreads();
    // bitonic sort, descending by value (ties: lower index first)
    for (int size = 2; size <= n2; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int i = threadIdx.x; i < n2; i += SAMPLE_NT) {
          const int j = i ^ stride;
          if (j > i) {
            const bool desc = (i & size) == 0;
            const float a = cval[i], c = cval[j];
            const int ai = cidx[i], ci = cidx[j];
            const bool a_first = a > c || (a == c && ai < ci);
            if (desc != a_first) {
              cval[i] = c; cval[j] = a; cidx[i] = ci; cidx[j] = ai;
            }
          }
        }
        __syncthreads();
      }
    }
    if (threadIdx.x == 0) {
      const int n = min(k, cnt);
      const float top = cval[0];
      // T = 1 probabilities for top-p / min-p
      float z = 0.f;
      for (int i = 0; i < n; ++i) z += __expf(cval[i] - top);
      const float topp = P.top_p[b], minp = P.min_p[b];
      int keep = n;
      if (topp < 1.f) {
        float c = 0.f;
        for (int i = 0; i < n; ++i) {
          c += __expf(cval[i] - top) / z;
          if (c >= topp) { keep = i + 1; break; }
        }
      }
      if (minp > 0.f) {
        int j = 1;
        while (j < keep && __expf(cval[j] - top) >= minp) ++j;
        keep = j;
      }
      // temperature, then draw
      float zt = 0.f;
      for (int i = 0; i < keep; ++i) zt += __expf((cval[i] - top) / temp);
      const unsigned long long r = splitmix64(P.seed[b] ^ (0xD1B54A32D192ED03ull * (unsigned long long)(P.step[b] + 1)));
      const float u = (float)(r >> 40) * (1.0f / 16777216.0f) * zt;
      float c = 0.f;
      int pick = keep - 1;
      for (int i = 0; i < keep; ++i) {
        c += __expf((cval[i] - top) / temp);
        if (u < c) { pick = i; break; }
      }
      chosen = cidx[pick];
      chosen_lp = (cval[pick] - top) / temp - __logf(zt);
      redi[0] = chosen;
      redv[0] = chosen_lp;
    }
    __syncthreads();
    chosen = redi[0];
    chosen_lp = redv[0];
  }
}

__device__ __forceinline__ void finish_sample(const SampleParams& P, int b, int chosen, float chosen_lp) {
  // a non-finite logit row (an overflowed activation upstream) must not turn into an out-of-range id:
  // the id is the next step's embedding row, read on device without a host check
  if ((unsigned)chosen >= (unsigned)P.V) {
    chosen = 0;
    if (P.err) *P.err = 1;  // the host fails the request (Runner.sampler_error)
  }
  const int seen = P.hist_count[b];
  P.out[b] = chosen;
  if (P.out_logprob) P.out_logprob[b] = chosen_lp;
  P.history[(long long)b * P.hist_cap + (seen % P.hist_cap)] = chosen;
  P.hist_count[b] = seen + 1;
  P.step[b] += 1;
  if (P.fb_step) decode_feedback_row(P.fb_step, P.fb_ld, b, chosen, 1, P.fb_block_table, P.fb_max_blocks, P.fb_bs,
                                     P.fb_host_ring, P.fb_ring, P.fb_sysfence);
}

__global__ __launch_bounds__(SAMPLE_NT) void sample_kernel(SampleParams P) {
  const int b = blockIdx.x;
  float* lg = (float*)P.logits + (long long)b * P.ld;
  apply_penalties_inplace(P, b, lg, P.V);
  int chosen;
  float chosen_lp;
  legacy_select(P, b, lg, P.V, chosen, chosen_lp);
  if (threadIdx.x == 0) finish_sample(P, b, chosen, chosen_lp);
}

// ---------------------------------------------------------------------------------------------
// Multi-block fast path (top_k in 1..64, or greedy): one 1024-thread block per 1024-logit slice,
// one logit per lane. Each wave sorts its 64 logits (64-lane bitonic network on DPP / permlane
// exchanges, order = value desc, index asc -- the host reference's stable argsort); the block's 16
// sorted lists merge through LDS in a tree into its exact top-64; the list goes out with sc1
// (agent-scope) stores and the block drawing the last agent-scope ticket merges every block's list
// and samples with wave scans (MI355X_MICROARCH.md "Valid forms" row 1, as attention's split
// combine). A row whose top_k is outside 1..64 is handed to legacy_select in that last block, on
// the untouched logits.
constexpr int FAST_K = 64;
constexpr int FAST_SLICE = SAMPLE_NT;

__device__ __forceinline__ bool cand_better(float av, int ai, float bv, int bi) {
  return av > bv || (av == bv && ai < bi);
}

// compare-exchange with lane ^ J; the lower lane of the pair ends with the better when lo_better
template <int J>
__device__ __forceinline__ void cand_cx(float& v, int& i, bool lo_better) {
  const int lane = threadIdx.x & 63;
  const float ov = xor_shfl<J>(v);
  const int oi = xor_shfl<J>(i);
  const bool want_better = ((lane & J) == 0) == lo_better;
  if (want_better == cand_better(ov, oi, v, i)) { v = ov; i = oi; }
}

// half-cleaners J, J/2, .., 1
template <int J>
__device__ __forceinline__ void cand_clean(float& v, int& i, bool lo_better) {
  cand_cx<J>(v, i, lo_better);
  if constexpr (J > 1) cand_clean<J / 2>(v, i, lo_better);
}

template <int SIZE>
__device__ __forceinline__ void cand_sort_stage(float& v, int& i, bool desc) {
  const int lane = threadIdx.x & 63;
  cand_clean<SIZE / 2>(v, i, ((lane & SIZE) == 0) == desc);
  if constexpr (SIZE < 64) cand_sort_stage<SIZE * 2>(v, i, desc);
}

// sort one candidate per lane across the wave: descending (lane 0 best) or ascending
__device__ __forceinline__ void wave_bitonic_sort(float& v, int& i, bool desc) { cand_sort_stage<2>(v, i, desc); }

// R (desc) := top-64 of R u C, where C is sorted ascending
__device__ __forceinline__ void wave_merge_asc(float& rv, int& ri, float cv, int ci) {
  if (cand_better(cv, ci, rv, ri)) { rv = cv; ri = ci; }  // bitonic: the 64 best of the union
  cand_clean<32>(rv, ri, true);
}

// R (desc) := top-64 of R u L, where L is sorted descending (lane l reads L[63 - l])
__device__ __forceinline__ void wave_merge_desc(float& rv, int& ri, const float* lv, const int* li) {
  const int lane = threadIdx.x & 63;
  wave_merge_asc(rv, ri, lv[63 - lane], li[63 - lane]);
}

__global__ __launch_bounds__(SAMPLE_NT) void sample_fast_kernel(SampleParams P) {
  __shared__ int pen_cnt[FAST_SLICE];
  __shared__ float lv[SAMPLE_NT / 64][FAST_K];
  __shared__ int li[SAMPLE_NT / 64][FAST_K];
  __shared__ int s_last;
  const int b = blockIdx.y, G = gridDim.x, blk = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const float* lg = P.logits + (long long)b * P.ld;
  const int V = P.V, base = blk * FAST_SLICE + wave * 64;
  const float temp = P.temperature[b];
  const int kk = P.top_k[b];
  const bool fast = temp <= 0.f || (kk >= 1 && kk <= FAST_K);

  if (fast) {
    const int ix = base + lane;
    float v = ix < V ? lg[ix] : -INFINITY;
    if (v != v) v = -INFINITY;  // NaN ranks last (every comparison with it is false)
    // penalties for the tokens of this slice (counts via LDS, applied in registers)
    const int seen = P.hist_count[b];
    const int win = min(min(seen, P.repeat_last_n[b]), P.hist_cap);
    const float rp = P.repeat_penalty[b], pp = P.presence_penalty[b], fp = P.frequency_penalty[b];
    if (win > 0 && (rp != 1.f || pp != 0.f || fp != 0.f)) {
      pen_cnt[tid] = 0;
      __syncthreads();
      const int* h = P.history + (long long)b * P.hist_cap;
      for (int i = tid; i < win; i += SAMPLE_NT) {
        const int tok = h[(seen - 1 - i) % P.hist_cap] - blk * FAST_SLICE;
        if (tok >= 0 && tok < FAST_SLICE) atomicAdd(&pen_cnt[tok], 1);
      }
      __syncthreads();
      const int cnt = pen_cnt[tid];
      if (cnt > 0 && ix < V) {
        if (rp != 1.f) v = v > 0.f ? v / rp : v * rp;
        v -= (float)cnt * fp + pp;
      }
    }
    float rv = v;
    int ri = ix < V ? ix : 0x7FFFFFFF;
    wave_bitonic_sort(rv, ri, true);
    // block tree merge of the 16 wave lists
    lv[wave][lane] = rv;
    li[wave][lane] = ri;
    for (int st = 1; st < SAMPLE_NT / 64; st <<= 1) {
      __syncthreads();
      if ((wave & (2 * st - 1)) == 0) {
        wave_merge_desc(rv, ri, lv[wave + st], li[wave + st]);
        lv[wave][lane] = rv;
        li[wave][lane] = ri;
      }
    }
    if (wave == 0) {  // sc1 stores of the block list; drained before the ticket
      float* wsv = P.ws + ((long long)b * G + blk) * 2 * FAST_K;
      __hip_atomic_store(wsv + lane, rv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((int*)wsv + FAST_K + lane, ri, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    int* cnt = P.counters + b;
    const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == G - 1;
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;

  if (!fast) {  // top_k outside 1..64: the whole row in this block, as sample_kernel
    float* lgw = (float*)P.logits + (long long)b * P.ld;
    apply_penalties_inplace(P, b, lgw, V);
    int chosen;
    float chosen_lp;
    legacy_select(P, b, lgw, V, chosen, chosen_lp);
    if (tid == 0) finish_sample(P, b, chosen, chosen_lp);
    return;
  }
  // ---- merge every block's list (sc1 loads), tree over the waves
  auto ldf = [](const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  auto ldi = [](const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  float rv = -INFINITY;
  int ri = 0x7FFFFFFF;
  for (int l = wave; l < G; l += SAMPLE_NT / 64) {
    const float* wsv = P.ws + ((long long)b * G + l) * 2 * FAST_K;
    const float cv = ldf(wsv + 63 - lane);
    const int ci = ldi((const int*)wsv + FAST_K + 63 - lane);
    wave_merge_asc(rv, ri, cv, ci);
  }
  __syncthreads();  // lv / li reuse
  lv[wave][lane] = rv;
  li[wave][lane] = ri;
  for (int st = 1; st < SAMPLE_NT / 64; st <<= 1) {
    __syncthreads();
    if ((wave & (2 * st - 1)) == 0) {
      wave_merge_desc(rv, ri, lv[wave + st], li[wave + st]);
      lv[wave][lane] = rv;
      li[wave][lane] = ri;
    }
  }
  if (wave != 0) return;
  // ---- wave 0: candidates sorted (lane = rank); top-p -> min-p -> temperature -> draw
  int chosen = __shfl(ri, 0, 64);
  float chosen_lp = 0.f;
  if (temp > 0.f) {
    const int n = min(kk, V);
    const float top = __shfl(rv, 0, 64);
    const bool in = lane < n;
    const float e1 = in ? __expf(rv - top) : 0.f;
    const float z = wave_sum(e1);
    int keep = n;
    const float topp = P.top_p[b], minp = P.min_p[b];
    if (topp < 1.f) {
      float c = e1 / z;  // inclusive prefix sum over ranks
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float t = __shfl_up(c, o, 64);
        if (lane >= o) c += t;
      }
      const unsigned long long hit = __ballot(in && c >= topp);
      if (hit) keep = __ffsll((long long)hit);  // first rank reaching top_p, inclusive
    }
    if (minp > 0.f) {
      const unsigned long long fail = __ballot(lane >= 1 && lane < keep && e1 < minp);
      if (fail) keep = __ffsll((long long)fail) - 1;
    }
    const float wt = lane < keep ? __expf((rv - top) / temp) : 0.f;
    const float zt = wave_sum(wt);
    float c = wt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float t = __shfl_up(c, o, 64);
      if (lane >= o) c += t;
    }
    const unsigned long long r = splitmix64(P.seed[b] ^ (0xD1B54A32D192ED03ull * (unsigned long long)(P.step[b] + 1)));
    const float u = (float)(r >> 40) * (1.0f / 16777216.0f) * zt;
    const unsigned long long hit = __ballot(lane < keep && u < c);
    const int pick = hit ? __ffsll((long long)hit) - 1 : keep - 1;
    chosen = __shfl(ri, pick, 64);
    chosen_lp = (__shfl(rv, pick, 64) - top) / temp - __logf(zt);
  }
  if (lane == 0) finish_sample(P, b, chosen, chosen_lp);
}

void sample(const SampleParams& P, hipStream_t s) {
  if (P.B <= 0) return;
  if (P.ws && P.counters) {  // multi-block path (rows with top_k outside 1..64 fall back inside it)
    const int G = (P.V + FAST_SLICE - 1) / FAST_SLICE;
    hipLaunchKernelGGL(sample_fast_kernel, dim3(G, P.B), dim3(SAMPLE_NT), 0, s, P);
    return;
  }
  hipLaunchKernelGGL(sample_kernel, dim3(P.B), dim3(SAMPLE_NT), 0, s, P);
}

__global__ __launch_bounds__(SAMPLE_NT) void argmax_kernel(const float* logits, int V, int ld, int* out) {
  __shared__ float sv[SAMPLE_NT / 64];
  __shared__ int si[SAMPLE_NT / 64];
  float best;
  int bi;
  block_argmax(logits + (long long)blockIdx.x * ld, V, sv, si, best, bi);
  if (threadIdx.x == 0) out[blockIdx.x] = bi;
}

void argmax(const float* logits, int B, int V, int ld, int* out, hipStream_t s) {
  if (B <= 0) return;
  hipLaunchKernelGGL(argmax_kernel, dim3(B), dim3(SAMPLE_NT), 0, s, logits, V, ld, out);
}

}  // namespace omx
