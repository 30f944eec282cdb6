// Batch-1 decode attention probe (round 6): where do the 5.7 us of a 150-key MHA attention launch go,
// and which geometry is fastest in a dependent chain? Standalone (hipcc, no torch):
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I csrc/kernels experiments/attn_probe/probe.hip -o /tmp/attn_probe
// Chain per "layer": producer (writes q, like the QKV GEMV's epilogue) -> attention (deferred split
// partials, the engine's B == 1 path) -> consumer (reads every partial slab, like the O GEMV's merge
// prologue). KV caches rotate over enough copies to miss the 256 MiB Infinity Cache. The attention's
// marginal cost = graph(with) - graph(without), per layer. Stamp mode: s_memrealtime (100 MHz) per block
// at kernel entry / operands in / KV in / merged / end, relative to the producer's last block end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.h"
#include "ops.h"

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

using namespace omx;

typedef unsigned long long u64;

__device__ __forceinline__ void stamp(u64* ts, int k) {
  if (ts && threadIdx.x == 0) ts[((long long)blockIdx.z * gridDim.y + blockIdx.y) * 8 + k] = __builtin_amdgcn_s_memrealtime();
}

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float key_sum16(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  v += dppf<0x140>(v);
  return v;
}

template <int DPL>
struct KRow {
  f16 v[DPL];
};
template <int DPL>
__device__ __forceinline__ void load_krow(const f16* p, KRow<DPL>& r) {
  const f16x8 t = __builtin_nontemporal_load((const f16x8*)p);
#pragma unroll
  for (int j = 0; j < 8; ++j) r.v[j] = t[j];
}
template <int DPL, int U>
struct KVStep {
  KRow<DPL> k[U], v[U];
};

// ---------------------------------------------------------------------------------------------
// baseline: the engine's attn_decode_kernel<128, 1> (fp16 KV, G = 1, deferred) with stamps
constexpr int BTW = 1024;
template <int D, int NW, int U>
__global__ __launch_bounds__(64 * NW) void attn_base(AttnParams P, u64* ts) {
  constexpr int LPK = 16, DPL = D / LPK, KPW = 64 / LPK, NG = KPW * NW, STEP = NG * U;
  __shared__ float sm[NW][D + 2];
  __shared__ int sbt[BTW];
  stamp(ts, 0);
  const int qi = blockIdx.x, split = blockIdx.z, h = blockIdx.y;
  const int kvh = h / (P.H / P.n_kv);
  const int seq = P.q_seq ? P.q_seq[qi] : qi;
  const int len = P.q_len[qi];
  const int S = gridDim.z;
  const int chunk = (len + S - 1) / S;
  const int t0 = split * chunk, t1 = min(len, t0 + chunk);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, tg = lane / LPK, li = lane % LPK;
  const int grp = wave * KPW + tg;
  float q[DPL];
  const float* qp = P.q + (long long)qi * P.ldq + h * D;
#pragma unroll
  for (int j = 0; j < DPL; ++j) q[j] = qp[li * DPL + j] * P.scale;
  float m = -INFINITY, l = 0.f, acc[DPL];
#pragma unroll
  for (int j = 0; j < DPL; ++j) acc[j] = 0.f;
  const int* bt = P.block_table + (long long)seq * P.max_blocks;
  const f16* kc = (const f16*)P.kc;
  const f16* vc = (const f16*)P.vc;
  const int bs = P.bs;
  for (int w0 = t0; w0 < t1; w0 += BTW * bs) {
    const int w1 = min(t1, w0 + BTW * bs);
    const int b0 = w0 / bs, nb = (w1 - 1) / bs - b0 + 1;
    __syncthreads();
    for (int i = threadIdx.x; i < nb; i += 64 * NW) sbt[i] = bt[b0 + i];
    __syncthreads();
    stamp(ts, 1);
    auto issue = [&](int ts_, KVStep<DPL, U>& st) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = min(ts_ + u * NG + grp, w1 - 1);
        const long long blk = sbt[t / bs - b0];
        const long long base = ((blk * P.n_kv + kvh) * bs + (t % bs)) * D + li * DPL;
        load_krow<DPL>(kc + base, st.k[u]);
        load_krow<DPL>(vc + base, st.v[u]);
      }
    };
    bool first = true;
    auto consume = [&](int ts_, const KVStep<DPL, U>& st) {
      float sc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = ts_ + u * NG + grp < w1;
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < DPL; ++j) s += q[j] * (float)st.k[u].v[j];
        s = key_sum16(s);
        sc[u] = ok ? s : -INFINITY;
      }
      if (first) {
        first = false;
        stamp(ts, 2);
      }
      float mn = m;
#pragma unroll
      for (int u = 0; u < U; ++u) mn = fmaxf(mn, sc[u]);
      float p[U];
      if (mn == -INFINITY) {
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = 0.f;
      } else {
        const float corr = __expf(m - mn);
        float ps = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          p[u] = __expf(sc[u] - mn);
          ps += p[u];
        }
        l = l * corr + ps;
#pragma unroll
        for (int j = 0; j < DPL; ++j) acc[j] *= corr;
        m = mn;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < DPL; ++j) acc[j] += p[u] * (float)st.v[u].v[j];
    };
    KVStep<DPL, U> A, B;
    int t_ = w0;
    issue(t_, A);
    while (true) {
      if (t_ + STEP < w1) issue(t_ + STEP, B);
      consume(t_, A);
      t_ += STEP;
      if (t_ >= w1) break;
      if (t_ + STEP < w1) issue(t_ + STEP, A);
      consume(t_, B);
      t_ += STEP;
      if (t_ >= w1) break;
    }
  }
#pragma unroll
  for (int sh = LPK; sh <= 32; sh <<= 1) {
    const float mo = __shfl_xor(m, sh, 64), lo = __shfl_xor(l, sh, 64);
    const float mn = fmaxf(m, mo);
    const float c0 = mn == -INFINITY ? 0.f : __expf(m - mn);
    const float c1 = mn == -INFINITY ? 0.f : __expf(mo - mn);
    l = l * c0 + lo * c1;
#pragma unroll
    for (int j = 0; j < DPL; ++j) acc[j] = acc[j] * c0 + __shfl_xor(acc[j], sh, 64) * c1;
    m = mn;
  }
  if (lane < LPK) {
#pragma unroll
    for (int j = 0; j < DPL; ++j) sm[wave][li * DPL + j] = acc[j];
    if (li == 0) {
      sm[wave][D] = m;
      sm[wave][D + 1] = l;
    }
  }
  __syncthreads();
  stamp(ts, 3);
  for (int d = threadIdx.x; d < D; d += 64 * NW) {
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, sm[w][D]);
    float L = 0.f, A = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const float c = __expf(sm[w][D] - M);
        L += sm[w][D + 1] * c;
        A += sm[w][d] * c;
      }
    }
    const long long row = (long long)qi * S + split;
    P.ws[row * P.H * D + h * D + d] = A;
    if (d == 0) *(f32x2*)(P.ws + (long long)P.NQ * S * P.H * D + (row * P.H + h) * 2) = (f32x2){M, L};
  }
  stamp(ts, 4);
}

// ---------------------------------------------------------------------------------------------
// v2: block-table entries loaded straight into registers one step ahead (no LDS staging, no barrier
// before the first K/V load), power-of-two page shifts, q loaded behind the K/V issue, the cross-wave
// merge only when NW > 1 (one wave: shuffles and direct stores).
template <int D, int NW, int U>
__global__ __launch_bounds__(64 * NW) void attn_v2(AttnParams P, u64* ts) {
  constexpr int LPK = 16, DPL = D / LPK, KPW = 64 / LPK, NG = KPW * NW, STEP = NG * U;
  __shared__ float sm[NW > 1 ? NW : 1][D + 2];
  stamp(ts, 0);
  const int qi = blockIdx.x, split = blockIdx.z, h = blockIdx.y;
  const int kvh = h / (P.H / P.n_kv);
  const int seq = P.q_seq ? P.q_seq[qi] : qi;
  const int len = P.q_len[qi];
  const int S = gridDim.z;
  const int chunk = (len + S - 1) / S;
  const int t0 = split * chunk, t1 = min(len, t0 + chunk);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, tg = lane >> 4, li = lane & 15;
  const int grp = wave * KPW + tg;
  const int bsh = __ffs(P.bs) - 1, bmask = P.bs - 1;
  const int* bt = P.block_table + (long long)seq * P.max_blocks;
  const f16* kc = (const f16*)P.kc;
  const f16* vc = (const f16*)P.vc;
  float m = -INFINITY, l = 0.f, acc[DPL];
#pragma unroll
  for (int j = 0; j < DPL; ++j) acc[j] = 0.f;
  if (t0 < t1) {
    auto ldbt = [&](int s0, int (&b)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) b[u] = bt[min(s0 + u * NG + grp, t1 - 1) >> bsh];
    };
    auto issue = [&](int s0, const int (&b)[U], KVStep<DPL, U>& st) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = min(s0 + u * NG + grp, t1 - 1);
        const long long base = ((((long long)b[u] * P.n_kv + kvh) << bsh) + (t & bmask)) * D + li * DPL;
        load_krow<DPL>(kc + base, st.k[u]);
        load_krow<DPL>(vc + base, st.v[u]);
      }
    };
    int bA[U], bB[U];
    ldbt(t0, bA);
    const float* qp = P.q + (long long)qi * P.ldq + h * D + li * DPL;
    const f32x4 q0 = *(const f32x4*)qp, q1 = *(const f32x4*)(qp + 4);
    KVStep<DPL, U> A, B;
    issue(t0, bA, A);
    if (t0 + STEP < t1) ldbt(t0 + STEP, bB);
    float q[DPL] = {q0.x * P.scale, q0.y * P.scale, q0.z * P.scale, q0.w * P.scale,
                    q1.x * P.scale, q1.y * P.scale, q1.z * P.scale, q1.w * P.scale};
    stamp(ts, 1);
    bool first = true;
    auto consume = [&](int s0, const KVStep<DPL, U>& st) {
      float sc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = s0 + u * NG + grp < t1;
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < DPL; ++j) s += q[j] * (float)st.k[u].v[j];
        s = key_sum16(s);
        sc[u] = ok ? s : -INFINITY;
      }
      if (first) {
        first = false;
        stamp(ts, 2);
      }
      float mn = m;
#pragma unroll
      for (int u = 0; u < U; ++u) mn = fmaxf(mn, sc[u]);
      float p[U];
      if (mn == -INFINITY) {
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = 0.f;
      } else {
        const float corr = __expf(m - mn);
        float ps = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          p[u] = __expf(sc[u] - mn);
          ps += p[u];
        }
        l = l * corr + ps;
#pragma unroll
        for (int j = 0; j < DPL; ++j) acc[j] *= corr;
        m = mn;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < DPL; ++j) acc[j] += p[u] * (float)st.v[u].v[j];
    };
    int s0 = t0;
    while (true) {
      if (s0 + STEP < t1) {
        issue(s0 + STEP, bB, B);
        if (s0 + 2 * STEP < t1) ldbt(s0 + 2 * STEP, bA);
      }
      consume(s0, A);
      s0 += STEP;
      if (s0 >= t1) break;
      if (s0 + STEP < t1) {
        issue(s0 + STEP, bA, A);
        if (s0 + 2 * STEP < t1) ldbt(s0 + 2 * STEP, bB);
      }
      consume(s0, B);
      s0 += STEP;
      if (s0 >= t1) break;
    }
  }
  // merge the wave's 4 key groups
#pragma unroll
  for (int sh = 16; sh <= 32; sh <<= 1) {
    const float mo = __shfl_xor(m, sh, 64), lo = __shfl_xor(l, sh, 64);
    const float mn = fmaxf(m, mo);
    const float c0 = mn == -INFINITY ? 0.f : __expf(m - mn);
    const float c1 = mn == -INFINITY ? 0.f : __expf(mo - mn);
    l = l * c0 + lo * c1;
#pragma unroll
    for (int j = 0; j < DPL; ++j) acc[j] = acc[j] * c0 + __shfl_xor(acc[j], sh, 64) * c1;
    m = mn;
  }
  const long long row = (long long)qi * S + split;
  float* out = P.ws + row * P.H * D + h * D;
  float* ml = P.ws + (long long)P.NQ * S * P.H * D + (row * P.H + h) * 2;
  if constexpr (NW == 1) {
    stamp(ts, 3);
    if (lane < 16) {
      *(f32x4*)(out + li * DPL) = (f32x4){acc[0], acc[1], acc[2], acc[3]};
      *(f32x4*)(out + li * DPL + 4) = (f32x4){acc[4], acc[5], acc[6], acc[7]};
      if (li == 0) *(f32x2*)ml = (f32x2){m, l};
    }
  } else {
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < DPL; ++j) sm[wave][li * DPL + j] = acc[j];
      if (li == 0) {
        sm[wave][D] = m;
        sm[wave][D + 1] = l;
      }
    }
    __syncthreads();
    stamp(ts, 3);
    for (int d = threadIdx.x; d < D; d += 64 * NW) {
      float M = -INFINITY;
#pragma unroll
      for (int w = 0; w < NW; ++w) M = fmaxf(M, sm[w][D]);
      float L = 0.f, Acc = 0.f;
      if (M != -INFINITY) {
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          const float c = __expf(sm[w][D] - M);
          L += sm[w][D + 1] * c;
          Acc += sm[w][d] * c;
        }
      }
      out[d] = Acc;
      if (d == 0) *(f32x2*)ml = (f32x2){M, L};
    }
  }
  stamp(ts, 4);
}

// ---------------------------------------------------------------------------------------------
// chain neighbours
__global__ void producer(float* q, int n, float v, u64* tend) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) q[i] = v + 1e-3f * (float)(i % 97);
  if (tend && threadIdx.x == 0) tend[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}
// reads every split slab of every head (the O GEMV prologue's merge reads)
__global__ void consumer(const float* ws, int S, int HD, int NH, float* sink) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // one of HD
  if (i >= HD) return;
  float a = 0.f;
  for (int s = 0; s < S; ++s) a += ws[(long long)s * HD + i];
  const float* ml = ws + (long long)S * HD;
  for (int s = 0; s < S; ++s) a += ml[(s * NH + i / 128) * 2];
  if (a == 1234.5f) sink[0] = a;
}

struct Cfg {
  const char* name;
  int kind;  // 0 base, 1 v2
  int NW, U;
};

template <int NW, int U>
void launch_kind(int kind, dim3 grid, const AttnParams& P, u64* ts, hipStream_t s) {
  if (kind == 0) hipLaunchKernelGGL((attn_base<128, NW, U>), grid, dim3(64 * NW), 0, s, P, ts);
  else hipLaunchKernelGGL((attn_v2<128, NW, U>), grid, dim3(64 * NW), 0, s, P, ts);
}
void launch(const Cfg& c, dim3 grid, const AttnParams& P, u64* ts, hipStream_t s) {
  if (c.NW == 8 && c.U == 4) launch_kind<8, 4>(c.kind, grid, P, ts, s);
  else if (c.NW == 8 && c.U == 8) launch_kind<8, 8>(c.kind, grid, P, ts, s);
  else if (c.NW == 4 && c.U == 4) launch_kind<4, 4>(c.kind, grid, P, ts, s);
  else if (c.NW == 4 && c.U == 2) launch_kind<4, 2>(c.kind, grid, P, ts, s);
  else if (c.NW == 2 && c.U == 4) launch_kind<2, 4>(c.kind, grid, P, ts, s);
  else if (c.NW == 2 && c.U == 8) launch_kind<2, 8>(c.kind, grid, P, ts, s);
  else if (c.NW == 1 && c.U == 8) launch_kind<1, 8>(c.kind, grid, P, ts, s);
  else if (c.NW == 1 && c.U == 4) launch_kind<1, 4>(c.kind, grid, P, ts, s);
  else { fprintf(stderr, "no instantiation NW=%d U=%d\n", c.NW, c.U); exit(1); }
}

// fp64 host reference of one split's partial for head h
static void ref_partial(const std::vector<float>& q, const std::vector<uint16_t>& kc, const std::vector<uint16_t>& vc,
                        const std::vector<int>& bt, int H, int D, int bs, int h, int t0, int t1, float scale,
                        std::vector<double>& A, double& M, double& L) {
  auto h2d = [](uint16_t b) { _Float16 f; memcpy(&f, &b, 2); return (double)(float)f; };
  M = -INFINITY;
  std::vector<double> sc(t1 > t0 ? t1 - t0 : 0);
  for (int t = t0; t < t1; ++t) {
    const long long base = (((long long)bt[t / bs] * H + h) * bs + t % bs) * D;
    double s = 0;
    for (int d = 0; d < D; ++d) s += (double)(q[h * D + d] * scale) * h2d(kc[base + d]);
    sc[t - t0] = s;
    M = std::max(M, s);
  }
  A.assign(D, 0.0);
  L = 0;
  for (int t = t0; t < t1; ++t) {
    const double p = std::exp(sc[t - t0] - M);
    L += p;
    const long long base = (((long long)bt[t / bs] * H + h) * bs + t % bs) * D;
    for (int d = 0; d < D; ++d) A[d] += p * h2d(vc[base + d]);
  }
}

int main(int argc, char** argv) {
  const int H = 32, D = 128, bs = 16, NL = 32;
  const float scale = 1.f / sqrtf((float)D);
  const Cfg cfgs[] = {{"base nw8 u4", 0, 8, 4}, {"v2 nw8 u4", 1, 8, 4}, {"v2 nw8 u8", 1, 8, 8}, {"v2 nw4 u4", 1, 4, 4}};
  const int lens[] = {2048, 4000};
  const int Ss[] = {4, 8};
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  float* q;
  CK(hipMalloc(&q, H * D * 4));
  float* sink;
  CK(hipMalloc(&sink, 64));
  u64 *tsb, *tend;
  CK(hipMalloc(&tsb, 8 * 8 * 4096));
  CK(hipMalloc(&tend, 8 * 64));
  float* ws;
  CK(hipMalloc(&ws, (size_t)8 * H * (D + 2) * 4));
  int* qlen;
  CK(hipMalloc(&qlen, 4));
  for (int L : lens) {
    const int nblk = (L + bs - 1) / bs;
    const size_t per = (size_t)nblk * H * bs * D;  // halves per K (or V) cache of one layer
    const size_t layer_bytes = per * 2 * 2;
    const int copies = std::max(2, (int)((700ull << 20) / (layer_bytes * NL)) + 1);
    // one big K and V arena: [copies * NL] layers, pages shuffled within a layer's block table
    std::vector<uint16_t> hk(per), hv(per);
    unsigned rs = 12345;
    auto rnd = [&]() { rs = rs * 1664525u + 1013904223u; return ((rs >> 9) & 0xFFFF) / 65536.f - 0.5f; };
    for (size_t i = 0; i < per; ++i) {
      _Float16 a = (_Float16)rnd(), b = (_Float16)rnd();
      memcpy(&hk[i], &a, 2);
      memcpy(&hv[i], &b, 2);
    }
    std::vector<int> hbt(nblk);
    for (int i = 0; i < nblk; ++i) hbt[i] = (i * 7) % nblk;  // a permutation when gcd(7, nblk) == 1
    if (nblk % 7 == 0)
      for (int i = 0; i < nblk; ++i) hbt[i] = nblk - 1 - i;
    const int nlay = copies * NL;
    uint16_t *dk, *dv;
    CK(hipMalloc(&dk, per * 2 * nlay));
    CK(hipMalloc(&dv, per * 2 * nlay));
    for (int i = 0; i < nlay; ++i) {
      CK(hipMemcpy(dk + per * i, hk.data(), per * 2, hipMemcpyHostToDevice));
      CK(hipMemcpy(dv + per * i, hv.data(), per * 2, hipMemcpyHostToDevice));
    }
    int* dbt;
    CK(hipMalloc(&dbt, nblk * 4));
    CK(hipMemcpy(dbt, hbt.data(), nblk * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(qlen, &L, 4, hipMemcpyHostToDevice));
    std::vector<float> hq(H * D);
    for (int i = 0; i < H * D; ++i) hq[i] = 0.5f + 1e-3f * (float)(i % 97);
    for (int S : Ss) {
      if ((L + S - 1) / S > 1024 || (S == 1 && L > 512)) continue;
      AttnParams P{};
      P.q = q;
      P.ldq = H * D;
      P.block_table = dbt;
      P.max_blocks = nblk;
      P.q_len = qlen;
      P.NQ = 1;
      P.H = H;
      P.n_kv = H;
      P.D = D;
      P.Dv = D;
      P.bs = bs;
      P.scale = scale;
      P.ws = ws;
      P.n_splits = S;
      P.defer = 1;
      dim3 grid(1, H, S);
      // correctness of every config on layer 0 vs fp64
      for (const Cfg& c : cfgs) {
        P.kc = dk;
        P.vc = dv;
        hipLaunchKernelGGL(producer, dim3(H * D / 256), dim3(256), 0, st, q, H * D, 0.5f, (u64*)nullptr);
        CK(hipMemsetAsync(ws, 0, (size_t)8 * H * (D + 2) * 4, st));
        launch(c, grid, P, nullptr, st);
        CK(hipStreamSynchronize(st));
        std::vector<float> hw((size_t)S * H * D + S * H * 2);
        CK(hipMemcpy(hw.data(), ws, hw.size() * 4, hipMemcpyDeviceToHost));
        double worst = 0;
        const int chunk = (L + S - 1) / S;
        for (int sp = 0; sp < S; ++sp)
          for (int h = 0; h < H; h += 5) {
            std::vector<double> A;
            double M, Lr;
            const int t0 = sp * chunk, t1 = std::min(L, t0 + chunk);
            ref_partial(hq, hk, hv, hbt, H, D, bs, h, t0, t1, scale, A, M, Lr);
            const float gm = hw[(size_t)S * H * D + (sp * H + h) * 2], gl = hw[(size_t)S * H * D + (sp * H + h) * 2 + 1];
            if (t1 <= t0) continue;
            for (int d = 0; d < D; ++d) {
              const double got = hw[((size_t)sp * H + h) * D + d] / gl, want = A[d] / Lr;
              worst = std::max(worst, fabs(got - want));
            }
            worst = std::max(worst, fabs(gm - M));
          }
        if (worst > 2e-3) {
          printf("L=%d S=%d %s: WRONG (max err %.3e)\n", L, S, c.name, worst);
          fflush(stdout);
        }
      }
      // timing: graph of copies x NL layers, with and without attention
      auto build = [&](int ci, bool with) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < nlay; ++i) {
          hipLaunchKernelGGL(producer, dim3(H * D / 256), dim3(256), 0, st, q, H * D, 0.5f, (u64*)nullptr);
          if (with) {
            AttnParams Pl = P;
            Pl.kc = dk + per * i;
            Pl.vc = dv + per * i;
            launch(cfgs[ci], grid, Pl, nullptr, st);
          }
          hipLaunchKernelGGL(consumer, dim3((H * D + 255) / 256), dim3(256), 0, st, ws, S, H * D, H, sink);
        }
        CK(hipStreamEndCapture(st, &g));
        hipGraphExec_t e;
        CK(hipGraphInstantiate(&e, g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
        return e;
      };
      auto time_graph = [&](hipGraphExec_t e) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(e, st));
        std::vector<float> v;
        for (int r = 0; r < 9; ++r) {
          CK(hipEventRecord(a, st));
          CK(hipGraphLaunch(e, st));
          CK(hipEventRecord(b, st));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          v.push_back(ms * 1e3f / nlay);
        }
        std::sort(v.begin(), v.end());
        CK(hipEventDestroy(a));
        CK(hipEventDestroy(b));
        return v[v.size() / 2];
      };
      hipGraphExec_t g0 = build(0, false);
      const float t_none = time_graph(g0);
      CK(hipGraphExecDestroy(g0));
      printf("L=%5d S=%d (%.2f MB/layer, %d copies)  chain w/o attention %.2f us/layer\n", L, S, layer_bytes / 1e6, copies,
             t_none);
      for (int ci = 0; ci < (int)(sizeof(cfgs) / sizeof(cfgs[0])); ++ci) {
        hipGraphExec_t g1 = build(ci, true);
        const float t = time_graph(g1);
        CK(hipGraphExecDestroy(g1));
        // stamps: one chained launch, cold (a fresh copy)
        CK(hipMemset(tsb, 0, 8 * 8 * 4096));
        AttnParams Pl = P;
        Pl.kc = dk + per * (nlay - 1);
        Pl.vc = dv + per * (nlay - 1);
        hipLaunchKernelGGL(producer, dim3(H * D / 256), dim3(256), 0, st, q, H * D, 0.5f, tend);
        launch(cfgs[ci], grid, Pl, tsb, st);
        CK(hipStreamSynchronize(st));
        std::vector<u64> hts(8 * H * S), hend(H * D / 256);
        CK(hipMemcpy(hts.data(), tsb, hts.size() * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hend.data(), tend, hend.size() * 8, hipMemcpyDeviceToHost));
        const u64 pe = *std::max_element(hend.begin(), hend.end());
        double med[5];
        for (int k = 0; k < 5; ++k) {
          std::vector<double> v;
          for (int b = 0; b < H * S; ++b)
            if (hts[b * 8 + k]) v.push_back(((double)(long long)(hts[b * 8 + k] - pe)) * 0.01);
          std::sort(v.begin(), v.end());
          med[k] = v.empty() ? -1 : (k == 4 ? v.back() : v[v.size() / 2]);
        }
        printf("   %-12s %6.2f us/layer (+%5.2f)   stamps (us after producer end; median, end=max): entry %.2f  ops %.2f  kv %.2f  merged %.2f  end %.2f\n",
               cfgs[ci].name, t, t - t_none, med[0], med[1], med[2], med[3], med[4]);
        fflush(stdout);
      }
    }
    CK(hipFree(dk));
    CK(hipFree(dv));
    CK(hipFree(dbt));
  }
  return 0;
}
