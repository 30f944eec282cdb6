// Wave-specialised batch-1 decode GEMV: loader waves stream the weights straight into LDS
// (global_load_lds_dwordx4, no VGPRs), compute waves dot them against the staged activations.
//
// Why (profiles/r3_gemv, scripts/gemv_timeline.py): a CU's vector-memory queue is shallow next to a
// decode GEMV's per-CU share (gate_up: 198 KB per CU). In the all-in-flight kernel (gemv.hip flight)
// every wave first issues all of its weight loads, and a wave cannot issue past a full queue -- so a
// wave's first instruction after its loads (the activation prologue, then the dot products) starts
// only when the CU's stream has nearly drained. Even with the activations loaded and drained BEFORE
// any weight request (the x-barrier variant) the prologue ended at 9.3 us of a 12.7 us gate_up: the
// waves were stuck issuing. Every dot product then ran after the stream: a 1.2 us (Q4_K) to 3.2 us
// (Q6_K down) compute tail per launch, plus the late activations.
//
// Here the block is NC compute waves + NC loader waves, one block per CU. Loader l owns a ring of S
// LDS slots for compute wave l; a slot holds one unit = the exact register tile a flight wave would
// load (4 rows x 16 super-blocks, every stream of the quant layout), written by the DMA at
// [load][lane] so compute lane i reads its own 16 bytes back with one ds_read_b128. Loaders stall on
// the full queue; compute waves never touch the vector-memory queue after their prologue (their
// activations and every epilogue operand are requested before the loaders start, x-first), so they
// consume each unit as it lands and the compute overlaps the stream.
// Handshake (LDS): ready[c][slot] = unit + 1 after the loader's counted vmcnt wait; freed[c][slot] =
// unit + 1 once compute wave c holds the unit in registers. Every spin is bounded (s_memrealtime):
// a lost wave cannot hang the GPU, it produces a wrong result instead.
#include "gemv_core.h"

namespace omx {

constexpr int WS_NC = 4;                     // compute waves (one per SIMD)
constexpr int WS_NT = 64 * 2 * WS_NC;        // + one loader wave per compute wave
constexpr int WS_MAX_PRE = 16;               // row tiles per compute wave (epilogue operands preloaded per lane)

typedef __attribute__((address_space(3))) void* lds_ptr;

// unit layout in LDS: L16 loads of 16 B per lane (1 KB each), then L4 loads of 4 B (256 B each)
template <int QT>
struct WsLayout {
  static constexpr int L16 = QT == QT_Q8_0 ? 17 : 9;
  static constexpr int L4 = QT == QT_Q6_K ? 17 : QT == QT_Q5_K ? 8 : 0;
  static constexpr int BYTES = 1024 * L16 + 256 * L4;
  static constexpr int LOADS = L16 + L4;
};

__device__ __forceinline__ void dma16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_ptr)lds, 16, 0, 0);
}
__device__ __forceinline__ void dma4(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_ptr)lds, 4, 0, 0);
}

// the loads of load_wtile<QT, 1, 1> for (row, super-block sb), into the slot at `u` (wave-uniform)
template <int QT>
__device__ __forceinline__ void dma_unit(const QMat& w, long long row, long long SB, long long sb, char* u) {
  constexpr int L16 = WsLayout<QT>::L16;
  if constexpr (QT == QT_Q8_0) {
    const uint8_t* q = w.s0 + row * SB * 256 + 32 * sb;
    dma16(w.s1 + row * SB * 16 + 16 * sb, u);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      dma16(q + 32LL * t * SB, u + 1024 * (1 + 2 * t));
      dma16(q + 32LL * t * SB + 16, u + 1024 * (2 + 2 * t));
    }
  } else if constexpr (QT == QT_Q6_K) {
    const uint8_t* q = w.s0 + row * SB * 128 + 16 * sb;
    const uint8_t* hq = w.s1 + row * SB * 64 + 8 * sb;
    dma16(w.s2 + row * SB * 16 + 16 * sb, u);
#pragma unroll
    for (int t = 0; t < 8; ++t) dma16(q + 16LL * t * SB, u + 1024 * (1 + t));
    char* u4 = u + 1024 * L16;
    dma4(w.s3 + ((row * SB * 2 + 2 * sb) & ~3LL), u4);  // fp16 d inside its aligned dword
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      dma4(hq + 8LL * t * SB, u4 + 256 * (1 + 2 * t));
      dma4(hq + 8LL * t * SB + 4, u4 + 256 * (2 + 2 * t));
    }
  } else if constexpr (QT == QT_Q5_K) {
    const uint8_t* q = w.s0 + row * SB * 128 + 16 * sb;
    const uint8_t* hq = w.s2 + row * SB * 32 + 4 * sb;
    dma16(w.s1 + row * SB * 16 + 16 * sb, u);
#pragma unroll
    for (int t = 0; t < 8; ++t) dma16(q + 16LL * t * SB, u + 1024 * (1 + t));
    char* u4 = u + 1024 * L16;
#pragma unroll
    for (int t = 0; t < 8; ++t) dma4(hq + 4LL * t * SB, u4 + 256 * t);
  } else {  // Q4_K, Q4_0
    const uint8_t* q = w.s0 + row * SB * 128 + 16 * sb;
    dma16(w.s1 + row * SB * 16 + 16 * sb, u);
#pragma unroll
    for (int t = 0; t < 8; ++t) dma16(q + 16LL * t * SB, u + 1024 * (1 + t));
  }
}

// unit -> the register tile the flight kernel would hold (lane-private 16 / 4 byte records)
template <int QT>
__device__ __forceinline__ void read_unit(const char* u, int lane, long long row, long long SB, long long sb,
                                          WTile<QT, 1, 1>& T) {
  constexpr int L16 = WsLayout<QT>::L16;
  const u32x4* v = (const u32x4*)u + lane;
  T.m[0][0] = v[0];
  if constexpr (QT == QT_Q8_0) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      T.a[0][0][t] = v[64 * (1 + 2 * t)];
      T.b[0][0][t] = v[64 * (2 + 2 * t)];
    }
  } else {
#pragma unroll
    for (int t = 0; t < 8; ++t) T.a[0][0][t] = v[64 * (1 + t)];
  }
  const unsigned* v4 = (const unsigned*)(u + 1024 * L16) + lane;
  if constexpr (QT == QT_Q6_K) {
    const unsigned dw = v4[0];
    T.d[0][0] = ((row * SB * 2 + 2 * sb) & 2) ? (dw >> 16) : (dw & 0xFFFF);
#pragma unroll
    for (int t = 0; t < 8; ++t) T.h[0][0][t] = (u32x2){v4[64 * (1 + 2 * t)], v4[64 * (2 + 2 * t)]};
  } else if constexpr (QT == QT_Q5_K) {
#pragma unroll
    for (int t = 0; t < 8; ++t) T.q5h[0][0][t] = v4[64 * t];
  }
}

// LDS flag handshake. Relaxed atomics plus compiler barriers, not acquire / release: a release
// would make the loader drain every DMA in flight (vmcnt(0)) before each signal. Ordering comes
// from the explicit counted waits: the loader signals after its vmcnt wait for the unit, the
// compute wave frees a slot after its lgkmcnt(0); LDS executes one wave's operations in order.
__device__ __forceinline__ bool lds_wait_geq(int* p, int want) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool ok = true;
  while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < want) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) { ok = false; break; }  // 200 ms: a lost wave
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
  return ok;
}
__device__ __forceinline__ void lds_set(int* p, int v) {
  asm volatile("" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// s_waitcnt vmcnt(N) (gfx9 encoding: vmcnt[3:0] + vmcnt[5:4] at bits 15:14, expcnt / lgkmcnt at max)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  constexpr int n = N > 63 ? 63 : N;
  __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8));
  asm volatile("" ::: "memory");
}

// per-row epilogue operands preloaded with the activations (the compute waves issue no global load
// once the loaders run: it would queue behind the weight stream)
struct WsPre {
  float y, b, bp, fq;
};

__device__ __forceinline__ void ws_epi(const GemvParams& P, int vn, float v, float pv, const WsPre& e, int pos,
                                       int slot) {
  switch (P.epi) {
    case EPI_STORE: P.y[vn] = v + e.b; break;
    case EPI_ADD: P.y[vn] = e.y + v + e.b; break;
    case EPI_GELU: P.y[vn] = gelu_tanh(v + e.b); break;
    case EPI_GLU:
      if ((vn & 1) == 0) P.y[vn / 2] = silu(v) * pv;
      break;
    case EPI_GEGLU:
      if ((vn & 1) == 0) P.y[vn / 2] = gelu_tanh(v) * pv;
      break;
    case EPI_QKV: {
      const int Eq = P.Eq, Ekv = P.Ekv, D = P.D;
      int which, hh, d;
      if (vn < Eq) { which = 0; hh = vn / D; d = vn % D; }
      else if (vn < Eq + Ekv) { which = 1; hh = (vn - Eq) / D; d = (vn - Eq) % D; }
      else { which = 2; hh = (vn - Eq - Ekv) / D; d = (vn - Eq - Ekv) % D; }
      v += e.b;
      float out = v;
      if (which < 2 && d < P.n_rot) {
        pv += e.bp;
        float sn, cs;
        sincosf((float)pos * e.fq, &sn, &cs);
        out = (d & 1) ? (pv * sn + v * cs) : (v * cs - pv * sn);
      }
      if (which == 0) {
        P.y[vn] = out;
      } else {
        const long long blk = slot / P.bs, off = slot % P.bs;
        const long long idx = ((blk * P.n_kv + hh) * P.bs + off) * D + d;
        if (which == 1) ((f16*)P.kc)[idx] = (f16)out;
        else ((f16*)P.vc)[idx] = (f16)out;
      }
      break;
    }
  }
}

// Side A (QA rows [0, PA.w.N)) and optionally side B (QB, same K and activations; nB = 0: none) over
// one combined space of 4-row tiles; NXG = activation groups per compute thread = K chunks of 4096.
// DBG (scripts/bench_gemv.py OMX_BENCH_DEBUG, microbenchmark only): 1 = compute waves skip the dot
// products (the DMA pipeline alone), 2 = loaders skip the DMA (the compute waves alone)
template <int QA, int QB, int NXG, int NRM, int DBG = 0>
__global__ __launch_bounds__(WS_NT) void qgemv_ws_kernel(GemvParams PA, GemvParams PB, int has_b) {
  constexpr int UBA = WsLayout<QA>::BYTES, UBB = WsLayout<QB>::BYTES;
  constexpr int UB = UBA > UBB ? UBA : UBB;
  constexpr int S = UB > 10240 ? 2 : 3;  // ring slots per compute wave (LDS: NC * S * UB <= 139 KB)
  constexpr int LA = WsLayout<QA>::LOADS, LB = WsLayout<QB>::LOADS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int K = PA.w.K, SB = n_sb(K), XS = SB * XPAD;
  const int nc = (SB + 15) / 16;
  const int RTA = (PA.w.N + 3) / 4, RT = RTA + (has_b ? (PB.w.N + 3) / 4 : 0);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, s = lane & 15;
  const bool loader = wave >= WS_NC;
  const int c = loader ? wave - WS_NC : wave;
  char* ring = smem + (size_t)c * S * UB;
  i32x4* lq = (i32x4*)(smem + (size_t)WS_NC * S * UB);  // [XS + 1] (slot XS: dummy)
  f32x2* lf = (f32x2*)(lq + XS + 1);
  float* red = (float*)(lf + XS + 1);                     // [NC][2]
  int* ready = (int*)(red + 2 * WS_NC);                   // [NC][S]
  int* freed = ready + WS_NC * S;                         // [NC][S]
  int* cnt = freed + WS_NC * S;                           // [2] compute-wave rendezvous
  // this wave pair's 4-row tiles: first_rt + i * stride
  const int first_rt = blockIdx.x * WS_NC + c, stride = gridDim.x * WS_NC;
  const int n_rt = first_rt < RT ? (RT - first_rt + stride - 1) / stride : 0;
  const int n_units = n_rt * nc;
  auto side_of = [&](int rt) { return rt >= RTA; };

  if (loader) {
    __builtin_amdgcn_s_barrier();  // the compute waves' activation requests are queued first
    for (int k = 0; k < n_units; ++k) {
      const int slot = k % S;
      if (k >= S && !lds_wait_geq(&freed[c * S + slot], k - S + 1)) break;
      const int i = k / nc, chunk = k - i * nc, rt = first_rt + i * stride;
      const long long sb = min(chunk * 16 + s, SB - 1);
      if constexpr ((DBG & 2) == 0) {
        if (!side_of(rt)) dma_unit<QA>(PA.w, min(rt * 4 + g, PA.w.N - 1), SB, sb, ring + slot * UB);
        else dma_unit<QB>(PB.w, min((rt - RTA) * 4 + g, PB.w.N - 1), SB, sb, ring + slot * UB);
      }
      if (k >= S - 1) {
        // unit k - S + 1 landed once at most the loads of the S - 1 younger units are outstanding; a
        // side-B unit among them has LB loads, so wait for the smaller count (conservative)
        wait_vmcnt<(S - 1) * (LA < LB ? LA : LB)>();
        if (lane == 0) lds_set(&ready[c * S + (k - S + 1) % S], k - S + 2);
      }
    }
    wait_vmcnt<0>();
    if (lane == 0)
      for (int k = n_units - S + 1 > 0 ? n_units - S + 1 : 0; k < n_units; ++k) lds_set(&ready[c * S + k % S], k + 1);
    return;
  }

  // ---- compute waves: activations + epilogue operands first, then the loaders may start
  const int tid = threadIdx.x;  // 0 .. 64 * NC - 1
  constexpr int NTC = 64 * WS_NC;
  constexpr bool nrm = NRM != 0, lnb = NRM == 2;
  f32x4 xv[NXG][4], nw[NXG][4], nb[NXG][4];
#pragma unroll
  for (int i = 0; i < NXG; ++i) {
    const int gi = min(tid + NTC * i, K / 16 - 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      xv[i][j] = *(const f32x4*)(PA.x + 16 * gi + 4 * j);
      if constexpr (nrm) nw[i][j] = *(const f32x4*)(PA.norm_w + 16 * gi + 4 * j);
      if constexpr (lnb) nb[i][j] = *(const f32x4*)(PA.norm_b + 16 * gi + 4 * j);
    }
  }
  // lane (4 i + g) holds the operands of row g of this wave's i-th tile. Branch-free: every lane
  // loads from a valid address (x when the operand is unused) and flags what it loaded; a divergent
  // branch around the loads makes the compiler drain them before the loaders may start.
  WsPre pre;
  int pfl = 0;
  {
    const int i = lane >> 2, rt = first_rt + i * stride;
    const bool in = i < n_rt, sbs = rt >= RTA;  // n_rt <= WS_MAX_PRE (ws_launch_n)
    const int n = min((sbs ? rt - RTA : rt) * 4 + (lane & 3), (sbs ? PB.w.N : PA.w.N) - 1);
    const int vn = n + (sbs ? PB.row_offset : PA.row_offset);
    const float* yb = PA.y;
    const float* bb = PA.bias;
    const int epi = PA.epi;
    int d = -1;
    if (epi == EPI_QKV) d = vn < PA.Eq ? vn % PA.D : vn < PA.Eq + PA.Ekv ? (vn - PA.Eq) % PA.D : -1;
    const bool uy = in && epi == EPI_ADD, ub = in && bb && epi != EPI_GLU && epi != EPI_GEGLU;
    const bool rope = in && epi == EPI_QKV && d >= 0 && d < PA.n_rot, ubp = rope && bb;
    const float* dummy = PA.x;
    pre.y = *(uy ? yb + vn : dummy);
    pre.b = *(ub ? bb + vn : dummy);
    pre.bp = *(ubp ? bb + (vn ^ 1) : dummy);
    pre.fq = *(rope ? PA.inv_freq + (d >> 1) : dummy);
    pfl = (uy ? 1 : 0) | (ub ? 2 : 0) | (ubp ? 4 : 0) | (rope ? 8 : 0);
  }
  const bool qkv = PA.epi == EPI_QKV;
  const int pos_raw = *(qkv ? PA.pos : (const int*)PA.x), slot_raw = *(qkv ? PA.slot : (const int*)PA.x);
  asm volatile("" ::: "memory");  // every activation / operand load issued before the loaders start
  if (tid < WS_NC * S) { ready[tid] = 0; freed[tid] = 0; }
  if (tid < 2) cnt[tid] = 0;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);  // no use of a loaded value may move above the barrier
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

#pragma unroll
  for (int i = 0; i < NXG; ++i) {
    const bool ok = 16 * (tid + NTC * i) < K;
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
    sm = wave_sum(sm);
    ss = wave_sum(ss);
    if (lane == 0) {
      red[2 * c] = sm;
      red[2 * c + 1] = ss;
      __hip_atomic_fetch_add(&cnt[0], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    lds_wait_geq(&cnt[0], WS_NC);
    sm = 0.f;
    ss = 0.f;
#pragma unroll
    for (int w = 0; w < WS_NC; ++w) {
      sm += red[2 * w];
      ss += red[2 * w + 1];
    }
    if (NRM == 2 || PA.norm == NORM_LAYER) {
      mean = sm / K;
      rstd = rsqrtf(fmaxf(ss / K - mean * mean, 0.f) + PA.eps);
    } else {
      rstd = rsqrtf(ss / K + PA.eps);
    }
  }
#pragma unroll
  for (int i = 0; i < NXG; ++i) {
    const int gi = tid + NTC * i;
    const int slot = gi < SB * 16 ? (gi >> 4) * XPAD + (gi & 15) : XS;
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
  if (lane == 0) __hip_atomic_fetch_add(&cnt[1], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  lds_wait_geq(&cnt[1], WS_NC);
  // the operand preloads returned right behind the activations (issued before any weight request);
  // collect them here so no wait inside the loop has to count them (it would then also count the
  // epilogue stores queued behind the weight stream)
  wait_vmcnt<0>();

  // ---- consume the units as they land
  float acc[1][1] = {{0.f}};
  for (int j = 0; j < n_units; ++j) {
    const int slot = j % S;
    if (!lds_wait_geq(&ready[c * S + slot], j + 1)) break;
    const int i = j / nc, chunk = j - i * nc, rt = first_rt + i * stride;
    const bool sb_side = side_of(rt);
    const int n = sb_side ? (rt - RTA) * 4 + g : rt * 4 + g;
    const int Ns = sb_side ? PB.w.N : PA.w.N, roff = sb_side ? PB.row_offset : PA.row_offset;
    const long long sb = min(chunk * 16 + s, SB - 1);
    const char* u = ring + slot * UB;
    if (!sb_side) {
      WTile<QA, 1, 1> T;
      read_unit<QA>(u, lane, min(n, PA.w.N - 1), SB, sb, T);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) lds_set(&freed[c * S + slot], j + 1);
      if constexpr (DBG & 1) acc[0][0] += (float)((T.a[0][0][0].x ^ T.a[0][0][7].w ^ T.m[0][0].y) & 1);
      else compute_wtile<QA, 1, 1, 1>(T, SB, chunk * 16, s, lq, lf, XS, acc);
    } else {
      WTile<QB, 1, 1> T;
      read_unit<QB>(u, lane, min(n, PB.w.N - 1), SB, sb, T);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) lds_set(&freed[c * S + slot], j + 1);
      if constexpr (DBG & 1) acc[0][0] += (float)((T.a[0][0][0].x ^ T.a[0][0][7].w ^ T.m[0][0].y) & 1);
      else compute_wtile<QB, 1, 1, 1>(T, SB, chunk * 16, s, lq, lf, XS, acc);
    }
    if (chunk == nc - 1) {
      float v = row16_sum(acc[0][0]);
      const float pv = __shfl_xor(v, 16, OMX_WAVE);  // pair partner: row n ^ 1 (group g ^ 1)
      const int src = 4 * i + g, fl = __shfl(pfl, src, OMX_WAVE);
      WsPre e;
      e.y = (fl & 1) ? __shfl(pre.y, src, OMX_WAVE) : 0.f;
      e.b = (fl & 2) ? __shfl(pre.b, src, OMX_WAVE) : 0.f;
      e.bp = (fl & 4) ? __shfl(pre.bp, src, OMX_WAVE) : 0.f;
      e.fq = (fl & 8) ? __shfl(pre.fq, src, OMX_WAVE) : 0.f;
      if (s == 0 && n < Ns) ws_epi(PA, n + roff, v, pv, e, qkv ? pos_raw : 0, qkv ? slot_raw : 0);
      acc[0][0] = 0.f;
    }
  }
}

template <int QA, int QB, int NXG>
static bool ws_launch_n(const GemvParams& A, const GemvParams& B, int has_b, hipStream_t s) {
  constexpr int UBA = WsLayout<QA>::BYTES, UBB = WsLayout<QB>::BYTES;
  constexpr int UB = UBA > UBB ? UBA : UBB;
  constexpr int S = UB > 10240 ? 2 : 3;
  const int SB = (A.w.K + 255) / 256, XS = SB * XPAD;
  const size_t lds = (size_t)WS_NC * S * UB + (size_t)(XS + 1) * 24 + 4 * 2 * WS_NC + 4 * (2 * WS_NC * S + 2);
  if (lds > 160 * 1024) return false;
  const int RT = (A.w.N + 3) / 4 + (has_b ? (B.w.N + 3) / 4 : 0);
  int ncu = 0, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    ncu = 256;
  const int gx = min(ncu, (RT + WS_NC - 1) / WS_NC);
  // every row tile of a compute wave has its epilogue operands preloaded (no global load may issue
  // inside the loop: it would queue behind the weight stream)
  if ((RT + gx * WS_NC - 1) / (gx * WS_NC) > WS_MAX_PRE) return false;
  const int nrm = A.norm == NORM_NONE ? 0 : (A.norm == NORM_LAYER && A.norm_b) ? 2 : 1;
  auto go = [&](auto kern) {
    static bool attr = false;  // one attribute call per instantiation (> 64 KB dynamic LDS)
    if (!attr) {
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    hipLaunchKernelGGL(kern, dim3(gx), dim3(WS_NT), lds, s, A, B, has_b);
  };
  if constexpr (QA == QB) {  // microbenchmark-only variants
    if (g_tune.debug == 1 && nrm == 0) { go(qgemv_ws_kernel<QA, QB, NXG, 0, 1>); return true; }
    if (g_tune.debug == 2 && nrm == 0) { go(qgemv_ws_kernel<QA, QB, NXG, 0, 2>); return true; }
    if (g_tune.debug == 1 && nrm == 1) { go(qgemv_ws_kernel<QA, QB, NXG, 1, 1>); return true; }
    if (g_tune.debug == 2 && nrm == 1) { go(qgemv_ws_kernel<QA, QB, NXG, 1, 2>); return true; }
  }
  if (nrm == 0) go(qgemv_ws_kernel<QA, QB, NXG, 0>);
  else if (nrm == 1) go(qgemv_ws_kernel<QA, QB, NXG, 1>);
  else go(qgemv_ws_kernel<QA, QB, NXG, 2>);
  return true;
}

template <int QA, int QB>
static bool ws_launch(const GemvParams& A, const GemvParams& B, int has_b, hipStream_t s) {
  switch (((A.w.K + 255) / 256 + 15) / 16) {
    case 1: return ws_launch_n<QA, QB, 1>(A, B, has_b, s);
    case 2: return ws_launch_n<QA, QB, 2>(A, B, has_b, s);
    case 3: return ws_launch_n<QA, QB, 3>(A, B, has_b, s);
    default: return false;
  }
}

static bool ws_eligible(const GemvParams& P) {
  const int q = P.w.qtype;
  if (g_tune.debug && g_tune.debug != 1 && g_tune.debug != 2) return false;
  return P.B == 1 && !P.expert_ids && !P.merge_S && !P.dbg_ts && !P.w.s4 &&
         (q == QT_Q4_K || q == QT_Q6_K || q == QT_Q4_0 || q == QT_Q8_0 || q == QT_Q5_K) &&
         ((P.w.K + 255) / 256 + 15) / 16 <= 3;
}

bool gemv_ws(const GemvParams& P, hipStream_t s) {
  if (!g_tune.ws || !ws_eligible(P)) return false;
  switch (P.w.qtype) {
    case QT_Q4_K: return ws_launch<QT_Q4_K, QT_Q4_K>(P, P, 0, s);
    case QT_Q6_K: return ws_launch<QT_Q6_K, QT_Q6_K>(P, P, 0, s);
    case QT_Q4_0: return ws_launch<QT_Q4_0, QT_Q4_0>(P, P, 0, s);
    case QT_Q8_0: return ws_launch<QT_Q8_0, QT_Q8_0>(P, P, 0, s);
    case QT_Q5_K: return ws_launch<QT_Q5_K, QT_Q5_K>(P, P, 0, s);
    default: return false;
  }
}

// the Q4_K_M / Q5_K_M QKV: q,k rows (Q4_K / Q5_K) + v rows (Q6_K) over the same activations
bool gemv_ws2(const GemvParams& A, const GemvParams& B, hipStream_t s) {
  // one epilogue parameter set serves both sides (kernel: PA's fields, per-side N / row_offset)
  if (!g_tune.ws || !ws_eligible(A) || !ws_eligible(B) || A.w.K != B.w.K || A.x != B.x || A.norm != B.norm ||
      A.norm_w != B.norm_w || A.epi != B.epi || A.y != B.y || A.bias != B.bias || A.kc != B.kc || A.vc != B.vc)
    return false;
  if (B.w.qtype != QT_Q6_K) return false;
  if (A.w.qtype == QT_Q4_K) return ws_launch<QT_Q4_K, QT_Q6_K>(A, B, 1, s);
  if (A.w.qtype == QT_Q5_K) return ws_launch<QT_Q5_K, QT_Q6_K>(A, B, 1, s);
  return false;
}

}  // namespace omx
