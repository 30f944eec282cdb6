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
#include "gemv8_core.h"

namespace omx {

// One block = KS groups of 4 waves on the same 16-row tiles (group kg owns super-blocks
// [kg * CH, (kg + 1) * CH)); J consecutive tiles per block, every weight load issued up front.
// MS: merge slabs of IN_MERGE (1 = plain fp32 input, no merge).
// BT: batch rows (continuous batching): every weight tile is read once and dotted with BT activation
// images (row b of the LDS image at b * XSP slots); rows >= P.B are computed but never stored.
template <int QT, int NSB, int J, int KS, int IN, int MS, int EMIT, bool WT = false, int BT = 1>
__device__ __forceinline__ void gemv8_body(const GemvParams& P, const int bx) {
  static_assert(BT == 1 || MS <= 1, "batched rows take the plain fp32 input (no deferred merge)");
  constexpr int NT = GEMV_NT * KS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const QMat& w = P.w;
  const int K = w.K, N = w.N, SB = n_sb(K), XS = SB * XPAD, XSP = x8_slots_dev(K);
  i32x4* lq = (i32x4*)smem;                           // [BT][XSP]
  f32x2* lf = (f32x2*)(smem + (size_t)BT * XSP * 16);  // [BT][XSP]
  float* stage = (float*)(lf + BT * XSP);             // [BT][32]: emitted values, their squares
  float* part = stage + 32 * BT;                      // [KS - 1][BT][GEMV_NT] partial sums of the K split
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, s = lane & 15;
  const int kg = KS > 1 ? wave / GEMV_NW : 0, gtid = tid - kg * GEMV_NT;
  const int CH = KS > 1 ? (SB + KS - 1) / KS : SB;
  const int sb0 = kg * CH, se = min(SB, sb0 + CH);
  const int n_tiles = (N + 15) / 16;
  const int rbase = (wave - kg * GEMV_NW) * 4 + g;
  const int tile0 = bx * J;

  // 1. activation operands FIRST (they return ahead of the weight stream)
  u32x4 xw[BT][X8_NWI];
  f32x4 stv[BT][X8_NSTW];
  constexpr int MG = IN == IN_MERGE ? NSB * KS : 1;  // groups per thread of the merge prologue
  constexpr int MSS = MS > 0 ? MS : 1;
  constexpr int AR = BT > 1 ? BT : MSS;  // merge slabs (batch 1) or batch rows of plain fp32 input
  f32x4 av[AR][MG][4];
  f32x2 ml[MSS][MG];
  const int nwords = XSP * 3 / 2;
  const size_t img_b = (size_t)XSP * 24;
  const int st_ld = x8_stat_ld_dev(K);
  const int blast = BT > 1 ? min(P.B, BT) - 1 : 0;  // rows >= P.B re-read the last real row (never stored)
  if constexpr (IN != IN_MERGE) {
#pragma unroll
    for (int b = 0; b < BT; ++b)
#pragma unroll
      for (int i = 0; i < X8_NWI; ++i)
        xw[b][i] = ((const u32x4*)((const char*)P.x8 + min(b, blast) * img_b))[min(tid + NT * i, nwords - 1)];
    if constexpr (IN == IN_X8_RMS) {
      const int n4 = K / 64;  // f32x4 of partials (K / 16 floats)
#pragma unroll
      for (int b = 0; b < BT; ++b)
#pragma unroll
        for (int i = 0; i < X8_NSTW; ++i)
          stv[b][i] = ((const f32x4*)(P.x8_stat + min(b, blast) * st_ld))[min(lane + 64 * i, n4 - 1)];
    }
  } else {
#pragma unroll
    for (int i = 0; i < MG; ++i) {
      const int gi = min(tid + NT * i, K / 16 - 1);
      if constexpr (MS > 1) {
        const int h = 16 * gi / P.merge_D, nh = K / P.merge_D;
#pragma unroll
        for (int sp = 0; sp < MS; ++sp) {
          ml[sp][i] = *(const f32x2*)(P.merge_ml + 2 * (sp * nh + h));
#pragma unroll
          for (int j = 0; j < 4; ++j) av[sp][i][j] = *(const f32x4*)(P.x + (long long)sp * K + 16 * gi + 4 * j);
        }
      } else {
#pragma unroll
        for (int b = 0; b < BT; ++b)
#pragma unroll
          for (int j = 0; j < 4; ++j) av[b][i][j] = *(const f32x4*)(P.x + (long long)min(b, blast) * P.ldx + 16 * gi + 4 * j);
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);

  // 2. every weight tile of this block in flight (surplus slots re-read the last tile, unused)
  WTile<QT, NSB, 1> T[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int t = min(tile0 + j, n_tiles - 1);
    load_wtile<QT, NSB, 1>(w, 0, t * 16 + rbase, N, SB, sb0, s, T[j], se);
  }
  __builtin_amdgcn_sched_barrier(0);

  // 3. the activation images into LDS (the copy waits for the activation loads only); a row's image
  //    is [XSP] int8 words then [XSP] (d, d * sum q) pairs, split here into the lq / lf planes
  float rstd[BT];
#pragma unroll
  for (int b = 0; b < BT; ++b) rstd[b] = 1.f;
  if constexpr (IN != IN_MERGE) {
#pragma unroll
    for (int b = 0; b < BT; ++b)
#pragma unroll
      for (int i = 0; i < X8_NWI; ++i) {
        const int wd = tid + NT * i;
        if (wd < nwords) {
          u32x4* dst = wd < XSP ? (u32x4*)lq + b * XSP + wd : (u32x4*)(lf + b * XSP) + (wd - XSP);
          *dst = xw[b][i];
        }
      }
    if constexpr (IN == IN_X8_RMS) {
      const int n4 = K / 64;
#pragma unroll
      for (int b = 0; b < BT; ++b) {
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < X8_NSTW; ++i)
          if (lane + 64 * i < n4) ss += stv[b][i].x + stv[b][i].y + stv[b][i].z + stv[b][i].w;
        rstd[b] = rsqrtf(wave_sum(ss) / K + P.eps);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < MG; ++i) {
      const int gi = tid + NT * i;
#pragma unroll
      for (int b = 0; b < BT; ++b) {
        f32x4 xv[4];
        if constexpr (MS > 1) {  // flash-decode merge: splits without keys carry m = -inf, l = 0
          float M = -INFINITY;
#pragma unroll
          for (int sp = 0; sp < MS; ++sp) M = fmaxf(M, ml[sp][i].x);
          float L = 0.f;
          f32x4 a[4] = {};
#pragma unroll
          for (int sp = 0; sp < MS; ++sp) {
            const float c = ml[sp][i].x == -INFINITY ? 0.f : __expf(ml[sp][i].x - M);
            L += c * ml[sp][i].y;
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] += c * av[sp][i][j];
          }
          const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) xv[j] = a[j] * inv;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) xv[j] = av[b][i][j];
        }
        const int slot = b * XSP + (gi < SB * 16 ? (gi >> 4) * XPAD + (gi & 15) : XS);
        float v[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[4 * j] = xv[j].x; v[4 * j + 1] = xv[j].y; v[4 * j + 2] = xv[j].z; v[4 * j + 3] = xv[j].w;
        }
        if (16 * gi >= K) {
#pragma unroll
          for (int j = 0; j < 16; ++j) v[j] = 0.f;
        }
        float amax = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) amax = fmaxf(amax, fabsf(v[j]));
        const float d = amax / 127.f, id = amax > 0.f ? 127.f / amax : 0.f;
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
    }
    // K padding groups beyond the threads' reach stay whatever they were: every group < SB * 16 is
    // written above (NT * MG >= SB * 16 by the launch rule), the pad / dummy slots are never read
  }
  __syncthreads();

  // 4. consume the tiles in issue order; epilogue (+ emission) per tile
  const int nb = blast + 1;  // rows stored / emitted
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int t = tile0 + j;
    if (t >= n_tiles) break;  // block-uniform
    float acc[1][BT];
#pragma unroll
    for (int b = 0; b < BT; ++b) acc[0][b] = 0.f;
    compute_wtile<QT, NSB, 1, BT>(T[j], SB, sb0, s, lq, lf, XSP, acc, se);
    if constexpr (KS > 1) {  // partial sums of groups 1.. meet group 0's in LDS
      if (kg > 0) {
#pragma unroll
        for (int b = 0; b < BT; ++b) part[((kg - 1) * BT + b) * GEMV_NT + gtid] = acc[0][b];
      }
      __syncthreads();
      if (kg == 0) {
#pragma unroll
        for (int k = 1; k < KS; ++k)
#pragma unroll
          for (int b = 0; b < BT; ++b) acc[0][b] += part[((k - 1) * BT + b) * GEMV_NT + gtid];
      }
    }
#pragma unroll
    for (int b = 0; b < BT; ++b) acc[0][b] *= rstd[b];
    if constexpr (EMIT == EM_NONE) {
      if (kg == 0) finish_rows<1, BT>(P, acc, t * 16 + rbase, N, 0, s);
    } else {
      const int n = t * 16 + rbase;
      float v[BT], pv[BT];
#pragma unroll
      for (int b = 0; b < BT; ++b) {
        v[b] = row16_sum(acc[0][b]);
        pv[b] = __shfl_xor(v[b], 16, OMX_WAVE);  // row rbase ^ 1 (GLU partner)
      }
      if constexpr (EMIT == EM_ADD) {
        if (kg == 0 && s == 0) {
#pragma unroll
          for (int b = 0; b < BT; ++b) {
            float nv = 0.f;
            if (n < N && b < nb) {
              float* dst = P.y + (long long)b * P.ldy + n;
              nv = *dst + v[b] + (P.bias ? P.bias[n] : 0.f);
              *dst = nv;
            }
            stage[32 * b + rbase] = n < N ? nv * P.emit8_nw[n] : 0.f;
            stage[32 * b + 16 + rbase] = nv * nv;
          }
        }
        __syncthreads();
        if (tid < nb)
          emit_group((char*)P.emit8 + (size_t)tid * x8_slots_dev(N) * 24, N, t, stage + 32 * tid, stage + 32 * tid + 16,
                     P.emit8_stat + tid * x8_stat_ld_dev(N));
        __syncthreads();  // the stage is reused by the next tile
      } else {  // EM_GLU: even row = gate, odd = up; 8 outputs per tile, a group per tile pair
        const int half = (t & 1) * 8;
        if (kg == 0 && s == 0 && (rbase & 1) == 0) {
#pragma unroll
          for (int b = 0; b < BT; ++b) {
            const float h = n < N ? (P.epi == EPI_GEGLU ? gelu_tanh(v[b]) : silu(v[b])) * pv[b] : 0.f;
            if (n < N && b < nb) P.y[(long long)b * P.ldy + (n >> 1)] = h;
            stage[32 * b + half + (rbase >> 1)] = h;
            if (half == 0 && t + 1 >= n_tiles) stage[32 * b + 8 + (rbase >> 1)] = 0.f;  // trailing half group
          }
        }
        if ((t & 1) || t + 1 >= n_tiles) {
          __syncthreads();
          if (tid < nb)
            emit_group<WT>((char*)P.emit8 + (size_t)tid * x8_slots_dev(N / 2) * 24, N / 2, t >> 1, stage + 32 * tid,
                           nullptr, nullptr);
          __syncthreads();
        }
      }
    }
    if constexpr (KS > 1) __syncthreads();  // part is reused by the next tile
  }
}

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
    if (G.nsb == 2 && G.J > 1) return false;
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
  if (in == IN_MERGE && (P.w.K > 4096 * 1 || P.w.K % 16)) return false;  // merge prologue: one group per thread
  if (in == IN_X8_RMS && (P.w.K > 8192 || P.w.K % 64)) return false;
  if (em == EM_ADD && (!P.emit8_nw || !P.emit8_stat || P.w.N % 16)) return false;
  if (em == EM_GLU && P.w.N % 32) return false;
  const int q = P.w.qtype;
  if (!(q == QT_Q4_K || q == QT_Q6_K || q == QT_Q4_0 || q == QT_Q8_0 || q == QT_Q5_K)) return false;
  if (!geometry(P, G)) return false;
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
  else if constexpr (NSB == 1 && KS == 1 && J == 1) {  // the O projection: merge slabs or plain fp32
    switch (P.merge_S) {
      case 2: launch_em<QT, 1, 1, 1, IN_MERGE, 2>(P, em, G.grid, s); break;
      case 4: launch_em<QT, 1, 1, 1, IN_MERGE, 4>(P, em, G.grid, s); break;
      case 8: launch_em<QT, 1, 1, 1, IN_MERGE, 8>(P, em, G.grid, s); break;
      default: launch_em<QT, 1, 1, 1, IN_MERGE, 1>(P, em, G.grid, s); break;
    }
  }
}

template <int QT>
void launch_q(const GemvParams& P, const Geo& G, hipStream_t s) {
  if (G.ks == 1 && G.nsb == 1 && G.J == 1) launch_in<QT, 1, 1, 1>(P, G, s);
  else if (G.ks == 1 && G.nsb == 1) launch_in<QT, 1, 2, 1>(P, G, s);
  else if (G.ks == 1 && G.nsb == 2) launch_in<QT, 2, 1, 1>(P, G, s);
  else if (G.ks == 2) launch_in<QT, 1, 1, 2>(P, G, s);
  else if (G.ks == 3) launch_in<QT, 1, 1, 3>(P, G, s);
  else launch_in<QT, 1, 1, 4>(P, G, s);
}

bool launchable(const GemvParams& P, const Geo& G) {
  // the merge / plain-fp32 input exists for the single-tile, unsplit geometry only
  return in_mode(P) != IN_MERGE || (G.ks == 1 && G.nsb == 1 && G.J == 1);
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
  switch (A.w.qtype) {
    case QT_Q4_K: return dual_b<QT_Q4_K>(A, B, gxa, gxb, s);
    case QT_Q5_K: return dual_b<QT_Q5_K>(A, B, gxa, gxb, s);
    case QT_Q4_0: return dual_b<QT_Q4_0>(A, B, gxa, gxb, s);
    default: return false;
  }
}

}  // namespace omx
