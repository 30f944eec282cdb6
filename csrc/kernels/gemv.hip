#include <atomic>
// Fused quantized GEMV for decode and small batches (M = B <= a few rows) on gfx950.
//
// y[b, n] = epilogue( sum_k W[n, k] * norm(x[b, :])[k] )
//
// Design (MI355X-first, see SURVEY.md §7.4 hard part 1 and docs/kernels.md):
//  * Weights use repack layout v2 (ollama_operator_amd/quant.py "device repack"): K padded to SB
//    super-blocks of 256, codes stored piece-major across super-blocks -- qs[row][t][sb][16 B].
//  * Lane mapping: a wave = 4 row groups of 16 lanes; lane s of a group owns super-blocks
//    s, s+16, ... (NSB of them per K chunk) of R rows and walks all 8 pieces t of each. One load
//    instruction for piece t therefore reads a contiguous 256 B run per row group, and t is a
//    compile-time constant: the K-quant scales / mins are decoded once per 256 weights, with
//    constant byte selects (v_cvt_f32_ubyteN), instead of once per 32-weight piece. The previous
//    lane-per-piece kernel spent ~95 VALU ops per piece-row (rocprofv3 PMC, profiles/r1_pmc):
//    VALU-bound next to an 8 us HBM floor. This one spends ~30.
//  * 4-bit codes keep the high nibble signed (byte ^ 0x80 at repack), so `q & 0xF0F0F0F0` feeds
//    v_dot4_i32_i8 directly (16 * (n - 8)): 2 VALU per dword to unpack both nibbles.
//  * Activation prologue once per block: x (fp32) optionally RMS/Layer-normalised (fused), int8-
//    quantised per 16-element group (fp32 scale + group sum for the K-quant mins / zero points),
//    staged in LDS with one pad slot per super-block (17 slots) so the 16 lanes of a group -- one
//    super-block apart -- hit distinct banks.
//  * Weight loads for the first tile are issued before the prologue; persistent blocks prefetch the
//    next (tile, K chunk) unit into a second register tile when the tile fits (DB), else rely on
//    other waves for latency hiding.
//  * Row sums: 16-lane DPP reduction (quad_perm / row_half_mirror / row_mirror), no LDS.
//  * Epilogues fused: residual add (+ MoE routing weight, atomics for top-k > 1), bias, SiLU-GLU
//    (gate/up rows interleaved at load), GELU, and QKV (RoPE on adjacent row pairs + fp16 paged KV
//    scatter). Pair partners come from the same lane (R = 2) or the neighbouring row group (R = 1).
// Reference parity: the reference delegates all of this to llama.cpp inside `ollama/ollama`
// (reference pkg/model/pod.go:10-12); numerics are checked against quant.py + an fp32 torch GEMV.
#include "gemv_core.h"

#include <stdexcept>

namespace omx {



GemvTuning g_tune;
void set_gemv_tuning(int blocks_per_cu, int rows, int debug, int ks, int xfirst, int xbar, int stream,
                     int stream_bpc, int pf, int ws) {
  g_tune.debug = debug > 0 ? debug : 0;
  (void)pf;  // cross-launch L2 prefetch: measured slower (profiles/r3_gemv), removed
  (void)stream;  // the streaming / wave-specialised variants live in experiments/kernels (slower, unbuilt)
  (void)stream_bpc;
  (void)ws;
  if (xfirst == 0 || xfirst == 1) g_tune.xfirst = xfirst;
  if (xbar == 0 || xbar == 1) g_tune.xbar = xbar;
  if (ks >= 0 && ks <= 4) g_tune.ks = ks;
  if (blocks_per_cu > 0) g_tune.blocks_per_cu = blocks_per_cu;
  if (rows == 1 || rows == 2) g_tune.rows = rows;
}


// ---------------------------------------------------------------------------------------------
// Block = GEMV_NW waves x 4 row groups x R rows per tile. Work unit = (tile, K chunk of
// 16*NSB super-blocks); blocks are persistent over units (tile += gridDim.x).
// DBG (microbenchmark only, scripts/bench_gemv.py): bit 0 = replace the dot products by an XOR of
// the loaded words (memory path alone), bit 1 = skip the activation prologue
template <int QT, int NSB, int R, int BT, int DBG = 0>
__global__ __launch_bounds__(GEMV_NT) void qgemv_kernel(GemvParams P) {
  constexpr int PB = (QT == QT_Q8_0 || QT == QT_Q6_K8) ? 8 : QT == QT_Q6_K ? 6 : QT == QT_Q5_K ? 5 : 4;  // VGPRs per piece
  constexpr bool DB = R * NSB * (8 * PB + 5) <= 80;               // room for a prefetch tile
  constexpr int ROWS_W = 4 * R, ROWS_B = GEMV_NW * ROWS_W;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const QMat& w = P.w;
  const int K = w.K, N = w.N, SB = n_sb(K);
  const int XS = SB * XPAD;
  i32x4* lq = (i32x4*)smem;                         // [BT][XS]
  f32x2* lf = (f32x2*)(smem + (size_t)BT * XS * 16);  // [BT][XS]
  float* red = (float*)(lf + BT * XS);              // [NT/64]
  const int b0 = blockIdx.y * BT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, s = lane & 15;
  const int nc = (SB + 16 * NSB - 1) / (16 * NSB);
  const int n_tiles = (N + ROWS_B - 1) / ROWS_B;
  const int rbase = wave * ROWS_W + g * R;

  long long row_base = 0;
  const float* x = P.x;
  if (P.expert_ids) {  // MoE: blockIdx.z = k-th selected expert of batch row b0
    const int e = P.expert_ids[b0 * P.n_sel + blockIdx.z];
    row_base = (long long)e * N;
    if (P.x_per_sel) x = P.x + (long long)blockIdx.z * P.x_sel_stride;
  }

  int tile = blockIdx.x, c = 0;
  WTile<QT, NSB, R> A;
  if (tile < n_tiles) load_wtile<QT, NSB, R>(w, row_base, tile * ROWS_B + rbase, N, SB, 0, s, A);

#pragma unroll
  for (int b = 0; b < BT; ++b) {
    if (DBG & 2) break;
    if (b0 + b < P.B) {
      stage_x<GEMV_NT>(P, x + (long long)(b0 + b) * P.ldx, K, SB, lq + b * XS, lf + b * XS, red);
    } else {
      for (int i = threadIdx.x; i < XS; i += GEMV_NT) {
        lq[b * XS + i] = (i32x4){0, 0, 0, 0};
        lf[b * XS + i] = (f32x2){0.f, 0.f};
      }
    }
  }
  __syncthreads();

  float acc[R][BT];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int b = 0; b < BT; ++b) acc[r][b] = 0.f;
  auto finish = [&](int t) {
    finish_rows<R, BT>(P, acc, t * ROWS_B + rbase, N, b0, s);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int b = 0; b < BT; ++b) acc[r][b] = 0.f;
  };

  if constexpr (DB) {
    // explicit ping-pong (a register copy would force a vmcnt(0) drain every unit)
    WTile<QT, NSB, R> Bt;
    auto step = [&](WTile<QT, NSB, R>& cur, WTile<QT, NSB, R>& nxt) {
      int nt = tile, ncc = c + 1;
      if (ncc == nc) { ncc = 0; nt += gridDim.x; }
      if (nt < n_tiles) load_wtile<QT, NSB, R>(w, row_base, nt * ROWS_B + rbase, N, SB, ncc * 16 * NSB, s, nxt);
      if constexpr (DBG & 1) {
        unsigned v = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) v ^= cur.a[0][0][t].x ^ cur.a[0][0][t].w;
        acc[0][0] += (float)(v & 1);
      } else {
        compute_wtile<QT, NSB, R, BT>(cur, SB, c * 16 * NSB, s, lq, lf, XS, acc);
      }
      if (c == nc - 1) finish(tile);
      tile = nt;
      c = ncc;
    };
    while (tile < n_tiles) {
      step(A, Bt);
      if (tile >= n_tiles) break;
      step(Bt, A);
    }
  } else {
    while (tile < n_tiles) {
      compute_wtile<QT, NSB, R, BT>(A, SB, c * 16 * NSB, s, lq, lf, XS, acc);
      if (c == nc - 1) finish(tile);
      if (++c == nc) { c = 0; tile += gridDim.x; }
      if (tile < n_tiles) load_wtile<QT, NSB, R>(w, row_base, tile * ROWS_B + rbase, N, SB, c * 16 * NSB, s, A);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Decode kernel, "all in flight" (B = 1, one K chunk). scripts/bench_gemv.py DBG variants showed the
// persistent kernel above streams at the HBM ceiling only without its prologue and its dot products
// (gate_up 9.0 us vs 15.1 us): vector loads return in issue order, so the prologue's activation
// loads -- issued after the weight tiles -- waited for every tile, and the 2-deep register ping-pong
// then left HBM idle while tiles computed. Here each thread first loads its activation groups (and
// norm weights) into registers, THEN issues the loads of all J weight tiles of its block, computes
// the norm + int8 quantisation from registers while the weights stream, and consumes the tiles in
// order with counted vmcnt waits (fully unrolled), so HBM sees the whole matrix requested up front.
// NRM: 0 = no norm (only x is loaded), 1 = RMSNorm (x, w), 2 = LayerNorm (x, w, b). Stand-in loads
// for absent norm operands would spend the wave's 63-deep vmcnt budget (NSB = 3: 69 loads per lane).
// KS > 1 (matrices with few row tiles, e.g. the K = 11008 down projection: 256 tiles = one 4-wave
// block per CU): the block has KS groups of GEMV_NW waves on the same rows, group kg owning the
// super-block range [kg*CH, (kg+1)*CH); partial sums meet in LDS before the epilogue. More waves per
// CU = more weight bytes in flight.
// MRG > 0 (B == 1 decode, O projection): x holds MRG unmerged flash-decode partial slabs
// (attention.hip `defer`); the prologue merges them per head in registers -- the merge rides on the
// activation round trip this kernel pays anyway, instead of an in-launch ticket + re-read (~2.5 us).
// JG > 1: the block holds JG independent groups of GEMV_NW * KS waves, each acting as its own
// (sub-)block over the tiles vb = bx * JG + jg (+ j * gxn * JG); they share the staged activations.
// XB (x barrier): every wave's activation loads are drained and the block meets at a barrier BEFORE
// any weight is requested. Measured (profiles/r3_gemv, scripts/gemv_timeline.py): a CU returns vector
// loads in issue order across its waves, so an activation load issued by any wave after another
// wave's weight burst waits for that whole burst -- the prologue ended only after the CU's entire
// weight share had streamed (gate_up 6.3 us, down Q6_K 8.2 us), and every dot product then ran after
// the stream instead of under it. With XB and one block per CU (JG / J sized so the grid = #CUs) the
// activations land in ~1 us and the tiles are consumed as they arrive.
// JG == 0: the group count is read from the launch (blockDim.x / (64 * GEMV_NW)).
template <int QT, int NSB, int R, int J, int NRM, int DBG = 0, int KS = 1, int MRG = 0, int JG = 1, int XB = 0>
__device__ __forceinline__ void flight_body(const GemvParams& P, const int bx, const int gxn) {
  static_assert(KS == 1 || JG == 1, "tile groups and the in-block K split do not combine");
  constexpr int ROWS_B = GEMV_NW * 4 * R;
  const int NT = JG == 0 ? (int)blockDim.x : GEMV_NT * KS * JG;
  const int JGr = JG == 0 ? (int)blockDim.x / GEMV_NT : JG;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const QMat& w = P.w;
  auto stamp = [&](int k) {
    if (P.dbg_ts && threadIdx.x == 0)
      P.dbg_ts[4 * ((long long)blockIdx.z * gxn + bx) + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  const int K = w.K, N = w.N, SB = n_sb(K);
  const int XS = SB * XPAD;
  i32x4* lq = (i32x4*)smem;                           // [XS + 1]: slot XS is a dummy
  f32x2* lf = (f32x2*)(smem + (size_t)(XS + 1) * 16);  // [XS + 1]
  float* red = (float*)(lf + XS + 1);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, s = lane & 15;
  const int jg = JG != 1 ? wave / GEMV_NW : 0;      // tile group
  const int kg = KS > 1 ? wave / GEMV_NW : 0, gtid = tid - kg * GEMV_NT;
  // K-split groups start on 16-super-block boundaries: a group's piece runs then begin where the row's
  // piece run begins (SB = 43 split 15 / 15 / 13 put every run 240 B off: the down GEMVs streamed at
  // 3.3 TB/s memory-path-only vs 4.5 at 16 / 16 / 16, profiles/r5_decode align probe)
  const int CH = ks_chunk(SB, KS);
  const int sb0 = kg * CH, se = min(SB, sb0 + CH);
  const int n_tiles = (N + ROWS_B - 1) / ROWS_B;
  const int rbase = (wave - kg * GEMV_NW - jg * GEMV_NW) * (4 * R) + g * R;
  const int vb = bx * JGr + jg, gv = gxn * JGr;    // this group's first tile and tile stride

  long long row_base = 0;
  const float* x = P.x;
  if (P.expert_ids) {  // MoE: blockIdx.z = k-th selected expert
    const int e = P.expert_ids[blockIdx.z];
    row_base = (long long)e * N;
    if (P.x_per_sel) x = P.x + (long long)blockIdx.z * P.x_sel_stride;
  }

  // 1. this thread's activation groups g = tid + NT i (i < NSB) and norm weights -> registers
  constexpr bool nrm = NRM != 0, lnb = NRM == 2;
  f32x4 xv[NSB][4], nw[NSB][4], nb[NSB][4];
  constexpr int MS = MRG > 0 ? MRG : 1;
  f32x4 av[MS][NSB][4];
  f32x2 ml[MS][NSB];
  // unconditional loads from clamped addresses (a conditional load would make the compiler drain it
  // before the weight loads are issued); out-of-range values are masked at use
#pragma unroll
  for (int i = 0; i < NSB; ++i) {
    const int gi = min(tid + NT * i, K / 16 - 1);
    if constexpr (MRG > 0) {
      const int h = 16 * gi / P.merge_D, nh = K / P.merge_D;
#pragma unroll
      for (int sp = 0; sp < MRG; ++sp) {
        ml[sp][i] = *(const f32x2*)(P.merge_ml + 2 * (sp * nh + h));
#pragma unroll
        for (int j = 0; j < 4; ++j) av[sp][i][j] = *(const f32x4*)(x + (long long)sp * K + 16 * gi + 4 * j);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (MRG == 0) xv[i][j] = *(const f32x4*)(x + 16 * gi + 4 * j);
      if constexpr (nrm) nw[i][j] = *(const f32x4*)(P.norm_w + 16 * gi + 4 * j);
      if constexpr (lnb) nb[i][j] = *(const f32x4*)(P.norm_b + 16 * gi + 4 * j);
    }
  }
  __builtin_amdgcn_sched_barrier(0);  // activations ahead of the weights
  if constexpr ((DBG & 4) != 0) __builtin_amdgcn_s_barrier();  // every wave's x requests queued first
  if constexpr (XB) {  // every activation byte of the block landed before the first weight request
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // x-first (GemvTuning::xfirst): wait for the activations BEFORE requesting any weight. The x lines
  // were just written by the previous kernel and miss L2; issued behind the whole matrix's requests
  // they return only after most of the weight stream (profiles/r1_defer/gemv_timeline.log: prologue
  // p50 4.6-8.3 us on the down projections), so every tile waits on them.
  if (P.xfirst) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // diagnostic (DBG & 16): every block of the grid has its activations before ANY block requests a
  // weight -- a bounded spin on a grid counter in the timeline buffer (scripts/gemv_timeline.py)
  if constexpr ((DBG & 16) != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && P.dbg_ts) {
      unsigned long long* cnt = P.dbg_ts + 4 * 4096;
      __hip_atomic_fetch_add(cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long want = (unsigned long long)gridDim.x * gridDim.z;
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want &&
             __builtin_amdgcn_s_memrealtime() - t0 < 10000)
        __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
  }
  __builtin_amdgcn_sched_barrier(0);
  // 2. every weight tile of this block in flight (surplus slots re-read the last tile, unused)
  WTile<QT, NSB, R> T[J];
  if constexpr ((DBG & 8) == 0) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int t = min(vb + j * gv, n_tiles - 1);
      load_wtile<QT, NSB, R>(w, row_base, t * ROWS_B + rbase, N, SB, sb0, s, T[j], se);
    }
  } else {  // diagnostic: no weight traffic at all (activation latency alone)
    for (int j = 0; j < J; ++j) T[j] = WTile<QT, NSB, R>{};
  }
  __builtin_amdgcn_sched_barrier(0);  // every load issued before the prologue's first wait
  if constexpr (MRG > 0) {  // flash-decode merge: splits without keys carry m = -inf, l = 0
#pragma unroll
    for (int i = 0; i < NSB; ++i) {
      float M = -INFINITY;
#pragma unroll
      for (int sp = 0; sp < MRG; ++sp) M = fmaxf(M, ml[sp][i].x);
      float L = 0.f;
      f32x4 a[4] = {};
#pragma unroll
      for (int sp = 0; sp < MRG; ++sp) {
        const float c = ml[sp][i].x == -INFINITY ? 0.f : __expf(ml[sp][i].x - M);
        L += c * ml[sp][i].y;
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] += c * av[sp][i][j];
      }
      const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[i][j] = a[j] * inv;
    }
  }
  // 3. norm statistics + quantisation from registers while the weights stream
#pragma unroll
  for (int i = 0; i < NSB; ++i) {
    const bool ok = 16 * (tid + NT * i) < K;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!ok) xv[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if constexpr (!nrm) nw[i][j] = (f32x4){1.f, 1.f, 1.f, 1.f};
      if constexpr (!lnb) nb[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  }
  float mean = 0.f, rstd = 1.f;
  if (nrm && !(DBG & 2)) {
    float sm = 0.f, ss = 0.f;
#pragma unroll
    for (int i = 0; i < NSB; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 v = xv[i][j];
        sm += v.x + v.y + v.z + v.w;
        ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      }
    ss = block_sum_rt(ss, red, NT / 64);
    if (NRM == 2 || P.norm == NORM_LAYER) {
      sm = block_sum_rt(sm, red, NT / 64);
      mean = sm / K;
      rstd = rsqrtf(fmaxf(ss / K - mean * mean, 0.f) + P.eps);
    } else {
      rstd = rsqrtf(ss / K + P.eps);
    }
  }
#pragma unroll
  for (int i = 0; i < NSB; ++i) {
    if constexpr (DBG & 2) continue;
    const int gi = tid + NT * i;
    // branch-free: surplus threads store to the dummy slot (a guarded block lets the compiler sink
    // the activation loads behind the weight loads, then drain them all with vmcnt(0))
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
  __syncthreads();
  stamp(1);
  if constexpr (KS > 1) {  // one tile per block: groups 1.. hand their partial sums to group 0
    static_assert(J == 1, "in-block K split is for single-tile blocks");
    float acc[R][1];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = 0.f;
    if constexpr (DBG & 1) {
      unsigned v = 0;
#pragma unroll
      for (int i = 0; i < NSB; ++i)
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) v ^= T[0].a[0][i][tt].x ^ T[0].a[0][i][tt].w ^ T[0].m[0][i].y;
      acc[0][0] = (float)(v & 1);
    } else {
      compute_wtile<QT, NSB, R, 1>(T[0], SB, sb0, s, lq, lf, XS, acc, se);
    }
    stamp(2);
    float* part = red + NT / 64;  // [KS-1][R][GEMV_NT]
    if (kg > 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) part[((kg - 1) * R + r) * GEMV_NT + gtid] = acc[r][0];
    }
    __syncthreads();
    if (kg == 0 && vb < n_tiles) {
#pragma unroll
      for (int k = 1; k < KS; ++k)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][0] += part[((k - 1) * R + r) * GEMV_NT + gtid];
      finish_rows<R, 1>(P, acc, vb * ROWS_B + rbase, N, 0, s);
    }
    stamp(3);
    return;
  }
  // 4. consume the tiles in issue order
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int t = vb + j * gv;
    if (t >= n_tiles) break;  // group-uniform (no barrier follows)
    float acc[R][1];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = 0.f;
    if constexpr (DBG & 1) {  // memory path only: consume every loaded word, no dot products
      unsigned v = 0;
#pragma unroll
      for (int i = 0; i < NSB; ++i)
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) {
          v ^= T[j].a[0][i][tt].x ^ T[j].a[0][i][tt].w ^ T[j].m[0][i].y;
          if constexpr (QT == QT_Q6_K) v ^= T[j].h[0][i][tt].x;
        }
      acc[0][0] = (float)(v & 1);
    } else {
      compute_wtile<QT, NSB, R, 1>(T[j], SB, 0, s, lq, lf, XS, acc);
    }
    if (j == 0) stamp(2);
    finish_rows<R, 1>(P, acc, t * ROWS_B + rbase, N, 0, s);
  }
  stamp(3);
}

template <int QT, int NSB, int R, int J, int NRM, int DBG = 0, int KS = 1, int MRG = 0, int XB = 0>
__global__ __launch_bounds__(GEMV_NT * KS) void qgemv_flight_kernel(GemvParams P) {
  flight_body<QT, NSB, R, J, NRM, DBG, KS, MRG, 1, XB>(P, blockIdx.x, gridDim.x);
}

// x-barrier flight kernel, one block per CU: 1-3 groups of 4 waves (blockDim.x = 256 * groups).
// Variants whose registers exceed the 168 VGPRs of 3 waves per SIMD (NSB = 2, 8-split merges,
// LayerNorm Q8_0 / Q6_K pairs) are built for one group (MJ = 1, 512 VGPRs) -- no scratch.
constexpr int XB_MAX_JG = 3;
template <int QT, int NSB, int J, int NRM, int MRG>
constexpr int xb_maxjg() {
  constexpr int PB = QT == QT_Q8_0 ? 8 : QT == QT_Q6_K ? 6 : QT == QT_Q5_K ? 5 : 4;
  constexpr int regs = J * NSB * (8 * PB + 5) + NSB * 16 * (1 + (NRM != 0) + (NRM == 2)) + MRG * NSB * 18 + 30;
  return regs <= 150 ? XB_MAX_JG : 1;
}
template <int QT, int NSB, int J, int NRM, int MRG>
__global__ __launch_bounds__((GEMV_NT * xb_maxjg<QT, NSB, J, NRM, MRG>())) void qgemv_flight_xb_kernel(GemvParams P) {
  flight_body<QT, NSB, 1, J, NRM, 0, 1, MRG, 0, 1>(P, blockIdx.x, gridDim.x);
}

// two matrices that read the same normalised x in ONE launch (Q4_K_M QKV: q,k rows Q4_K + v rows
// Q6_K): blocks [0, gxa) run A, the rest B -- one launch ramp / drain instead of two (v alone was
// 6.3 us for 13.8 MB, rocprofv3 profiles/r1_defer)
template <int QA, int QB, int NSB, int NRM>
__global__ __launch_bounds__(GEMV_NT) void qgemv_flight_dual_kernel(GemvParams PA, GemvParams PB, int gxa) {
  if ((int)blockIdx.x < gxa) flight_body<QA, NSB, 1, 1, NRM>(PA, blockIdx.x, gxa);
  else flight_body<QB, NSB, 1, 1, NRM>(PB, (int)blockIdx.x - gxa, (int)gridDim.x - gxa);
}

// x-barrier dual launch: one block per CU, JG tile groups per block; side A takes JA tiles per
// group, side B JB (q,k rows Q4_K: 512 tiles, v rows Q6_K: 256 tiles -> JA = 2, JB = 1)
template <int QA, int QB, int NSB, int NRM, int JA, int JB>
__global__ __launch_bounds__(GEMV_NT * XB_MAX_JG) void qgemv_flight_dual_xb_kernel(GemvParams PA, GemvParams PB,
                                                                                   int gxa) {
  if ((int)blockIdx.x < gxa) flight_body<QA, NSB, 1, JA, NRM, 0, 1, 0, 0, 1>(PA, blockIdx.x, gxa);
  else flight_body<QB, NSB, 1, JB, NRM, 0, 1, 0, 0, 1>(PB, (int)blockIdx.x - gxa, (int)gridDim.x - gxa);
}

// register tiles a block keeps in flight: ~150 VGPRs of weight tiles per lane
template <int QT, int NSB, int R>
constexpr int flight_jmax() {
  constexpr int PB = (QT == QT_Q8_0 || QT == QT_Q6_K8) ? 8 : QT == QT_Q6_K ? 6 : QT == QT_Q5_K ? 5 : 4;
  constexpr int regs = R * NSB * (8 * PB + 5);
  return regs * 3 <= 150 ? 3 : regs * 2 <= 150 ? 2 : 1;
}

static size_t lds_bytes(int K, int BT, int JG = 1) {
  return (size_t)BT * ((K + 255) / 256) * XPAD * 24 + 24 + 4 * GEMV_NW * JG;
}
// flight kernel with an in-block K split: activation slots + reduction slots + partial sums
static size_t lds_bytes_ks(int K, int KS, int R) {
  return (size_t)((K + 255) / 256) * XPAD * 24 + 24 + 4 * GEMV_NW * KS + (size_t)4 * (KS - 1) * R * GEMV_NT;
}

template <int QT, int NSB, int R, int BT, int DBG = 0>
static void launch_t(const GemvParams& P, hipStream_t s) {
  const int N = P.w.N;
  const int tiles = (N + 4 * GEMV_NW * R - 1) / (4 * GEMV_NW * R);
  const int by = (P.B + BT - 1) / BT;
  const int bz = P.expert_ids ? P.n_sel : 1;
  int gx = tiles;
  const int slots = 256 * g_tune.blocks_per_cu;
  const int cap = slots / (by * bz) > 0 ? slots / (by * bz) : 1;
  if (gx > cap) gx = cap;
  hipLaunchKernelGGL((qgemv_kernel<QT, NSB, R, BT, DBG>), dim3(gx, by, bz), dim3(GEMV_NT), lds_bytes(P.w.K, BT), s, P);
}

template <int QT, int NSB, int R, int J, int NRM>
static void launch_flight_n(const GemvParams& P, int gx, hipStream_t s) {
  const int bz = P.expert_ids ? P.n_sel : 1;
  const size_t lds = lds_bytes(P.w.K, 1);
  if constexpr (NSB == 1 && R == 1 && NRM == 0) {
    switch (P.merge_S) {  // deferred flash-decode merge in the prologue (O projection)
      case 0: break;
      case 2: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 0, 1, 2>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      case 4: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 0, 1, 4>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      case 8: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 0, 1, 8>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      default: return;  // rejected by gemv() before launch
    }
  }
  if constexpr (R == 1 && (QT == QT_Q4_K || QT == QT_Q6_K) && (NSB == 1 || NSB == 3) && NRM < 2) {
    switch (g_tune.debug) {  // microbenchmark-only variants (scripts/bench_gemv.py OMX_BENCH_DEBUG)
      case 1: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 1>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      case 2: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 2>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      case 3: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 3>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      case 4: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 4>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      case 9: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 9>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      case 16: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM, 16>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P); return;
      default: break;
    }
  }
  hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, R, J, NRM>), dim3(gx, 1, bz), dim3(GEMV_NT), lds, s, P);
}

template <int QT, int NSB, int KS, int NRM>
static void launch_flight_ks_n(const GemvParams& P, int gx, hipStream_t s) {
  const int bz = P.expert_ids ? P.n_sel : 1;
  const size_t lds = lds_bytes_ks(P.w.K, KS, 1);
  if constexpr ((QT == QT_Q4_K || QT == QT_Q6_K) && NRM == 0) {
    switch (g_tune.debug) {  // microbenchmark-only variants, as launch_flight_n
      case 1: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, 1, 1, NRM, 1, KS>), dim3(gx, 1, bz), dim3(GEMV_NT * KS), lds, s, P); return;
      case 2: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, 1, 1, NRM, 2, KS>), dim3(gx, 1, bz), dim3(GEMV_NT * KS), lds, s, P); return;
      case 3: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, 1, 1, NRM, 3, KS>), dim3(gx, 1, bz), dim3(GEMV_NT * KS), lds, s, P); return;
      case 4: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, 1, 1, NRM, 4, KS>), dim3(gx, 1, bz), dim3(GEMV_NT * KS), lds, s, P); return;
      case 9: hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, 1, 1, NRM, 9, KS>), dim3(gx, 1, bz), dim3(GEMV_NT * KS), lds, s, P); return;
      case 16:
        hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, 1, 1, NRM, 16, KS>), dim3(gx, 1, bz), dim3(GEMV_NT * KS), lds, s, P);
        return;
      default: break;
    }
  }
  if (g_tune.xbar && !P.expert_ids)
    hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, 1, 1, NRM, 0, KS, 0, 1>), dim3(gx, 1, bz), dim3(GEMV_NT * KS), lds, s, P);
  else
    hipLaunchKernelGGL((qgemv_flight_kernel<QT, NSB, 1, 1, NRM, 0, KS>), dim3(gx, 1, bz), dim3(GEMV_NT * KS), lds, s, P);
}

static int cu_count() {
  static int n = 0;
  if (n <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// (JG, J) of an x-barrier launch: the smallest per-block capacity JG * J (tile groups x tiles per
// group) that fits the tiles in one block per CU; J <= 2 keeps three 4-wave groups within the
// 168-VGPR budget of 3 waves per SIMD. false: the matrix needs more (old launch shape).
static bool xb_shape(int tiles, int jmax, int& JG, int& J, int& gx) {
  const int ncu = cu_count();
  const int cap = (tiles + ncu - 1) / ncu;
  if (cap <= XB_MAX_JG) {
    J = 1;
    JG = cap;
  } else {
    J = 2;
    JG = (cap + 1) / 2;
  }
  if (JG > XB_MAX_JG || J > jmax) return false;
  gx = (tiles + JG * J - 1) / (JG * J);
  return true;
}

// launches the variant if its register class admits JG groups; false otherwise
template <int QT, int NSB, int J, int NRM, int MRG>
static bool launch_xb_m(const GemvParams& P, int JG, int gx, hipStream_t s) {
  if (JG > xb_maxjg<QT, NSB, J, NRM, MRG>()) return false;
  hipLaunchKernelGGL((qgemv_flight_xb_kernel<QT, NSB, J, NRM, MRG>), dim3(gx), dim3(GEMV_NT * JG),
                     lds_bytes(P.w.K, 1, JG), s, P);
  return true;
}

template <int QT, int NSB, int J, int NRM>
static bool launch_xb_n(const GemvParams& P, int JG, int gx, hipStream_t s) {
  if constexpr (NSB == 1 && J == 1 && NRM == 0) {
    switch (P.merge_S) {  // deferred flash-decode merge in the prologue (O projection)
      case 0: break;
      case 2: return launch_xb_m<QT, NSB, J, NRM, 2>(P, JG, gx, s);
      case 4: return launch_xb_m<QT, NSB, J, NRM, 4>(P, JG, gx, s);
      case 8: return launch_xb_m<QT, NSB, J, NRM, 8>(P, JG, gx, s);
      default: return false;
    }
  }
  return launch_xb_m<QT, NSB, J, NRM, 0>(P, JG, gx, s);
}

template <int QT, int NSB, int J>
static bool launch_xb_j(const GemvParams& P, int JG, int gx, hipStream_t s) {
  if (P.norm == NORM_NONE) return launch_xb_n<QT, NSB, J, 0>(P, JG, gx, s);
  if (P.norm == NORM_LAYER && P.norm_b) return launch_xb_n<QT, NSB, J, 2>(P, JG, gx, s);
  return launch_xb_n<QT, NSB, J, 1>(P, JG, gx, s);
}

// batch-1 decode GEMV as one x-barrier block per CU (see flight_body XB); false = not covered
template <int QT>
static bool launch_flight_xb(const GemvParams& P, int need, hipStream_t s) {
  if constexpr (QT == QT_Q6_K8) {
    return false;
  } else {
    if (!g_tune.xbar || P.expert_ids || g_tune.debug || need > 2) return false;
    const int tiles = (P.w.N + 4 * GEMV_NW - 1) / (4 * GEMV_NW);
    int JG, J, gx;
    if (need == 1) {
      if (!xb_shape(tiles, flight_jmax<QT, 1, 1>() >= 2 ? 2 : 1, JG, J, gx)) return false;
      if (J == 1) return launch_xb_j<QT, 1, 1>(P, JG, gx, s);
      if constexpr (flight_jmax<QT, 1, 1>() >= 2) return launch_xb_j<QT, 1, 2>(P, JG, gx, s);
      return false;
    }
    if (P.merge_S || !xb_shape(tiles, 1, JG, J, gx)) return false;
    return launch_xb_j<QT, 2, 1>(P, JG, gx, s);
  }
}

template <int QT, int NSB, int R, int J>
static void launch_flight_j(const GemvParams& P, int gx, hipStream_t s) {
  if (P.norm == NORM_NONE) launch_flight_n<QT, NSB, R, J, 0>(P, gx, s);
  else if (P.norm == NORM_LAYER && P.norm_b) launch_flight_n<QT, NSB, R, J, 2>(P, gx, s);
  else launch_flight_n<QT, NSB, R, J, 1>(P, gx, s);
}

// grid: at least one block per CU while the matrix has the tiles, then up to J tiles per block
// in-block K split for single-row-tile matrices: KS groups of 4 waves, each NSB' = ceil(need / KS)
static int flight_ks(int need, int tiles, int bz) {
  if (g_tune.ks > 0) return g_tune.ks;
  // K <= 4096 (need 1): a split leaves half of every row group's lanes idle and doubles the VALU
  // work (measured: O 4.4 -> 5.0 us, V Q6_K 5.0 -> 7.8 us); enough tiles fill the CUs anyway
  if (need < 2 || tiles * bz > 256 * 2) return 1;
  // need 4 (K 12289..16384: Mixtral expert down, Llama-2-13B down): KS 4 x NSB 1 for Q6_K only
  // (launch_flight_split) -- Mixtral expert down Q6_K 30.6 -> 29.5 us, Q4_K 17.2 -> 19.9 us
  return need >= 4 ? 4 : need >= 3 ? 3 : 2;
}

// VGPRs a K-split flight instantiation needs (weight tile + activation / norm registers + ~24 of
// addressing, accumulators and the prefetch register) against the 512 / KS per lane that KS waves per
// SIMD leave. Calibrated on the built code objects (tests/test_isa.py): the Q8_0 / Q6_K LayerNorm
// variants above budget (KS = 4 NSB = 1, KS = 2 NSB = 2) were the only ones spilling to scratch.
template <int QT, int NSB, int KS, int NRM>
constexpr bool flight_ks_fits() {
  constexpr int PB = (QT == QT_Q8_0 || QT == QT_Q6_K8) ? 8 : QT == QT_Q6_K ? 6 : QT == QT_Q5_K ? 5 : 4;
  return NSB * (8 * PB + 5) + NSB * 16 * (1 + (NRM != 0) + (NRM == 2)) + 28 <= 512 / KS;
}

template <int QT, int NSB, int KS>
static bool launch_flight_ks_fit(const GemvParams& P, int gx, hipStream_t s) {
  const int nrm = P.norm == NORM_NONE ? 0 : (P.norm == NORM_LAYER && P.norm_b) ? 2 : 1;
  if (nrm == 0) {
    if constexpr (flight_ks_fits<QT, NSB, KS, 0>()) { launch_flight_ks_n<QT, NSB, KS, 0>(P, gx, s); return true; }
  } else if (nrm == 1) {
    if constexpr (flight_ks_fits<QT, NSB, KS, 1>()) { launch_flight_ks_n<QT, NSB, KS, 1>(P, gx, s); return true; }
  } else {
    if constexpr (flight_ks_fits<QT, NSB, KS, 2>()) { launch_flight_ks_n<QT, NSB, KS, 2>(P, gx, s); return true; }
  }
  return false;  // the variant would spill: the caller takes the unsplit kernel
}

template <int QT>
static bool launch_flight_split(const GemvParams& P, int need, hipStream_t s) {
  const int tiles = (P.w.N + 4 * GEMV_NW - 1) / (4 * GEMV_NW);
  const int bz = P.expert_ids ? P.n_sel : 1;
  int ks = flight_ks(need, tiles, bz);
  if (ks == 4 && QT != QT_Q6_K && g_tune.ks <= 0) ks = 2;  // Q4_K need 4: KS 2 x NSB 2
  if (ks <= 1) return false;
  const int nsb = (need + ks - 1) / ks;  // 16 * nsb >= ceil(SB / ks)
  if (ks == 2 && nsb == 1) return launch_flight_ks_fit<QT, 1, 2>(P, tiles, s);
  if (ks == 2 && nsb == 2) return launch_flight_ks_fit<QT, 2, 2>(P, tiles, s);
  if (ks == 3 && nsb == 1) return launch_flight_ks_fit<QT, 1, 3>(P, tiles, s);
  if (ks == 4 && nsb == 1) return launch_flight_ks_fit<QT, 1, 4>(P, tiles, s);
  return false;
}

template <int QT, int NSB, int R>
static void launch_flight(const GemvParams& P, hipStream_t s) {
  constexpr int JM = flight_jmax<QT, NSB, R>();
  const int tiles = (P.w.N + 4 * GEMV_NW * R - 1) / (4 * GEMV_NW * R);
  const int bz = P.expert_ids ? P.n_sel : 1;
  const int want = (256 * g_tune.blocks_per_cu + bz - 1) / bz;  // blocks per (z) slice
  int J = (tiles + want - 1) / want;
  J = J < 1 ? 1 : J > JM ? JM : J;
  const int gx = (tiles + J - 1) / J;
  if (J == 1) launch_flight_j<QT, NSB, R, 1>(P, gx, s);
  else if (J == 2) launch_flight_j<QT, NSB, R, (JM >= 2 ? 2 : 1)>(P, gx, s);
  else launch_flight_j<QT, NSB, R, JM>(P, gx, s);
}

template <int QT, int R, int BT>
static void launch_nsb(const GemvParams& P, hipStream_t s) {
  const int SB = (P.w.K + 255) / 256;
  const int need = (SB + 15) / 16;
  if constexpr (R == 2) {  // two rows per group only while both register tiles stay resident
    if (need == 1) launch_t<QT, 1, 2, BT>(P, s);
    else if (need == 2) launch_t<QT, 2, 2, BT>(P, s);
    else launch_nsb<QT, 1, BT>(P, s);
    return;
  } else {
    switch (need) {
      case 1: launch_t<QT, 1, R, BT>(P, s); return;
      case 2: launch_t<QT, 2, R, BT>(P, s); return;
      case 3: launch_t<QT, 3, R, BT>(P, s); return;
      default: launch_t<QT, 4, R, BT>(P, s); return;  // K > 12288: chunks of 64 super-blocks
    }
  }
}

template <int QT>
static void launch_q(const GemvParams& P, hipStream_t s) {
  if (P.merge_S > 0) {  // only the single-chunk B == 1 flight kernel merges (merge_supported())
    if (launch_flight_xb<QT>(P, 1, s)) return;
    launch_flight<QT, 1, 1>(P, s);
    return;
  }
  if (P.B == 1 || P.expert_ids != nullptr) {  // decode (and MoE: experts differ per batch row)
    const int need = ((P.w.K + 255) / 256 + 15) / 16;
    if (P.B == 1 && need <= 4) {  // whole K in one chunk: all-in-flight kernel
      if (g_tune.rows == 2 && need == 1) { launch_flight<QT, 1, 2>(P, s); return; }
      if (launch_flight_split<QT>(P, need, s)) return;
      if (launch_flight_xb<QT>(P, need, s)) return;
      switch (need) {
        case 1: launch_flight<QT, 1, 1>(P, s); return;
        case 2: launch_flight<QT, 2, 1>(P, s); return;
        case 3: launch_flight<QT, 3, 1>(P, s); return;
        default: launch_flight<QT, 4, 1>(P, s); return;
      }
    }
    if (g_tune.rows == 2 && QT != QT_Q6_K8) launch_nsb<QT, (QT == QT_Q6_K8 ? 1 : 2), 1>(P, s);
    else launch_nsb<QT, 1, 1>(P, s);
    return;
  }
  if constexpr (QT != QT_Q6_K8) {  // widened codes serve batch-1 only (eff_qtype)
    // continuous-batching rows: all-in-flight small-batch kernel (gemv_batch.hip)
    if (gemv_batch(P, s)) return;
    // batch tiles: the weights are unpacked once per piece and dotted against BT activation rows;
    // BT bounded by the LDS the staged activations take
    if (lds_bytes(P.w.K, 4) <= 96 * 1024) launch_nsb<QT, 1, 4>(P, s);
    else if (lds_bytes(P.w.K, 2) <= 120 * 1024) launch_nsb<QT, 1, 2>(P, s);
    else launch_nsb<QT, 1, 1>(P, s);
  }
}

template <int QA, int QB, int NSB>
static void launch_dual_n(const GemvParams& A, const GemvParams& Bp, hipStream_t s) {
  const int ta = (A.w.N + 4 * GEMV_NW - 1) / (4 * GEMV_NW), tb = (Bp.w.N + 4 * GEMV_NW - 1) / (4 * GEMV_NW);
  hipLaunchKernelGGL((qgemv_flight_dual_kernel<QA, QB, NSB, 1>), dim3(ta + tb), dim3(GEMV_NT), lds_bytes(A.w.K, 1),
                     s, A, Bp, ta);
}

// x-barrier dual launch for the Q4_K_M / Q5_K_M QKV (q,k rows Q4_K or Q5_K, v rows Q6_K): the group
// count and per-side tiles per group that put the most blocks on distinct CUs
template <int QA, int QB>
static bool launch_dual_xb(const GemvParams& A, const GemvParams& Bp, int need, hipStream_t s) {
  if constexpr (!((QA == QT_Q4_K || QA == QT_Q5_K) && QB == QT_Q6_K)) {
    return false;
  } else {
    if (!g_tune.xbar || need != 1) return false;
    const int ta = (A.w.N + 4 * GEMV_NW - 1) / (4 * GEMV_NW), tb = (Bp.w.N + 4 * GEMV_NW - 1) / (4 * GEMV_NW);
    const int ncu = cu_count();
    int best = -1, bJG = 0, bJA = 0, bJB = 0;
    for (int JG = XB_MAX_JG; JG >= 1; --JG)
      for (int JA = 1; JA <= 2; ++JA)
        for (int JB = 1; JB <= 2; ++JB) {
          const int blocks = (ta + JG * JA - 1) / (JG * JA) + (tb + JG * JB - 1) / (JG * JB);
          if (blocks <= ncu && blocks > best) { best = blocks; bJG = JG; bJA = JA; bJB = JB; }
        }
    if (best < 0) return false;
    const int gxa = (ta + bJG * bJA - 1) / (bJG * bJA);
    const size_t lds = lds_bytes(A.w.K, 1, bJG);
    const dim3 blk(GEMV_NT * bJG), grid(best);
    if (bJA == 1 && bJB == 1) hipLaunchKernelGGL((qgemv_flight_dual_xb_kernel<QA, QB, 1, 1, 1, 1>), grid, blk, lds, s, A, Bp, gxa);
    else if (bJA == 1) hipLaunchKernelGGL((qgemv_flight_dual_xb_kernel<QA, QB, 1, 1, 1, 2>), grid, blk, lds, s, A, Bp, gxa);
    else if (bJB == 1) hipLaunchKernelGGL((qgemv_flight_dual_xb_kernel<QA, QB, 1, 1, 2, 1>), grid, blk, lds, s, A, Bp, gxa);
    else hipLaunchKernelGGL((qgemv_flight_dual_xb_kernel<QA, QB, 1, 1, 2, 2>), grid, blk, lds, s, A, Bp, gxa);
    return true;
  }
}

template <int QA, int QB>
static void launch_dual_q(const GemvParams& A, const GemvParams& Bp, int need, hipStream_t s) {
  if (launch_dual_xb<QA, QB>(A, Bp, need, s)) return;
  if (need == 1) launch_dual_n<QA, QB, 1>(A, Bp, s);
  else launch_dual_n<QA, QB, 2>(A, Bp, s);
}

// batch-1 GEMVs of a Q6_K matrix with widened codes read them (QT_Q6_K8, qmat.h)
static int eff_qtype(const GemvParams& P) {
  return P.w.qtype == QT_Q6_K && P.w.s4 && P.B == 1 && !P.expert_ids ? (int)QT_Q6_K8 : P.w.qtype;
}

template <int QA>
static bool launch_dual_a(const GemvParams& A, const GemvParams& Bp, int need, hipStream_t s) {
  switch (eff_qtype(Bp)) {
    case QT_Q4_K: if (QA != QT_Q4_K) { launch_dual_q<QA, QT_Q4_K>(A, Bp, need, s); return true; } break;
    case QT_Q6_K: if (QA != QT_Q6_K) { launch_dual_q<QA, QT_Q6_K>(A, Bp, need, s); return true; } break;
    case QT_Q5_K: if (QA != QT_Q5_K) { launch_dual_q<QA, QT_Q5_K>(A, Bp, need, s); return true; } break;
    case QT_Q6_K8: if (QA != QT_Q6_K8) { launch_dual_q<QA, QT_Q6_K8>(A, Bp, need, s); return true; } break;
    case QT_Q4_0: if (QA != QT_Q4_0) { launch_dual_q<QA, QT_Q4_0>(A, Bp, need, s); return true; } break;
    case QT_Q8_0: if (QA != QT_Q8_0) { launch_dual_q<QA, QT_Q8_0>(A, Bp, need, s); return true; } break;
    default: break;
  }
  return false;
}

void gemv2(const GemvParams& A0, const GemvParams& B0, hipStream_t s) {
  if (A0.x8 && gemv8_2(A0, B0, s)) return;  // int8 activation chain (gemv8.hip)
  if (A0.B > 1 && gemv_mb2(A0, B0, s)) return;  // batched decode chain: q,k + v on the matrix cores
  GemvParams A = A0, Bp = B0;
  A.xfirst = Bp.xfirst = g_tune.xfirst;
  const int need = ((A.w.K + 255) / 256 + 15) / 16;
  const bool ok = A.B == 1 && Bp.B == 1 && A.w.K == Bp.w.K && need <= 2 && A.norm == NORM_RMS &&
                  Bp.norm == NORM_RMS && !A.expert_ids && !Bp.expert_ids && !A.merge_S && !Bp.merge_S &&
                  A.x == Bp.x && g_tune.debug == 0;
  if (ok) {
    bool done = false;
    switch (eff_qtype(A)) {
      case QT_Q4_K: done = launch_dual_a<QT_Q4_K>(A, Bp, need, s); break;
      case QT_Q6_K: done = launch_dual_a<QT_Q6_K>(A, Bp, need, s); break;
      case QT_Q5_K: done = launch_dual_a<QT_Q5_K>(A, Bp, need, s); break;
      case QT_Q6_K8: done = launch_dual_a<QT_Q6_K8>(A, Bp, need, s); break;
      case QT_Q4_0: done = launch_dual_a<QT_Q4_0>(A, Bp, need, s); break;
      case QT_Q8_0: done = launch_dual_a<QT_Q8_0>(A, Bp, need, s); break;
      default: break;
    }
    if (done) {
      count_launch(LC_GEMV_FLIGHT);
      return;
    }
  }
  gemv(A, s);
  gemv(Bp, s);
}

bool gemv_merge_supported(int B, int K, int D, int S) {
  return B == 1 && K <= 4096 && D % 16 == 0 && K % D == 0 && (S == 2 || S == 4 || S == 8);
}

static std::atomic<long long> g_launches[LC_N];
void count_launch(int which) { g_launches[which].fetch_add(1, std::memory_order_relaxed); }
long long launch_count(int which) { return which >= 0 && which < LC_N ? g_launches[which].load() : -1; }
void reset_launch_counts() {
  for (auto& c : g_launches) c.store(0);
}

void gemv(const GemvParams& P0, hipStream_t s) {
  // int8 activation chain (gemv8.hip); also the batch-1 deferred-merge residual add (Phi-2's O)
  const bool merge_add = P0.merge_S > 1 && P0.epi == EPI_ADD && P0.B == 1 && !P0.expert_ids;
  if ((P0.x8 || P0.emit8 || merge_add) && gemv8(P0, s)) return;
  if (P0.emit8) throw std::runtime_error("gemv: int8 activation emitter not covered by gemv8");
  if (P0.w.qtype == QT_F16) {  // fp16 weights (vision tower): the stream-order GEMM only
    if (!dq_gemm(P0, s)) throw std::runtime_error("gemv: F16 weights need >= 128 rows and an fp16 workspace");
    return;
  }
  GemvParams P = P0;
  P.xfirst = g_tune.xfirst;
  if (P.merge_S > 0) {
    // flight grid for K <= 4096 is one chunk, R = 1, no K split: the merge variant covers exactly it
    if (!gemv_merge_supported(P.B, P.w.K, P.merge_D, P.merge_S) || P.norm != NORM_NONE || P.expert_ids) return;
  }
  if (P.B > 1 && gemv_mb(P, s)) return;  // continuous-batching rows on the matrix cores (layout M)
  if (gemm_eligible(P)) {
    gemm(P, s);
    return;
  }
  count_launch(LC_GEMV_FLIGHT);
  switch (eff_qtype(P)) {
    case QT_Q6_K8: launch_q<QT_Q6_K8>(P, s); break;
    case QT_Q4_K: launch_q<QT_Q4_K>(P, s); break;
    case QT_Q6_K: launch_q<QT_Q6_K>(P, s); break;
    case QT_Q5_K: launch_q<QT_Q5_K>(P, s); break;
    case QT_Q4_0: launch_q<QT_Q4_0>(P, s); break;
    case QT_Q8_0: launch_q<QT_Q8_0>(P, s); break;
    default: break;
  }
}

}  // namespace omx
