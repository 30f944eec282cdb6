// The batch-1 / few-row int8-chain GEMV body (gemv8.hip) and its prefetched epilogues.
#pragma once
#include "gemv8_core.h"

namespace omx {

// Epilogue operands, loaded at block entry ahead of the activation image and the weight stream. The
// epilogues used to read them after the tile: the residual and the next norm's weight (EM_ADD), the
// bias, and RoPE's position / frequency plus the KV slot (EPI_QKV) -- each a dependent round trip at
// the block's tail, several in series behind branch-local vmcnt(0) waits (disassembly of the QKV
// GEMV: five load + vmcnt(0) pairs after the last dot product). Lane s of a row group writes batch
// row b = s (BT rows), so a lane's position / slot are those of row min(s, B - 1).
template <int J, int BT>
struct EpiPre {
  float res[J][BT];  // EM_ADD: current residual y[b][n]
  float nw[J];       // EM_ADD: emit8_nw[n]
  float bias[J];     // bias[vn] (0 when none)
  float pbias[J];    // EPI_QKV: bias[vn ^ 1] (RoPE pair partner)
  float fr[J];       // EPI_QKV: inv_freq[d / 2] of this row (0 beyond n_rot)
  float cs[J], sn[J];
  float c1[J], c2[J];  // IN_X8_LN: the row's LayerNorm constants (GemvParams::ln_c1 / ln_c2)
  int pos, slot;     // EPI_QKV: row min(s, B - 1)
};

// PRE = false: the EM_ADD operands are read in the epilogue instead (the register-heaviest
// instantiations, 2+ batch rows at a 3-4 way K split, would spill holding them)
template <int EMIT, int J, int BT, bool PRE = true, int IN = IN_X8>
__device__ __forceinline__ void epi_prefetch(const GemvParams& P, int tile0, int rbase, int s, EpiPre<J, BT>& E) {
  const int N = P.w.N, bl = min(s, P.B - 1);
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int n = min((tile0 + j) * 16 + rbase, N - 1), vn = n + P.row_offset;
    E.bias[j] = P.bias && PRE ? P.bias[vn] : 0.f;
    if constexpr (IN == IN_X8_LN) {
      E.c1[j] = P.ln_c1[n];
      E.c2[j] = P.ln_c2[n];
    }
    if constexpr (EMIT == EM_ADD && PRE) {
#pragma unroll
      for (int b = 0; b < BT; ++b) E.res[j][b] = P.y[(long long)min(b, P.B - 1) * P.ldy + n];
      E.nw[j] = P.emit8_nw[n];
    }
    if constexpr (EMIT == EM_NONE) {
      E.pbias[j] = 0.f;
      E.fr[j] = 0.f;
      if (P.epi == EPI_QKV) {
        const int sec = vn < P.Eq ? 0 : vn < P.Eq + P.Ekv ? P.Eq : P.Eq + P.Ekv;
        const int d = (vn - sec) % P.D;
        if (P.bias) E.pbias[j] = P.bias[vn ^ 1];
        if (sec < P.Eq + P.Ekv && d < P.n_rot) E.fr[j] = P.inv_freq[d >> 1];
      }
    }
  }
  if constexpr (EMIT == EM_NONE) {
    E.pos = 0;
    E.slot = 0;
    if (P.epi == EPI_QKV) {
      E.pos = P.pos[bl];
      E.slot = P.slot[bl];
    }
  }
}

// after the activation wait (the VALU is idle until the first weight piece lands)
template <int EMIT, int J, int BT>
__device__ __forceinline__ void epi_prepare(const GemvParams& P, EpiPre<J, BT>& E) {
  if constexpr (EMIT == EM_NONE) {
    if (P.epi == EPI_QKV) {
      // pinned: hipcc otherwise hoists the int -> float conversion of the position right behind its
      // load, i.e. a vmcnt wait BEFORE the weight stream is issued (one round trip per launch)
      int p = E.pos;
      asm volatile("" : "+v"(p)::"memory");
#pragma unroll
      for (int j = 0; j < J; ++j) {
        float f = E.fr[j];
        asm volatile("" : "+v"(f));
        sincosf((float)p * f, &E.sn[j], &E.cs[j]);
      }
    }
  }
}

// EM_NONE rows: the 16 lanes of a row group reduce; lane s == b writes batch row b (EPI_QKV: RoPE +
// paged K/V scatter; EPI_STORE: + bias; anything else: the shared epi_apply)
template <int J, int BT>
__device__ __forceinline__ void epi_rows(const GemvParams& P, float (&acc)[1][BT], int n, int s, int j,
                                         const EpiPre<J, BT>& E) {
  float v[BT], pv[BT];
#pragma unroll
  for (int b = 0; b < BT; ++b) {
    v[b] = row16_sum(acc[0][b]);
    pv[b] = __shfl_xor(v[b], 16, OMX_WAVE);  // row n ^ 1 (RoPE / GLU partner)
  }
  if (n >= P.w.N) return;
  const int vn = n + P.row_offset;
#pragma unroll
  for (int b = 0; b < BT; ++b) {
    if (s != b || b >= P.B) continue;
    if (P.epi == EPI_STORE) {
      P.y[(long long)b * P.ldy + vn] = v[b] + E.bias[j];
    } else if (P.epi == EPI_QKV) {
      const int Eq = P.Eq, Ekv = P.Ekv, D = P.D;
      const int which = vn < Eq ? 0 : vn < Eq + Ekv ? 1 : 2;
      const int rel = vn - (which == 0 ? 0 : which == 1 ? Eq : Eq + Ekv), hh = rel / D, d = rel % D;
      const float x = v[b] + E.bias[j];
      float out = x;
      if (which < 2 && d < P.n_rot) {
        const float px = pv[b] + E.pbias[j];
        out = (d & 1) ? (px * E.sn[j] + x * E.cs[j]) : (x * E.cs[j] - px * E.sn[j]);
      }
      if (which == 0) {
        P.y[(long long)b * P.ldy + vn] = out;
      } else {
        const long long blk = E.slot / P.bs, off = E.slot % P.bs;
        const long long idx = ((blk * P.n_kv + hh) * P.bs + off) * (P.Dc > 0 ? P.Dc : D) + d;
        if (which == 1) kv_store(P.kc, idx, out, P.kv8);
        else kv_store(P.vc, idx, out, P.kv8);
      }
    } else {
      epi_apply(P, b, vn, v[b], pv[b], 0);
    }
  }
}

// One block = KS groups of 4 waves on the same 16-row tiles (group kg owns super-blocks
// [kg * CH, (kg + 1) * CH)); J consecutive tiles per block, every weight load issued up front.
// MS: merge slabs of IN_MERGE (1 = plain fp32 input, no merge).
// BT: batch rows (continuous batching): every weight tile is read once and dotted with BT activation
// images (row b of the LDS image at b * XSP slots); rows >= P.B are computed but never stored.
template <int QT, int NSB, int J, int KS, int IN, int MS, int EMIT, int BT = 1>
__device__ __forceinline__ void gemv8_body(const GemvParams& P, const int bx) {
  static_assert(BT == 1 || MS <= 1, "batched rows take the plain fp32 input (no deferred merge)");
  static_assert(IN != IN_X8_LN || BT == 1, "LayerNorm'd images: batch 1 (Phi-2 decode)");
  static_assert(EMIT != EM_ACT || IN == IN_X8_LN, "EM_ACT: Phi-2's FFN up only");
  constexpr int NT = GEMV_NT * KS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const QMat& w = P.w;
  const int K = w.K, N = w.N, SB = n_sb(K), XS = SB * XPAD, XSP = x8_slots_dev(K);
  i32x4* lq = (i32x4*)smem;                           // [BT][XSP]
  f32x2* lf = (f32x2*)(smem + (size_t)BT * XSP * 16);  // [BT][XSP]
  float* stage = (float*)(lf + BT * XSP);             // [BT][48]: emitted values, their squares, plain values
  float* part = stage + 48 * BT;                      // [KS - 1][BT][GEMV_NT] partial sums of the K split
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, s = lane & 15;
  const int kg = KS > 1 ? wave / GEMV_NW : 0, gtid = tid - kg * GEMV_NT;
  // lanes stop at the last super-block holding weights: a padded K (weights.py ffn_pad) keeps its runs
  // line-aligned without streaming the zero super-blocks
  const int SBv = P.k_valid > 0 && P.k_valid < K ? n_sb(P.k_valid) : SB;
  // K split across blocks (GemvParams::kb, batch 1 only): block part kp of a tile streams super-blocks
  // [pa, pe), split again over the KS in-block groups
  const int KB = BT == 1 && P.kb > 1 ? P.kb : 1;
  const int kp = KB > 1 ? bx % KB : 0;
  int pa = 0, pe = SBv;
  if (KB > 1) {
    const int SBp = (SBv + KB - 1) / KB;
    pa = kp * SBp;
    pe = min(SBv, pa + SBp);
  }
  // K-split groups (ks_chunk): aligned to 16 super-blocks when the row stride keeps piece runs on lines
  const int CH = KB > 1 ? ks_chunk(pe - pa, KS) : ks_chunk(SB, KS);
  const int sb0 = pa + kg * CH, se = min(pe, sb0 + CH);
  const int n_tiles = (N + 15) / 16;
  const int rbase = (wave - kg * GEMV_NW) * 4 + g;
  const int tile0 = (KB > 1 ? bx / KB : bx) * J;

  // 0. epilogue operands (EpiPre), then 1. the activation operands: both return ahead of the weights
  constexpr bool PRE = BT == 1 || KS <= 2;
  EpiPre<J, BT> pre;
  epi_prefetch<EMIT, J, BT, PRE, IN>(P, tile0, rbase, s, pre);
  constexpr int NWI = x8_nwi(NSB, KS);
  u32x4 xw[BT][NWI];
  f32x4 stv[BT][X8_NSTW];
  f32x4 sxv[IN == IN_X8_LN ? X8_NSTW : 1];  // IN_X8_LN: the per-group sums
  // groups per thread of the merge prologue: the block's NT = GEMV_NT * KS threads cover KS * 4096
  // elements per group slot (O at K = 5120, Llama-2-13B, takes KS = 2)
  constexpr int MG = IN == IN_MERGE ? NSB : 1;
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
      for (int i = 0; i < NWI; ++i)
        xw[b][i] = ((const u32x4*)((const char*)P.x8 + min(b, blast) * img_b))[min(tid + NT * i, nwords - 1)];
    if constexpr (IN == IN_X8_RMS || IN == IN_X8_LN) {
      const int n4 = K / 64;  // f32x4 of partials (K / 16 floats)
#pragma unroll
      for (int b = 0; b < BT; ++b)
#pragma unroll
        for (int i = 0; i < X8_NSTW; ++i)
          stv[b][i] = ((const f32x4*)(P.x8_stat + min(b, blast) * st_ld))[min(lane + 64 * i, n4 - 1)];
      if constexpr (IN == IN_X8_LN) {
#pragma unroll
        for (int i = 0; i < X8_NSTW; ++i) sxv[i] = ((const f32x4*)P.x8_sum)[min(lane + 64 * i, n4 - 1)];
      }
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
  float rstd[BT], mu_rstd = 0.f;  // IN_X8_LN: mean * rstd (batch 1)
#pragma unroll
  for (int b = 0; b < BT; ++b) rstd[b] = 1.f;
  if constexpr (IN != IN_MERGE) {
#pragma unroll
    for (int b = 0; b < BT; ++b)
#pragma unroll
      for (int i = 0; i < NWI; ++i) {
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
    } else if constexpr (IN == IN_X8_LN) {
      const int n4 = K / 64;
      float ss = 0.f, sx = 0.f;
#pragma unroll
      for (int i = 0; i < X8_NSTW; ++i)
        if (lane + 64 * i < n4) {
          ss += stv[0][i].x + stv[0][i].y + stv[0][i].z + stv[0][i].w;
          sx += sxv[i].x + sxv[i].y + sxv[i].z + sxv[i].w;
        }
      const float mu = wave_sum(sx) / K;
      rstd[0] = rsqrtf(fmaxf(wave_sum(ss) / K - mu * mu, 0.f) + P.eps);
      mu_rstd = mu * rstd[0];
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
  epi_prepare<EMIT, J, BT>(P, pre);
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
    // memory path only (batch-1 microbenchmark): fold the tile's registers (the loads stay live), no dots;
    // compiled for BT == 1 alone (the branch costs the batched instantiations registers)
    if (BT == 1 && P.dbg8 == 1) {
      unsigned f = 0;
#pragma unroll
      for (int i = 0; i < NSB; ++i)
#pragma unroll
        for (int t = 0; t < 8; ++t) f ^= T[j].a[0][i][t].x ^ T[j].a[0][i][t].w ^ T[j].m[0][i].y;
      acc[0][0] += (float)(f & 1);
    } else {
      compute_wtile<QT, NSB, 1, BT, (BT == 1 || KS <= 2)>(T[j], SB, sb0, s, lq, lf, XSP, acc, se);
    }
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
    if constexpr (BT == 1 && J == 1 && IN != IN_MERGE && IN != IN_X8_LN && (EMIT == EM_ADD || EMIT == EM_NONE)) {
      if (KB > 1) {  // the tile's K parts meet: sc1 partial stores, agent-scope ticket, last block sums
        __shared__ int s_last;
        const float v = row16_sum(acc[0][0]);
        float* slot = P.kb_ws + ((long long)t * 16 + rbase) * KB;
        if (kg == 0 && s == 0) __hip_atomic_store(slot + kp, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
          const int old = __hip_atomic_fetch_add(P.kb_cnt + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const int last = old == KB - 1;
          if (last) __hip_atomic_store(P.kb_cnt + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
          s_last = last;
        }
        __syncthreads();
        if (!s_last) return;  // block-uniform
        float tot = 0.f;
        if (kg == 0 && s == 0)
          for (int p = 0; p < KB; ++p) tot += __hip_atomic_load(slot + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc[0][0] = tot;  // lane s == 0 of the row group carries the row's sum, the others 0
      }
    }
    // LayerNorm: rstd * (dot - mu * c1) + c2, the row's constant terms on one lane of its 16
    if constexpr (IN == IN_X8_LN) {
      if (s == 0) acc[0][0] += pre.c2[j] - mu_rstd * pre.c1[j];
    }
    if constexpr (EMIT == EM_NONE) {
      if (kg == 0) epi_rows<J, BT>(P, acc, t * 16 + rbase, s, j, pre);
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
              nv = (PRE ? pre.res[j][b] + pre.bias[j] : *dst + (P.bias ? P.bias[n] : 0.f)) + v[b];
              *dst = nv;
            }
            stage[48 * b + rbase] = n < N ? nv * (PRE ? pre.nw[j] : P.emit8_nw[n]) : 0.f;
            stage[48 * b + 16 + rbase] = nv * nv;
            stage[48 * b + 32 + rbase] = nv;
          }
        }
        __syncthreads();
        if (tid < 16 * nb) {  // batch row tid / 16 on 16 lanes of wave 0
          const int b = tid >> 4, i = tid & 15;
          emit_group16((char*)P.emit8 + (size_t)b * x8_slots_dev(N) * 24, N, t, stage[48 * b + i], stage[48 * b + 16 + i],
                       P.emit8_stat + b * x8_stat_ld_dev(N), i, stage[48 * b + 32 + i],
                       P.emit8_sum ? P.emit8_sum + b * x8_stat_ld_dev(N) : nullptr);
        }
        __syncthreads();  // the stage is reused by the next tile
      } else if constexpr (EMIT == EM_ACT) {  // one group per tile: act(v + bias) (EPI_GELU)
        if (kg == 0 && s == 0) {
          const float h = n < N ? gelu_tanh(v[0] + pre.bias[j]) : 0.f;
          if (n < N) P.y[n] = h;
          stage[rbase] = h;
        }
        __syncthreads();
        if (tid < 16) {
          const int Kc = P.emit8_k > 0 ? P.emit8_k : N;  // the consumer's (possibly padded) K
          emit_group16(P.emit8, Kc, t, stage[tid], 0.f, nullptr, tid);
        }
        __syncthreads();
      } else {  // EM_GLU: even row = gate, odd = up; 8 outputs per tile, a group per tile pair
        const int half = (t & 1) * 8;
        if (kg == 0 && s == 0 && (rbase & 1) == 0) {
#pragma unroll
          for (int b = 0; b < BT; ++b) {
            const float h = n < N ? (P.epi == EPI_GEGLU ? gelu_tanh(v[b]) : silu(v[b])) * pv[b] : 0.f;
            if (n < N && b < nb) P.y[(long long)b * P.ldy + (n >> 1)] = h;
            stage[48 * b + half + (rbase >> 1)] = h;
            if (half == 0 && t + 1 >= n_tiles) stage[48 * b + 8 + (rbase >> 1)] = 0.f;  // trailing half group
          }
        }
        if ((t & 1) || t + 1 >= n_tiles) {
          __syncthreads();
          if (tid < 16 * nb) {
            const int b = tid >> 4, i = tid & 15;
            const int Kc = P.emit8_k > 0 ? P.emit8_k : N / 2;  // the consumer's (possibly padded) K
            emit_group16((char*)P.emit8 + (size_t)b * x8_slots_dev(Kc) * 24, Kc, t >> 1, stage[48 * b + i], 0.f,
                         nullptr, i);
          }
          __syncthreads();
        }
      }
    }
    if constexpr (KS > 1) __syncthreads();  // part is reused by the next tile
  }
}

}  // namespace omx
