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
#include "gemv8_body.h"

namespace omx {

template <int QT, int NSB, int J, int KS, int IN, int MS, int EMIT, int BT>
__global__ __launch_bounds__(GEMV_NT * KS) void qgemv8_kernel(GemvParams P) {
  gemv8_body<QT, NSB, J, KS, IN, MS, EMIT, BT>(P, blockIdx.x);
}

// q,k rows + v rows of different quant types (Q4_K_M QKV) over the same image: one launch. Phi-2: QKV
// and the FFN up (EMB = EM_ACT, emitting down's image) over the same LayerNorm'd image
// NSB = 2: 4096 < K <= 8192 (Llama-2-13B's QKV at K = 5120, two super-blocks per lane on both sides)
template <int QA, int QB, int IN, int BT, int EMB = EM_NONE, int NSB = 1>
__global__ __launch_bounds__(GEMV_NT) void qgemv8_dual_kernel(GemvParams PA, GemvParams PB, int gxa) {
  if ((int)blockIdx.x < gxa) gemv8_body<QA, NSB, 1, 1, IN, 0, EM_NONE, BT>(PA, blockIdx.x);
  else gemv8_body<QB, NSB, 1, 1, IN, 0, EMB, BT>(PB, (int)blockIdx.x - gxa);
}

// ------------------------------------------------------------------------------------------------
// host side
namespace {

size_t lds8(int K, int KS, int BT = 1) { return BT * x8_bytes(K) + (size_t)BT * (48 + (KS - 1) * GEMV_NT) * 4; }

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
  if (P.epi == EPI_GELU) return EM_ACT;
  return -1;
}

int in_mode(const GemvParams& P) {
  if (P.x8) return P.x8_sum ? IN_X8_LN : P.x8_stat ? IN_X8_RMS : IN_X8;
  if (P.norm != NORM_NONE) return -1;  // fp32 input with a norm: gemv.hip's prologue
  return IN_MERGE;                      // merge slabs (O) or a plain fp32 row
}

// launch geometry: (NSB, KS) from K; J tiles per block
struct Geo {
  int nsb = 0, ks = 0, J = 0, grid = 0;
};

// microbenchmarks only (scripts/bench_gemv8.py OMX_BENCH_GEO): force (NSB, KS) of the K-split plain-image
// launches (down) where that geometry covers K; 0 = the rule below
static int g_geo_nsb = 0, g_geo_ks = 0;

bool geometry(const GemvParams& P, Geo& G) {
  const int SB = (P.w.K + 255) / 256, need = (SB + 15) / 16;
  const int tiles = (P.w.N + 15) / 16;
  if (g_geo_nsb > 0 && g_geo_ks > 1 && need > 2 && P.x8 && !P.x8_stat && g_geo_nsb * g_geo_ks >= need) {
    G.nsb = g_geo_nsb;
    G.ks = g_geo_ks;
    G.J = 1;
    G.grid = tiles;
    return true;
  }
  if (need == 1) { G.nsb = 1; G.ks = 1; }
  else if (need == 2) { G.nsb = tiles > 512 ? 2 : 1; G.ks = tiles > 512 ? 1 : 2; }
  else if (need == 4 && P.w.qtype == QT_Q4_K && P.x8 && !P.x8_stat && P.B == 1) {
    // Llama-2-13B's Q4_K ffn_down (K = 13824, 54 SBs): 2 super-blocks per lane over a 2-way split, 14.4
    // vs 16.7 us at 4 x 1 (the Q6_K rows and the 3-way 7B shapes measured slower: profiles/r6_gemv8/geo.log)
    G.nsb = 2;
    G.ks = 2;
  } else if (need <= 4) { G.nsb = 1; G.ks = need; }
  else if (need <= 8) { G.nsb = 2; G.ks = (need + 1) / 2; }  // Llama-2-70B ffn_down (K = 28672): 4 x 32 SBs
  else return false;
  if (G.ks > 1) {
    G.J = 1;
  } else {
    const int want = 256 * g_tune.blocks_per_cu;
    G.J = (tiles + want - 1) / want;
    G.J = G.J < 1 ? 1 : G.J > 2 ? 2 : G.J;
    if (emit_mode(P) == EM_GLU) G.J = 2;  // a block owns whole groups (two tiles each)
    // two super-blocks per lane and two tiles: the GLU producer at 4096 < K <= 8192 only (Llama-2-13B
    // gate_up, K = 5120), from the RMS image, at most 2 batch rows (launch_glu_nsb2)
    if (G.nsb == 2 && G.J > 1) {
      if (emit_mode(P) == EM_GLU) {
        if (in_mode(P) != IN_X8_RMS || P.B > 2) return false;
      } else {
        G.J = 1;  // > 512 tiles: one tile per block still fills the chip (QKV at K = 5120: 960 blocks)
      }
    }
  }
  G.grid = (tiles + G.J - 1) / G.J;
  return true;
}

bool covered(const GemvParams& P, Geo& G) {
  if (P.B < 1 || P.B > X8_MAX_B || P.expert_ids || P.w.s0 == nullptr || P.dbg_ts) return false;
  const int em = emit_mode(P), in = in_mode(P);
  if (em < 0 || in < 0) return false;
  if (P.B > 1 && in == IN_MERGE && P.merge_S > 0) return false;  // batched rows: plain fp32 attention rows
  // nothing for this path to do -- except the batch-1 deferred-merge residual add without emission
  // (Phi-2's O: its consumer reads the residual through down's emission)
  if (!P.x8 && !P.emit8 && !(in == IN_MERGE && P.merge_S > 1 && P.epi == EPI_ADD && P.B == 1)) return false;
  if (in == IN_MERGE && P.merge_S > 0 && !(P.merge_S == 2 || P.merge_S == 4 || P.merge_S == 8)) return false;
  if (in == IN_MERGE && P.w.K % 16) return false;
  if (in == IN_X8_RMS && (P.w.K > 8192 || P.w.K % 64)) return false;
  // LayerNorm'd images (Phi-2): batch 1, constants present, K split at most in 2
  if (in == IN_X8_LN && (P.B != 1 || !P.x8_stat || !P.ln_c1 || !P.ln_c2 || P.w.K > 8192 || P.w.K % 64)) return false;
  if (em == EM_ACT && (in != IN_X8_LN || P.w.N % 16 || P.row_offset)) return false;
  if (em == EM_ADD && (!P.emit8_nw || !P.emit8_stat || P.w.N % 16)) return false;
  if (em == EM_GLU && P.w.N % 32) return false;
  const int q = P.w.qtype;
  if (!(q == QT_Q4_K || q == QT_Q6_K || q == QT_Q4_0 || q == QT_Q8_0 || q == QT_Q5_K)) return false;
  if (!geometry(P, G)) return false;
  // merge prologue: one 16-element group per thread and group slot (NSB slots); the deferred merge
  // (merge_S > 1) exists for the unsplit geometry only
  if (in == IN_MERGE && (P.w.K > GEMV_NT * G.ks * G.nsb * 16 || (P.merge_S > 1 && G.ks > 2))) return false;
  if (em == EM_GLU && G.J != 2) return false;  // a block owns whole groups: two tiles, unsplit K
  if (in != IN_MERGE && (size_t)G.ks * GEMV_NT * x8_nwi(G.nsb, G.ks) * 16 < x8_bytes(P.w.K)) return false;
  if (bt_of(P.B) >= 3 && !bt4_ok(q, G.ks, in)) return false;
  if (in == IN_X8_LN && (G.ks > 2 || (G.nsb == 2 && G.J == 2))) return false;
  // two super-blocks per lane at a 3-4 way K split (K > 16384): the plain image in (down), batch 1; at
  // the 4-way split (1024 threads, <= 128 VGPRs) only the Q4_0 / Q4_K tiles fit without spilling
  // (tests/test_isa.py)
  if (G.nsb == 2 && G.ks > 1 &&
      (in != IN_X8 || (em != EM_ADD && em != EM_NONE) || P.B > 1 || (G.ks == 4 && q != QT_Q4_0 && q != QT_Q4_K)))
    return false;
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
  else if (in == IN_X8_LN) {  // batch 1; no emission (QKV, LM head) or the activated FFN up
    if constexpr (KS <= 2) {
      if (em == EM_ACT) launch_k<QT, NSB, J, KS, IN_X8_LN, 0, EM_ACT, 1>(P, G.grid, s);
      else launch_k<QT, NSB, J, KS, IN_X8_LN, 0, EM_NONE, 1>(P, G.grid, s);
    }
  }
  else if constexpr (NSB == 1 && KS == 2 && J == 1) {  // O at 4096 < K <= 8192: merge slabs or plain fp32
    switch (P.merge_S) {
      case 2: launch_em<QT, 1, 1, 2, IN_MERGE, 2>(P, em, G.grid, s); break;
      case 4: launch_em<QT, 1, 1, 2, IN_MERGE, 4>(P, em, G.grid, s); break;
      case 8: launch_em<QT, 1, 1, 2, IN_MERGE, 8>(P, em, G.grid, s); break;
      default: launch_em<QT, 1, 1, 2, IN_MERGE, 1>(P, em, G.grid, s); break;
    }
  } else if constexpr (NSB == 1 && KS == 1 && J == 1) {  // the O projection: merge slabs or plain fp32
    switch (P.merge_S) {
      case 2: launch_em<QT, 1, 1, 1, IN_MERGE, 2>(P, em, G.grid, s); break;
      case 4: launch_em<QT, 1, 1, 1, IN_MERGE, 4>(P, em, G.grid, s); break;
      case 8: launch_em<QT, 1, 1, 1, IN_MERGE, 8>(P, em, G.grid, s); break;
      default: launch_em<QT, 1, 1, 1, IN_MERGE, 1>(P, em, G.grid, s); break;
    }
  }
}

template <int QT>
void launch_glu_nsb2(const GemvParams& P, const Geo& G, hipStream_t s) {
  if (bt_of(P.B) == 1) launch_k<QT, 2, 2, 1, IN_X8_RMS, 0, EM_GLU, 1>(P, G.grid, s);
  else launch_k<QT, 2, 2, 1, IN_X8_RMS, 0, EM_GLU, 2>(P, G.grid, s);
}

// K > 16384 (Llama-2-70B ffn_down): two super-blocks per lane, K split in 3-4, IN_X8, batch 1
template <int QT, int KS>
void launch_wide(const GemvParams& P, const Geo& G, hipStream_t s) {
  if constexpr (KS <= 3 || QT == QT_Q4_0 || QT == QT_Q4_K) {
    if (emit_mode(P) == EM_ADD) launch_k<QT, 2, 1, KS, IN_X8, 0, EM_ADD, 1>(P, G.grid, s);
    else launch_k<QT, 2, 1, KS, IN_X8, 0, EM_NONE, 1>(P, G.grid, s);
  }
}

template <int QT>
void launch_q(const GemvParams& P, const Geo& G, hipStream_t s) {
  if (G.nsb == 2 && G.ks == 2) launch_wide<QT, 2>(P, G, s);
  else if (G.nsb == 2 && G.ks == 3) launch_wide<QT, 3>(P, G, s);
  else if (G.nsb == 2 && G.ks == 4) launch_wide<QT, 4>(P, G, s);
  else if (G.ks == 1 && G.nsb == 2 && G.J == 2) launch_glu_nsb2<QT>(P, G, s);
  else if (G.ks == 1 && G.nsb == 1 && G.J == 1) launch_in<QT, 1, 1, 1>(P, G, s);
  else if (G.ks == 1 && G.nsb == 1) launch_in<QT, 1, 2, 1>(P, G, s);
  else if (G.ks == 1 && G.nsb == 2) launch_in<QT, 2, 1, 1>(P, G, s);
  else if (G.ks == 2) launch_in<QT, 1, 1, 2>(P, G, s);
  else if (G.ks == 3) launch_in<QT, 1, 1, 3>(P, G, s);
  else launch_in<QT, 1, 1, 4>(P, G, s);
}

bool launchable(const GemvParams& P, const Geo& G) {
  // the merge / plain-fp32 input exists for single-tile blocks, unsplit or split in 2 (K <= 8192)
  return in_mode(P) != IN_MERGE || (G.ks <= 2 && G.nsb == 1 && G.J == 1);
}

template <int QA, int QB, int IN, int BT, int EMB = EM_NONE, int NSB = 1>
void launch_dual_k(const GemvParams& A, const GemvParams& B, int gxa, int gxb, hipStream_t s) {
  const size_t lds = lds8(A.w.K, 1, BT);
  auto k = qgemv8_dual_kernel<QA, QB, IN, BT, EMB, NSB>;
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
  if ((A.w.K + 255) / 256 > 16) {  // two super-blocks per lane (gemv8_2: RMS image, <= 2 rows)
    if (bt_of(A.B) == 1) launch_dual_k<QA, QB, IN_X8_RMS, 1, EM_NONE, 2>(A, B, gxa, gxb, s);
    else launch_dual_k<QA, QB, IN_X8_RMS, 2, EM_NONE, 2>(A, B, gxa, gxb, s);
    return;
  }
  if (A.x8_sum) launch_dual_k<QA, QB, IN_X8_LN, 1, EM_ACT>(A, B, gxa, gxb, s);  // Phi-2 QKV + FFN up
  else if (A.x8_stat) launch_dual_in<QA, QB, IN_X8_RMS>(A, B, gxa, gxb, s);
  else launch_dual_in<QA, QB, IN_X8>(A, B, gxa, gxb, s);
}

template <int QA>
bool dual_b(const GemvParams& A, const GemvParams& B, int gxa, int gxb, hipStream_t s) {
  switch (B.w.qtype) {
    case QT_Q6_K: launch_dual<QA, QT_Q6_K>(A, B, gxa, gxb, s); return true;
    case QT_Q4_K: launch_dual<QA, QT_Q4_K>(A, B, gxa, gxb, s); return true;
    case QT_Q8_0: launch_dual<QA, QT_Q8_0>(A, B, gxa, gxb, s); return true;
    case QT_Q4_0: launch_dual<QA, QT_Q4_0>(A, B, gxa, gxb, s); return true;
    default: return false;
  }
}

}  // namespace

// K split across blocks (GemvParams::kb): -1 = OMX_GEMV8_KB, read once (0 / unset = auto, 1 = off, 2 = on
// wherever covered)
static int g_kb = -1;

static int kb_mode() {
  if (g_kb < 0) {
    const char* e = getenv("OMX_GEMV8_KB");
    g_kb = e ? atoi(e) : 0;
  }
  return g_kb;
}

// two blocks per row tile for a batch-1 K-split launch; each block streams half of K over 2 in-block
// groups and the tile's last block sums the halves (profiles/r6_gemv8/kb.log). Measured: Phi-2's ffn_down
// (160 tiles) 6.96 -> 9.63 us, the 7B shapes slower too -- the ticket hand-off costs more than the extra
// blocks win -- and only Llama-2-13B's Q6_K ffn_down (54 super-blocks) faster, 24.3 -> 22.0 us: the auto
// rule takes that shape alone
static int choose_kb(const GemvParams& P, const Geo& G) {
  const int mode = kb_mode();
  if (mode == 1 || !P.kb_ws || !P.kb_cnt || P.B != 1 || G.J != 1 || G.ks < 2 || G.nsb != 1) return 1;
  const int in = in_mode(P), em = emit_mode(P);
  if ((in != IN_X8 && in != IN_X8_RMS) || (em != EM_ADD && em != EM_NONE)) return 1;
  if ((size_t)2 * GEMV_NT * X8_NWI * 16 < x8_bytes(P.w.K) || P.w.N > 65536) return 1;  // image fit; kb_ws rows
  const int need = ((P.w.K + 255) / 256 + 15) / 16;
  return mode == 2 || (P.w.qtype == QT_Q6_K && need == 4) ? 2 : 1;
}

void set_gemv8_kb(int mode) { g_kb = mode; }

// the deferred flash-decode merge in the int8-chain O projection: K = H * D up to 8192 (Llama-2-13B /
// 70B: a 2-way in-block K split), 2 / 4 / 8 slabs
bool gemv8_merge_supported(int K, int D, int S) {
  return K <= 8192 && K % 16 == 0 && D % 16 == 0 && D > 0 && K % D == 0 && (S == 2 || S == 4 || S == 8);
}

void set_gemv8_geo(int nsb, int ks) {
  g_geo_nsb = nsb;
  g_geo_ks = ks;
}

bool gemv8_supported(const GemvParams& P) {
  Geo G;
  return covered(P, G) && launchable(P, G);
}

bool gemv8(const GemvParams& P0, hipStream_t s) {
  Geo G;
  if (!covered(P0, G) || !launchable(P0, G)) return false;
  GemvParams P = P0;
  P.kb = choose_kb(P0, G);
  if (P.kb > 1) {  // each block: 1 / kb of K over 2 in-block groups
    G.ks = 2;
    G.grid *= P.kb;
  }
  count_launch(P.B > 1 ? LC_GEMV8_ROWS : LC_GEMV8_ROW1);
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
  if (!A.x8 || !B.x8 || A.x8 != B.x8 || A.emit8 || A.w.K != B.w.K || A.B != B.B) return false;
  // LayerNorm'd images (Phi-2): B is the FFN up emitting down's image; otherwise neither side emits
  if (A.x8_sum != B.x8_sum || (A.x8_sum ? emit_mode(B) != EM_ACT : B.emit8 != nullptr)) return false;
  if (!covered(A, GA) || !covered(B, GB)) return false;
  const int need = ((A.w.K + 255) / 256 + 15) / 16;  // 16-super-block groups of K
  if (need == 2) {  // 4096 < K <= 8192: both sides two super-blocks per lane, RMS image, <= 2 rows
    if (in_mode(A) != IN_X8_RMS || A.B > 2) return false;
  } else if (GA.nsb != 1 || GA.ks != 1 || GB.nsb != 1 || GB.ks != 1) {
    return false;
  }
  const int gxa = (A.w.N + 15) / 16, gxb = (B.w.N + 15) / 16;  // one tile per block on both sides
  count_launch(LC_GEMV8_DUAL);
  switch (A.w.qtype) {
    case QT_Q4_K: return dual_b<QT_Q4_K>(A, B, gxa, gxb, s);
    case QT_Q5_K: return dual_b<QT_Q5_K>(A, B, gxa, gxb, s);
    case QT_Q4_0: return dual_b<QT_Q4_0>(A, B, gxa, gxb, s);
    default: return false;
  }
}

}  // namespace omx
