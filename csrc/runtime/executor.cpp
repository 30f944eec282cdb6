#include "executor.h"

#include <cmath>
#include <cstdlib>
#include <stdexcept>
#include <vector>

namespace omx {

static GemvParams base_params(const QMat& w, int B, const float* x, int ldx, const Workspace& ws) {
  GemvParams P{};
  P.xws = ws.x16;
  P.xws_elems = ws.x16_elems;
  P.gws = ws.gws;
  P.gws_elems = ws.gws_elems;
  P.w16ws = ws.w16;
  P.w16_elems = ws.w16_elems;
  P.yws = ws.yws;
  P.yws_elems = ws.yws_elems;
  P.w = w;
  P.B = B;
  P.x = x;
  P.ldx = ldx;
  P.eps = 1e-5f;
  P.n_sel = 1;
  P.kb_ws = ws.kb_ws;
  P.kb_cnt = ws.kb_cnt;
  return P;
}

// Batched decode chain (gemv_mfma.hip): each residual-adding projection (O, down) also emits the
// next RMSNorm'd GEMV's activations as fp16(resid * norm_w) plus per-tile sum-of-squares partials;
// the consumer (gate_up, next QKV, LM head) reads them straight from global memory and applies
// rsqrt(mean + eps) to its outputs -- no per-block activation staging, no separate norm launch.
bool Executor::chain(const StepInputs& in) const {
  return !x8(in) && ws.mb_ok && mb_enabled() && in.B >= 3 && in.B <= MB_CHAIN_MAX && !in.prefill && cfg.tp == 1 && cfg.arch == 0 &&
         cfg.n_expert == 0 && ws.xa16 && ws.h16 && ws.a16 && ws.st[0] && ws.st[1];
}

// a partial slab st[0] / st[1] is [16][n] sum-of-squares partials, 16 row scales 2^e (the emission range
// guard, gemv_mfma.hip emit_range_exp) and 16 range exponents for the next producer; 16 * n + 32 floats
static void chain_in(GemvParams& P, const void* x16, int ld16, const float* xstat, int n_stat) {
  P.x16 = x16;
  P.ld16 = ld16;
  P.zrow16 = MB_CHAIN_MAX;
  P.xstat = xstat;
  P.xstat_n = n_stat;
  P.xscale = xstat ? xstat + 16 * n_stat : nullptr;
}

// prev: the slab holding the partials of the residual before this producer's add (null: scale 1)
static void chain_emit(GemvParams& P, void* e16, int ld, const float* nw, float* st, const float* prev) {
  const int n = (P.w.N + 15) / 16;
  P.emit16 = e16;
  P.ld_emit = ld;
  P.emit_nw = nw;
  P.emit_stat = st;
  P.emit_scale = st + 16 * n;
  P.emit_prev = prev;
  P.emit_prev_n = prev ? n : 0;
}

// every projection of the chain takes the matrix-core kernel (a fallback kernel would neither emit nor
// read the fp16 activations): checked once when the workspace is bound
bool Executor::chain_capable() const {
  if (cfg.tp != 1 || cfg.arch != 0 || cfg.n_expert != 0 || layers.empty()) return false;
  static const float dummy[4] = {0.f, 0.f, 0.f, 0.f};
  auto ok = [&](const QMat& w, int epi, int norm, bool x16, bool emit) {
    GemvParams P{};
    P.w = w;
    P.B = 4;
    P.epi = epi;
    P.norm = norm;
    P.n_sel = 1;
    if (x16) chain_in(P, dummy, 256, norm == NORM_RMS ? dummy : nullptr, (cfg.E + 15) / 16);
    if (emit) chain_emit(P, (void*)dummy, 256, dummy, (float*)dummy, nullptr);
    return gemv_mb_supported(P);
  };
  for (const LayerW& L : layers) {
    if (!ok(L.wqk, EPI_QKV, NORM_RMS, true, false) || !ok(L.wo, EPI_ADD, NORM_NONE, true, true) ||
        !ok(L.wgu, EPI_GLU, NORM_RMS, true, false) || !ok(L.wdown, EPI_ADD, NORM_NONE, true, true))
      return false;
    if (!L.qkv_fused && !ok(L.wv, EPI_QKV, NORM_RMS, true, false)) return false;
    if (!ok(L.wqk, EPI_QKV, NORM_RMS, false, false)) return false;  // layer 0 reads fp32 resid
  }
  return ok(lm_head, EPI_STORE, NORM_RMS, true, false);
}

// Int8 activation chain (gemv8.hip): O and down emit the next RMSNorm'd GEMV's input as an int8 image
// (+ sum-of-squares partials), gate_up emits down's; consumers skip the fp32 activation prologue.
// Layer 0's QKV reads the embedding rows through gemv.hip's prologue. Batch 1, and up to ws.x8_bmax
// (<= X8_MAX_B) continuous-batching rows, which then read each weight tile once for every row.
// Under tensor parallelism the chain runs inside forward_tp only (the custom all-reduce is what emits
// the QKV / gate_up / LM-head images there: ar_allreduce_add_emit); the RCCL prefill path keeps fp32.
bool Executor::x8(const StepInputs& in) const {
  if (cfg.arch == 1) return ws.x8_ok && in.B == 1 && !in.prefill && cfg.tp == 1 && ln8();
  return ws.x8_ok && (in.B == 1 || in.B <= ws.x8_bmax) && !in.prefill && (cfg.tp == 1 || ar_active_) &&
         cfg.arch == 0 && cfg.n_expert == 0;
}

// Phi-2 (parallel attention/FFN block, LayerNorm): the same chain, batch 1. down emits the next layer's
// image of resid * attn_norm_w with sums and sums of squares (the LayerNorm's mean and variance); QKV
// and FFN up both consume it (rstd * (dot - mu * c1) + c2, GemvParams::ln_c1 / ln_c2), FFN up emits
// gelu(.) for down. O adds to the residual without emitting (its consumer is down, through resid).
bool Executor::ln8() const {
  if (cfg.arch != 1 || cfg.tp != 1 || cfg.n_expert != 0 || !ws.x8sum || cfg.E % 16) return false;
  for (const LayerW& L : layers)
    if (!L.c1_qkv || !L.c2_qkv || !L.c1_up || !L.c2_up || !L.attn_norm || !L.attn_norm_b) return false;
  return true;
}

// layer 0's QKV input image written by the embedding gather (E % 16 == 0, a dense llama-family stack)
bool Executor::x8_layer0(const StepInputs& in) const {
  return x8(in) && !layers.empty() && cfg.E % 16 == 0 && layers[0].attn_norm && ws.x8e && ws.x8st &&
         (cfg.arch != 1 || ws.x8sum);
}

static void x8_in(GemvParams& P, const void* img, const float* stat) {
  P.x8 = img;
  P.x8_stat = stat;
}

static void x8_emit(GemvParams& P, void* img, const float* nw, float* stat) {
  P.emit8 = img;
  P.emit8_nw = nw;
  P.emit8_stat = stat;
}

// consumers fall back to gemv.hip's fp32 prologue on their own (the producers keep writing the fp32
// residual / GLU rows too); an emitter the int8 kernel does not cover would leave its consumer a stale
// image, so the chain is on only when every emitter is covered
bool Executor::x8_capable(int B) const {
  if (cfg.arch == 1 && B == 1 && ln8() && ws.x8e && ws.x8f && ws.x8st) {  // the emitters: FFN up, down
    static const float dummy[4] = {0.f, 0.f, 0.f, 0.f};
    for (const LayerW& L : layers) {
      GemvParams U{};
      U.w = L.wgu;
      U.B = 1;
      U.epi = EPI_GELU;
      U.n_sel = 1;
      x8_in(U, dummy, dummy);
      U.x8_sum = U.ln_c1 = U.ln_c2 = dummy;
      U.emit8 = (void*)dummy;
      GemvParams D{};
      D.w = L.wdown;
      D.B = 1;
      D.epi = EPI_ADD;
      D.n_sel = 1;
      x8_in(D, dummy, nullptr);
      x8_emit(D, (void*)dummy, dummy, (float*)dummy);
      D.emit8_sum = (float*)dummy;
      if (!gemv8_supported(U) || !gemv8_supported(D)) return false;
    }
    return true;
  }
  if (cfg.arch != 0 || cfg.n_expert != 0 || layers.empty() || !ws.x8e || !ws.x8f || !ws.x8st) return false;
  const bool tp = cfg.tp > 1;  // O and down write partial sums to the all-reduce slabs, which emits
  static const float dummy[4] = {0.f, 0.f, 0.f, 0.f};
  for (const LayerW& L : layers) {
    GemvParams O{};
    O.w = L.wo;
    O.B = B;
    O.epi = EPI_ADD;
    O.n_sel = 1;
    x8_emit(O, (void*)dummy, dummy, (float*)dummy);  // (TP: O only writes slab partials, not checked)
    GemvParams G{};
    G.w = L.wgu;
    G.B = B;
    G.epi = cfg.glu_act ? EPI_GEGLU : EPI_GLU;
    G.n_sel = 1;
    x8_in(G, dummy, dummy);
    G.emit8 = (void*)dummy;
    GemvParams D{};
    D.w = L.wdown;
    D.B = B;
    D.epi = tp ? EPI_STORE : EPI_ADD;
    D.n_sel = 1;
    x8_in(D, dummy, nullptr);
    if (!tp) x8_emit(D, (void*)dummy, dummy, (float*)dummy);
    if ((!tp && !gemv8_supported(O)) || !gemv8_supported(G) || !gemv8_supported(D)) return false;
  }
  // TP: the all-reduce emits the images (ar_allreduce_add_emit covers E % 16 == 0, <= 4 rows)
  return !tp || (cfg.E % 16 == 0 && B <= 4);
}

void Executor::embed(const StepInputs& in, hipStream_t s) {
  // the batched fp16 chain: the embedded rows' partials go to st[1], read by layer 0's O emission
  // the int8 chain: the gather also writes layer 0's QKV input image (x8_layer0), as the producers do
  // for every later layer, so layer 0 takes the same int8 GEMV instead of the fp32-prologue one
  const bool q8 = x8_layer0(in);
  embed_rows(tok_embd, in.tokens, in.B, ws.resid, cfg.E, s, cfg.embed_scale, ws.ext, chain(in) ? ws.st[1] : nullptr,
             q8 ? ws.x8e : nullptr, q8 ? layers[0].attn_norm : nullptr, q8 ? ws.x8st : nullptr,
             q8 && cfg.arch == 1 ? ws.x8sum : nullptr);
}

void Executor::attn_block(int i, const StepInputs& in, hipStream_t s) {
  const LayerW& L = layers[i];
  const int B = in.B, E = cfg.E, Eq = cfg.H * cfg.D, Ekv = cfg.Hkv * cfg.D;
  const bool phi = cfg.arch == 1;
  // --- QKV projection: fused norm prologue, RoPE + paged K/V scatter epilogue
  GemvParams P = base_params(L.wqk, B, ws.resid, E, ws);
  P.norm = phi ? NORM_LAYER : NORM_RMS;
  P.norm_w = L.attn_norm;
  P.norm_b = L.attn_norm_b;
  P.eps = cfg.eps;
  P.epi = EPI_QKV;
  P.y = ws.qbuf;
  P.ldy = Eq;
  P.bias = L.qkv_bias;
  P.pos = in.pos;
  P.slot = in.slot;
  P.kc = L.kc;
  P.vc = L.vc;
  P.inv_freq = inv_freq;
  P.Eq = Eq;
  P.Ekv = Ekv;
  P.D = cfg.D;
  P.Dc = cfg.Dc;
  P.kv8 = cfg.kv8;
  P.n_rot = cfg.n_rot;
  P.n_kv = cfg.Hkv;
  P.bs = in.bs;  // the next GEMV of the step (gemv.hip cross-launch prefetch)
  const bool ch = chain(in);
  const bool q8 = x8(in);
  if (ch && i > 0) chain_in(P, ws.xa16, ws.ld_e, ws.st[1], (E + 15) / 16);  // emitted by layer i-1's down
  if (ch) P.rexp_out = ws.st[1] + 16 * ((E + 15) / 16) + 16;  // O's range exponents (layer 0: from resid)
  if (q8 && (i > 0 || x8_layer0(in))) {  // emitted by layer i-1's down / the embed
    x8_in(P, ws.x8e, ws.x8st);
    if (phi) {
      P.x8_sum = ws.x8sum;
      P.ln_c1 = L.c1_qkv;
      P.ln_c2 = L.c2_qkv;
    }
  }
  if (!L.qkv_fused) {  // q,k and v rows of different quant types: one dual launch at B == 1
    GemvParams V = P;
    V.w = L.wv;
    V.row_offset = Eq + Ekv;
    gemv2(P, V, s);
  } else if (!phi) {
    gemv(P, s);
  }
  if (phi) {  // parallel block: FFN up reads the same normed input, before O touches resid
    GemvParams U = base_params(L.wgu, B, ws.resid, E, ws);
    U.norm = NORM_LAYER;
    U.norm_w = L.attn_norm;
    U.norm_b = L.attn_norm_b;
    U.eps = cfg.eps;
    U.epi = EPI_GELU;
    U.bias = L.bup;
    U.y = ws.hbuf;
    U.ldy = cfg.F;
    if (q8 && (i > 0 || x8_layer0(in))) {  // same image as QKV; emits down's input
      x8_in(U, ws.x8e, ws.x8st);
      U.x8_sum = ws.x8sum;
      U.ln_c1 = L.c1_up;
      U.ln_c2 = L.c2_up;
      U.emit8 = ws.x8f;
      U.emit8_k = cfg.F;
    }
    // on the chain QKV and up share one launch over the same image (gemv8_2), else two
    if (!(L.qkv_fused && P.x8 && U.x8 && gemv8_2(P, U, s))) {
      if (L.qkv_fused) gemv(P, s);
      gemv(U, s);
    }
  }
  // --- attention over the paged cache
  AttnParams A{};
  A.q = ws.qbuf;
  A.ldq = Eq;
  A.kc = L.kc;
  A.vc = L.vc;
  A.block_table = in.block_table;
  A.max_blocks = in.max_blocks;
  A.q_seq = in.q_seq;
  A.q_len = in.q_len;
  A.NQ = B;
  A.H = cfg.H;
  A.n_kv = cfg.Hkv;
  A.D = cfg.Dc > 0 ? cfg.Dc : cfg.D;
  A.kv8 = cfg.kv8;
  A.Dv = cfg.D;
  A.bs = in.bs;
  A.scale = 1.0f / std::sqrt((float)cfg.D);
  A.window = cfg.window;
  A.out = ws.abuf;
  A.ldo = Eq;
  A.ws = ws.attn_ws;
  A.n_splits = ws.n_splits;
  A.counters = ws.attn_cnt;
  A.prefill = in.prefill;
  // deferred split merge (B == 1): the O projection's prologue merges the partial slabs
  const bool defer = ws.defer && B == 1 && ws.n_splits > 1;
  if (defer && !gemv_merge_supported(B, Eq, cfg.D, ws.n_splits) &&
      !(x8(in) && cfg.tp == 1 && gemv8_merge_supported(Eq, cfg.D, ws.n_splits)))
    throw std::runtime_error("deferred attention merge: unsupported (K, D, splits)");
  A.defer = defer;
  if (ch) A.out16 = ws.a16;
  if (in.prefill && !segments.empty()) {  // several sequences' prompts: flash attention per segment
    for (const auto& sg : segments) {
      AttnParams As = A;
      As.q = A.q + (long long)sg.first * A.ldq;
      As.out = A.out + (long long)sg.first * A.ldo;
      As.q_len = A.q_len + sg.first;
      As.q_seq = A.q_seq ? A.q_seq + sg.first : nullptr;
      As.NQ = sg.second;
      attention_decode(As, s);
    }
  } else {
    attention_decode(A, s);
  }
  // --- output projection (+ residual, or partial sum under TP); Phi-2 on the int8 chain: launched with
  // ffn_down as one pair kernel (ffn_block, gemv8_pair.hip) when covered
  if (phi && phi_pair(i, in)) return;
  GemvParams O = o_params(i, in);
  if (ch) {
    chain_in(O, ws.a16, ws.ld_q, nullptr, 0);
    // range exponents of the residual before O: written by this layer's QKV (st[1] + 16 n + 16)
    chain_emit(O, ws.xa16, ws.ld_e, L.ffn_norm, ws.st[0], nullptr);  // gate_up's RMSNorm input
    O.rexp_in = ws.st[1] + 16 * ((E + 15) / 16) + 16;
  }
  if (q8 && cfg.tp == 1 && !phi) x8_emit(O, ws.x8e, L.ffn_norm, ws.x8st);  // gate_up's RMSNorm input, int8
  gemv(O, s);
}

// the O projection's GEMV: merge slabs of the deferred split (B == 1) or the attention rows
GemvParams Executor::o_params(int i, const StepInputs& in) const {
  const LayerW& L = layers[i];
  const int B = in.B, Eq = cfg.H * cfg.D;
  const bool defer = ws.defer && B == 1 && ws.n_splits > 1;
  GemvParams O = base_params(L.wo, B, defer ? ws.attn_ws : ws.abuf, Eq, ws);
  if (defer) {
    O.merge_S = ws.n_splits;
    O.merge_ml = ws.attn_ws + (size_t)ws.n_splits * Eq;
    O.merge_D = cfg.D;
  }
  O.bias = L.bo;
  if (cfg.tp > 1) {
    O.epi = EPI_STORE;
    O.y = tp_dst(0, B);
  } else {
    O.epi = EPI_ADD;
    O.y = ws.resid;
  }
  O.ldy = cfg.E;
  return O;
}

// Phi-2's ffn_down on the int8 chain: FFN up's image in, the next layer's QKV / up (or the LM head) image out
GemvParams Executor::phi_down_params(int i, const StepInputs& in) const {
  const LayerW& L = layers[i];
  GemvParams Dn = base_params(L.wdown, in.B, ws.hbuf, cfg.F, ws);
  Dn.epi = cfg.tp > 1 ? EPI_STORE : EPI_ADD;
  Dn.bias = L.bdown;
  Dn.y = cfg.tp > 1 ? tp_dst(1, in.B) : ws.resid;
  Dn.ldy = cfg.E;
  Dn.k_valid = cfg.F_valid;
  if (x8(in)) {
    const bool last = i + 1 >= (int)layers.size();
    x8_in(Dn, ws.x8f, nullptr);
    x8_emit(Dn, ws.x8e, last ? out_norm : layers[i + 1].attn_norm, ws.x8st);
    Dn.emit8_sum = ws.x8sum;
  }
  return Dn;
}

// O and ffn_down of a Phi-2 layer in one launch (gemv8_pair.hip): the int8 chain at batch 1, OMX_PHI_PAIR
// unset or 1
bool Executor::phi_pair(int i, const StepInputs& in) const {
  static const int on = [] {
    const char* e = getenv("OMX_PHI_PAIR");
    return e ? atoi(e) : 1;
  }();
  if (!on || cfg.arch != 1 || cfg.tp != 1 || in.prefill || in.B != 1 || !x8(in)) return false;
  return gemv8_pair_supported(phi_down_params(i, in), o_params(i, in));
}

void Executor::ffn_block(int i, const StepInputs& in, hipStream_t s) {
  const LayerW& L = layers[i];
  const int B = in.B, E = cfg.E, F = cfg.F;
  float* dst = cfg.tp > 1 ? tp_dst(1, B) : ws.resid;
  const int dst_epi = cfg.tp > 1 ? EPI_STORE : EPI_ADD;
  if (cfg.arch == 1) {  // phi2: up+GELU already done in attn_block
    const GemvParams Dn = phi_down_params(i, in);
    if (phi_pair(i, in)) {  // O (skipped in attn_block) + down, one launch
      if (!gemv8_pair(Dn, o_params(i, in), s)) throw std::runtime_error("phi2: O + down pair launch declined");
      return;
    }
    gemv(Dn, s);
    return;
  }
  if (cfg.n_expert > 0) {
    const int X = cfg.n_expert, k = cfg.n_expert_used;
    GemvParams R = base_params(L.router, B, ws.resid, E, ws);
    R.norm = NORM_RMS;
    R.norm_w = L.ffn_norm;
    R.eps = cfg.eps;
    if (!moe_router(R, k, ws.eids, ws.ew, s)) {  // one fused launch: norm + logits + top-k (moe.hip)
      R.epi = EPI_STORE;
      R.y = ws.rlogits;
      R.ldy = X;
      gemv(R, s);
      moe_route(ws.rlogits, B, X, k, ws.eids, ws.ew, s);
    }
    if (B >= GEMM_MIN_B && ws.x16 && ws.moe_rows) {
      // prefill: grouped MFMA GEMM over expert-homogeneous tiles of the sorted (token, expert)
      // pairs -- each expert's weights stream once per 128 routed rows, not once per pair
      const int pairs = B * k;
      moe_sort(ws.eids, pairs, X, ws.moe_rows, ws.moe_tiles, ws.moe_ntiles, MOE_TILE_M, s);
      auto grouped = [&](GemvParams& P) {
        P.n_sel = k;
        P.moe_rows = ws.moe_rows;
        P.moe_tiles = ws.moe_tiles;
        P.moe_ntiles = ws.moe_ntiles;
        P.moe_max_tiles = (pairs + MOE_TILE_M - 1) / MOE_TILE_M + X;
      };
      GemvParams G = base_params(L.gu_exps, pairs, ws.resid, E, ws);
      G.norm = NORM_RMS;
      G.norm_w = L.ffn_norm;
      G.eps = cfg.eps;
      G.epi = EPI_GLU;
      G.y = ws.hbuf;  // [pair (sorted)][F]
      G.ldy = F;
      grouped(G);
      G.moe_gather = 1;
      // long prompts: per-expert hipBLASLt GEMMs (gemm.hip moe_gemm_lib) need the routed counts on the
      // host -- one small D2H copy + sync per layer (prefill is never graph-captured)
      std::vector<int> counts;
      hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
      (void)hipStreamIsCapturing(s, &cap);
      const int lm = moe_lib_min_m();
      if (lm > 0 && pairs >= lm && ws.w16 && ws.yws && cap == hipStreamCaptureStatusNone) {
        std::vector<int> e_host(pairs);
        if (hipMemcpyAsync(e_host.data(), ws.eids, sizeof(int) * pairs, hipMemcpyDeviceToHost, s) == hipSuccess &&
            hipStreamSynchronize(s) == hipSuccess) {
          counts.assign(X, 0);
          for (int v : e_host)
            if (v >= 0 && v < X) ++counts[v];
        }
      }
      const bool lib = !counts.empty() && moe_gemm_lib(G, counts.data(), X, s);
      if (!lib) moe_gemm(G, s);
      if (cfg.tp > 1) hipMemsetAsync(dst, 0, sizeof(float) * (size_t)B * E, s);
      GemvParams Dn = base_params(L.down_exps, pairs, ws.hbuf, F, ws);
      Dn.epi = EPI_ADD;  // routing-weighted, atomically accumulated per token
      Dn.y = dst;
      Dn.ldy = E;
      Dn.expert_ids = ws.eids;
      Dn.expert_w = ws.ew;
      grouped(Dn);
      Dn.moe_scatter = 1;
      if (!(lib && moe_gemm_lib(Dn, counts.data(), X, s))) moe_gemm(Dn, s);
      return;
    }
    GemvParams G = base_params(L.gu_exps, B, ws.resid, E, ws);
    G.norm = NORM_RMS;
    G.norm_w = L.ffn_norm;
    G.eps = cfg.eps;
    G.epi = EPI_GLU;
    G.y = ws.hbuf;
    G.ldy = k * F;
    G.expert_ids = ws.eids;
    G.n_sel = k;
    G.y_sel_stride = F;
    gemv(G, s);
    if (cfg.tp > 1) hipMemsetAsync(dst, 0, sizeof(float) * (size_t)B * E, s);
    GemvParams Dn = base_params(L.down_exps, B, ws.hbuf, k * F, ws);
    Dn.epi = EPI_ADD;  // expert-weighted, atomically accumulated
    Dn.y = dst;
    Dn.ldy = E;
    Dn.expert_ids = ws.eids;
    Dn.expert_w = ws.ew;
    Dn.n_sel = k;
    Dn.x_per_sel = 1;
    Dn.x_sel_stride = F;
    gemv(Dn, s);  // expert launches take no prefetch (their rows depend on the routing)
    return;
  }
  const bool ch = chain(in);
  const bool q8 = x8(in);
  GemvParams G = base_params(L.wgu, B, ws.resid, E, ws);
  G.norm = NORM_RMS;
  G.norm_w = L.ffn_norm;
  G.eps = cfg.eps;
  G.epi = cfg.glu_act ? EPI_GEGLU : EPI_GLU;
  G.y = ws.hbuf;
  G.ldy = F;
  if (ch) {
    chain_in(G, ws.xa16, ws.ld_e, ws.st[0], (E + 15) / 16);
    G.rexp_out = ws.st[0] + 16 * ((E + 15) / 16) + 16;  // down's range exponents
    G.y16 = ws.h16;
    G.ld16y = ws.ld_f;
  }
  if (q8) {
    x8_in(G, ws.x8e, ws.x8st);
    G.emit8 = ws.x8f;  // down's input
    G.emit8_k = F;     // down's K (ffn_down padded to whole 16-super-block groups: weights.py ffn_pad)
  }
  GemvParams Dn = base_params(L.wdown, B, ws.hbuf, F, ws);
  Dn.epi = dst_epi;
  Dn.y = dst;
  Dn.ldy = E;
  Dn.k_valid = cfg.F_valid;
  if (ch) {  // the next RMSNorm'd GEMV: layer i+1's QKV, or the LM head
    chain_in(Dn, ws.h16, ws.ld_f, nullptr, 0);
    chain_emit(Dn, ws.xa16, ws.ld_e, i + 1 < (int)layers.size() ? layers[i + 1].attn_norm : out_norm, ws.st[1],
               nullptr);
    Dn.rexp_in = ws.st[0] + 16 * ((E + 15) / 16) + 16;  // written by this layer's gate_up
  }
  if (q8 && cfg.tp > 1) {
    x8_in(Dn, ws.x8f, nullptr);  // partial sums to the slab: the all-reduce emits the next image
  } else if (q8) {
    x8_in(Dn, ws.x8f, nullptr);
    x8_emit(Dn, ws.x8e, i + 1 < (int)layers.size() ? layers[i + 1].attn_norm : out_norm, ws.x8st);
  }
  gemv(G, s);
  gemv(Dn, s);
}

void Executor::head(const StepInputs& in, hipStream_t s) {
  const int E = cfg.E;
  const float* x = ws.resid;
  if (in.n_logits <= 0) return;
  if (in.logit_idx) {
    gather_rows(ws.resid, E, in.logit_idx, in.n_logits, E, ws.lbuf, s);
    x = ws.lbuf;
  }
  GemvParams P = base_params(lm_head, in.n_logits, x, E, ws);
  P.norm = cfg.arch == 1 ? NORM_LAYER : NORM_RMS;
  P.norm_w = out_norm;
  P.norm_b = out_norm_b;
  P.eps = cfg.eps;
  P.epi = EPI_STORE;
  P.bias = lm_bias;
  P.y = in.logits;
  P.ldy = lm_head.N;
  if (chain(in) && x == ws.resid && in.n_logits == in.B && cfg.n_layer > 0)
    chain_in(P, ws.xa16, ws.ld_e, ws.st[1], (E + 15) / 16);
  if (x8(in) && x == ws.resid && in.n_logits == in.B && cfg.n_layer > 0) {
    if (cfg.arch != 1) {
      x8_in(P, ws.x8e, ws.x8st);
    } else if (lm_c1 && lm_c2 && out_norm && out_norm_b) {  // else the fp32 LayerNorm prologue
      x8_in(P, ws.x8e, ws.x8st);
      P.x8_sum = ws.x8sum;
      P.ln_c1 = lm_c1;
      P.ln_c2 = lm_c2;
    }
  }
  gemv(P, s);
}

float* Executor::tp_dst(int slab, int B) const {
  if (ar_active_) return ws.ar.data[ws.ar.rank] + (long long)slab * ws.ar.slab_floats;
  return ws.ypart;  // RCCL path: the caller all-reduces ypart between stages
}

bool Executor::ar_fits(int B) const {
  return ws.ar_on && (long long)B * cfg.E <= ws.ar.slab_floats && (long long)B * cfg.V <= ws.ar.slab_floats;
}

void Executor::forward_tp(const StepInputs& in, hipStream_t s) {
  if (cfg.tp <= 1 || !ws.ar_on) throw std::runtime_error("forward_tp needs tp > 1 and the custom all-reduce");
  if (!ar_fits(in.B)) throw std::runtime_error("forward_tp: batch exceeds the all-reduce slabs");
  if (in.B > ws.max_B) throw std::runtime_error("batch exceeds workspace");
  const int n = in.B * cfg.E;
  struct Active {  // the stages write partial sums to the slabs only inside forward_tp
    int& f;
    explicit Active(int& x) : f(x) { f = 1; }
    ~Active() { f = 0; }
  } active(ar_active_);
  embed(in, s);
  const bool q8 = x8(in);
  for (int i = 0; i < cfg.n_layer; ++i) {
    attn_block(i, in, s);
    // resid += sum of the ranks' O partials; on the int8 chain the same kernel emits gate_up's image
    // (the consumers read that image whenever the chain is on: an emission the kernel declines must
    // fail loudly, never leave them a stale one)
    if (q8) {
      if (!ar_allreduce_add_emit(ws.ar, 0, ws.resid, cfg.E, in.B, ws.x8e, layers[i].ffn_norm, ws.x8st, s))
        throw std::runtime_error("forward_tp: int8-chain all-reduce emission not covered");
    } else {
      ar_allreduce_add(ws.ar, 0, ws.resid, n, s);
    }
    ffn_block(i, in, s);
    const float* nxt = i + 1 < cfg.n_layer ? layers[i + 1].attn_norm : out_norm;  // next QKV / LM head
    if (q8) {
      if (!ar_allreduce_add_emit(ws.ar, 1, ws.resid, cfg.E, in.B, ws.x8e, nxt, ws.x8st, s))
        throw std::runtime_error("forward_tp: int8-chain all-reduce emission not covered");
    } else {
      ar_allreduce_add(ws.ar, 1, ws.resid, n, s);
    }
  }
  if (in.n_logits > 0) {
    StepInputs h = in;
    h.logits = ws.ar.data[ws.ar.rank] + 2LL * ws.ar.slab_floats;  // this rank's vocab shard -> slab 2
    head(h, s);
    ar_allgather(ws.ar, 2, in.full_logits, in.n_logits, cfg.V, in.ld_full, s);
  }
}

void Executor::forward(const StepInputs& in, hipStream_t s) {
  if (cfg.tp != 1) throw std::runtime_error("Executor::forward is the TP=1 path; TP steps are driven per block");
  if (in.B > ws.max_B) throw std::runtime_error("batch exceeds workspace");
  embed(in, s);
  for (int i = 0; i < cfg.n_layer; ++i) {
    attn_block(i, in, s);
    ffn_block(i, in, s);
  }
  head(in, s);
}

}  // namespace omx
