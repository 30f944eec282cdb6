// Stage implementations of the CPU serving backend (see cpu_engine.h). Mirrors the gfx950 executor
// (csrc/runtime/executor.cpp) and its torch twin (ollama_operator_amd/ops/reference.py) stage for
// stage: fused-norm projections, RoPE on adjacent pairs (NEOX heads are row-permuted at load), fp16
// paged KV scatter, GQA attention over the block table, SiLU-GLU (interleaved gate/up rows), GELU,
// top-k MoE, and the row-parallel partial sums of tensor parallelism (ypart).
#include <immintrin.h>
#include <omp.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <stdexcept>

#include "cpu_engine.h"

namespace omxcpu {

static inline float h2f(uint16_t h) { return _cvtsh_ss(h); }
static inline uint16_t f2h(float f) { return _cvtss_sh(f, _MM_FROUND_TO_NEAREST_INT); }

static void norm_rows(const float* x, int ldx, int B, int n, const float* w, const float* b, bool layer, float eps,
                      float* out, int ldo) {
  for (int r = 0; r < B; ++r) {
    const float* xr = x + (long long)r * ldx;
    float* o = out + (long long)r * ldo;
    double s = 0.0, ss = 0.0;
    for (int i = 0; i < n; ++i) {
      s += xr[i];
      ss += (double)xr[i] * xr[i];
    }
    float mean = 0.f, rstd;
    if (layer) {
      mean = (float)(s / n);
      rstd = 1.f / std::sqrt(std::max((float)(ss / n) - mean * mean, 0.f) + eps);
    } else {
      rstd = 1.f / std::sqrt((float)(ss / n) + eps);
    }
    for (int i = 0; i < n; ++i) o[i] = (xr[i] - mean) * rstd * w[i] + (b ? b[i] : 0.f);
  }
}

static inline float gelu(float x) {
  return 0.5f * x * (1.f + std::tanh(0.7978845608028654f * (x + 0.044715f * x * x * x)));
}
static inline float silu(float x) { return x / (1.f + std::exp(-x)); }

float* Engine::dst(int B) { return cfg.tp > 1 ? buf.ypart : buf.resid; }

void Engine::embed(int B) {
  for (int b = 0; b < B && !buf.ext; ++b)
    if (buf.tokens[b] < 0) throw std::runtime_error("negative token id without external embeddings");
#pragma omp parallel for schedule(static) if (B > 1)
  for (int b = 0; b < B; ++b) {
    float* r = buf.resid + (long long)b * cfg.E;
    if (buf.tokens[b] < 0) {  // external embedding row -(id + 1): copied as is
      const float* src = buf.ext + (long long)(-buf.tokens[b] - 1) * cfg.E;
      std::copy(src, src + cfg.E, r);
      continue;
    }
    dequant_row(tok_embd, buf.tokens[b], r);
    if (cfg.embed_scale != 1.f)
      for (int j = 0; j < cfg.E; ++j) r[j] *= cfg.embed_scale;
  }
}

void Engine::attn(int i, int B) {
  const Layer& L = layers[i];
  const int E = cfg.E, H = cfg.H, Hkv = cfg.Hkv, D = cfg.D, Eq = H * D, Ekv = Hkv * D;
  const bool phi = cfg.arch == 1;
  xn_.resize((size_t)B * E);
  norm_rows(buf.resid, E, B, E, L.attn_norm, L.attn_norm_b, phi, cfg.eps, xn_.data(), E);
  const int W = Eq + 2 * Ekv;
  tmp_.resize((size_t)B * W);
  float* qkv = tmp_.data();
  gemm(L.wqk, 0, L.wqk.N, xn_.data(), E, B, qkv, W, false);
  if (!L.qkv_fused) gemm(L.wv, 0, L.wv.N, xn_.data(), E, B, qkv + Eq + Ekv, W, false);
  if (L.qkv_bias)
    for (int b = 0; b < B; ++b)
      for (int j = 0; j < W; ++j) qkv[(long long)b * W + j] += L.qkv_bias[j];
  // RoPE on adjacent pairs of q and k heads, then q -> qbuf, k/v -> paged fp16 cache
  const int bs = buf.bs;
  for (int b = 0; b < B; ++b) {
    float* r = qkv + (long long)b * W;
    const float p = (float)buf.pos[b];
    for (int h = 0; h < H + Hkv; ++h) {
      float* v = r + h * D;
      for (int d = 0; d < cfg.n_rot; d += 2) {
        const float ang = p * inv_freq[d >> 1];
        const float cs = std::cos(ang), sn = std::sin(ang);
        const float a = v[d], c = v[d + 1];
        v[d] = a * cs - c * sn;
        v[d + 1] = a * sn + c * cs;
      }
    }
    memcpy(buf.qbuf + (long long)b * Eq, r, sizeof(float) * Eq);
    const long long slot = buf.slot[b], blk = slot / bs, off = slot % bs;
    for (int h = 0; h < Hkv; ++h) {
      const long long idx = ((blk * Hkv + h) * bs + off) * D;
      for (int d = 0; d < D; ++d) {
        L.kc[idx + d] = f2h(r[Eq + h * D + d]);
        L.vc[idx + d] = f2h(r[Eq + Ekv + h * D + d]);
      }
    }
  }
  if (phi) {  // parallel block: FFN up + GELU reads the same normed input
    const int F = cfg.F;
    gemm(L.wgu, 0, L.wgu.N, xn_.data(), E, B, buf.hbuf, F, false);
#pragma omp parallel for schedule(static)
    for (int b = 0; b < B; ++b)
      for (int j = 0; j < F; ++j) {
        float& h = buf.hbuf[(long long)b * F + j];
        h = gelu(h + (L.bup ? L.bup[j] : 0.f));
      }
  }
  // attention: one (row, head) per task, keys gathered through the block table
  const int G = H / Hkv;
  const float scale = 1.f / std::sqrt((float)D);
#pragma omp parallel
  {
    std::vector<float> sc, acc(D);
#pragma omp for schedule(dynamic, 1) collapse(2)
    for (int b = 0; b < B; ++b)
      for (int h = 0; h < H; ++h) {
        const int len = buf.q_len[b], row = buf.q_seq[b];
        const int start = cfg.window > 0 ? std::max(0, len - cfg.window) : 0;
        const int* bt = buf.block_table + (long long)row * buf.max_blocks;
        const float* q = buf.qbuf + (long long)b * Eq + h * D;
        const int kvh = h / G;
        sc.resize(len - start);
        float m = -INFINITY;
        for (int t = start; t < len; ++t) {
          const long long base = (((long long)bt[t / bs] * Hkv + kvh) * bs + t % bs) * D;
          float s = 0.f;
          for (int d = 0; d < D; ++d) s += q[d] * h2f(L.kc[base + d]);
          s *= scale;
          sc[t - start] = s;
          m = std::max(m, s);
        }
        float l = 0.f;
        std::fill(acc.begin(), acc.end(), 0.f);
        for (int t = start; t < len; ++t) {
          const float p = std::exp(sc[t - start] - m);
          l += p;
          const long long base = (((long long)bt[t / bs] * Hkv + kvh) * bs + t % bs) * D;
          for (int d = 0; d < D; ++d) acc[d] += p * h2f(L.vc[base + d]);
        }
        float* o = buf.abuf + (long long)b * Eq + h * D;
        const float inv = l > 0.f ? 1.f / l : 0.f;
        for (int d = 0; d < D; ++d) o[d] = acc[d] * inv;
      }
  }
  // output projection (+ bias) into the residual (or the TP partial-sum buffer)
  float* y = dst(B);
  const bool add = cfg.tp <= 1;
  gemm(L.wo, 0, L.wo.N, buf.abuf, Eq, B, y, E, add);
  if (L.bo)
    for (int b = 0; b < B; ++b)
      for (int j = 0; j < E; ++j) y[(long long)b * E + j] += L.bo[j];
}

void Engine::ffn(int i, int B) {
  const Layer& L = layers[i];
  const int E = cfg.E, F = cfg.F;
  float* y = dst(B);
  const bool add = cfg.tp <= 1;
  if (cfg.arch == 1) {  // phi2: up + GELU already in hbuf
    gemm(L.wdown, 0, L.wdown.N, buf.hbuf, F, B, y, E, add);
    if (L.bdown)
      for (int b = 0; b < B; ++b)
        for (int j = 0; j < E; ++j) y[(long long)b * E + j] += L.bdown[j];
    return;
  }
  xn_.resize((size_t)B * E);
  norm_rows(buf.resid, E, B, E, L.ffn_norm, nullptr, false, cfg.eps, xn_.data(), E);
  if (cfg.n_expert > 0) {
    const int X = cfg.n_expert, k = cfg.n_expert_used;
    std::vector<float> lg((size_t)B * X);
    gemm(L.router, 0, X, xn_.data(), E, B, lg.data(), X, false);
    if (!add) memset(y, 0, sizeof(float) * (size_t)B * E);
    gu_.resize((size_t)2 * F);
    std::vector<float> h(F), out(E);
    for (int b = 0; b < B; ++b) {
      const float* l = lg.data() + (long long)b * X;
      const float mx = *std::max_element(l, l + X);
      std::vector<float> p(X);
      float Z = 0.f;
      for (int e = 0; e < X; ++e) Z += (p[e] = std::exp(l[e] - mx));
      std::vector<int> idx(X);
      for (int e = 0; e < X; ++e) idx[e] = e;
      std::partial_sort(idx.begin(), idx.begin() + k, idx.end(), [&](int a, int c) { return p[a] > p[c]; });
      float ws = 0.f;
      for (int j = 0; j < k; ++j) ws += p[idx[j]];
      for (int j = 0; j < k; ++j) {
        const int e = idx[j];
        gemm(L.gu_exps, (long long)e * 2 * F, 2 * F, xn_.data() + (long long)b * E, E, 1, gu_.data(), 2 * F, false);
        for (int f = 0; f < F; ++f) h[f] = silu(gu_[2 * f]) * gu_[2 * f + 1];
        gemm(L.down_exps, (long long)e * E, E, h.data(), F, 1, out.data(), E, false);
        const float wgt = p[e] / ws;
        for (int c = 0; c < E; ++c) y[(long long)b * E + c] += wgt * out[c];
      }
    }
    return;
  }
  gu_.resize((size_t)B * 2 * F);
  gemm(L.wgu, 0, 2 * F, xn_.data(), E, B, gu_.data(), 2 * F, false);
#pragma omp parallel for schedule(static)
  for (int b = 0; b < B; ++b)
    for (int f = 0; f < F; ++f)
      buf.hbuf[(long long)b * F + f] = (cfg.glu_act ? gelu(gu_[(long long)b * 2 * F + 2 * f])
                                                   : silu(gu_[(long long)b * 2 * F + 2 * f])) *
                                       gu_[(long long)b * 2 * F + 2 * f + 1];
  gemm(L.wdown, 0, E, buf.hbuf, F, B, y, E, add);
}

void Engine::head(int n_logits, bool use_idx) {
  if (n_logits <= 0) return;
  const int E = cfg.E;
  xn_.resize((size_t)n_logits * E);
  for (int r = 0; r < n_logits; ++r) {
    const int src = use_idx ? buf.logit_idx[r] : r;
    norm_rows(buf.resid + (long long)src * E, E, 1, E, out_norm, out_norm_b, cfg.arch == 1, cfg.eps,
              xn_.data() + (long long)r * E, E);
  }
  gemm(lm_head, 0, lm_head.N, xn_.data(), E, n_logits, buf.logits, buf.ld_logits, false);
  if (lm_bias)
    for (int r = 0; r < n_logits; ++r)
      for (int j = 0; j < lm_head.N; ++j) buf.logits[(long long)r * buf.ld_logits + j] += lm_bias[j];
}

void Engine::forward(int B, int n_logits, bool use_idx) {
  if (cfg.tp != 1) throw std::runtime_error("forward is the TP=1 path; TP steps are driven per stage");
  if (B > buf.max_B) throw std::runtime_error("batch exceeds workspace");
  embed(B);
  for (int i = 0; i < cfg.n_layer; ++i) {
    attn(i, B);
    ffn(i, B);
  }
  head(n_logits, use_idx);
}

}  // namespace omxcpu
