// Native CPU serving backend (BASELINE config 1: `image: phi` on kind, CPU-only server).
//
// The same stage API as the gfx950 executor (csrc/runtime/executor.h) over the same buffers and the
// same repacked weight streams (quant.py "device repack", layout v2), so the Python runner, paged KV
// cache, sampler and tensor-parallel stage loop are shared unchanged. Weights stay quantised in
// memory (Phi-2 Q4_0: 1.6 GB, not the 10.7 GB an fp32 dequantisation takes); every projection is an
// int8 dot product of the unpacked codes against Q8_K-style activations (one fp32 scale per 256,
// int16 sums per 16), with AVX-512 VNNI (vpdpbusd) when the CPU has it and AVX2 otherwise, threaded
// over output rows with OpenMP. Prefill rows share each unpacked weight super-block (B rows per
// unpack), so a prompt streams the weights once per row tile instead of once per token.
// Reference parity: replaces the llama.cpp CPU runner inside `ollama/ollama` (reference
// pkg/model/pod.go:10-12; demo recordings docs/public/demo*.cast are CPU-only Phi-2).
#pragma once
#include <stdint.h>

#include <vector>

namespace omxcpu {

enum QType : int { QT_Q4_0 = 2, QT_Q8_0 = 8, QT_Q4_K = 12, QT_Q5_K = 13, QT_Q6_K = 14 };

struct QMat {
  const uint8_t* s[4] = {nullptr, nullptr, nullptr, nullptr};
  int N = 0, K = 0, qtype = 0;
};

struct Config {
  int arch = 0;  // 0 llama family, 1 phi2
  int E = 0, H = 0, Hkv = 0, D = 0, n_rot = 0, F = 0, n_layer = 0, V = 0;
  float eps = 1e-5f;
  int n_expert = 0, n_expert_used = 0, window = 0, tp = 1;
  float embed_scale = 1.f;  // Gemma: sqrt(E)
  int glu_act = 0;          // 0 SiLU-GLU, 1 GELU-GLU (Gemma)
};

struct Layer {
  const float *attn_norm = nullptr, *attn_norm_b = nullptr, *ffn_norm = nullptr;
  QMat wqk, wv;
  int qkv_fused = 1;
  const float* qkv_bias = nullptr;
  QMat wo;
  const float* bo = nullptr;
  QMat wgu;
  const float* bup = nullptr;
  QMat wdown;
  const float* bdown = nullptr;
  QMat router, gu_exps, down_exps;
  uint16_t *kc = nullptr, *vc = nullptr;  // fp16 [nblk][Hkv][bs][D]
};

struct Buffers {
  float *resid = nullptr, *qbuf = nullptr, *abuf = nullptr, *hbuf = nullptr, *ypart = nullptr;
  float *logits = nullptr;
  const float* ext = nullptr;  // [*][E] external embedding rows for negative token ids (image patches)
  int max_B = 0, ld_logits = 0;
  // step inputs (int32 [B] each)
  const int *tokens = nullptr, *pos = nullptr, *slot = nullptr, *q_len = nullptr, *q_seq = nullptr;
  const int *logit_idx = nullptr, *block_table = nullptr;
  int max_blocks = 0, bs = 16;
};

class Engine {
 public:
  Config cfg;
  std::vector<Layer> layers;
  QMat tok_embd, lm_head;
  const float *out_norm = nullptr, *out_norm_b = nullptr, *lm_bias = nullptr, *inv_freq = nullptr;
  Buffers buf;

  void embed(int B);
  void attn(int i, int B);
  void ffn(int i, int B);
  void head(int n_logits, bool use_idx);
  void forward(int B, int n_logits, bool use_idx);

 private:
  std::vector<float> xn_, tmp_, gu_, att_;  // scratch, grown on demand
  float* dst(int B);                        // resid (tp == 1) or ypart
};

// y[b][n] (ldy) = sum_k W[n][k] x[b][k]  for the B rows of x (ldx), rows [0, N) of W (row_base offset
// for stacked MoE experts). accumulate: y += instead of y =.
void gemm(const QMat& w, long long row_base, int N, const float* x, int ldx, int B, float* y, int ldy,
          bool accumulate);
void dequant_row(const QMat& w, long long row, float* out);  // one full row (K floats)
const char* isa();                                           // "avx512vnni" / "avx2"
int threads();

}  // namespace omxcpu
