// Native step executor: the per-token launch sequence of a transformer on gfx950 kernels.
// Python owns the device memory (torch tensors) and hands raw pointers in; the executor only
// enqueues kernels on a stream, so a whole step is capturable into one hipGraph.
// Reference parity: replaces the llama.cpp runner inside `ollama/ollama` (reference
// pkg/model/pod.go:10-12; SURVEY.md §3.4 hot loop).
#pragma once
#include <hip/hip_runtime_api.h>

#include <vector>

#include "../kernels/ops.h"

namespace omx {

struct ExecConfig {
  int arch = 0;          // 0 llama-family (llama/mistral/mixtral), 1 phi2
  int E = 0, H = 0, Hkv = 0, D = 0, n_rot = 0, F = 0, n_layer = 0, V = 0;  // per-rank (TP) sizes
  int Dc = 0;            // KV cache row stride (head dim padded to a multiple of 16; 0 = D)
  int kv8 = 0;           // fp8 e4m3 KV cache (OMX_KV_CACHE_TYPE=fp8), else fp16
  float eps = 1e-5f;
  int n_expert = 0, n_expert_used = 0;
  int window = 0;
  int tp = 1;            // >1: O/down projections write partial sums to ypart (caller all-reduces)
  float embed_scale = 1.f;  // token embeddings x this (Gemma: sqrt(E))
  int glu_act = 0;          // 0 SiLU-GLU, 1 GELU-GLU (Gemma GeGLU)
  int F_valid = 0;          // FFN width before ffn_down's K padding (weights.py ffn_pad; 0 = F)
};

struct LayerW {
  const float* attn_norm = nullptr;
  const float* attn_norm_b = nullptr;
  const float* ffn_norm = nullptr;
  QMat wqk{};            // q,k rows (and v rows too when qkv_fused)
  QMat wv{};             // v rows when not fused (different quant type)
  int qkv_fused = 1;
  const float* qkv_bias = nullptr;
  QMat wo{};
  const float* bo = nullptr;
  QMat wgu{};            // llama: gate/up rows interleaved; phi2: up
  const float* bup = nullptr;
  QMat wdown{};
  const float* bdown = nullptr;
  QMat router{};         // MoE router [X][E]
  QMat gu_exps{};        // [X][2F][E] interleaved gate/up per expert
  QMat down_exps{};      // [X][E][F]
  void* kc = nullptr;    // fp16 [nblk][Hkv][bs][D]
  void* vc = nullptr;
  // phi2 int8 chain: LayerNorm constants of the two attn_norm consumers (GemvParams::ln_c1 / ln_c2)
  const float* c1_qkv = nullptr;
  const float* c2_qkv = nullptr;
  const float* c1_up = nullptr;
  const float* c2_up = nullptr;
};

struct Workspace {
  float* resid = nullptr;    // [maxB][E]
  float* qbuf = nullptr;     // [maxB][H*D]
  float* abuf = nullptr;     // [maxB][H*D]
  float* hbuf = nullptr;     // [maxB][n_sel][F]
  float* ypart = nullptr;    // [maxB][E] (TP partial sums)
  float* lbuf = nullptr;     // [maxB][E] gathered rows for the LM head
  float* rlogits = nullptr;  // [maxB][X]
  int* eids = nullptr;       // [maxB][n_sel]
  float* ew = nullptr;       // [maxB][n_sel]
  float* attn_ws = nullptr;  // split-K workspace
  int* attn_cnt = nullptr;   // [maxB][H] split arrival tickets (zero-initialised)
  void* x16 = nullptr;       // [maxB][max K] fp16 activations for the prefill MFMA GEMM
  long long x16_elems = 0;
  float* gws = nullptr;      // split-K partial slabs for small-M prefill GEMMs
  int* moe_rows = nullptr;   // [maxB*k] MoE prefill: pairs sorted by expert
  int* moe_tiles = nullptr;  // [(maxB*k/128 + X + 1)*3] expert row tiles
  int* moe_ntiles = nullptr; // [1]
  long long gws_elems = 0;
  const float* ext = nullptr;  // [*][E] external embedding rows (negative token ids), e.g. image patches
  void* w16 = nullptr;       // large-M prefill library GEMM: fp16 dequantised weight [N][K] scratch
  long long w16_elems = 0;
  float* yws = nullptr;      //   and its fp32 output slab [M][N]
  long long yws_elems = 0;
  int max_B = 0;
  int n_splits = 1;
  int defer = 0;             // B == 1: attention leaves n_splits partials, the O GEMV merges them
  // TP decode: one-shot all-reduce over peer-mapped slabs (allreduce.hip). The O / down projections
  // write their partial sums into this rank's slab 0 / 1, the vocab-sharded LM head into slab 2.
  ARParams ar{};
  int ar_on = 0;
  // batched decode chain on the matrix cores (gemv_mfma.hip, 2 <= B <= MB_CHAIN_MAX, tp == 1): fp16
  // activation rows [MB_CHAIN_MAX + 1][ld] (row MB_CHAIN_MAX all zero) and RMS partial slabs
  int mb_ok = 0;             // every dense projection has its layout M copy
  void* xa16 = nullptr;      // fp16(resid * next norm weight) [17][ld_e]
  void* h16 = nullptr;       // fp16 GLU output [17][ld_f]
  void* a16 = nullptr;       // fp16 attention output [17][ld_q]
  float* st[2] = {nullptr, nullptr};  // sum-of-squares partials [E / 16][16] (after O / after down)
  int ld_e = 0, ld_f = 0, ld_q = 0;
  // batch-1 int8 activation chain (gemv8.hip): images of the E-wide (QKV / gate_up / LM head input)
  // and F-wide (down input) activations, RMS partials [E / 16]; x8_ok once every emitter is covered
  void* x8e = nullptr;
  void* x8f = nullptr;
  float* x8st = nullptr;
  float* x8sum = nullptr;    // phi2: per-group sums of the E-wide rows (LayerNorm mean), x8st's layout
  float* kb_ws = nullptr;    // gemv8 K split across blocks: row partials [N][2] and tile tickets (zeroed)
  int* kb_cnt = nullptr;
  int x8_ok = 0;
  int x8_bmax = 1;           // batch rows the chain takes (continuous batching: up to X8_MAX_B)
};
constexpr int MB_CHAIN_MAX = 16;

struct StepInputs {
  int B = 0;
  const int* tokens = nullptr;    // [B]
  const int* pos = nullptr;       // [B]
  const int* slot = nullptr;      // [B]
  const int* q_len = nullptr;     // [B] = pos + 1
  const int* q_seq = nullptr;     // [B] row of block_table
  const int* block_table = nullptr;
  int max_blocks = 0;
  int bs = 16;
  int prefill = 0;                // one sequence, contiguous positions (MFMA flash attention)
  int n_logits = 0;               // rows that need logits
  const int* logit_idx = nullptr; // [n_logits] (null = first n_logits rows)
  float* logits = nullptr;        // [n_logits][V]
  float* full_logits = nullptr;   // TP: [n_logits][ld_full] all-gathered vocab
  int ld_full = 0;
};

class Executor {
 public:
  ExecConfig cfg;
  std::vector<LayerW> layers;
  QMat tok_embd{};
  const float* out_norm = nullptr;
  const float* out_norm_b = nullptr;
  QMat lm_head{};
  const float* lm_bias = nullptr;
  const float* inv_freq = nullptr;
  const float* lm_c1 = nullptr;  // phi2 int8 chain: the LM head's LayerNorm constants (out_norm)
  const float* lm_c2 = nullptr;
  Workspace ws;

  void embed(const StepInputs& in, hipStream_t s);
  void attn_block(int i, const StepInputs& in, hipStream_t s);
  void ffn_block(int i, const StepInputs& in, hipStream_t s);
  void head(const StepInputs& in, hipStream_t s);
  void forward(const StepInputs& in, hipStream_t s);     // tp == 1 only
  void forward_tp(const StepInputs& in, hipStream_t s);  // tp > 1, custom all-reduce (graph-capturable)
  bool ar_fits(int B) const;                             // decode batch B fits the AR slabs
  bool chain_capable() const;                            // every projection takes the fp16 matrix-core chain
  bool x8_capable(int B = 1) const;                               // every emitter of the int8 chain takes gemv8
  StepInputs bound{};                                    // pre-bound step inputs (set_inputs)
  // batched admission (Runner.admit_many): the rows of a prefill step are several sequences' contiguous
  // prompt segments {first row, rows}; attention runs the MFMA flash kernel once per segment. Empty: one
  // sequence (or a decode step). Host-side: admission steps are never graph-captured.
  std::vector<std::pair<int, int>> segments;

 private:
  float* tp_dst(int slab, int B) const;  // where a row-parallel projection leaves its partial sums
  bool chain(const StepInputs& in) const;  // this step runs the fp16 matrix-core decode chain
  bool x8_layer0(const StepInputs& in) const;  // the embed writes layer 0's int8 QKV image
  bool x8(const StepInputs& in) const;     // this step runs the batch-1 int8 activation chain
  bool ln8() const;                        // the phi2 (LayerNorm) form of that chain is set up
  GemvParams o_params(int i, const StepInputs& in) const;         // layer i's O projection GEMV
  GemvParams phi_down_params(int i, const StepInputs& in) const;  // phi2 layer i's ffn_down GEMV
  bool phi_pair(int i, const StepInputs& in) const;               // phi2: O + down as one launch
  int ar_active_ = 0;
};

}  // namespace omx
