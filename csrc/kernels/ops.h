// Host-visible interface of the gfx950 kernels. Plain C++ types only: this header is included by
// the HIP kernel sources (hipcc) and by the torch bindings / executor (host compiler).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#include "qmat.h"

namespace omx {

enum { NORM_NONE = 0, NORM_RMS = 1, NORM_LAYER = 2 };
// EPI_GELU: tanh approximation (Phi-2 / Gemma); EPI_GELU_ERF: exact erf GELU (LLaVA projector, CLIP with
// use_gelu); EPI_QGELU: x * sigmoid(1.702 x) (OpenAI CLIP "quick GELU"). The last two: prefill GEMM only
enum { EPI_STORE = 0, EPI_ADD = 1, EPI_GLU = 2, EPI_GELU = 3, EPI_QKV = 4, EPI_GEGLU = 5, EPI_GELU_ERF = 6, EPI_QGELU = 7 };

struct GemvParams {
  QMat w;
  int B;                       // activation rows
  const float* x;              // [B][ldx] fp32
  int ldx;
  int norm;                    // NORM_*
  const float* norm_w;
  const float* norm_b;
  float eps;
  int epi;                     // EPI_*
  float* y;                    // output / residual (EPI_QKV: q output [B][ldy])
  int ldy;
  const float* bias;           // [virtual N] or null
  int row_offset;              // row index of w's row 0 in the virtual concatenated matrix
  // EPI_QKV
  const int* pos;              // [B]
  const int* slot;             // [B] flat KV slot (block * bs + offset)
  void* kc;                    // fp16 [nblk][n_kv][bs][D] (this layer)
  void* vc;
  const float* inv_freq;       // [n_rot/2]
  int Eq, Ekv, D, n_rot, n_kv, bs;
  int Dc;                      // KV cache row stride (head dim padded to 16 on the GPU; 0 = D)
  int kv8;                     // KV cache elements are fp8 e4m3 (OCP e4m3fn, 1 byte) instead of fp16
  // MoE: blockIdx.z = k-th selected expert of batch row b
  const int* expert_ids;       // [B][n_sel] or null
  const float* expert_w;       // [B][n_sel] routing weights (EPI_ADD scale) or null
  int n_sel;
  int x_per_sel;               // x has one row-block per selected expert (down proj)
  long long x_sel_stride;      // elements between experts' x (within batch row b)
  long long y_sel_stride;      // elements between experts' y (EPI_GLU output)
  // prefill GEMM path: fp16 activation scratch, >= B * K halves (null -> always the GEMV)
  void* xws;
  long long xws_elems;          // its capacity in halves (0: exactly B * K assumed)
  // split-K partial slabs for small-M GEMMs: fp32 [splits][B][N], capacity gws_elems (0 -> no split)
  float* gws;
  long long gws_elems;
  // library GEMM path for large M (gemm.hip gemm_lib, blas.cpp): the weight dequantised once per call
  // into fp16 scratch [N][K], one hipBLASLt fp16 x fp16 -> fp32 GEMM into yws [M][N], then the fused
  // epilogue; null / too small -> the fused dequant MFMA GEMM
  void* w16ws;
  long long w16_elems;
  float* yws;
  long long yws_elems;
  // MoE prefill grouped GEMM (gemm.hip GROUPED): rows are the B*k (token, expert) pairs sorted by
  // expert (moe_sort); x / y rows are in sorted order except that moe_scatter writes output row
  // pair = moe_rows[pos] to token pair / n_sel with routing weight expert_w[pair]
  const int* moe_rows;         // [B*k] sorted position -> pair index (token * k + j)
  const int* moe_tiles;        // [max_tiles][3] {expert, first sorted row, rows}
  const int* moe_ntiles;       // device count of valid tiles
  int moe_max_tiles;
  int moe_gather;              // x row of sorted position pos = moe_rows[pos] / n_sel (else pos)
  int moe_scatter;             // output row of pos = token (EPI_ADD, weighted, atomic) (else pos)
  // deferred attention merge (B == 1 decode): x = acc slabs [merge_S][K], merge_ml = [merge_S][K/D]{m, l};
  // the activation prologue computes x[k] = sum_s e^(m_s - M) acc_s[k] / sum_s e^(m_s - M) l_s
  int merge_S;                 // 0 = x is the activation itself
  const float* merge_ml;
  int merge_D;                 // head dim (elements per {m, l} pair)
  // timeline probe (scripts/gemv_timeline.py): per block 4 x s_memrealtime (100 MHz) at entry,
  // prologue done, first tile computed, exit; null in production
  unsigned long long* dbg_ts;
  int xfirst;                  // activations waited for before any weight load (GemvTuning::xfirst)
  // batched matrix-core decode chain (gemv_mfma.hip, 2 <= B <= 16; null = unused):
  const void* x16;             // consumer: activations already in fp16 [B][ld16] (times norm_w when norm = RMS)
  int ld16;
  int zrow16;                  //   index of an all-zero row of x16 (>= B): the A-operand lanes of rows >= B
  const float* xstat;          // consumer: per-row sum-of-squares partials [xstat_n][16] of the un-normed x
  int xstat_n;                 //   (RMSNorm scale rsqrt(sum / K + eps) applied to the outputs)
  void* emit16;                // producer (EPI_ADD): also writes fp16(new_resid * emit_nw) [B][ld_emit]
  int ld_emit;
  const float* emit_nw;
  float* emit_stat;            //   and its per-16-row-tile sum-of-squares partials [tiles][16]
  // fp16 range guard of the emission: row b is stored times 2^-e_b, with e_b from the RMS of the residual
  // BEFORE the add (emit_prev: that row's partials [B][emit_prev_n], the previous emission's slab), and
  // 2^e_b goes to emit_scale[b]; the consumer multiplies its outputs by xscale[b] (= that emit_scale).
  // e_b = 0 while the old RMS is below 8, so ordinary rows are stored exactly as without it.
  const float* emit_prev;
  int emit_prev_n;
  float* emit_scale;
  const float* xscale;
  // cheaper form used by the engine: the consumer that reduces the old row's partials for its RMSNorm
  // anyway (QKV, gate_up) writes e_b to rexp_out[b]; the producer reads rexp_in[b] instead of emit_prev
  float* rexp_out;
  const float* rexp_in;
  void* y16;                   // EPI_GLU / EPI_GEGLU: fp16 output [B][ld16y] instead of y
  int ld16y;
  // batch-1 int8 activation chain (gemv8.hip): the producer of a GEMV's input writes it already
  // int8-quantised per 16-element group, in the consumer's LDS image layout (x8_bytes(K)); an RMSNorm'd
  // input carries (x * norm_w) and per-group sum-of-squares partials of the un-normed x, and the
  // consumer scales its outputs by rsqrt(sum / K + eps)
  const void* x8;              // consumer: activation image (null = fp32 x / merge prologue)
  const float* x8_stat;        //   RMS partials [K / 16] (null = no norm)
  void* emit8;                 // producer: image of this GEMV's output (EPI_ADD: new residual * emit8_nw;
  const float* emit8_nw;       //   EPI_GLU / EPI_GEGLU: the GLU output)
  float* emit8_stat;           //   EPI_ADD: per-16-row sum-of-squares partials of the new residual
  int k_valid;                 // K columns holding weights (0 = K): ffn_down's zero padding past it is not
                               // streamed by the int8-chain GEMV (gemv8_body.h)
  int emit8_k;                 //   EPI_GLU: K of the consumer's image (0 = N / 2; larger when ffn_down's K is
                               //   padded: the image slots past N / 2 stay zero)
  int dbg8;                    // microbenchmarks only (scripts/bench_gemv8.py): 1 = gemv8 memory path alone
                               // (weights loaded and folded, no dot products); 0 in production
  // LayerNorm'd consumers (Phi-2 int8 chain, batch 1): the image holds x * ln_w and the producer also
  // writes per-group sums of x (x8_sum, same layout as x8_stat). With mu = sum / K and
  // rstd = rsqrt(sumsq / K - mu^2 + eps), W . LN(x) = rstd * (W . (x * ln_w) - mu * c1) + c2 for the
  // per-row constants c1 = W . ln_w, c2 = W . ln_b (computed at load: engine/weights.py ln_consts)
  const float* x8_sum;         // consumer: per-group sums of x (non-null = LayerNorm input)
  const float* ln_c1;          //   [N] W . ln_w
  const float* ln_c2;          //   [N] W . ln_b (+ nothing else: the GEMV's own bias stays in `bias`)
  float* emit8_sum;            // producer (EPI_ADD): per-16-row sums of the new residual (LN consumers)
  // K split across blocks (gemv8.hip, batch 1, K-split launches of < 256 row tiles): kb blocks share a tile,
  // each streams 1 / kb of K; row partials meet in kb_ws [N][kb] and the last block of a tile (agent-scope
  // ticket in kb_cnt[tile], zero-initialised, re-armed) sums them and runs the epilogue. Set by gemv8
  float* kb_ws;
  int* kb_cnt;
  int kb;
};
// int8 activation image of a K-wide row (gemv8.hip): [slots] i32x4 codes + [slots] {scale, scale * sum}
// with one pad slot per 256-element super-block and a trailing dummy slot (the GEMV's LDS layout)
inline int x8_slots(int K) { return ((((K + 255) / 256) * 17 + 1) + 1) & ~1; }
inline size_t x8_bytes(int K) { return (size_t)x8_slots(K) * 24; }
inline int x8_stat_ld(int K) { return ((K >> 4) + 3) & ~3; }  // RMS-partial floats per batch row
// batch-1 decode GEMV on the int8 activation chain; false = not covered (caller takes gemv.hip)
bool gemv8(const GemvParams& P, hipStream_t s);
bool gemv8_2(const GemvParams& A, const GemvParams& B, hipStream_t s);  // q,k + v rows, one launch
bool gemv8_supported(const GemvParams& P);
// Phi-2's parallel block, batch 1 (gemv8_pair.hip): the attention output projection O (merge slabs or plain
// fp32 input) and ffn_down (int8 image) add into the same residual row in ONE launch, which then emits the
// next LayerNorm'd image (sums + sums of squares). D: the down GEMV's params (EPI_ADD + emission), O: the
// O GEMV's (EPI_ADD, same y). false = not covered (the caller launches both)
bool gemv8_pair(const GemvParams& D, const GemvParams& O, hipStream_t s);
bool gemv8_pair_supported(const GemvParams& D, const GemvParams& O);
void set_gemv8_kb(int mode);  // K split across blocks: 0 auto (< 256 row tiles), 1 off, 2 wherever covered
void set_gemv8_geo(int nsb, int ks);  // microbenchmarks: force (NSB, KS) of K-split plain-image launches
struct AttnParams;

// y = epi(W x): the quantised GEMV for small B (decode), the MFMA dequant GEMM for B >= GEMM_MIN_B
// when an fp16 activation workspace is given (prefill); same epilogues either way.
void gemv(const GemvParams& P, hipStream_t s);
bool gemv_merge_supported(int B, int K, int D, int S);
bool gemv8_merge_supported(int K, int D, int S);  // the same merge in the int8-chain O GEMV (K <= 8192)
// two GEMVs over the same x (same K, RMS norm prologue) in one launch when B == 1, else two launches
void gemv2(const GemvParams& A, const GemvParams& B, hipStream_t s);
constexpr int GEMM_MIN_B = 16;
// prefill rows from which the library GEMM path is taken (0 = never); OMX_GEMM_LIB_MIN_M overrides
void set_gemm_lib_min_m(int m);
int gemm_lib_min_m();
// MoE prefill: routed (token, expert) pairs from which each expert's GEMM runs on hipBLASLt over its
// dequantised weights (gemm.hip moe_gemm_lib; 0 = never, the grouped tile GEMM). OMX_MOE_LIB_MIN_M
void set_moe_lib_min_m(int m);
int moe_lib_min_m();
// D[M][N] (fp32, row-major) = X[M][K] . W[N][K]^T, X and W fp16 row-major, on hipBLASLt; false when
// no algorithm fits (the caller falls back)
// m_cap: rows of x16 / d the buffers hold (>= M); when the M-bucket's algorithm does not accept M
// exactly, the GEMM runs the bucket's rows (<= m_cap) instead of paying a heuristic query
bool blas_gemm_tn(const void* w16, const void* x16, float* d, int M, int N, int K, void* ws, size_t ws_bytes,
                  hipStream_t s, int m_cap = 0);
// plan (heuristic algorithm) every power-of-two M bucket from min_M to max_M ahead of serving: the first
// GEMM of a bucket would otherwise pay the heuristic query inside a request's TTFT
void blas_prepare(int N, int K, int min_M, int max_M, size_t ws_bytes);
bool blas_plan_ok(int M, int N, int K, size_t ws_bytes, int m_cap = 0);  // a plan exists (created if needed)
// batched decode GEMV on the matrix cores (gemv_mfma.hip): 2 <= B <= 16 rows, needs the layout M
// copy (QMat::mt) built by repack_m; false = shape not covered (the caller takes the int8 GEMV)
bool gemv_mb(const GemvParams& P, hipStream_t s);
bool gemv_mb2(const GemvParams& A, const GemvParams& B, hipStream_t s);  // two matrices, one launch
bool gemv_mb_supported(const GemvParams& P);
void set_mb_enable(int on);
void set_mb_tuning(int dbg, int bpc);  // microbenchmark variants (gemv_mfma.hip DBG), blocks per CU
bool mb_enabled();
size_t mfma_layout_bytes(int qtype, int N, int K);  // 0 = no layout M for this quant type
void repack_m(const QMat& w, void* out, hipStream_t s);
bool gemm_eligible(const GemvParams& P);
void gemm(const GemvParams& P, hipStream_t s);
// stream-order dequant MFMA GEMM (gemm_dq.hip): M >= 128, dense v2 matrices; false = not covered
bool dq_gemm(const GemvParams& P, hipStream_t s);
bool dq_gemm_enabled();
void set_dq_gemm(int on);
void set_dq_ring(int on);  // 1: the register-ring dq kernel (gemm_dq_impl.h), 0: the glds kernel
void set_dq_tuning(int cfg, int sk);  // microbenchmarks: force tile config (-1 auto) and split-K (0 auto)
void gemm_finalize(const GemvParams& P, int sk, hipStream_t s);  // sums sk split-K slabs + epilogue

// launch-shape knobs for the decode GEMV (tuned on MI355X; see scripts/bench_gemv.py)
struct GemvTuning {
  int blocks_per_cu = 4;  // persistent-grid cap = 256 CUs x this (scripts/bench_gemv.py sweep)
  int rows = 1;           // rows per 16-lane row group in B == 1 launches (1 or 2)
  int debug = 0;          // microbenchmark-only kernel variants (gemv.hip DBG)
  int ks = 0;             // in-block K split of the flight kernel: 0 = auto, 1 = off, 2..4 = forced
  int xfirst = 0;         // 1: decode GEMVs wait for their activations before streaming weights
  int xbar = 0;           // 1: batch-1 decode GEMVs as x-barrier launches, one block per CU (gemv.hip XB)
};
extern GemvTuning g_tune;
void set_gemv_tuning(int blocks_per_cu, int rows, int debug, int ks = -1, int xfirst = -1, int xbar = -1,
                     int stream = -1, int stream_bpc = -1, int pf = -1, int ws = -1);

// Dequantize rows of a repacked matrix (embedding gather / fp16 copies)
// rows[i] < 0: row -(rows[i] + 1) of ext [*][w.K] (external embeddings, e.g. image patches)
// img8 / img_nw / img_stat (optional, the int8 decode chain): the gathered rows also go out as layer 0's
// QKV input image (x8_bytes(K) per row: int8(row * img_nw) per 16-group + RMS partials, x8_stat_ld(K)
// floats per row), exactly what the residual-adding producers emit for the later layers
// img_sum (optional): per-group sums of the rows too, for a LayerNorm'd consumer (GemvParams::x8_sum)
void embed_rows(const QMat& w, const int* rows, int n, float* out, int ldo, hipStream_t s, float scale = 1.f,
                const float* ext = nullptr, float* stat = nullptr, void* img8 = nullptr, const float* img_nw = nullptr,
                float* img_stat = nullptr, float* img_sum = nullptr);
// rows [row0, row0 + w.N) of w (an expert's slice of a stacked MoE matrix); perm: prep_x16 K order
void dequant_f16(const QMat& w, void* out_f16, hipStream_t s, int perm = 0, long long row0 = 0);

struct AttnParams {
  const float* q;              // [NQ][ldq] fp32 (roped)
  int ldq;
  const void* kc;              // fp16 [nblk][n_kv][bs][D]
  const void* vc;
  const int* block_table;      // [nseq][max_blocks]
  int max_blocks;
  const int* q_seq;            // [NQ] sequence row of each query (null -> identity)
  const int* q_len;            // [NQ] visible keys (= pos + 1)
  int NQ, H, n_kv, D, bs;       // D: KV cache row stride (the kernel's head dim, a multiple of 16)
  int Dv;                      // valid head dim (<= D; q / out head stride): Orca Mini D = 100 in 112 (0 = D)
  float scale;
  int window;                  // sliding window (0 = none)
  float* out;                  // [NQ][ldo] fp32
  int ldo;
  void* out16;                 // optional fp16 copy [NQ][ldo] (the batched matrix-core O projection reads it)
  float* ws;                   // split workspace: [NQ][H][S][D + 2] fp32
  int n_splits;                // <= 64
  int* counters;               // [NQ][H] arrival tickets (one per block row), zero before first use (self re-arming)
  int prefill;                 // all NQ queries: one sequence, contiguous positions (MFMA flash path)
  int kps;                     // target keys per split (0 -> g_attn_kps)
  int defer;                   // write exactly n_splits unmerged partials (attention_ws_floats layout
                               // [NQ][S][H*D] then [NQ][S][H][2] {m, l}); the consumer merges them
  int kv8;                     // kc / vc hold fp8 e4m3 (OCP e4m3fn) instead of fp16
};
void attention_decode(const AttnParams& P, hipStream_t s);
size_t attention_ws_floats(int NQ, int H, int D, int n_splits);
extern int g_attn_kps;  // decode keys per flash-decode split (scripts/bench_attn.py sweep)
void set_attn_tuning(int kps, int hpb = -1);

struct SampleParams {
  const float* logits;         // [B][V] (modified in place by penalties)
  int B, V, ld;
  const float* temperature;    // [B]
  const int* top_k;            // [B]
  const float* top_p;          // [B]
  const float* min_p;          // [B]
  const float* repeat_penalty; // [B]
  const float* presence_penalty;   // [B]
  const float* frequency_penalty;  // [B]
  int* history;                // [B][hist_cap] ring of recent tokens
  int* hist_count;             // [B] tokens seen so far (ring write index)
  int hist_cap;
  const int* repeat_last_n;    // [B]
  const unsigned long long* seed;  // [B]
  int* step;                   // [B] RNG counter, incremented per sample
  int* out;                    // [B] sampled token
  float* out_logprob;          // [B] or null
  // multi-block path (null = single-block kernel): candidate lists [B][ceil(V/1024)][2][64] and
  // per-row tickets [B] (zero-initialised; re-armed by the kernel)
  float* ws = nullptr;
  int* counters = nullptr;
  // optional error word: set to 1 when a row's choice was out of range (non-finite logits); the id
  // itself is clamped to 0 so the next step's embedding read stays in bounds, the host fails the request
  int* err = nullptr;
  // optional decode feedback (null fb_step = none): the row's finishing lane also feeds the token back
  // (feedback.h) -- token into the step block, host ring (row 0), advance to the next position -- so a
  // decode step has no separate feedback launch
  int* fb_step = nullptr;
  int fb_ld = 0, fb_max_blocks = 0, fb_bs = 0, fb_ring = 0;
  const int* fb_block_table = nullptr;
  int* fb_host_ring = nullptr;
  int fb_sysfence = 1;           // system-scope fence after the host-ring store (feedback.h; the runner
                                 // passes 0: its host reads a slot only after the step's event)
};
constexpr int SAMPLE_WS_FLOATS_PER_ROW(int V) { return ((V + 1023) / 1024) * 2 * 64; }
void sample(const SampleParams& P, hipStream_t s);
void argmax(const float* logits, int B, int V, int ld, int* out, hipStream_t s);

void moe_route(const float* logits, int B, int X, int k, int* ids, float* w, hipStream_t s);
// fused RMSNorm + router logits + top-k softmax (P.w = router [X <= 64][K], P.x = resid, P.norm_w)
bool moe_router(const GemvParams& P, int k, int* ids, float* w, hipStream_t s);  // false: shape not covered
void gather_rows(const float* x, int ld, const int* idx, int rows, int n, float* out, hipStream_t s);
void moe_sort(const int* eids, int n_pairs, int X, int* rows, int* tiles, int* n_tiles, int tile_m, hipStream_t s);
// grouped dequant GEMM over expert-homogeneous row tiles (P.moe_* set; P.B = number of pairs)
void moe_gemm(const GemvParams& P, hipStream_t s);
// MoE prefill on hipBLASLt: one dequant + library GEMM per expert over its contiguous sorted rows
// (host counts from moe_sort's order: ascending expert, counts[e] rows each), the grouped-GEMM
// epilogue (GLU in sorted order / routing-weighted atomic scatter) in the finalize pass; false = shape
// or workspace not covered (the caller runs moe_gemm)
bool moe_gemm_lib(const GemvParams& P, const int* counts, int X, hipStream_t s);
constexpr int MOE_TILE_M = 128;

// One-shot all-reduce / all-gather over peer-mapped (hipIpc) slabs for TP decode (allreduce.hip)
constexpr int AR_MAX_RANKS = 8;
constexpr int AR_MAX_BLOCKS = 64;
constexpr int AR_SLABS = 3;  // call sites rotate over 3 slabs: one barrier per call suffices
struct ARParams {
  float* data[AR_MAX_RANKS];      // rank r's slab buffer [AR_SLABS][slab_floats] (peer-mapped for r != rank)
  unsigned* flags[AR_MAX_RANKS];  // rank r's flags [AR_MAX_BLOCKS][AR_MAX_RANKS] (uncached, peer-mapped)
  unsigned* epoch;                // this rank's per-block barrier counters [AR_MAX_BLOCKS] (zeroed once)
  int* err;                       // this rank's error word: 1 + peer that never arrived (0 = ok)
  int* err_host;                  // host-mapped mirror of err (null: none); the host polls it without a HIP call
  int rank, world;
  long long slab_floats;
  unsigned long long timeout_ticks;  // 100 MHz wall-clock ticks a barrier may wait
};
// y[0:n] += sum_r slab_r[slab][0:n]  (n % 4 == 0), same bits on every rank
void ar_allreduce_add(const ARParams& P, int slab, float* y, int n, hipStream_t s);
// the same, then the new residual rows b < B (E each) are emitted as the int8 chain's image of
// (y * nw) + RMS partials (gemv8.hip consumer layout, row b at b * x8_bytes(E)); false = not covered
bool ar_allreduce_add_emit(const ARParams& P, int slab, float* y, int E, int B, void* img, const float* nw, float* stat,
                           hipStream_t s);
// out[row][r * n_local + j] = slab_r[slab][row * n_local + j]
void ar_allgather(const ARParams& P, int slab, float* out, int rows, int n_local, int ld_out, hipStream_t s);

// Launch counters: which kernel family a host call actually enqueued (a tested path must not silently
// become another one -- e.g. dq_gemm() declining and gemm() taking the old tile kernel). Counted on
// the host per enqueue (a captured graph counts at capture); tests reset, run, and assert.
enum {
  LC_DQ_GEMM = 0,    // gemm_dq.hip stream-order MFMA prefill GEMM
  LC_GEMM_TILE,      // gemm.hip 128 x 128 tile GEMM (< 128 rows, or a declined dq shape)
  LC_GEMM_LIB,       // hipBLASLt path (OMX_GEMM_LIB_MIN_M)
  LC_GEMV8_ROW1,     // gemv8.hip int8 chain, one row
  LC_GEMV8_ROWS,     // gemv8.hip int8 chain, 2..4 batched rows
  LC_GEMV8_DUAL,     // gemv8.hip q,k + v dual launch
  LC_GEMV_MB,        // gemv_mfma.hip layout-M matrix-core batched GEMV (single or dual)
  LC_GEMV_FLIGHT,    // gemv.hip / gemv_batch.hip fp32-prologue GEMVs
  LC_ATTN_DECODE,    // attention.hip split flash-decode kernel
  LC_ATTN_PREFILL,   // attention.hip MFMA flash prefill
  LC_GEMV8_PAIR,     // gemv8_pair.hip Phi-2 O + ffn_down in one launch
  LC_N
};
void count_launch(int which);
long long launch_count(int which);
void reset_launch_counts();

// small elementwise helpers
void add_inplace(float* y, const float* x, long long n, hipStream_t s);
void widen_q6k(const QMat& w, void* out, hipStream_t s);  // out: N * SB * 256 bytes
void rmsnorm(const float* x, const float* w, float eps, int rows, int n, float* out, hipStream_t s);

}  // namespace omx
