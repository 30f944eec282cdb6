// Batch-1 decode: the QKV projection and the attention in ONE launch (Llama family, short context).
//
// Every block is an ordinary int8-chain QKV GEMV block (gemv8_body: one 16-row tile, image + RMS
// partials in, RoPE + paged K/V scatter out) whose q / k / v stores are write-through (sc1). A tile
// belongs to one KV group (G query heads + their K and V head: (G + 2) * 8 tiles); after its stores
// drain, the block takes a ticket on its group's counter, and the block drawing the group's LAST
// ticket runs that group's attention over the paged cache (attn8_core.h attn_group) and writes the
// group's slice of the O projection's int8 image. No block ever waits: the hand-off is a
// last-arriver ticket (MI355X_MICROARCH.md "Valid forms" table row 1: every storing wave
// vmcnt(0) -> workgroup barrier -> one agent-scope add; the last adder reads with sc1 loads).
//
// Why: as separate launches the attention kernel (5.7 us per layer at ~150 keys, profiles/r5_a) is
// pure latency on 64 blocks -- q + block table, then K/V, then the cross-wave merge -- plus its own
// launch boundary, and the O projection after it pays a merge prologue over the split slabs. Here
// the attention runs in the QKV launch's tail on 32 (MHA) blocks while the other blocks drain, and
// O reads a ready int8 image like every other consumer of the chain (gemv8.hip IN_X8).
// Unlike attn8.hip (QKV + attention + O, one block per CU, every block waiting for the attention:
// measured slower than three launches, profiles/r4_decode), the QKV part keeps the standalone
// kernel's geometry and nothing spins.
//
// Covered: B == 1, head dim 128, no sliding window, G = H / H_kv in {1, 4, 8}, <= A8_MAXBT blocks of
// keys (the host fuses only short contexts; attn_group raises the error word past that bound).
// Reference parity: the attention block of llama.cpp's decode graph inside `ollama/ollama`
// (reference pkg/model/pod.go:10-12); numerics vs the fp32 torch twin (tests/test_qkv_attn_gpu.py).
#include "attn8_core.h"
#include "gemv8_body.h"

namespace omx {

// KV group of the 16-row tile starting at virtual row vr (q rows: head / G; k, v rows: their head)
template <int G>
__device__ __forceinline__ int tile_group(int vr, int Eq, int Ekv) {
  if (vr < Eq) return vr / A8_D / G;
  if (vr < Eq + Ekv) return (vr - Eq) / A8_D;
  return (vr - Eq - Ekv) / A8_D;
}

// blocks [0, gxa): P.A rows (q,k, or q,k,v when fused); blocks [gxa, grid): P.B rows (v)
template <int QA, int QB, int G>
__global__ __launch_bounds__(GEMV_NT) void qkv_attn_kernel(Attn8Params P, int gxa) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bx = blockIdx.x;
  int vr;
  if (bx < gxa) {
    gemv8_body<QA, 1, 1, 1, IN_X8_RMS, 0, EM_NONE, true, 1>(P.A, bx);
    vr = bx * 16 + P.A.row_offset;
  } else {
    if constexpr (QB != 0) gemv8_body<QB, 1, 1, 1, IN_X8_RMS, 0, EM_NONE, true, 1>(P.B, bx - gxa);
    vr = (bx - gxa) * 16 + P.B.row_offset;
  }
  const int g = tile_group<G>(vr, P.A.Eq, P.A.Ekv);
  constexpr unsigned TPG = (G + 2) * A8_TPH;  // tiles per KV group
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 q / k / v stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(P.sync + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == TPG - 1;
    if (s_last) __hip_atomic_store(P.sync + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  }
  __syncthreads();  // also: the GEMV body's LDS image is dead, attn_group reuses smem
  if (s_last) attn_group<G>(P, g, smem);
}

namespace {

template <int QA, int QB, int G>
void launch_qa(const Attn8Params& P, int gxa, int gxb, size_t lds, hipStream_t s) {
  count_launch(LC_QKV_ATTN);
  hipLaunchKernelGGL((qkv_attn_kernel<QA, QB, G>), dim3(gxa + gxb), dim3(GEMV_NT), lds, s, P, gxa);
}

template <int QA, int QB>
bool qa_g(const Attn8Params& P, int gxa, int gxb, size_t lds, hipStream_t s) {
  switch (P.H / P.Hkv) {
    case 1: launch_qa<QA, QB, 1>(P, gxa, gxb, lds, s); return true;
    case 4: launch_qa<QA, QB, 4>(P, gxa, gxb, lds, s); return true;
    case 8: launch_qa<QA, QB, 8>(P, gxa, gxb, lds, s); return true;
    default: return false;
  }
}

bool qtype_ok(int q) { return q == QT_Q4_K || q == QT_Q6_K || q == QT_Q4_0 || q == QT_Q8_0 || q == QT_Q5_K; }

}  // namespace

bool qkv_attn(const GemvParams& A, const GemvParams& B, const AttnParams& At, void* img, void* sync, hipStream_t s) {
  if (!sync || !img || At.kv8 || A.kv8 || A.B != 1 || !A.x8 || !A.x8_stat || A.epi != EPI_QKV || A.emit8 || A.D != A8_D ||
      At.D != A8_D || At.window > 0 || At.NQ != 1 || A.w.K % 64 || A.w.K > 8192 || At.H % At.n_kv ||
      At.n_kv > 64 || A.row_offset != 0 || !qtype_ok(A.w.qtype))
    return false;
  const int G = At.H / At.n_kv;
  if (G != 1 && G != 4 && G != 8) return false;
  const bool fused = B.w.s0 == nullptr;
  const int Eq = At.H * A8_D, Ekv = At.n_kv * A8_D;
  if (A.Eq != Eq || A.Ekv != Ekv) return false;
  if (fused && A.w.N != Eq + 2 * Ekv) return false;
  if (!fused && (A.w.N != Eq + Ekv || B.w.N != Ekv || B.w.K != A.w.K || B.row_offset != Eq + Ekv || B.x8 != A.x8 ||
                 !qtype_ok(B.w.qtype)))
    return false;
  // one super-block per lane, no K split (the gemv8 geometry for K <= 4096)
  if (((A.w.K + 255) / 256 + 15) / 16 != 1) return false;
  Attn8Params P{};
  P.A = A;
  P.B = B;
  P.O.x8 = img;         // attn_group writes the O projection's input image here
  P.O.w.K = At.H * A8_D;
  P.block_table = At.block_table;
  P.max_blocks = At.max_blocks;
  P.q_seq = At.q_seq;
  P.q_len = At.q_len;
  P.scale = At.scale;
  P.H = At.H;
  P.Hkv = At.n_kv;
  P.sync = (unsigned*)sync + 16;  // [0, Hkv) group tickets, [66] error word (shared layout with attn8)
  const int gxa = (A.w.N + 15) / 16, gxb = fused ? 0 : (B.w.N + 15) / 16;
  const size_t img_lds = x8_bytes(A.w.K) + 32 * 4;
  const size_t att = (size_t)(4 * G * (A8_D + 2) + G * A8_D) * 4 + A8_MAXBT * 4;
  const size_t lds = img_lds > att ? img_lds : att;
  switch (A.w.qtype) {
    case QT_Q4_K:
      if (fused) return qa_g<QT_Q4_K, 0>(P, gxa, gxb, lds, s);
      if (B.w.qtype == QT_Q6_K) return qa_g<QT_Q4_K, QT_Q6_K>(P, gxa, gxb, lds, s);
      if (B.w.qtype == QT_Q4_K) return qa_g<QT_Q4_K, QT_Q4_K>(P, gxa, gxb, lds, s);
      return false;
    case QT_Q5_K:
      if (fused) return qa_g<QT_Q5_K, 0>(P, gxa, gxb, lds, s);
      if (B.w.qtype == QT_Q6_K) return qa_g<QT_Q5_K, QT_Q6_K>(P, gxa, gxb, lds, s);
      return false;
    case QT_Q4_0:
      if (fused) return qa_g<QT_Q4_0, 0>(P, gxa, gxb, lds, s);
      return false;
    case QT_Q8_0:
      if (fused) return qa_g<QT_Q8_0, 0>(P, gxa, gxb, lds, s);
      return false;
    default: return false;
  }
}

}  // namespace omx
