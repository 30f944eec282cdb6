// Fused output epilogues shared by the decode GEMV (gemv.hip) and the prefill MFMA GEMM (gemm.hip):
// one output element (batch row bb, virtual matrix row vn) with its pair partner (row vn ^ 1) for
// the epilogues that combine adjacent rows (SiLU-GLU gate/up, RoPE pairs).
#pragma once
#include "common.h"
#include "ops.h"

namespace omx {

// `zsel`: MoE selected-expert slot of this output (blockIdx.z in the GEMV), 0 otherwise.
// One epilogue kind per instantiation: kernels that unroll many outputs per thread (gemm_dq.hip)
// dispatch on P.epi once and keep the unrolled body small.
template <int E>
__device__ __forceinline__ void epi_apply_t(const GemvParams& P, int bb, int vn, float v, float pv, int zsel) {
  if constexpr (E == EPI_STORE) {
    if (P.bias) v += P.bias[vn];
    P.y[(long long)bb * P.ldy + vn] = v;
  } else if constexpr (E == EPI_ADD) {
    if (P.bias) v += P.bias[vn];
    if (P.expert_w) v *= P.expert_w[bb * P.n_sel + zsel];
    float* dst = P.y + (long long)bb * P.ldy + vn;
    if (P.expert_ids && P.n_sel > 1) atomicAdd(dst, v);
    else *dst += v;
  } else if constexpr (E == EPI_GELU) {
    if (P.bias) v += P.bias[vn];
    P.y[(long long)bb * P.ldy + vn] = gelu_tanh(v);
  } else if constexpr (E == EPI_GELU_ERF) {
    if (P.bias) v += P.bias[vn];
    P.y[(long long)bb * P.ldy + vn] = 0.5f * v * (1.f + erff(v * 0.70710678f));
  } else if constexpr (E == EPI_QGELU) {
    if (P.bias) v += P.bias[vn];
    P.y[(long long)bb * P.ldy + vn] = v / (1.f + __expf(-1.702f * v));
  } else if constexpr (E == EPI_GLU) {
    if ((vn & 1) == 0)  // even row = gate, odd row = up
      P.y[(long long)bb * P.ldy + (long long)zsel * P.y_sel_stride + vn / 2] = silu(v) * pv;
  } else if constexpr (E == EPI_GEGLU) {  // Gemma: gelu(gate) * up
    if ((vn & 1) == 0)
      P.y[(long long)bb * P.ldy + (long long)zsel * P.y_sel_stride + vn / 2] = gelu_tanh(v) * pv;
  } else {  // EPI_QKV
    const int Eq = P.Eq, Ekv = P.Ekv, D = P.D;
    int which, hh, d;
    if (vn < Eq) { which = 0; hh = vn / D; d = vn % D; }
    else if (vn < Eq + Ekv) { which = 1; hh = (vn - Eq) / D; d = (vn - Eq) % D; }
    else { which = 2; hh = (vn - Eq - Ekv) / D; d = (vn - Eq - Ekv) % D; }
    if (P.bias) v += P.bias[vn];
    float out = v;
    if (which < 2 && d < P.n_rot) {
      if (P.bias) pv += P.bias[vn ^ 1];
      const float ang = (float)P.pos[bb] * P.inv_freq[d >> 1];
      float sn, cs;
      sincosf(ang, &sn, &cs);
      out = (d & 1) ? (pv * sn + v * cs) : (v * cs - pv * sn);
    }
    if (which == 0) {
      P.y[(long long)bb * P.ldy + vn] = out;
    } else {
      const int slot = P.slot[bb];
      const long long blk = slot / P.bs, off = slot % P.bs;
      const long long idx = ((blk * P.n_kv + hh) * P.bs + off) * (P.Dc > 0 ? P.Dc : D) + d;
      // two explicit stores: a pointer select here is lowered to an indexed scratch array
      if (which == 1) kv_store(P.kc, idx, out, P.kv8);
      else kv_store(P.vc, idx, out, P.kv8);
    }
  }
}

__device__ __forceinline__ void epi_apply(const GemvParams& P, int bb, int vn, float v, float pv, int zsel) {
  switch (P.epi) {
    case EPI_STORE: epi_apply_t<EPI_STORE>(P, bb, vn, v, pv, zsel); break;
    case EPI_ADD: epi_apply_t<EPI_ADD>(P, bb, vn, v, pv, zsel); break;
    case EPI_GELU: epi_apply_t<EPI_GELU>(P, bb, vn, v, pv, zsel); break;
    case EPI_GLU: epi_apply_t<EPI_GLU>(P, bb, vn, v, pv, zsel); break;
    case EPI_GEGLU: epi_apply_t<EPI_GEGLU>(P, bb, vn, v, pv, zsel); break;
    case EPI_QKV: epi_apply_t<EPI_QKV>(P, bb, vn, v, pv, zsel); break;
    case EPI_GELU_ERF: epi_apply_t<EPI_GELU_ERF>(P, bb, vn, v, pv, zsel); break;
    case EPI_QGELU: epi_apply_t<EPI_QGELU>(P, bb, vn, v, pv, zsel); break;
  }
}

}  // namespace omx
