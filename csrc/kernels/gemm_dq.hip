// Stream-order dequant prefill GEMM: dispatcher and knobs. Kernels and the tile x split-K chooser are in
// gemm_dq_impl.h (design notes there), instantiated once per weight type in gemm_dq_<type>.hip.
#include <cstdlib>

#include "common.h"
#include "ops.h"

namespace omx {

int g_dq_enable = -1;  // -1: OMX_GEMM_DQ (default on), read once
int g_dq_cfg = -2;     // OMX_DQ_CFG: force tile config 0..3 (microbenchmarks); -2 = not read yet
int g_dq_sk = 0;       // > 0: force the split-K factor (microbenchmarks, set_dq_tuning)
int g_dq_dbg = 0;      // OMX_DQ_DBG=1: no operand reloads after the first K step (timing probe only)
int g_dq_ring = 1;     // OMX_DQ_RING (default 1): the register-ring kernel (gemm_dq_impl.h), 0 = the glds one

void run_dq_q4k(const GemvParams& P, f16* xp, int Kp, hipStream_t s);  // gemm_dq_q4k.hip
void run_dq_q5k(const GemvParams& P, f16* xp, int Kp, hipStream_t s);  // gemm_dq_q5k.hip
void run_dq_q6k(const GemvParams& P, f16* xp, int Kp, hipStream_t s);  // gemm_dq_q6k.hip
void run_dq_q40(const GemvParams& P, f16* xp, int Kp, hipStream_t s);  // gemm_dq_q40.hip
void run_dq_q80(const GemvParams& P, f16* xp, int Kp, hipStream_t s);  // gemm_dq_q80.hip
void run_dq_f16(const GemvParams& P, f16* xp, int Kp, hipStream_t s);  // gemm_dq_f16.hip

bool dq_gemm_enabled() {
  if (g_dq_enable < 0) {
    const char* e = getenv("OMX_GEMM_DQ");
    g_dq_enable = e ? atoi(e) != 0 : 1;
  }
  if (g_dq_cfg == -2) {
    const char* c = getenv("OMX_DQ_CFG");
    g_dq_cfg = c ? atoi(c) : -1;
    const char* d = getenv("OMX_DQ_DBG");
    g_dq_dbg = d ? atoi(d) : 0;
    const char* r = getenv("OMX_DQ_RING");
    g_dq_ring = r ? atoi(r) : g_dq_ring;
  }
  return g_dq_enable != 0;
}

void set_dq_gemm(int on) { g_dq_enable = on ? 1 : 0; }

void set_dq_ring(int on) {
  dq_gemm_enabled();  // env defaults read first, then overridden
  g_dq_ring = on ? 1 : 0;
}

void set_dq_tuning(int cfg, int sk) {
  dq_gemm_enabled();  // env defaults read first, then overridden
  g_dq_cfg = cfg;
  g_dq_sk = sk;
}

bool dq_gemm(const GemvParams& P, hipStream_t s) {
  if (!dq_gemm_enabled() || P.B < 128 || !P.xws || P.expert_ids || P.moe_tiles) return false;
  const int qt = P.w.qtype;
  if (qt != QT_Q4_K && qt != QT_Q5_K && qt != QT_Q6_K && qt != QT_Q4_0 && qt != QT_Q8_0 && qt != QT_F16) return false;
  const int Kp = ((P.w.K + 255) >> 8) * 256;
  const long long cap = P.xws_elems ? P.xws_elems : (long long)P.B * P.w.K;
  if ((long long)P.B * Kp > cap) return false;
  f16* xp = (f16*)P.xws;
  count_launch(LC_DQ_GEMM);
  switch (qt) {
    case QT_Q4_K: run_dq_q4k(P, xp, Kp, s); break;
    case QT_Q5_K: run_dq_q5k(P, xp, Kp, s); break;
    case QT_Q6_K: run_dq_q6k(P, xp, Kp, s); break;
    case QT_Q4_0: run_dq_q40(P, xp, Kp, s); break;
    case QT_F16: run_dq_f16(P, xp, Kp, s); break;
    default: run_dq_q80(P, xp, Kp, s); break;
  }
  return true;
}

}  // namespace omx
