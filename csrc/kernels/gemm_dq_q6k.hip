// QT_Q6_K instantiation of the stream-order dequant prefill GEMM (gemm_dq_impl.h)
#include "gemm_dq_impl.h"

namespace omx {

void run_dq_q6k(const GemvParams& P, f16* xp, int Kp, hipStream_t s) { run_dq<QT_Q6_K>(P, xp, Kp, s); }

}  // namespace omx
