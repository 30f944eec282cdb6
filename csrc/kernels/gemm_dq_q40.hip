// QT_Q4_0 instantiation of the stream-order dequant prefill GEMM (gemm_dq_impl.h)
#include "gemm_dq_impl.h"

namespace omx {

void run_dq_q40(const GemvParams& P, f16* xp, int Kp, hipStream_t s) { run_dq<QT_Q4_0>(P, xp, Kp, s); }

}  // namespace omx
