// QT_F16 instantiation of the stream-order dequant prefill GEMM (gemm_dq_impl.h)
#include "gemm_dq_impl.h"

namespace omx {

void run_dq_f16(const GemvParams& P, f16* xp, int Kp, hipStream_t s) { run_dq<QT_F16>(P, xp, Kp, s); }

}  // namespace omx
