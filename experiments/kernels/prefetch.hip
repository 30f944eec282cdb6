// Infinity-Cache (MALL) weight prefetch for batch-1 decode.
//
// Batch-1 decode streams ~4 GB of distinct weights per token, each GEMV reading its matrix exactly once.
// Every GEMV launch pays a ramp (blocks issue their first loads into an idle memory system) and a tail
// (the last blocks drain while the rest of the chip idles): profiles/r5_decode puts these at 2-4 us per
// launch against a 5-13 us stream. A side stream that reads the NEXT launch's weights while the current
// one runs moves those bytes into the 256 MiB MALL (memory-attached, so it caches every HBM stack's
// lines), turning the next launch's ramp and tail into MALL-latency ones and keeping HBM busy across the
// kernel boundary. This kernel is that reader: a grid-stride 16-B load stream whose values are folded
// into a register and (practically never) stored, so the loads cannot be elided.
#include <hip/hip_runtime.h>

#include "ops.h"

namespace omx {

__global__ __launch_bounds__(256) void mall_touch_kernel(const uint4* __restrict__ p, size_t n16, unsigned* sink) {
  unsigned acc = 0;
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {  // 4 loads in flight per lane
    const uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= a.x ^ b.y ^ c.z ^ d.w;
  }
  for (; i < n16; i += stride) acc ^= p[i].x;
  if (acc == 0x9E3779B9u) sink[threadIdx.x] = acc;  // keeps the loads live; a vector store
}

void mall_prefetch(const void* p, size_t bytes, int blocks, unsigned* sink, hipStream_t s) {
  const size_t n16 = bytes / 16;
  if (!p || n16 == 0 || blocks <= 0) return;
  count_launch(LC_MALL_PREFETCH);
  hipLaunchKernelGGL(mall_touch_kernel, dim3(blocks), dim3(256), 0, s, (const uint4*)p, n16, sink);
}

}  // namespace omx
