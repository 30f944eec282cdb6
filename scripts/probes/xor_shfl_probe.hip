// Pins csrc/kernels/wave_shuffle.h: xor_shfl<J>(x)[lane] must equal x[lane ^ J] for every J.
// hipcc --offload-arch=gfx950 -O3 -I csrc scripts/probes/xor_shfl_probe.hip -o /tmp/xor_probe && /tmp/xor_probe
#include <cstdio>
#include "kernels/wave_shuffle.h"

__global__ void probe(int* out) {
  const int x = 1000 + (int)threadIdx.x;
  out[0 * 64 + threadIdx.x] = omx::xor_shfl<1>(x);
  out[1 * 64 + threadIdx.x] = omx::xor_shfl<2>(x);
  out[2 * 64 + threadIdx.x] = omx::xor_shfl<4>(x);
  out[3 * 64 + threadIdx.x] = omx::xor_shfl<8>(x);
  out[4 * 64 + threadIdx.x] = omx::xor_shfl<16>(x);
  out[5 * 64 + threadIdx.x] = omx::xor_shfl<32>(x);
}

int main() {
  int* d;
  int h[6 * 64];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  int bad = 0;
  for (int s = 0; s < 6; ++s)
    for (int l = 0; l < 64; ++l) {
      const int want = 1000 + (l ^ (1 << s));
      if (h[s * 64 + l] != want) {
        if (bad < 16) printf("J=%d lane %d: got %d want %d\n", 1 << s, l, h[s * 64 + l] - 1000, want - 1000);
        ++bad;
      }
    }
  printf(bad ? "xor_shfl probe: %d mismatches\n" : "xor_shfl probe: OK\n", bad);
  hipFree(d);
  return bad ? 1 : 0;
}
