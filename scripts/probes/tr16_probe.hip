// Probe of ds_read_b64_tr_b16 semantics on gfx950: LDS holds value = 64*row + col (as int16);
// lane L of each 16-lane group supplies the address of (row = (L&15)>>2, cols 4*(L&3)..+3) of a
// 64-column image; prints what every lane receives.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s4 __attribute__((ext_vector_type(4)));
__global__ void k(int* out, int mode) {
  __shared__ __attribute__((aligned(16))) short lds[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) lds[i] = (short)i;
  __syncthreads();
  const int L = threadIdx.x & 15, g = threadIdx.x >> 4;
  int row, col;
  if (mode == 0) { row = L >> 2; col = 4 * (L & 3); }      // documented: lane 4q+p -> row q, cols 4p
  else { row = L & 3; col = 4 * (L >> 2); }                // alternative: lane 4p+q -> row q, cols 4p
  row += 4 * g;
  const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4*)(lds + row * 64 + col));
  for (int j = 0; j < 4; ++j) out[threadIdx.x * 4 + j] = v[j];
}
int main() {
  int* d; hipMalloc(&d, 64 * 4 * 4);
  int h[256];
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("mode %d (%s):\n", mode, mode == 0 ? "lane 4q+p -> row q, cols 4p" : "lane 4p+q -> row q, cols 4p");
    for (int l = 0; l < 20; ++l) {
      printf("  lane %2d:", l);
      for (int j = 0; j < 4; ++j) printf(" (r%d,c%d)", h[l * 4 + j] / 64, h[l * 4 + j] % 64);
      printf("\n");
    }
  }
  return 0;
}
