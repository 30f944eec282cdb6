// Lane exchange x[lane ^ J] across a wave64 without the LDS crossbar (ds_bpermute costs LDS latency
// on every dependent step of a sorting network). All forms are direction-free compositions:
//   J = 1, 2   DPP quad_perm
//   J = 4      row_half_mirror (l ^ 7) then quad reverse (l ^ 3)
//   J = 8      row_mirror (l ^ 15) then row_half_mirror (l ^ 7)
//   J = 16     v_permlane16_swap (gfx950): odd rows of one copy <-> even rows of the other
//   J = 32     v_permlane32_swap (gfx950): upper half of one copy <-> lower half of the other
// Semantics pinned by scripts/probes/xor_shfl_probe.hip.
#pragma once
#include <hip/hip_runtime.h>

namespace omx {

template <int CTRL>
__device__ __forceinline__ int dpp_mov(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}

template <int J>
__device__ __forceinline__ int xor_shfl(int v) {
  static_assert(J == 1 || J == 2 || J == 4 || J == 8 || J == 16 || J == 32, "xor_shfl: J");
  if constexpr (J == 1) {
    return dpp_mov<0xB1>(v);  // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    return dpp_mov<0x4E>(v);  // quad_perm [2,3,0,1]
  } else if constexpr (J == 4) {
    return dpp_mov<0x1B>(dpp_mov<0x141>(v));  // half-mirror, then quad_perm [3,2,1,0]
  } else if constexpr (J == 8) {
    return dpp_mov<0x141>(dpp_mov<0x140>(v));  // mirror, then half-mirror
  } else if constexpr (J == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (threadIdx.x & 16) ? (int)r[0] : (int)r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (threadIdx.x & 32) ? (int)r[0] : (int)r[1];
  }
}

template <int J>
__device__ __forceinline__ float xor_shfl(float v) {
  return __int_as_float(xor_shfl<J>(__float_as_int(v)));
}

}  // namespace omx
