// Phi-2's parallel attention/FFN block at batch 1: the attention output projection (O) and ffn_down add
// into the same residual row, and nothing reads that row between them. Separate launches paid two kernel
// boundaries and two partly filled grids per layer (O 5.7 us for 3.7 MB, down 6.8 us for 14.7 MB:
// profiles/r6_phi2/step_breakdown_phi2.txt). Here one block per 16-row tile runs both: wave group 0 streams
// O's rows against the merged attention output, groups 1..3 split ffn_down's K against FFN up's int8 image,
// the four partial sums meet in LDS, and group 0 writes resid + O + down + both biases and emits the next
// layer's LayerNorm'd image (x * ln_w, per-group sums and sums of squares: executor.cpp ln8).
//
// The O input is merged here from the deferred flash-decode slabs (or read as the plain fp32 row): four
// threads per 16-element group (one f32x4 of every slab each), the group's int8 scale found by a 4-lane
// max -- so 8 slabs fit the 1024-thread block's register budget. Weight tiles, dot products and the
// emission are the gemv8 ones (gemv_core.h, gemv8_core.h).
#include "gemv8_core.h"

namespace omx {

namespace {

constexpr int PAIR_KS = 4;                     // wave groups: 0 = O, 1..3 = ffn_down's K split
constexpr int PAIR_NT = GEMV_NT * PAIR_KS;
constexpr int PAIR_DW = 2;                     // down image words per thread (K <= 20480)

size_t pair_lds(int Ko, int Kd) { return x8_bytes(Ko) + x8_bytes(Kd) + (size_t)(48 + 3 * GEMV_NT) * 4; }

template <int QT, int MS>
__global__ __launch_bounds__(PAIR_NT) void qgemv8_pair_kernel(GemvParams D, GemvParams O) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int N = D.w.N, Ko = O.w.K, Kd = D.w.K;
  const int SBo = n_sb(Ko), SBd = n_sb(Kd);
  const int XSPo = x8_slots_dev(Ko), XSPd = x8_slots_dev(Kd);
  i32x4* lqo = (i32x4*)smem;
  f32x2* lfo = (f32x2*)(smem + (size_t)XSPo * 16);
  char* imd = smem + (size_t)XSPo * 24;
  i32x4* lqd = (i32x4*)imd;
  f32x2* lfd = (f32x2*)(imd + (size_t)XSPd * 16);
  float* stage = (float*)(imd + (size_t)XSPd * 24);  // [48]: emitted values, squares, plain values
  float* part = stage + 48;                          // [3][GEMV_NT] partial sums of groups 1..3
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, s = lane & 15;
  const int kg = wave / GEMV_NW, gtid = tid - kg * GEMV_NT;
  const int rbase = (wave - kg * GEMV_NW) * 4 + g;
  const int t = blockIdx.x;
  const int n = t * 16 + rbase, nc = min(n, N - 1);
  const int SBdv = D.k_valid > 0 && D.k_valid < Kd ? n_sb(D.k_valid) : SBd;
  const int CH = ks_chunk(SBd, PAIR_KS - 1);
  const int sb0 = kg > 0 ? (kg - 1) * CH : 0, se = kg > 0 ? min(SBdv, sb0 + CH) : SBo;

  // 0. epilogue operands (group 0), then 1. the activation operands, ahead of the weight stream
  float res = 0.f, nw = 0.f, bias = 0.f;
  if (kg == 0) {
    res = D.y[nc];
    nw = D.emit8_nw[nc];
    bias = (D.bias ? D.bias[nc] : 0.f) + (O.bias ? O.bias[nc] : 0.f);
  }
  // O's input: thread -> 16-element group gi = tid / 4, quarter qq = tid % 4 (elements 16 gi + 4 qq ..)
  const int gi = tid >> 2, qq = tid & 3;
  const bool og = gi < Ko / 16;
  const int gic = og ? gi : 0;
  f32x4 av[MS];
  f32x2 ml[MS];
  {
    const int h = MS > 1 ? 16 * gic / O.merge_D : 0, nh = MS > 1 ? Ko / O.merge_D : 0;
#pragma unroll
    for (int sp = 0; sp < MS; ++sp) {
      if constexpr (MS > 1) ml[sp] = *(const f32x2*)(O.merge_ml + 2 * (sp * nh + h));
      av[sp] = *(const f32x4*)(O.x + (long long)sp * Ko + 16 * gic + 4 * qq);
    }
  }
  const int nwd = XSPd * 3 / 2;  // 16-B words of down's image
  u32x4 xw[PAIR_DW];
#pragma unroll
  for (int i = 0; i < PAIR_DW; ++i) xw[i] = ((const u32x4*)D.x8)[min(tid + PAIR_NT * i, nwd - 1)];
  __builtin_amdgcn_sched_barrier(0);

  // 2. this wave group's weight tile in flight
  WTile<QT, 1, 1> T;
  if (kg == 0) load_wtile<QT, 1, 1>(O.w, 0, n, N, SBo, 0, s, T, SBo);
  else load_wtile<QT, 1, 1>(D.w, 0, n, N, SBd, sb0, s, T, se);
  __builtin_amdgcn_sched_barrier(0);

  // 3. images into LDS: down's copied, O's merged + quantised (4 lanes per group)
#pragma unroll
  for (int i = 0; i < PAIR_DW; ++i) {
    const int wd = tid + PAIR_NT * i;
    if (wd < nwd) {
      u32x4* dst = wd < XSPd ? (u32x4*)lqd + wd : (u32x4*)lfd + (wd - XSPd);
      *dst = xw[i];
    }
  }
  {
    f32x4 x;
    if constexpr (MS > 1) {  // flash-decode merge: splits without keys carry m = -inf, l = 0
      float M = -INFINITY;
#pragma unroll
      for (int sp = 0; sp < MS; ++sp) M = fmaxf(M, ml[sp].x);
      float L = 0.f;
      x = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sp = 0; sp < MS; ++sp) {
        const float c = ml[sp].x == -INFINITY ? 0.f : __expf(ml[sp].x - M);
        L += c * ml[sp].y;
        x += c * av[sp];
      }
      x *= L > 0.f ? 1.f / L : 0.f;
    } else {
      x = av[0];
    }
    if (!og) x = (f32x4){0.f, 0.f, 0.f, 0.f};
    float amax = fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)));
    amax = fmaxf(amax, __shfl_xor(amax, 1, 4));
    amax = fmaxf(amax, __shfl_xor(amax, 2, 4));
    const float d = amax / 127.f, id = amax > 0.f ? 127.f / amax : 0.f;
    const int q0 = (int)rintf(x.x * id), q1 = (int)rintf(x.y * id), q2 = (int)rintf(x.z * id),
              q3 = (int)rintf(x.w * id);
    int qs = q0 + q1 + q2 + q3;
    qs += __shfl_xor(qs, 1, 4);
    qs += __shfl_xor(qs, 2, 4);
    if (og) {
      const int slot = (gi >> 4) * XPAD + (gi & 15);
      ((int*)(lqo + slot))[qq] = (q0 & 0xFF) | ((q1 & 0xFF) << 8) | ((q2 & 0xFF) << 16) | ((q3 & 0xFF) << 24);
      if (qq == 0) lfo[slot] = (f32x2){d, d * (float)qs};
    }
  }
  __syncthreads();

  // 4. dot products, the groups' partials meet in LDS, group 0 writes the row and the emission
  float acc[1][1] = {{0.f}};
  if (kg == 0) compute_wtile<QT, 1, 1, 1>(T, SBo, 0, s, lqo, lfo, XSPo, acc, SBo);
  else compute_wtile<QT, 1, 1, 1>(T, SBd, sb0, s, lqd, lfd, XSPd, acc, se);
  if (kg > 0) part[(kg - 1) * GEMV_NT + gtid] = acc[0][0];
  __syncthreads();
  if (kg == 0) {
    float a = acc[0][0];
#pragma unroll
    for (int k = 0; k < PAIR_KS - 1; ++k) a += part[k * GEMV_NT + gtid];
    const float v = row16_sum(a);
    if (s == 0) {
      float nv = 0.f;
      if (n < N) {
        nv = res + bias + v;
        D.y[n] = nv;
      }
      stage[rbase] = n < N ? nv * nw : 0.f;
      stage[16 + rbase] = nv * nv;
      stage[32 + rbase] = nv;
    }
  }
  __syncthreads();
  if (tid < 16)
    emit_group16(D.emit8, N, t, stage[tid], stage[16 + tid], D.emit8_stat, tid, stage[32 + tid], D.emit8_sum);
}

template <int QT>
void launch_pair(const GemvParams& D, const GemvParams& O, hipStream_t s) {
  const size_t lds = pair_lds(O.w.K, D.w.K);
  const dim3 grid((D.w.N + 15) / 16), block(PAIR_NT);
  switch (O.merge_S > 1 ? O.merge_S : 1) {
    case 2: hipLaunchKernelGGL((qgemv8_pair_kernel<QT, 2>), grid, block, lds, s, D, O); break;
    case 4: hipLaunchKernelGGL((qgemv8_pair_kernel<QT, 4>), grid, block, lds, s, D, O); break;
    case 8:  // Q8_0's 32-B pieces and 8 merge slabs exceed the 1024-thread block's 128 VGPRs (declined)
      if constexpr (QT != QT_Q8_0) hipLaunchKernelGGL((qgemv8_pair_kernel<QT, 8>), grid, block, lds, s, D, O);
      break;
    default: hipLaunchKernelGGL((qgemv8_pair_kernel<QT, 1>), grid, block, lds, s, D, O); break;
  }
}

}  // namespace

bool gemv8_pair_supported(const GemvParams& D, const GemvParams& O) {
  const int q = D.w.qtype;
  if (!(q == QT_Q4_0 || q == QT_Q4_K || q == QT_Q8_0) || O.w.qtype != q) return false;
  if (D.B != 1 || O.B != 1 || D.w.N != O.w.N || D.y != O.y || D.epi != EPI_ADD || O.epi != EPI_ADD) return false;
  if (!D.x8 || D.x8_stat || D.x8_sum || !D.emit8 || !D.emit8_nw || !D.emit8_stat || D.expert_ids || D.dbg_ts) return false;
  if (O.x8 || O.norm != NORM_NONE || O.expert_ids || O.emit8 || !O.x) return false;
  if (D.w.N % 16 || O.w.s0 == nullptr || D.w.s0 == nullptr) return false;
  const int Ko = O.w.K, Kd = D.w.K;
  if (Ko % 64 || Ko > 16 * 256 || Ko / 4 > PAIR_NT) return false;  // O: one group of <= 16 super-blocks
  const int MS = O.merge_S > 1 ? O.merge_S : 1;
  if (MS != 1 && MS != 2 && MS != 4 && MS != 8) return false;
  if (q == QT_Q8_0 && MS == 8) return false;
  if (MS > 1 && (O.merge_D <= 0 || O.merge_D % 16 || Ko % O.merge_D)) return false;
  if ((Kd + 255) / 256 > 16 * (PAIR_KS - 1) || (size_t)x8_slots(Kd) * 3 / 2 > (size_t)PAIR_DW * PAIR_NT) return false;
  return pair_lds(Ko, Kd) <= 64 * 1024;
}

bool gemv8_pair(const GemvParams& D, const GemvParams& O, hipStream_t s) {
  if (!gemv8_pair_supported(D, O)) return false;
  count_launch(LC_GEMV8_PAIR);
  switch (D.w.qtype) {
    case QT_Q4_0: launch_pair<QT_Q4_0>(D, O, s); return true;
    case QT_Q4_K: launch_pair<QT_Q4_K>(D, O, s); return true;
    case QT_Q8_0: launch_pair<QT_Q8_0>(D, O, s); return true;
    default: return false;
  }
}

}  // namespace omx
