// One-shot intra-node all-reduce / all-gather for tensor-parallel decode over xGMI.
//
// Why not RCCL for the decode step: a TP=8 70B token makes 2 * 80 all-reduces of 32 KB each. RCCL's
// ring/tree pays several xGMI hops and a host-visible launch per call; one-shot over peer-mapped
// memory is one hop: every rank reads the other ranks' partial sums straight out of their HBM
// (hipIpc-mapped pointers) and reduces locally. With 7 point-to-point links per MI355X, the 7 remote
// reads of a rank go over 7 different links in parallel, so the op costs ~one link latency plus
// n * 4 B / 153 GB/s — about 3 us for 32 KB. Large (prefill) messages keep RCCL (engine/runner.py).
//
// Protocol (no host involvement, graph-capturable, epoch counters so replays need no reset):
//  * Each rank owns a slab buffer of AR_SLABS slabs and a flag array flags[AR_MAX_BLOCKS][AR_MAX_RANKS]
//    in uncached device memory; the producing GEMV of call k writes its partial sums straight into
//    this rank's slab (executor.cpp: attention -> slab 0, FFN -> slab 1, logits gather -> slab 2).
//  * Block b of the kernel on rank r: epoch e = epoch[b] + 1 (local counter; all ranks run the same
//    sequence of AR calls with the same grid, so epoch[b] agrees across ranks). Thread p < world
//    does a system-scope release (the slab written by the producing GEMV is visible to peers), then
//    stores e into peer p's flags[b][r], then spins (bounded) until its own flags[b][p] >= e, then a
//    system-scope acquire. After the block barrier every peer's slab is complete.
//  * Sum in fixed rank order 0..world-1, so every rank produces bit-identical results (TP ranks must
//    sample the same token from the same logits).
//  * Slab reuse needs no end barrier as long as consecutive calls use different slabs: a rank's
//    producer for call k runs after its barrier of call k-1 returned, i.e. after every peer entered
//    call k-1 and so finished reading call k-2's slabs. The per-step sequence 0,1,0,1,...,0,1,2 keeps
//    consecutive slabs distinct, also across steps (2 -> 0).
//  * Spins are bounded (timeout_ticks of the 100 MHz wall clock): a dead peer turns into an error
//    flag (err[0] = 1 + rank of the first missing peer) and a finished kernel, never a hung GPU.
//    Once err is set every later collective on this rank skips its slab reads and leaves y untouched
//    (the group is out of step: reading would mix slabs of different calls). The host notices on the
//    next poll: the TP watchdog (parallel/tp.py `_watchdog`, leader) and the per-generate check
//    (engine/runner.py, every rank) raise TPCollectiveError / exit non-zero, so the pod restarts.
// Reference parity: the reference has replica parallelism only (pkg/model/model.go:149-186); this is
// the MI355X-native TP collective the north star adds.
#include "common.h"
#include "gemv8_core.h"
#include "ops.h"

namespace omx {

constexpr int AR_NT = 256;

// returns false (block-uniform) when this rank's collectives have failed: a barrier timed out now
// or in an earlier call -- the caller must not read peers' slabs then
__device__ __forceinline__ bool ar_barrier(const ARParams& P) {
  const int t = threadIdx.x, b = blockIdx.x;
  const unsigned e = P.epoch[b] + 1u;
  if (t < P.world) {
    // make this rank's slab (written by earlier kernels in stream order) visible system-wide
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(P.flags[t] + b * AR_MAX_RANKS + P.rank, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned* mine = P.flags[P.rank] + b * AR_MAX_RANKS + t;
    const unsigned long long t0 = wall_clock64();
    // a barrier that already timed out on this rank fails fast instead of waiting again
    const bool failed = __hip_atomic_load(P.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    while (!failed && (int)(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      if (wall_clock64() - t0 > P.timeout_ticks) {
        __hip_atomic_store(P.err, 1 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (P.err_host) __hip_atomic_store(P.err_host, 1 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  if (t == 0) P.epoch[b] = e;
  // every thread re-reads the error word after the barrier: a timeout by any thread of this block
  // (or an earlier call) is visible here, so the whole block takes the same branch
  return __hip_atomic_load(P.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
}

template <int W>
__global__ __launch_bounds__(AR_NT) void ar_add_kernel(ARParams P, int slab, float* __restrict__ y, int n) {
  if (!ar_barrier(P)) return;
  const long long off = (long long)slab * P.slab_floats;
  const int n4 = n >> 2;
  for (int i = blockIdx.x * AR_NT + threadIdx.x; i < n4; i += gridDim.x * AR_NT) {
    f32x4 v[W];
#pragma unroll
    for (int r = 0; r < W; ++r) v[r] = *(const f32x4*)(P.data[r] + off + 4LL * i);  // all loads in flight
    f32x4 s = v[0];
#pragma unroll
    for (int r = 1; r < W; ++r) s += v[r];  // rank order: identical on every rank
    f32x4* yp = (f32x4*)(y + 4LL * i);
    *yp = *yp + s;
  }
}

// The same sum + residual add, fused with the int8 activation chain's emission (gemv8.hip): thread
// = one 16-element group of the new residual row, which it also quantises into the next RMSNorm'd
// GEMV's image (x * norm_w, ops.h x8_bytes layout) with the group's sum of squares -- what the O /
// down producers emit at TP = 1, so under TP the QKV / gate_up / LM-head GEMVs read an int8 image too
// and no separate norm or quantisation pass runs. Rows b = 0..B-1 of E each (n = B * E).
template <int W>
__global__ __launch_bounds__(AR_NT) void ar_add_emit_kernel(ARParams P, int slab, float* __restrict__ y, int E, int B,
                                                            void* img, const float* __restrict__ nw, float* stat) {
  if (!ar_barrier(P)) return;
  const long long off = (long long)slab * P.slab_floats;
  const int gpr = E >> 4;  // groups per row
  for (int gi = blockIdx.x * AR_NT + threadIdx.x; gi < B * gpr; gi += gridDim.x * AR_NT) {
    const int b = gi / gpr, G = gi - b * gpr;
    const long long e0 = (long long)b * E + 16LL * G;
    f32x4 v[W][4];
#pragma unroll
    for (int r = 0; r < W; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[r][j] = *(const f32x4*)(P.data[r] + off + e0 + 4 * j);  // all loads in flight
    f32x4 yv[4], wv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      yv[j] = *(const f32x4*)(y + e0 + 4 * j);
      wv[j] = *(const f32x4*)(nw + 16LL * G + 4 * j);
    }
    float o[16], sq[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 sacc = v[0][j];
#pragma unroll
      for (int r = 1; r < W; ++r) sacc += v[r][j];  // rank order: identical on every rank
      const f32x4 nv = yv[j] + sacc;
      *(f32x4*)(y + e0 + 4 * j) = nv;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o[4 * j + k] = nv[k] * wv[j][k];
        sq[4 * j + k] = nv[k] * nv[k];
      }
    }
    emit_group((char*)img + (size_t)b * x8_slots_dev(E) * 24, E, G, o, sq, stat + (size_t)b * x8_stat_ld_dev(E));
  }
}

// out[row][r * n_local + j] = slab_r[row][j]  (vocab-sharded logits -> full rows)
__global__ __launch_bounds__(AR_NT) void ar_gather_kernel(ARParams P, int slab, float* __restrict__ out, int rows,
                                                          int n_local, int ld_out) {
  if (!ar_barrier(P)) return;
  const long long off = (long long)slab * P.slab_floats;
  const long long per = (long long)rows * n_local;
  const long long total = per * P.world;
  for (long long i = (long long)blockIdx.x * AR_NT + threadIdx.x; i < total; i += (long long)gridDim.x * AR_NT) {
    const int r = (int)(i / per);
    const long long k = i - r * per;
    const int row = (int)(k / n_local), j = (int)(k - (long long)row * n_local);
    out[(long long)row * ld_out + (long long)r * n_local + j] = P.data[r][off + k];
  }
}

static int ar_grid(long long work) {
  long long g = (work + AR_NT - 1) / AR_NT;
  return (int)(g < 1 ? 1 : g > AR_MAX_BLOCKS ? AR_MAX_BLOCKS : g);
}

void ar_allreduce_add(const ARParams& P, int slab, float* y, int n, hipStream_t s) {
  const int g = ar_grid((n / 4 + 1) / 2);  // ~2 float4 per thread: latency-bound, keep blocks few
  switch (P.world) {
#define AR_CASE(W) \
  case W: ar_add_kernel<W><<<g, AR_NT, 0, s>>>(P, slab, y, n); break;
    AR_CASE(1) AR_CASE(2) AR_CASE(3) AR_CASE(4) AR_CASE(5) AR_CASE(6) AR_CASE(7) AR_CASE(8)
#undef AR_CASE
    default: break;
  }
}

bool ar_allreduce_add_emit(const ARParams& P, int slab, float* y, int E, int B, void* img, const float* nw, float* stat,
                           hipStream_t s) {
  if (E % 16 || !img || !nw || !stat || B < 1 || B > X8_MAX_B) return false;
  const int g = ar_grid((long long)B * E / 16);  // one 16-element group per thread
  switch (P.world) {
#define AR_CASE(W) \
  case W: ar_add_emit_kernel<W><<<g, AR_NT, 0, s>>>(P, slab, y, E, B, img, nw, stat); return true;
    AR_CASE(1) AR_CASE(2) AR_CASE(3) AR_CASE(4) AR_CASE(5) AR_CASE(6) AR_CASE(7) AR_CASE(8)
#undef AR_CASE
    default: return false;
  }
}

void ar_allgather(const ARParams& P, int slab, float* out, int rows, int n_local, int ld_out, hipStream_t s) {
  const int g = ar_grid((long long)rows * n_local * P.world / 8);
  ar_gather_kernel<<<g, AR_NT, 0, s>>>(P, slab, out, rows, n_local, ld_out);
}

}  // namespace omx
