// Decode-step token feedback for one row, run by the sampler's finishing lane (sampling.hip,
// SampleParams::fb_step; it replaced a separate feedback launch per decode step). step: int32 [6][ld] =
// (pos, slot, q_len, q_seq, logit_idx, tokens), engine/runner.py d_step.
// host_ring (row 0 only): the sampled token also goes straight to host-mapped pinned memory,
// slot = input position % ring, so the host reads it after the step's event (no D2H copy command).
#pragma once
#include <hip/hip_runtime.h>

// sysfence: a system-scope fence after the host-ring store (0: the store alone; the host reads the ring
// only after the step's event, whose completion signal is itself a system-scope release)
__device__ __forceinline__ void decode_feedback_row(int* step, int ld, int b, int tok, int advance,
                                                    const int* block_table, int max_blocks, int bs,
                                                    int* host_ring, int ring, int sysfence = 1) {
  step[5 * ld + b] = tok;
  if (host_ring && b == 0) {
    __hip_atomic_store(host_ring + step[0] % ring, tok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (sysfence) __threadfence_system();
  }
  if (!advance) return;
  const int pos = step[b] + 1;
  const int row = step[3 * ld + b];
  const int bi = min(pos / bs, max_blocks - 1);  // past the context end the host re-uploads anyway
  step[b] = pos;
  step[ld + b] = block_table[(long long)row * max_blocks + bi] * bs + pos % bs;
  step[2 * ld + b] = pos + 1;
}
