// Repacked quantized matrix descriptor (plain C++; shared by kernels and host code).
// Streams (see ollama_operator_amd/quant.py `repack`), all row-major over N rows of K weights:
//  Q4_K: s0 = qs [N][K/2],  s1 = meta [N][K/16]  (d, dmin, scales12 per 256 weights)
//  Q5_K: s0 = qs [N][K/2] (unsigned nibbles), s1 = meta [N][K/16] (as Q4_K), s2 = qh [N][K/8]
//        (4 B per piece, quant.py _q5k_qh_split)
//  Q6_K: s0 = ql [N][K/2],  s1 = qh [N][K/4], s2 = sc [N][K/16], s3 = d [N][K/128]
//  Q4_0: s0 = qs [N][K/2],  s1 = d [N][K/16]
//  Q8_0: s0 = qs [N][K],    s1 = d [N][K/16]
// MoE expert matrices are stored as X consecutive [N][...] blocks in every stream; the kernel
// offsets the row index by expert * N.
#pragma once
#include <stdint.h>

// QT_Q6_K8 is internal (no ggml type): a Q6_K matrix whose codes were widened at load to signed int8
// (q - 32), 32 B per piece (lo 16 weights | hi 16 weights) in s4, piece-major as Q8_0; scales stay in
// s2 (int8 per 16) / s3 (fp16 per 256). Opt-in (OMX_Q6K_WIDEN=1) for the batch-1 GEMV: it trades the
// 6-bit unpack chain (~5 us per down-projection launch, profiles/r2_gemv) for +30 % bytes, and in the
// engine that measured slower (down 13.2 -> 14.6 us). Prefill GEMM and batched GEMV read 6-bit streams.
// QT_F16 (ggml F16): plain fp16 rows [N][SB * 256] (K zero-padded to whole super-blocks) in s0; taken by
// the prefill GEMM only (gemm_dq.hip), e.g. the CLIP vision tower (models/clip.py)
enum QType : int { QT_F16 = 1, QT_Q4_0 = 2, QT_Q8_0 = 8, QT_Q4_K = 12, QT_Q5_K = 13, QT_Q6_K = 14, QT_Q6_K8 = 114 };

struct QMat {
  const uint8_t* s0;
  const uint8_t* s1;
  const uint8_t* s2;
  const uint8_t* s3;
  int N, K, qtype;
  const uint8_t* s4;  // optional widened Q6_K codes (QT_Q6_K8), null otherwise
  const uint8_t* mt;  // optional layout M copy for the batched MFMA decode GEMV (gemv_mfma.hip), or null
};
