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

enum QType : int { QT_Q4_0 = 2, QT_Q8_0 = 8, QT_Q4_K = 12, QT_Q5_K = 13, QT_Q6_K = 14 };

struct QMat {
  const uint8_t* s0;
  const uint8_t* s1;
  const uint8_t* s2;
  const uint8_t* s3;
  int N, K, qtype;
};
