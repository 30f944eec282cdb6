// Quantised GEMM/GEMV on the CPU over the repacked (layout v2) weight streams -- see cpu_engine.h.
//
// Per 256-weight super-block (SB) of a weight row the codes are unpacked once into natural order
// (32-byte AVX2 vectors, one per 32-weight sub-block) and dotted against every activation row of the
// call: u8 codes x s8 activations via vpmaddubsw (pairs, s16) then vpmaddwd with the sub-block's
// integer scale (K-quants) or with ones (Q4_0 / Q8_0, whose per-32 fp16 scales are applied in
// fp32). Activations are quantised per SB (Q8_K style: fp32 scale, int8 codes, int16 sums per 16)
// so the K-quant mins / zero points reduce to integer dot products of the sums.
//
// Layout v2 (ollama_operator_amd/quant.py `repack`, csrc/kernels/qmat.h): stream 0 holds each
// row's codes piece-major, piece t (16 B) of SB sb at byte (t * SB + sb) * 16 (Q8_0: 32 B).
//   Q4_K / Q4_0 bytes are stored ^ 0x80 (signed high nibble for the GPU dot); Q5_K unsigned.
//   Q4_K / Q5_K piece t: lo nibbles = sub-block 2(t/2), weights 16(t%2)..+16; hi nibbles = sub-block
//   2(t/2) + 1. Q4_0 / Q8_0 piece t = 32-weight block t of the SB. Q6_K piece t: lo nibbles = weights
//   128(t/4) + 16(t%4) + i, hi = the same + 64; high 2 bits in qh (8 B per piece, quant.py
//   _q6k_qh_split: weight i -> (qh[i % 4] >> 2(i / 4)) & 3, lo in bytes 0-3, hi in bytes 4-7).
#include <immintrin.h>
#include <omp.h>
#include <string.h>

#include <cmath>
#include <vector>

#include "cpu_engine.h"

namespace omxcpu {

static inline float h2f(uint16_t h) { return _cvtsh_ss(h); }

int threads() { return omp_get_max_threads(); }
const char* isa() { return "avx2"; }

// ------------------------------------------------------------------------------------------------
// activations: [B][SB] blocks of 256 int8 codes, fp32 scale, int16 sums per 16
struct QAct {
  int SB = 0, B = 0;
  std::vector<int8_t> q;      // [B][SB * 256]
  std::vector<float> d;       // [B][SB]
  std::vector<int16_t> bsum;  // [B][SB * 16]
};

static void quantize_rows(const float* x, int ldx, int B, int K, QAct& a) {
  const int SB = (K + 255) / 256;
  a.SB = SB;
  a.B = B;
  a.q.resize((size_t)B * SB * 256);
  a.d.resize((size_t)B * SB);
  a.bsum.resize((size_t)B * SB * 16);
#pragma omp parallel for schedule(static) if (B * SB >= 64)
  for (int i = 0; i < B * SB; ++i) {
    const int b = i / SB, sb = i % SB;
    const float* xs = x + (long long)b * ldx + sb * 256;
    const int n = K - sb * 256 < 256 ? K - sb * 256 : 256;
    float v[256];
    memcpy(v, xs, sizeof(float) * n);
    for (int j = n; j < 256; ++j) v[j] = 0.f;
    float amax = 0.f;
    for (int j = 0; j < 256; ++j) amax = fmaxf(amax, fabsf(v[j]));
    const float d = amax / 127.f, id = amax > 0.f ? 127.f / amax : 0.f;
    int8_t* q = a.q.data() + (size_t)i * 256;
    int16_t* bs = a.bsum.data() + (size_t)i * 16;
    for (int g = 0; g < 16; ++g) {
      int s = 0;
      for (int j = 0; j < 16; ++j) {
        const int c = (int)nearbyintf(v[16 * g + j] * id);
        q[16 * g + j] = (int8_t)c;
        s += c;
      }
      bs[g] = (int16_t)s;
    }
    a.d[i] = d;
  }
}

// ------------------------------------------------------------------------------------------------
// one unpacked SB: 8 vectors of 32 codes (sub-block order), integer or fp32 scales
struct USB {
  __m256i c[8];
  int sc[16];     // K-quants: integer scale per 32 (Q4_K/Q5_K: 8 used) or per 16 (Q6_K)
  int mn[8];      // Q4_K/Q5_K mins
  float d, dmin;  // super-block scales
  __m256 bdv;     // Q4_0/Q8_0 per-32 block scales
};

// [sum of the 8 lanes of p[0]], ..., [sum of p[7]] -> one vector (block order)
static inline __m256i hsum8(const __m256i* p) {
  const __m256i t0 = _mm256_hadd_epi32(p[0], p[1]), t1 = _mm256_hadd_epi32(p[2], p[3]);
  const __m256i t2 = _mm256_hadd_epi32(p[4], p[5]), t3 = _mm256_hadd_epi32(p[6], p[7]);
  const __m256i u0 = _mm256_hadd_epi32(t0, t1), u1 = _mm256_hadd_epi32(t2, t3);
  return _mm256_add_epi32(_mm256_permute2x128_si256(u0, u1, 0x20), _mm256_permute2x128_si256(u0, u1, 0x31));
}

static inline __m256i load2(const uint8_t* a, const uint8_t* b) {
  return _mm256_inserti128_si256(_mm256_castsi128_si256(_mm_loadu_si128((const __m128i*)a)),
                                 _mm_loadu_si128((const __m128i*)b), 1);
}

static inline void kscales(const uint8_t* m, int* sc, int* mn, float& d, float& dmin) {
  uint16_t dd, dm;
  memcpy(&dd, m, 2);
  memcpy(&dm, m + 2, 2);
  d = h2f(dd);
  dmin = h2f(dm);
  const uint8_t* s = m + 4;  // 12 bytes, ggml get_scale_min_k4
  for (int j = 0; j < 8; ++j) {
    if (j < 4) {
      sc[j] = s[j] & 63;
      mn[j] = s[j + 4] & 63;
    } else {
      sc[j] = (s[j + 4] & 0xF) | ((s[j - 4] >> 6) << 4);
      mn[j] = (s[j + 4] >> 4) | ((s[j] >> 6) << 4);
    }
  }
}

template <int QT>
static inline __attribute__((always_inline)) void unpack(const QMat& w, long long row, int sb, int SB, USB& u) {
  const __m256i m4 = _mm256_set1_epi8(0x0F), x80 = _mm256_set1_epi8((char)0x80);
  switch (QT) {
    case QT_Q4_K: {
      const uint8_t* qs = w.s[0] + row * SB * 128;
      kscales(w.s[1] + row * SB * 16 + 16 * sb, u.sc, u.mn, u.d, u.dmin);
      for (int c = 0; c < 4; ++c) {
        const __m256i p = _mm256_xor_si256(load2(qs + (2 * c * SB + sb) * 16, qs + ((2 * c + 1) * SB + sb) * 16), x80);
        u.c[2 * c] = _mm256_and_si256(p, m4);
        u.c[2 * c + 1] = _mm256_and_si256(_mm256_srli_epi16(p, 4), m4);
      }
      break;
    }
    case QT_Q5_K: {
      const uint8_t* qs = w.s[0] + row * SB * 128;
      const uint8_t* qh = w.s[2] + row * SB * 32;
      kscales(w.s[1] + row * SB * 16 + 16 * sb, u.sc, u.mn, u.d, u.dmin);
      // 5th bits: piece t byte j holds bit k (lo) / 4 + k (hi) for weight i = 4k + j
      const __m256i kshift = _mm256_setr_epi32(0, 1, 2, 3, 0, 1, 2, 3);
      const __m256i one = _mm256_set1_epi8(1);
      for (int c = 0; c < 4; ++c) {
        const __m256i p = load2(qs + (2 * c * SB + sb) * 16, qs + ((2 * c + 1) * SB + sb) * 16);
        unsigned h0, h1;
        memcpy(&h0, qh + (2 * c * SB + sb) * 4, 4);
        memcpy(&h1, qh + ((2 * c + 1) * SB + sb) * 4, 4);
        const __m256i H = _mm256_setr_epi32(h0, h0, h0, h0, h1, h1, h1, h1);  // dword k of each half
        const __m256i hl = _mm256_and_si256(_mm256_srlv_epi32(H, kshift), one);
        const __m256i hh = _mm256_and_si256(_mm256_srlv_epi32(H, _mm256_add_epi32(kshift, _mm256_set1_epi32(4))), one);
        u.c[2 * c] = _mm256_or_si256(_mm256_and_si256(p, m4), _mm256_slli_epi16(hl, 4));
        u.c[2 * c + 1] = _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(p, 4), m4), _mm256_slli_epi16(hh, 4));
      }
      break;
    }
    case QT_Q6_K: {
      const uint8_t* ql = w.s[0] + row * SB * 128;
      const uint8_t* qh = w.s[1] + row * SB * 64;
      const int8_t* sc = (const int8_t*)(w.s[2] + row * SB * 16 + 16 * sb);
      uint16_t dd;
      memcpy(&dd, w.s[3] + row * SB * 2 + 2 * sb, 2);
      u.d = h2f(dd);
      for (int g = 0; g < 16; ++g) u.sc[g] = sc[g];
      // vector v (32 weights) = group pair: lo groups of pieces (t, t+1) share n; map to the natural
      // 32-weight runs: c[2n*2 + ...]; we store per piece pair (t even): lo -> weights 128n+16s..+32
      const __m256i kshift = _mm256_setr_epi32(0, 2, 4, 6, 0, 2, 4, 6), m3 = _mm256_set1_epi8(3);
      for (int t = 0; t < 8; t += 2) {
        const int n = t >> 2, s = t & 3;  // s in {0, 2}
        const __m256i p = load2(ql + (t * SB + sb) * 16, ql + ((t + 1) * SB + sb) * 16);
        unsigned hl0, hh0, hl1, hh1;
        memcpy(&hl0, qh + (t * SB + sb) * 8, 4);
        memcpy(&hh0, qh + (t * SB + sb) * 8 + 4, 4);
        memcpy(&hl1, qh + ((t + 1) * SB + sb) * 8, 4);
        memcpy(&hh1, qh + ((t + 1) * SB + sb) * 8 + 4, 4);
        // byte 4k + j of a 16-weight half = weight 4k + j: high bits (H byte j >> 2k) & 3, i.e. dword k
        // of the broadcast H shifted right by 2k
        const __m256i HL = _mm256_setr_epi32(hl0, hl0, hl0, hl0, hl1, hl1, hl1, hl1);
        const __m256i HH = _mm256_setr_epi32(hh0, hh0, hh0, hh0, hh1, hh1, hh1, hh1);
        const __m256i bl = _mm256_and_si256(_mm256_srlv_epi32(HL, kshift), m3);
        const __m256i bh = _mm256_and_si256(_mm256_srlv_epi32(HH, kshift), m3);
        // vectors in 32-weight natural runs: run r = weights 32r..32r+32 of the SB
        // lo of pieces t, t+1 -> weights 128n + 16s .. + 32  -> run 4n + s/2
        // hi of pieces t, t+1 -> weights 128n + 64 + 16s ..   -> run 4n + 2 + s/2
        u.c[4 * n + s / 2] = _mm256_or_si256(_mm256_and_si256(p, m4), _mm256_slli_epi16(bl, 4));
        u.c[4 * n + 2 + s / 2] = _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(p, 4), m4), _mm256_slli_epi16(bh, 4));
      }
      break;
    }
    case QT_Q4_0: {
      const uint8_t* qs = w.s[0] + row * SB * 128;
      // 8 fp16 block scales in one conversion
      u.bdv = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i*)(w.s[1] + row * SB * 16 + 16 * sb)));
      for (int t = 0; t < 8; t += 2) {  // blocks t, t+1 per 256-bit op: [lo_t | lo_t1], [hi_t | hi_t1]
        const __m256i p = _mm256_xor_si256(load2(qs + (t * SB + sb) * 16, qs + ((t + 1) * SB + sb) * 16), x80);
        const __m256i lo = _mm256_and_si256(p, m4), hi = _mm256_and_si256(_mm256_srli_epi16(p, 4), m4);
        u.c[t] = _mm256_permute2x128_si256(lo, hi, 0x20);      // block t natural order
        u.c[t + 1] = _mm256_permute2x128_si256(lo, hi, 0x31);  // block t + 1
      }
      break;
    }
    case QT_Q8_0: {
      const uint8_t* qs = w.s[0] + row * SB * 256;
      u.bdv = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i*)(w.s[1] + row * SB * 16 + 16 * sb)));
      for (int t = 0; t < 8; ++t) u.c[t] = _mm256_loadu_si256((const __m256i*)(qs + (t * SB + sb) * 32));
      break;
    }
    default: break;
  }
}

static inline int hsum_i32(__m256i v) {
  __m128i s = _mm_add_epi32(_mm256_castsi256_si128(v), _mm256_extracti128_si256(v, 1));
  s = _mm_add_epi32(s, _mm_shuffle_epi32(s, 0x4E));
  s = _mm_add_epi32(s, _mm_shuffle_epi32(s, 0xB1));
  return _mm_cvtsi128_si32(s);
}
static inline float hsum_f32(__m256 v) {
  __m128 s = _mm_add_ps(_mm256_castps256_ps128(v), _mm256_extractf128_ps(v, 1));
  s = _mm_add_ps(s, _mm_movehl_ps(s, s));
  s = _mm_add_ss(s, _mm_movehdup_ps(s));
  return _mm_cvtss_f32(s);
}

// dot of one unpacked SB with one activation SB; returns the fp32 contribution
template <int QT>
static inline __attribute__((always_inline)) float dot_sb(const USB& u, const int8_t* xq, float dx, const int16_t* bs) {
  switch (QT) {
    case QT_Q4_K:
    case QT_Q5_K: {
      __m256i acc = _mm256_setzero_si256();
      for (int s = 0; s < 8; ++s) {
        const __m256i x = _mm256_loadu_si256((const __m256i*)(xq + 32 * s));
        acc = _mm256_add_epi32(acc, _mm256_madd_epi16(_mm256_maddubs_epi16(u.c[s], x), _mm256_set1_epi16((short)u.sc[s])));
      }
      int msum = 0;
      for (int s = 0; s < 8; ++s) msum += u.mn[s] * (bs[2 * s] + bs[2 * s + 1]);
      return dx * (u.d * (float)hsum_i32(acc) - u.dmin * (float)msum);
    }
    case QT_Q6_K: {
      // run r (32 weights) = 16-groups 2r, 2r + 1 with scales sc[2r], sc[2r + 1]
      __m256i acc = _mm256_setzero_si256();
      for (int r = 0; r < 8; ++r) {
        const __m256i x = _mm256_loadu_si256((const __m256i*)(xq + 32 * r));
        const __m256i sc = _mm256_setr_m128i(_mm_set1_epi16((short)u.sc[2 * r]), _mm_set1_epi16((short)u.sc[2 * r + 1]));
        acc = _mm256_add_epi32(acc, _mm256_madd_epi16(_mm256_maddubs_epi16(u.c[r], x), sc));
      }
      int off = 0;
      for (int g = 0; g < 16; ++g) off += u.sc[g] * bs[g];
      return dx * u.d * (float)(hsum_i32(acc) - 32 * off);
    }
    default: return 0.f;
  }
}

// Q4_0 / Q8_0: per-block contributions of one SB as a vector (reduced once per row):
// dx * d_t * (sum_i q_i x_i - 8 * sum_i x_i) for the 8 blocks t
template <int QT>
static inline __attribute__((always_inline)) __m256 dot_blocks(const USB& u, const int8_t* xq, float dx,
                                                               const int16_t* bs) {
  const __m256i ones = _mm256_set1_epi16(1);
  __m256i p[8];
  for (int t = 0; t < 8; ++t) {
    const __m256i x = _mm256_loadu_si256((const __m256i*)(xq + 32 * t));
    if constexpr (QT == QT_Q8_0) {
      const __m256i aw = _mm256_sign_epi8(u.c[t], u.c[t]);  // |w| (u8), the sign moves onto x
      p[t] = _mm256_madd_epi16(_mm256_maddubs_epi16(aw, _mm256_sign_epi8(x, u.c[t])), ones);
    } else {
      p[t] = _mm256_madd_epi16(_mm256_maddubs_epi16(u.c[t], x), ones);
    }
  }
  __m256 v = _mm256_cvtepi32_ps(hsum8(p));
  if constexpr (QT == QT_Q4_0) {  // zero point 8: subtract 8 * (sum of the block's activations)
    const __m256i bs32 = _mm256_madd_epi16(_mm256_loadu_si256((const __m256i*)bs), ones);  // pairs of 16
    v = _mm256_fnmadd_ps(_mm256_set1_ps(8.f), _mm256_cvtepi32_ps(bs32), v);
  }
  return _mm256_mul_ps(v, _mm256_mul_ps(u.bdv, _mm256_set1_ps(dx)));
}

// streams of the next super-block a row step reads (prefetched ahead of the unpack)
template <int QT>
static inline void prefetch_sb(const QMat& w, long long row, int sb, int SB) {
  if (sb >= SB) return;
  if constexpr (QT == QT_Q8_0) {
    const uint8_t* qs = w.s[0] + row * SB * 256;
    for (int t = 0; t < 8; ++t) _mm_prefetch((const char*)(qs + (t * SB + sb) * 32), _MM_HINT_T0);
  } else {
    const uint8_t* qs = w.s[0] + row * SB * 128;
    for (int t = 0; t < 8; ++t) _mm_prefetch((const char*)(qs + (t * SB + sb) * 16), _MM_HINT_T0);
  }
}

template <int QT>
static void gemm_t(const QMat& w, long long row_base, int N, const QAct& a, float* y, int ldy, bool accumulate) {
  const int SB = a.SB, B = a.B;
  // rows in contiguous slices: each thread streams its own part of the matrix
  constexpr bool BLK = QT == QT_Q4_0 || QT == QT_Q8_0;  // fp32 per-block scales: vector accumulators
#pragma omp parallel
  {
    // per-thread accumulators on the thread's own stack (small heap blocks of different threads
    // share cache lines: written every super-block, that false sharing cost 4x at 8 threads)
    alignas(64) float acc_s[64];
    alignas(64) __m256 vacc_s[64];
    std::vector<float> accv(B > 64 ? B + 16 : 0);
    std::vector<__m256> vaccv(BLK && B > 64 ? B + 2 : 0);
    float* acc = B > 64 ? accv.data() : acc_s;
    __m256* vacc = B > 64 ? vaccv.data() : vacc_s;
#pragma omp for schedule(static)
    for (int n = 0; n < N; ++n) {
      const long long row = row_base + n;
      for (int b = 0; b < B; ++b) {
        acc[b] = 0.f;
        if constexpr (BLK) vacc[b] = _mm256_setzero_ps();
      }
      for (int sb = 0; sb < SB; ++sb) {
        prefetch_sb<QT>(w, row, sb + 2, SB);
        USB u;
        unpack<QT>(w, row, sb, SB, u);
        for (int b = 0; b < B; ++b) {
          const size_t i = (size_t)b * SB + sb;
          if constexpr (BLK)
            vacc[b] = _mm256_add_ps(vacc[b], dot_blocks<QT>(u, a.q.data() + i * 256, a.d[i], a.bsum.data() + i * 16));
          else
            acc[b] += dot_sb<QT>(u, a.q.data() + i * 256, a.d[i], a.bsum.data() + i * 16);
        }
      }
      for (int b = 0; b < B; ++b) {
        if constexpr (BLK) acc[b] = hsum_f32(vacc[b]);
        float* o = y + (long long)b * ldy + n;
        *o = accumulate ? *o + acc[b] : acc[b];
      }
    }
  }
}

void gemm(const QMat& w, long long row_base, int N, const float* x, int ldx, int B, float* y, int ldy,
          bool accumulate) {
  static thread_local QAct act;
  quantize_rows(x, ldx, B, w.K, act);
  switch (w.qtype) {
    case QT_Q4_0: gemm_t<QT_Q4_0>(w, row_base, N, act, y, ldy, accumulate); break;
    case QT_Q8_0: gemm_t<QT_Q8_0>(w, row_base, N, act, y, ldy, accumulate); break;
    case QT_Q4_K: gemm_t<QT_Q4_K>(w, row_base, N, act, y, ldy, accumulate); break;
    case QT_Q5_K: gemm_t<QT_Q5_K>(w, row_base, N, act, y, ldy, accumulate); break;
    case QT_Q6_K: gemm_t<QT_Q6_K>(w, row_base, N, act, y, ldy, accumulate); break;
    default: break;
  }
}

template <int QT>
static void dequant_row_t(const QMat& w, long long row, float* out) {
  const int SB = (w.K + 255) / 256;
  for (int sb = 0; sb < SB; ++sb) {
    USB u;
    unpack<QT>(w, row, sb, SB, u);
    alignas(32) uint8_t c[256];
    for (int r = 0; r < 8; ++r) _mm256_store_si256((__m256i*)(c + 32 * r), u.c[r]);
    alignas(32) float bd[8];
    if constexpr (QT == QT_Q4_0 || QT == QT_Q8_0) _mm256_store_ps(bd, u.bdv);
    const int n = w.K - sb * 256 < 256 ? w.K - sb * 256 : 256;
    float* o = out + sb * 256;
    for (int j = 0; j < n; ++j) {
      const int s = j / 32;
      switch (QT) {
        case QT_Q4_K:
        case QT_Q5_K: o[j] = u.d * u.sc[s] * c[j] - u.dmin * u.mn[s]; break;
        case QT_Q6_K: o[j] = u.d * u.sc[j / 16] * ((int)c[j] - 32); break;
        case QT_Q4_0: o[j] = bd[s] * ((int)c[j] - 8); break;
        case QT_Q8_0: o[j] = bd[s] * (int8_t)c[j]; break;
        default: o[j] = 0.f;
      }
    }
  }
}

void dequant_row(const QMat& w, long long row, float* out) {
  switch (w.qtype) {
    case QT_Q4_0: dequant_row_t<QT_Q4_0>(w, row, out); break;
    case QT_Q8_0: dequant_row_t<QT_Q8_0>(w, row, out); break;
    case QT_Q4_K: dequant_row_t<QT_Q4_K>(w, row, out); break;
    case QT_Q5_K: dequant_row_t<QT_Q5_K>(w, row, out); break;
    case QT_Q6_K: dequant_row_t<QT_Q6_K>(w, row, out); break;
    default: break;
  }
}

}  // namespace omxcpu
