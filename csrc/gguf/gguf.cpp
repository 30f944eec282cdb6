// Native GGUF loader: mmap + bounds-checked tensor index + multi-threaded
// repack of ggml quant blocks into the 16-B-aligned device streams of csrc/kernels/qmat.h, with
// row selection/permutation (q/k NEOX pairing, gate/up interleave, TP row shards) and K-block
// slicing (TP column shards) fused into the same pass over the mapped file.
#include "gguf.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace omx {

namespace {

struct Cur {
  const uint8_t* p;
  size_t n, pos = 0;
  void need(size_t k) {
    if (k > n || pos + k > n) throw std::runtime_error("truncated GGUF header");
  }
  template <class T>
  T get() {
    need(sizeof(T));
    T v;
    std::memcpy(&v, p + pos, sizeof(T));
    pos += sizeof(T);
    return v;
  }
  std::string str() {
    const uint64_t len = get<uint64_t>();
    if (len > (1u << 24)) throw std::runtime_error("GGUF string too long");
    need(len);
    std::string s((const char*)p + pos, len);
    pos += len;
    return s;
  }
  void skip_value(uint32_t t, int depth = 0) {
    static const int sz[] = {1, 1, 2, 2, 4, 4, 4, 1, -1, -1, 8, 8, 8};
    if (t > 12) throw std::runtime_error("bad GGUF value type");
    if (t == 8) { (void)str(); return; }
    if (t == 9) {
      if (depth > 2) throw std::runtime_error("GGUF arrays nested too deep");
      const uint32_t et = get<uint32_t>();
      const uint64_t cnt = get<uint64_t>();
      if (cnt > (1ull << 28)) throw std::runtime_error("GGUF array too long");
      if (et == 8 || et == 9) {
        for (uint64_t i = 0; i < cnt; ++i) skip_value(et, depth + 1);
      } else {
        if (et > 12) throw std::runtime_error("bad GGUF array type");
        need(cnt * sz[et]);
        pos += cnt * sz[et];
      }
      return;
    }
    need(sz[t]);
    pos += sz[t];
  }
};

void block_geom(int t, int& blk, int& nb) {
  switch (t) {
    case 0: blk = 1; nb = 4; return;
    case 1: case 30: blk = 1; nb = 2; return;
    case 2: blk = 32; nb = 18; return;
    case 3: blk = 32; nb = 20; return;
    case 6: blk = 32; nb = 22; return;
    case 7: blk = 32; nb = 24; return;
    case 8: blk = 32; nb = 34; return;
    case 10: blk = 256; nb = 84; return;
    case 11: blk = 256; nb = 110; return;
    case 12: blk = 256; nb = 144; return;
    case 13: blk = 256; nb = 176; return;
    case 14: blk = 256; nb = 210; return;
    case 15: blk = 256; nb = 292; return;
    default: throw std::runtime_error("unsupported ggml type " + std::to_string(t));
  }
}

}  // namespace

GGUFMap::GGUFMap(const std::string& path) {
  fd_ = ::open(path.c_str(), O_RDONLY);
  if (fd_ < 0) throw std::runtime_error("cannot open " + path);
  struct stat st;
  if (fstat(fd_, &st) != 0) throw std::runtime_error("stat failed");
  size_ = (size_t)st.st_size;
  base_ = (const uint8_t*)mmap(nullptr, size_, PROT_READ, MAP_SHARED, fd_, 0);
  if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed");
  Cur c{base_, size_};
  if (c.get<uint32_t>() != 0x46554747u) throw std::runtime_error("not a GGUF file");
  version_ = c.get<uint32_t>();
  if (version_ != 2 && version_ != 3) throw std::runtime_error("unsupported GGUF version");
  const uint64_t nt = c.get<uint64_t>(), nkv = c.get<uint64_t>();
  if (nt > (1u << 20) || nkv > (1u << 20)) throw std::runtime_error("implausible GGUF counts");
  uint64_t align = 32;
  for (uint64_t i = 0; i < nkv; ++i) {
    const std::string key = c.str();
    const uint32_t t = c.get<uint32_t>();
    if (key == "general.alignment" && t == 4) {
      align = c.get<uint32_t>();
      if (align == 0 || (align & (align - 1))) throw std::runtime_error("bad alignment");
    } else {
      c.skip_value(t);
    }
  }
  std::vector<TensorEntry> tmp;
  for (uint64_t i = 0; i < nt; ++i) {
    TensorEntry e;
    e.name = c.str();
    const uint32_t nd = c.get<uint32_t>();
    if (nd == 0 || nd > 4) throw std::runtime_error("bad n_dims for " + e.name);
    e.n_elements = 1;
    for (uint32_t d = 0; d < nd; ++d) {
      e.dims.push_back((int64_t)c.get<uint64_t>());
      if (e.dims.back() <= 0) throw std::runtime_error("bad dim for " + e.name);
      e.n_elements *= e.dims.back();
    }
    e.type = (int)c.get<uint32_t>();
    e.offset = c.get<uint64_t>();
    int blk, nb;
    block_geom(e.type, blk, nb);
    if (e.n_elements % blk) throw std::runtime_error("tensor not block aligned: " + e.name);
    e.nbytes = e.n_elements / blk * nb;
    tmp.push_back(e);
  }
  data_offset_ = (c.pos + align - 1) / align * align;
  for (auto& e : tmp) {
    e.offset += data_offset_;
    if (e.offset + e.nbytes > size_) throw std::runtime_error("tensor data out of file: " + e.name);
    index_[e.name] = tensors_.size();
    tensors_.push_back(e);
  }
}

GGUFMap::~GGUFMap() {
  if (base_ && base_ != MAP_FAILED) munmap((void*)base_, size_);
  if (fd_ >= 0) ::close(fd_);
}

void GGUFMap::release(const TensorEntry& e) const {
  const uintptr_t page = (uintptr_t)sysconf(_SC_PAGESIZE);
  const uintptr_t lo = ((uintptr_t)(base_ + e.offset) + page - 1) / page * page;
  const uintptr_t hi = (uintptr_t)(base_ + e.offset + e.nbytes) / page * page;
  if (hi > lo) (void)madvise((void*)lo, hi - lo, MADV_DONTNEED);
}

const TensorEntry& GGUFMap::get(const std::string& name) const {
  auto it = index_.find(name);
  if (it == index_.end()) throw std::runtime_error("no tensor " + name);
  return tensors_[it->second];
}

// Stream geometry (layout v2, see ollama_operator_amd/quant.py "device repack"): K padded to SB
// super-blocks of 256; codes piece-major across super-blocks, scales per super-block.
static void stream_bytes(int qt, int64_t K, int64_t out[4]) {
  const int64_t SB = (K + 255) / 256;
  out[0] = out[1] = out[2] = out[3] = 0;
  switch (qt) {
    case 12: out[0] = 128 * SB; out[1] = 16 * SB; break;
    case 13: out[0] = 128 * SB; out[1] = 16 * SB; out[2] = 32 * SB; break;
    case 14: out[0] = 128 * SB; out[1] = 64 * SB; out[2] = 16 * SB; out[3] = 2 * SB; break;
    case 2: out[0] = 128 * SB; out[1] = 16 * SB; break;
    case 8: out[0] = 256 * SB; out[1] = 16 * SB; break;
    default: throw std::runtime_error("repack: unsupported type");
  }
}

static inline void copy_xor80(uint8_t* d, const uint8_t* s) {  // high nibble -> signed (n - 8)
  for (int i = 0; i < 16; ++i) d[i] = s[i] ^ 0x80;
}

// Q5_K high bits of one super-block (32 B, ggml order: bit j of qh[l] = weight l of sub-block j)
// -> 8 pieces x 4 B: piece t = 2c + h, byte j holds lo (sub-block 2c) weights 16h + 4k + j at bit k and
// hi (sub-block 2c + 1) weights at bit 4 + k (quant.py _q5k_qh_split).
static void q5k_split_qh(const uint8_t* qh, uint8_t* dst, int64_t piece_stride) {
  for (int t = 0; t < 8; ++t) {
    const int c = t >> 1, h = t & 1;
    uint8_t o[4] = {0, 0, 0, 0};
    for (int i = 0; i < 16; ++i) {
      const int v = qh[16 * h + i];
      o[i & 3] |= (uint8_t)((((v >> (2 * c)) & 1) << (i >> 2)) | (((v >> (2 * c + 1)) & 1) << (4 + (i >> 2))));
    }
    std::memcpy(dst + t * piece_stride, o, 4);
  }
}

// Q6_K high bits of one super-block (64 B, ggml order) -> 8 pieces x (H0 | H1), 8 B each.
static void q6k_split_qh(const uint8_t* qh, uint8_t* dst, int64_t piece_stride) {
  for (int n = 0; n < 2; ++n)
    for (int sub = 0; sub < 4; ++sub) {
      uint8_t o[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int half = 0; half < 2; ++half) {
        const int f = (sub >> 1) + 2 * half;
        for (int i = 0; i < 16; ++i) {
          const int bits = (qh[n * 32 + (sub & 1) * 16 + i] >> (2 * f)) & 3;
          o[half * 4 + (i & 3)] |= (uint8_t)(bits << (2 * (i >> 2)));
        }
      }
      std::memcpy(dst + (4 * n + sub) * piece_stride, o, 8);
    }
}

void repack_rows(const uint8_t* src, int qtype, int64_t K_src, const int64_t* rows, const int64_t* dst_rows,
                 int64_t n_rows, int64_t kb0, int64_t kb1, uint8_t* const dst[4], int n_threads, int64_t K_out) {
  int blk, nb;
  block_geom(qtype, blk, nb);
  const int64_t nblk_src = K_src / blk;
  if (kb0 < 0 || kb1 > nblk_src || kb0 >= kb1) throw std::runtime_error("repack: bad K block range");
  const int64_t K = (kb1 - kb0) * blk;
  if (K_out < K) K_out = K;
  const int64_t SB = (K_out + 255) / 256;  // the destination's super-blocks per row (stride of every stream)
  int64_t sb[4];
  stream_bytes(qtype, K_out, sb);
  const int64_t row_bytes = nblk_src * nb;
  auto work = [&](int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      const uint8_t* s = src + rows[r] * row_bytes + kb0 * nb;
      const int64_t o = dst_rows ? dst_rows[r] : r;
      uint8_t* d0 = dst[0] + o * sb[0];
      uint8_t* d1 = dst[1] + o * sb[1];
      uint8_t* d2 = dst[2] ? dst[2] + o * sb[2] : nullptr;
      uint8_t* d3 = dst[3] ? dst[3] + o * sb[3] : nullptr;
      for (int64_t b = 0; b < kb1 - kb0; ++b, s += nb) {
        switch (qtype) {
          case 12:  // d,dmin,scales | qs (8 pieces)
            std::memcpy(d1 + 16 * b, s, 16);
            for (int t = 0; t < 8; ++t) copy_xor80(d0 + (t * SB + b) * 16, s + 16 + 16 * t);
            break;
          case 13:  // d,dmin,scales | qh | qs (unsigned nibbles: the 5th bit is OR-ed in by the kernels)
            std::memcpy(d1 + 16 * b, s, 16);
            q5k_split_qh(s + 16, d2 + b * 4, SB * 4);
            for (int t = 0; t < 8; ++t) std::memcpy(d0 + (t * SB + b) * 16, s + 48 + 16 * t, 16);
            break;
          case 14:  // ql | qh | sc | d
            for (int t = 0; t < 8; ++t) std::memcpy(d0 + (t * SB + b) * 16, s + 16 * t, 16);
            q6k_split_qh(s + 128, d1 + b * 8, SB * 8);
            std::memcpy(d2 + 16 * b, s + 192, 16);
            std::memcpy(d3 + 2 * b, s + 208, 2);
            break;
          case 2: {  // d | qs ; 32-weight block b = piece (b & 7) of super-block b >> 3
            const int64_t g = b >> 3, t = b & 7;
            std::memcpy(d1 + 16 * g + 2 * t, s, 2);
            copy_xor80(d0 + (t * SB + g) * 16, s + 2);
            break;
          }
          case 8: {
            const int64_t g = b >> 3, t = b & 7;
            std::memcpy(d1 + 16 * g + 2 * t, s, 2);
            std::memcpy(d0 + (t * SB + g) * 32, s + 2, 32);
            break;
          }
        }
      }
    }
  };
  n_threads = std::max(1, std::min<int>(n_threads, (int)std::min<int64_t>(n_rows, 64)));
  if (n_threads == 1) {
    work(0, n_rows);
    return;
  }
  std::vector<std::thread> th;
  const int64_t per = (n_rows + n_threads - 1) / n_threads;
  for (int t = 0; t < n_threads; ++t) {
    const int64_t a = t * per, b = std::min(n_rows, a + per);
    if (a < b) th.emplace_back(work, a, b);
  }
  for (auto& t : th) t.join();
}

}  // namespace omx
