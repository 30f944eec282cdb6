#pragma once
#include <stdint.h>

#include <string>
#include <unordered_map>
#include <vector>

namespace omx {

struct TensorEntry {
  std::string name;
  std::vector<int64_t> dims;  // ggml order (ne0 first)
  int type = 0;
  int64_t n_elements = 0;
  uint64_t offset = 0;        // absolute file offset
  uint64_t nbytes = 0;
};

class GGUFMap {
 public:
  explicit GGUFMap(const std::string& path);
  ~GGUFMap();
  GGUFMap(const GGUFMap&) = delete;
  GGUFMap& operator=(const GGUFMap&) = delete;

  const std::vector<TensorEntry>& tensors() const { return tensors_; }
  const TensorEntry& get(const std::string& name) const;
  const uint8_t* data(const TensorEntry& e) const { return base_ + e.offset; }
  size_t size() const { return size_; }
  uint32_t version() const { return version_; }
  // drop this process's resident pages of a tensor's bytes (madvise MADV_DONTNEED on the read-only
  // mapping; a later read faults them back in from the page cache): a loaded model does not keep the
  // blob resident next to its repacked copy
  void release(const TensorEntry& e) const;

 private:
  int fd_ = -1;
  const uint8_t* base_ = nullptr;
  size_t size_ = 0;
  uint32_t version_ = 0;
  uint64_t data_offset_ = 0;
  std::vector<TensorEntry> tensors_;
  std::unordered_map<std::string, size_t> index_;
};

// Repack source rows `rows[0..n_rows)` of a block-quantized matrix with K_src weights per row,
// keeping K blocks [kb0, kb1), into the device stream layout (qmat.h) at dst[0..3]; source row
// rows[i] lands in destination row dst_rows[i] (or i when dst_rows is null).
// K_out > K: the destination rows hold K_out weights (whole super-blocks); the blocks past K stay as the
// caller zeroed them (zero codes and scales: zero weights). The GPU loader pads ffn_down's K this way so
// every piece run of the decode GEMV starts on a 256-B boundary (Llama-2-7B: 43 -> 48 super-blocks).
void repack_rows(const uint8_t* src, int qtype, int64_t K_src, const int64_t* rows, const int64_t* dst_rows,
                 int64_t n_rows, int64_t kb0, int64_t kb1, uint8_t* const dst[4], int n_threads, int64_t K_out = 0);

}  // namespace omx
