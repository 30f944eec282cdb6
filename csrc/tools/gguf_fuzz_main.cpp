// Host-only fuzz / sanitizer driver for the native GGUF loader (untrusted model
// files are parsed by C++). Built with -fsanitize=address,undefined by tests/test_gguf_fuzz.py and
// `make asan`; every argument is a (possibly corrupted) GGUF file. A file must either parse or be
// rejected with std::exception -- any sanitizer report or crash fails the run.
#include <cstdio>
#include <exception>
#include <vector>

#include "../gguf/gguf.h"

int main(int argc, char** argv) {
  int parsed = 0, rejected = 0;
  for (int i = 1; i < argc; ++i) {
    try {
      omx::GGUFMap g(argv[i]);
      // touch every tensor's bytes and repack one row of each native quant type
      unsigned long long sum = 0;
      for (const auto& e : g.tensors()) {
        const uint8_t* p = g.data(e);
        for (uint64_t b = 0; b < e.nbytes; b += 4096) sum += p[b];
        if (!e.dims.empty() && (e.type == 2 || e.type == 8 || e.type == 12 || e.type == 14)) {
          const int64_t K = e.dims[0];
          const int blk = (e.type == 2 || e.type == 8) ? 32 : 256;
          if (K % blk == 0 && e.n_elements / K >= 1) {
            const int64_t SB = (K + 255) / 256;
            std::vector<uint8_t> d0(256 * SB), d1(64 * SB), d2(16 * SB), d3(2 * SB);
            uint8_t* dst[4] = {d0.data(), d1.data(), d2.data(), d3.data()};
            const int64_t row = 0;
            omx::repack_rows(p, e.type, K, &row, nullptr, 1, 0, K / blk, dst, 1);
            sum += d0[0];
          }
        }
      }
      std::printf("%s: ok tensors=%zu sum=%llu\n", argv[i], g.tensors().size(), sum);
      ++parsed;
    } catch (const std::exception& ex) {
      std::printf("%s: rejected: %s\n", argv[i], ex.what());
      ++rejected;
    }
  }
  std::printf("parsed=%d rejected=%d\n", parsed, rejected);
  return 0;
}
