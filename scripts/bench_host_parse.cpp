// Host entropy-stage timing (no GPU): parses the given lossy .webp files through the same
// wg::vp8_parse the batch path uses and prints ms per frame.  Build:
//   g++ -O2 -std=c++17 -Igo-webp_amd/csrc -Iinclude scripts/bench_host_parse.cpp \
//       go-webp_amd/csrc/build/host/container.o go-webp_amd/csrc/build/host/vp8_parse.o -o /tmp/bench_host_parse
#include <chrono>
#include <cstdio>
#include <fstream>
#include <iterator>
#include <vector>

#include "host/host.h"

int main(int argc, char** argv) {
  std::vector<std::vector<uint8_t>> files;
  for (int i = 1; i < argc; ++i) {
    std::ifstream f(argv[i], std::ios::binary);
    files.emplace_back(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  }
  for (int rep = 0; rep < 3; ++rep) {
    const auto t0 = std::chrono::steady_clock::now();
    size_t nb = 0, nmb = 0;
    for (auto& d : files) {
      wg::Container c;
      wg_features ft;
      wg::parse_container(d.data(), d.size(), &c, &ft);
      wg::SparseFrame sf;
      const int st = wg::vp8_parse(d.data() + c.payload_off, c.payload_size, 0, nullptr, nullptr, &sf);
      if (st) {
        std::printf("status %d\n", st);
        return 1;
      }
      nb += sf.blocks.size() / 16;
      nmb += sf.mbs.size();
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("%zu frames: %.2f ms/frame, %.1f non-zero blocks/MB\n", files.size(), 1e3 * dt / files.size(),
                (double)nb / (double)nmb);
  }
  return 0;
}
