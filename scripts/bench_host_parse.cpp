// Host entropy-stage timing (no GPU): the batch host stage (wg::parse_all into a staging
// arena, the code behind wg_batch_create) over the given .webp files.  Prints ms per frame on
// one thread, the batch rate on T threads, and the device-input bytes per MB.  Build:
//   g++ -O2 -std=c++17 -Igo-webp_amd/csrc/host -Iinclude scripts/bench_host_parse.cpp \
//       go-webp_amd/csrc/host/*.cpp -lpthread -o /tmp/bench_host_parse
//   /tmp/bench_host_parse [-t THREADS] [-n FRAMES] [-r REPS] files...   (best of REPS batches)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>

#include "batch.h"
#include "host.h"

int main(int argc, char** argv) {
  int threads = 8, nframes = 64, reps = 3;
  std::vector<std::vector<uint8_t>> files;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "-t") && i + 1 < argc) {
      threads = std::atoi(argv[++i]);
      continue;
    }
    if (!std::strcmp(argv[i], "-r") && i + 1 < argc) {
      reps = std::atoi(argv[++i]);
      continue;
    }
    if (!std::strcmp(argv[i], "-n") && i + 1 < argc) {
      nframes = std::atoi(argv[++i]);
      continue;
    }
    std::ifstream f(argv[i], std::ios::binary);
    files.emplace_back(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  }
  if (files.empty()) return 1;
  std::vector<const uint8_t*> ptrs;
  std::vector<size_t> sizes;
  for (int i = 0; i < nframes; ++i) {
    ptrs.push_back(files[(size_t)i % files.size()].data());
    sizes.push_back(files[(size_t)i % files.size()].size());
  }
  wg_decoder_options opt{};
  opt.colorspace = 1;
  auto alloc = [](size_t b) { return std::malloc(b); };
  auto release = [](void* p) { std::free(p); };
  for (int pass = 0; pass < 2; ++pass) {
    const int t = pass == 0 ? 1 : threads;
    const int n = pass == 0 ? (int)files.size() : nframes;
    wg::WorkerPool pool(t);
    wg::StagingArena arena(alloc, release);
    std::vector<wg::FrameParse> out;
    double best = 1e30;
    for (int rep = 0; rep < reps; ++rep) {  // the first batch grows the arena (and faults it in)
      arena.begin_batch();
      const auto t0 = std::chrono::steady_clock::now();
      wg::parse_all(ptrs.data(), sizes.data(), n, opt, &pool, &arena, out);
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      size_t nb = 0, nmb = 0, bytes = 0;
      for (auto& f : out) {
        if (f.status) {
          std::printf("status %d\n", f.status);
          return 1;
        }
        nb += f.n_blocks;
        nmb += (size_t)f.info.mb_w * f.info.mb_h;
        bytes += f.input.bytes;
      }
      best = std::min(best, dt);
      if (rep + 1 == reps)
        std::printf("%d thread(s), %d frames: best of %d %.2f ms/frame (%.1f frames/s), %.2f blocks/MB, %.1f B/MB staged\n",
                    t, n, reps, 1e3 * best / n * t, n / best, (double)nb / (double)nmb, (double)bytes / (double)nmb);
    }
  }
  return 0;
}
