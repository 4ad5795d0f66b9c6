// Mutation fuzz of the host stages (container, VP8 / VP8L / ALPH entropy stages, ANIM
// demux) for tests/test_host_fuzz.py, built with ASan + UBSan: truncations and bit flips
// of every fixture must return a status, never crash, and successful VP8 parses must
// satisfy the invariants K1 relies on (record count, row index, one 16-coefficient block
// per set non-zero bit).  The meta-code amplification fixture (status/crafted_65536_groups)
// runs here too: it must parse within ASan's default memory.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <random>
#include <vector>
#include "host.h"
int main(int argc, char** argv) {
  std::mt19937 rng(1234);
  const int iters = atoi(getenv("WG_FUZZ_ITERS") ? getenv("WG_FUZZ_ITERS") : "300");
  long runs = 0;
  for (int i = 1; i < argc; ++i) {
    std::ifstream f(argv[i], std::ios::binary);
    std::vector<uint8_t> orig((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (orig.size() > 400000) continue;
    for (int it = 0; it < iters; ++it) {
      std::vector<uint8_t> d = orig;
      int mode = it % 3;
      if (mode == 0) d.resize(rng() % (d.size() + 1));
      else {
        int nflip = 1 + rng() % 8;
        for (int k = 0; k < nflip && !d.empty(); ++k) d[rng() % d.size()] ^= (uint8_t)(1u << (rng() % 8));
      }
      wg::Container c; wg_features ft;
      {
        wg::AnimInfo ai;
        std::vector<wg::AnimFrame> af;
        if (wg::anim_demux(d.data(), d.size(), &ai, &af) == 0)
          for (const auto& fr : af)
            if (fr.off > d.size() || fr.size > d.size() - fr.off) { printf("frame out of range\n"); return 1; }
      }
      if (wg::parse_container(d.data(), d.size(), &c, &ft) != 0) { ++runs; continue; }
      if (c.is_lossless) {
        wg::VP8LFrame lf;
        wg::vp8l_parse(d.data() + c.payload_off, c.payload_size, &lf);
      } else {
        wg_vp8_info info; wg::SparseFrame sf;
        // every third run bounded to a random crop bottom (the WebPDecode crop path)
        const int crop_bottom = it % 3 == 1 ? (int)(rng() % 64) : -1;
        int st = wg::vp8_parse(d.data(), d.size(), 0, &info, nullptr, &sf, crop_bottom);
        if (st == 0) {
          // device-side invariants the kernels rely on
          size_t nmb = (size_t)info.mb_w * info.mb_h;
          if (sf.mbs.size() != nmb || sf.row_block0.size() != (size_t)info.mb_h) { printf("bad sizes\n"); return 1; }
          size_t tot = 0;
          for (size_t m = 0; m < nmb; ++m) tot += __builtin_popcount(sf.mbs[m].flags & wg::kNzMask);
          if (tot * 16 != sf.blocks.size()) { printf("block count mismatch\n"); return 1; }
        }
        if (c.alpha_size) {
          wg::AlphaHeader ah;
          if (wg::parse_alpha_header(d.data() + c.alpha_off, c.alpha_size, ft.width, ft.height, &ah) && ah.method == 1) {
            wg::VP8LFrame af;
            wg::vp8l_parse_alpha(d.data() + c.alpha_off + 1, c.alpha_size - 1, ft.width, ft.height, &af);
          }
        }
      }
      ++runs;
    }
  }
  printf("%ld fuzz runs OK\n", runs);
}
