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
#include "batch.h"
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
      {
        wg::StagingArena arena([](size_t b) { return std::malloc(b); }, [](void* q) { std::free(q); }, 1 << 20);
        wg::StagingArena::Cursor cur;
        wg::FrameParse fp;
        wg_decoder_options opt{};
        opt.colorspace = 1;
        if (it % 5 == 2) {  // a crop window, sometimes invalid
          opt.use_cropping = 1;
          opt.crop_left = (int)(rng() % 40) - 4;
          opt.crop_top = (int)(rng() % 40) - 4;
          opt.crop_width = (int)(rng() % 80);
          opt.crop_height = (int)(rng() % 80);
        }
        wg::parse_one(d.data(), d.size(), opt, &arena, &cur, &fp);
        arena.release(&cur);
      }
      if (wg::parse_container(d.data(), d.size(), &c, &ft) != 0) { ++runs; continue; }
      if (c.is_lossless) {
        wg::VP8LFrame lf;
        wg::vp8l_parse(d.data() + c.payload_off, c.payload_size, &lf);
      } else {
        wg::SparseFrame sf;
        // every third run bounded to a random crop bottom (the WebPDecode crop path)
        const int crop_bottom = it % 3 == 1 ? (int)(rng() % 64) : -1;
        int st = wg::vp8_parse(d.data(), d.size(), 0, &sf, crop_bottom);
        const wg_vp8_info& info = sf.info;
        if (st == 0) {
          // device-side invariants the kernels rely on
          size_t nmb = (size_t)info.mb_w * info.mb_h;
          if (sf.mbs.size() != nmb || sf.row_block0.size() != (size_t)info.mb_h) { printf("bad sizes\n"); return 1; }
          size_t tot = 0;
          for (int y = 0; y < info.mb_h; ++y) {
            if (sf.row_block0[(size_t)y] != tot) { printf("row index mismatch\n"); return 1; }
            for (int x = 0; x < info.mb_w; ++x)
              tot += __builtin_popcount(sf.mbs[(size_t)y * info.mb_w + x].flags & (wg::kNzMask | wg::kY2Bit));
          }
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
