// Host entropy stage of VP8L (lossless): header, transform side images, prefix codes and
// the symbol walk -- everything that is a serial walk over the bit stream.  The main image
// leaves as one token per pixel (device_format.h kTok*: a literal's index, a color-cache key,
// or a backward-reference distance): the color cache and the LZ77 copies are resolved on the
// device (K7, vp8l_resolve.hip), and so are the inverse transforms (K3).  Side images
// (transform data, the meta prefix-code image) are resolved here: the host needs them.
//
// Semantics follow the VP8L format as libwebp 1.6.0 decodes it (the reference's
// pkg/vp8/vp8l_dec.c.go translates it; its DecodeImageStream is an unimplemented stub):
//   header                ReadImageInfo            vp8l_dec.c.go:108-116
//   transforms            ReadTransform            (libwebp vp8l_dec.c), ExpandColorMap :1196-1219
//   prefix codes          ReadHuffmanCode(s), ReadHuffmanCodeLengths
//   pixel decode          DecodeImageData          :1105-1153 (literal / back-reference / cache)
//   distance mapping      PlaneCodeToDistance      :157-167, kCodeToPlane :76
//   copy length/distance  GetCopyDistance          :140-150
//   color cache hash      VP8LHashPix              color_cache.go:46-48
#include <algorithm>
#include <cstring>
#include <vector>

#include "host.h"

namespace wg {
namespace {

constexpr int kNumLiteralCodes = 256;
constexpr int kNumLengthCodes = 24;
constexpr int kNumDistanceCodes = 40;
constexpr int kMaxCodeLength = 15;
constexpr int kRootBits = 8;
constexpr int kCodeLengthCodes = 19;
constexpr int kMaxCacheBits = 11;
constexpr int kMaxAlphabet = kNumLiteralCodes + kNumLengthCodes + (1 << kMaxCacheBits);
constexpr uint8_t kCodeLengthCodeOrder[kCodeLengthCodes] = {17, 18, 0, 1, 2, 3, 4, 5, 16, 6,
                                                            7,  8,  9, 10, 11, 12, 13, 14, 15};
// (dy, 8 - dx) pairs of the 120 short-distance plane codes (VP8L spec, kCodeToPlane).
constexpr uint8_t kCodeToPlane[120] = {
    0x18, 0x07, 0x17, 0x19, 0x28, 0x06, 0x27, 0x29, 0x16, 0x1a, 0x26, 0x2a, 0x38, 0x05, 0x37, 0x39, 0x15, 0x1b,
    0x36, 0x3a, 0x25, 0x2b, 0x48, 0x04, 0x47, 0x49, 0x14, 0x1c, 0x35, 0x3b, 0x46, 0x4a, 0x24, 0x2c, 0x58, 0x45,
    0x4b, 0x34, 0x3c, 0x03, 0x57, 0x59, 0x13, 0x1d, 0x56, 0x5a, 0x23, 0x2d, 0x44, 0x4c, 0x55, 0x5b, 0x33, 0x3d,
    0x68, 0x02, 0x67, 0x69, 0x12, 0x1e, 0x66, 0x6a, 0x22, 0x2e, 0x54, 0x5c, 0x43, 0x4d, 0x65, 0x6b, 0x32, 0x3e,
    0x78, 0x01, 0x77, 0x79, 0x53, 0x5d, 0x11, 0x1f, 0x64, 0x6c, 0x42, 0x4e, 0x76, 0x7a, 0x21, 0x2f, 0x75, 0x7b,
    0x31, 0x3f, 0x63, 0x6d, 0x52, 0x5e, 0x00, 0x74, 0x7c, 0x41, 0x4f, 0x10, 0x20, 0x62, 0x6e, 0x30, 0x73, 0x7d,
    0x51, 0x5f, 0x40, 0x72, 0x7e, 0x61, 0x6f, 0x50, 0x71, 0x7f, 0x60, 0x70};

inline int div_round_up(int n, int bits) { return (n + (1 << bits) - 1) >> bits; }

// LSB-first bit reader over the VP8L payload.
class BitReader {
 public:
  BitReader(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  uint32_t read(int nbits) {
    if (nbits == 0) return 0;
    if (avail_ < nbits) fill();
    if (avail_ < nbits) {
      eos_ = true;
      avail_ = 0;
      val_ = 0;
      return 0;
    }
    const uint32_t v = (uint32_t)(val_ & ((1ull << nbits) - 1));
    val_ >>= nbits;
    avail_ -= nbits;
    return v;
  }
  // At least kMaxCodeLength bits (zero-padded past the end) for a table lookup.
  uint32_t peek15() {
    if (avail_ < kMaxCodeLength) fill();
    return (uint32_t)(val_ & 0x7fff);
  }
  void skip(int nbits) {
    if (nbits > avail_) {
      eos_ = true;
      avail_ = 0;
      val_ = 0;
      return;
    }
    val_ >>= nbits;
    avail_ -= nbits;
  }
  bool eos() const { return eos_; }

 private:
  void fill() {  // 32 bits at a time away from the end, then byte by byte
    if (avail_ <= 32 && pos_ + 4 <= n_) {
      uint32_t w;
      std::memcpy(&w, p_ + pos_, 4);
      val_ |= (uint64_t)w << avail_;
      pos_ += 4;
      avail_ += 32;
    }
    while (avail_ <= 56 && pos_ < n_) {
      val_ |= (uint64_t)p_[pos_++] << avail_;
      avail_ += 8;
    }
  }
  const uint8_t* p_;
  size_t n_, pos_ = 0;
  uint64_t val_ = 0;
  int avail_ = 0;
  bool eos_ = false;
};

// Canonical prefix code, two-level lookup (8-bit root, per-prefix second level).
// Entry: bit 31 = link, otherwise (length << 16) | symbol; link: (sub_bits << 16) | offset.
class PrefixCode {
 public:
  // Returns false for an invalid code (over-subscribed, incomplete, or empty), the cases
  // libwebp's BuildHuffmanTable rejects.  A single used symbol decodes with 0 bits.
  bool build(const int* lengths, int n) {
    table_.assign(1u << kRootBits, 0);
    single_ = false;
    int count[kMaxCodeLength + 1] = {0};
    int used = 0, last = -1;
    for (int s = 0; s < n; ++s) {
      if (lengths[s] < 0 || lengths[s] > kMaxCodeLength) return false;
      if (lengths[s] > 0) {
        ++count[lengths[s]];
        ++used;
        last = s;
      }
    }
    if (used == 0) return false;
    if (used == 1) {  // single symbol: 0 bits
      std::fill(table_.begin(), table_.end(), (uint32_t)last);
      single_ = true;
      return true;
    }
    // completeness (Kraft sum == 1)
    int left = 1;
    for (int len = 1; len <= kMaxCodeLength; ++len) {
      left <<= 1;
      left -= count[len];
      if (left < 0) return false;
    }
    if (left != 0) return false;
    // canonical codes, sorted by (length, symbol)
    int next[kMaxCodeLength + 2] = {0};
    int code = 0;
    for (int len = 1; len <= kMaxCodeLength; ++len) {
      code = (code + count[len - 1]) << 1;
      next[len] = code;
    }
    // second-level sizes: for each root prefix, the longest code under it
    int sub_max[1 << kRootBits] = {0};
    syms_.clear();
    for (int s = 0; s < n; ++s) {
      const int len = lengths[s];
      if (!len) continue;
      const uint32_t c = (uint32_t)next[len]++;
      uint32_t r = 0;
      for (int b = 0; b < len; ++b) r |= ((c >> b) & 1u) << (len - 1 - b);
      syms_.push_back(Sym{r, s, len});
      if (len > kRootBits) {
        const uint32_t root = r & ((1u << kRootBits) - 1);
        sub_max[root] = std::max(sub_max[root], len - kRootBits);
      }
    }
    for (uint32_t root = 0; root < (1u << kRootBits); ++root) {
      if (!sub_max[root]) continue;
      const uint32_t off = (uint32_t)table_.size();
      table_[root] = 0x80000000u | ((uint32_t)sub_max[root] << 16) | off;
      table_.resize(off + (1u << sub_max[root]), 0);
    }
    for (const Sym& sy : syms_) {
      const uint32_t r = sy.rev;
      const int len = sy.len;
      const uint32_t e = ((uint32_t)len << 16) | (uint32_t)sy.sym;
      if (len <= kRootBits) {
        for (uint32_t k = r; k < (1u << kRootBits); k += 1u << len) table_[k] = e;
      } else {
        const uint32_t link = table_[r & ((1u << kRootBits) - 1)];
        const int sb = (int)((link >> 16) & 0x7fff);
        const uint32_t off = link & 0xffff;
        const uint32_t hi = r >> kRootBits;
        const int hl = len - kRootBits;
        for (uint32_t k = hi; k < (1u << sb); k += 1u << hl) table_[off + k] = e;
      }
    }
    return true;
  }
  // One used symbol (decodes with 0 bits): libwebp's htrees[c][0].bits == 0.
  bool single() const { return single_; }
  int read(BitReader& br) const {
    const uint32_t bits = br.peek15();
    uint32_t e = table_[bits & ((1u << kRootBits) - 1)];
    if (e & 0x80000000u) {
      const int sb = (int)((e >> 16) & 0x7fff);
      e = table_[(e & 0xffff) + ((bits >> kRootBits) & ((1u << sb) - 1))];
    }
    br.skip((int)(e >> 16));
    return (int)(e & 0xffff);
  }

 private:
  struct Sym {
    uint32_t rev;  // code, bit-reversed (LSB-first stream order)
    int sym, len;
  };
  std::vector<uint32_t> table_;
  std::vector<Sym> syms_;  // build() scratch, kept for reuse
  bool single_ = false;
};

struct HTreeGroup {
  PrefixCode code[5];  // green+length+cache, red, blue, alpha, distance
};

struct Decoder {
  BitReader br;
  int status = WG_STATUS_OK;
  // The headerless ALPH stream: libwebp decodes it with DecodeAlphaData (8-bit path) when
  // it only has a color-indexing transform and trivial red/blue/alpha codes.
  bool alpha_stream = false;
  bool in_main_pixels = false;  // the level-0 pixel loop has started (alpha error mapping)
  size_t fail_pos = SIZE_MAX;   // main image: first pixel of the symbol that failed
  std::vector<int> lengths;     // code lengths of the code being read (libwebp's code_lengths)
  // Called once the main image's header, transforms and codes are read, before its pixels
  // (libwebp's DecodeInto runs the output options between VP8LDecodeHeader and
  // VP8LDecodeImage, webp.go:528-544): a non-OK status stops the decode there.
  int (*pre_pixels)(void* ctx) = nullptr;
  void* pre_pixels_ctx = nullptr;
  int pre_pixels_status = WG_STATUS_OK;
  PrefixCode scratch;           // codes of meta groups the image never selects: read, validated, dropped
  explicit Decoder(const uint8_t* p, size_t n) : br(p, n), lengths(kMaxAlphabet, 0) {}
  bool fail(int st) {
    if (status == WG_STATUS_OK) status = st;
    return false;
  }
  // Non-incremental WebPDecode reports every end-of-stream as a bitstream error
  // (DecodeImageStream / DecodeImageData, vp8l_dec.c.go:1180-1187).
  bool check_eos() { return br.eos() ? fail(WG_STATUS_BITSTREAM_ERROR) : true; }

  bool read_code_lengths(const int* cl_lengths, int num_symbols, int* lens) {
    PrefixCode cl;
    if (!cl.build(cl_lengths, kCodeLengthCodes)) return fail(WG_STATUS_BITSTREAM_ERROR);
    int max_symbol = num_symbols;
    if (br.read(1)) {
      const int length_nbits = 2 + 2 * (int)br.read(3);
      max_symbol = 2 + (int)br.read(length_nbits);
      if (max_symbol > num_symbols) return fail(WG_STATUS_BITSTREAM_ERROR);
    }
    int symbol = 0, prev = 8;
    while (symbol < num_symbols) {
      if (max_symbol-- == 0) break;
      if (br.eos()) return fail(WG_STATUS_BITSTREAM_ERROR);
      const int code_len = cl.read(br);
      if (code_len < 16) {
        lens[symbol++] = code_len;
        if (code_len != 0) prev = code_len;
      } else {
        static const int kExtra[3] = {2, 3, 7}, kOffset[3] = {3, 3, 11};
        const int slot = code_len - 16;
        const int repeat = (int)br.read(kExtra[slot]) + kOffset[slot];
        if (symbol + repeat > num_symbols) return fail(WG_STATUS_BITSTREAM_ERROR);
        const int v = code_len == 16 ? prev : 0;
        for (int r = 0; r < repeat; ++r) lens[symbol++] = v;
      }
    }
    return check_eos();
  }

  // ReadHuffmanCode (libwebp 1.6.0 vp8l_dec.c; the reference's vp8l_dec.c.go:309-319 for the
  // simple code).  A simple-code symbol >= alphabet_size lands outside the range the table
  // is built over, so it is ignored; a code left with no symbol is invalid.
  bool read_code(int alphabet_size, PrefixCode* out) {
    int* lens = lengths.data();
    std::fill(lens, lens + alphabet_size, 0);
    if (br.read(1)) {  // simple code: one or two symbols of length 1
      const int num_symbols = (int)br.read(1) + 1;
      const int first_bits = br.read(1) ? 8 : 1;
      const int s0 = (int)br.read(first_bits);
      if (s0 < alphabet_size) lens[s0] = 1;
      if (num_symbols == 2) {
        const int s1 = (int)br.read(8);
        if (s1 < alphabet_size) lens[s1] = 1;
      }
    } else {
      int cl_lengths[kCodeLengthCodes] = {0};
      const int num_codes = (int)br.read(4) + 4;
      for (int i = 0; i < num_codes; ++i) cl_lengths[kCodeLengthCodeOrder[i]] = (int)br.read(3);
      if (!read_code_lengths(cl_lengths, alphabet_size, lens)) return false;
    }
    if (!check_eos()) return false;
    if (!out->build(lens, alphabet_size)) return fail(WG_STATUS_BITSTREAM_ERROR);
    return true;
  }

  static int copy_distance(int sym, BitReader& br) {
    if (sym < 4) return sym + 1;
    const int extra = (sym - 2) >> 1;
    const int offset = (2 + (sym & 1)) << extra;
    return offset + (int)br.read(extra) + 1;
  }

  static int plane_code_to_distance(int xsize, int plane_code) {
    if (plane_code > 120) return plane_code - 120;
    const int dc = kCodeToPlane[plane_code - 1];
    const int dist = (dc >> 4) * xsize + (8 - (dc & 0xf));
    return dist >= 1 ? dist : 1;
  }

  // The main image's symbol walk (DecodeImageData, vp8l_dec.c.go:1038-1189) without its
  // pixel values: per pixel a token -- kTokLiteral | index into f->lits, kTokCache | key, or
  // kTokCopy | distance (each pixel of a back-reference gets its own source distance).  The
  // color cache lookups/inserts (vp8l_dec.c.go:1105-1109, 1141-1153) and the copies
  // (CopyBlock32b, :915) are left to the device.  Pixels after a failing symbol are kTokUnset
  // (value 0; they are never shown: see VP8LFrame::fail_pixel).
  template <class GroupAt>
  bool decode_tokens(size_t total, int xsize, uint32_t mask, int cache_size, bool rba_single, VP8LFrame* f,
                     const GroupAt& group_at) {
    f->tokens.resize(total);  // no fill: every token is written below
    f->lits.clear();
    uint32_t* data = f->tokens.data();
    // The 8-bit alpha path (DecodeAlphaData) checks the end of stream only after storing a
    // symbol's pixels: a stream that runs out on the symbol completing the image still
    // decodes.  Everywhere else a symbol that reads past the end fails at its first pixel.
    const bool late_eos = alpha_stream && f->transforms.size() == 1 &&
                          f->transforms[0].type == kVP8LColorIndexing && cache_size == 0 && rba_single;
    size_t pos = 0;
    auto bad = [&](size_t at) {
      fail_pos = at;
      std::fill(data + at, data + total, kTokUnset);
      return fail(WG_STATUS_BITSTREAM_ERROR);
    };
    int x = 0, y = 0;
    const HTreeGroup* hg = &group_at(0, 0);
    while (pos < total) {
      const size_t start = pos;
      if ((x & mask) == 0) hg = &group_at(x, y);
      const int code = hg->code[0].read(br);
      if (code < kNumLiteralCodes) {
        const uint32_t r = (uint32_t)hg->code[1].read(br);
        const uint32_t b = (uint32_t)hg->code[2].read(br);
        const uint32_t a = (uint32_t)hg->code[3].read(br);
        if (br.eos() && !(late_eos && pos + 1 == total)) return bad(start);
        data[pos++] = kTokLiteral | (uint32_t)f->lits.size();
        f->lits.push_back((a << 24) | (r << 16) | ((uint32_t)code << 8) | b);
        if (++x >= xsize) {
          x = 0;
          ++y;
        }
      } else if (code < kNumLiteralCodes + kNumLengthCodes) {
        const int length = copy_distance(code - kNumLiteralCodes, br);
        const int dist_sym = hg->code[4].read(br);
        const int dist = plane_code_to_distance(xsize, copy_distance(dist_sym, br));
        if (br.eos() && !late_eos) return bad(start);
        if ((size_t)dist > pos || total - pos < (size_t)length) return bad(start);
        if (br.eos() && pos + (size_t)length < total) return bad(start);
        const uint32_t t = kTokCopy | (uint32_t)dist;
        for (int i = 0; i < length; ++i) data[pos++] = t;
        x += length;
        while (x >= xsize) {
          x -= xsize;
          ++y;
        }
        if (pos < total && (x & mask)) hg = &group_at(x, y);
      } else {
        if (br.eos()) return bad(start);
        const int key = code - (kNumLiteralCodes + kNumLengthCodes);
        if (key >= cache_size) return bad(start);
        data[pos++] = kTokCache | (uint32_t)key;
        if (++x >= xsize) {
          x = 0;
          ++y;
        }
      }
    }
    return true;
  }

  // One entropy-coded image: the main image when `level0` (as tokens into f->tokens /
  // f->lits), else a side image (pixel values into *out).
  bool decode_stream(int xsize, int ysize, bool level0, VP8LFrame* f, std::vector<uint32_t>* out) {
    if (level0) {
      unsigned seen = 0;
      while (br.read(1)) {
        const int type = (int)br.read(2);
        if (seen & (1u << type)) return fail(WG_STATUS_BITSTREAM_ERROR);
        seen |= 1u << type;
        VP8LTransform t;
        t.type = type;
        t.xsize = xsize;
        t.ysize = ysize;
        if (type == kVP8LPredictor || type == kVP8LCrossColor) {
          t.bits = (int)br.read(3) + 2;
          if (!decode_stream(div_round_up(xsize, t.bits), div_round_up(ysize, t.bits), false, nullptr, &t.data))
            return false;
        } else if (type == kVP8LColorIndexing) {
          const int num_colors = (int)br.read(8) + 1;
          t.bits = num_colors > 16 ? 0 : num_colors > 4 ? 1 : num_colors > 2 ? 2 : 3;
          std::vector<uint32_t> pal;
          if (!decode_stream(num_colors, 1, false, nullptr, &pal)) return false;
          // ExpandColorMap: per-byte running sum, padded to 1 << (8 >> bits) with 0
          const int final_num = 1 << (8 >> t.bits);
          t.data.assign((size_t)final_num, 0u);
          uint32_t prev = 0;
          for (int i = 0; i < num_colors; ++i) {
            const uint32_t a = pal[(size_t)i];
            const uint32_t v = (((a & 0xff00ff00u) + (prev & 0xff00ff00u)) & 0xff00ff00u) |
                               (((a & 0x00ff00ffu) + (prev & 0x00ff00ffu)) & 0x00ff00ffu);
            t.data[(size_t)i] = i == 0 ? a : v;
            prev = t.data[(size_t)i];
          }
          xsize = div_round_up(xsize, t.bits);
        } else {
          t.bits = 0;  // subtract green: no data
        }
        f->transforms.push_back(std::move(t));
        if (!check_eos()) return false;
      }
      f->coded_width = xsize;
    }
    // color cache
    int cache_bits = 0;
    if (br.read(1)) {
      cache_bits = (int)br.read(4);
      if (cache_bits < 1 || cache_bits > kMaxCacheBits) return fail(WG_STATUS_BITSTREAM_ERROR);
    }
    // prefix codes (meta codes only on the main image).  Tables are built only for the
    // groups the meta image selects, renumbered densely in order of first use; the codes
    // of the other group indices are still read and validated (ReadHuffmanCodes' mapping),
    // so a large index costs parse time, not memory.
    int huff_bits = 0, huff_xsize = 0;
    std::vector<uint32_t> huff_image;
    int num_groups = 1, num_groups_max = 1;
    std::vector<int> mapping;  // group index -> dense index, -1 = never selected
    if (level0 && br.read(1)) {
      huff_bits = (int)br.read(3) + 2;
      huff_xsize = div_round_up(xsize, huff_bits);
      if (!decode_stream(huff_xsize, div_round_up(ysize, huff_bits), false, nullptr, &huff_image)) return false;
      for (uint32_t& p : huff_image) {
        p = (p >> 8) & 0xffff;
        num_groups_max = std::max(num_groups_max, (int)p + 1);
      }
      mapping.assign((size_t)num_groups_max, -1);
      num_groups = 0;
      for (uint32_t& p : huff_image) {
        int& m = mapping[p];
        if (m < 0) m = num_groups++;
        p = (uint32_t)m;
      }
    }
    if (!check_eos()) return false;
    // libwebp itself keeps unused groups unless num_groups_max > 1000 or > the pixel count;
    // the groups it keeps decide whether its 8-bit alpha path applies (Is8bOptimizable).
    const bool libwebp_maps =
        !mapping.empty() && (num_groups_max > 1000 || (int64_t)num_groups_max > (int64_t)xsize * ysize);
    const int cache_size = cache_bits ? 1 << cache_bits : 0;
    std::vector<HTreeGroup> groups((size_t)num_groups);
    const int alphabet[5] = {kNumLiteralCodes + kNumLengthCodes + cache_size, kNumLiteralCodes, kNumLiteralCodes,
                             kNumLiteralCodes, kNumDistanceCodes};
    bool rba_single = true;  // every kept group's red, blue and alpha codes have one symbol
    for (int gi = 0; gi < num_groups_max; ++gi) {
      const int m = mapping.empty() ? gi : mapping[(size_t)gi];
      for (int j = 0; j < 5; ++j) {
        PrefixCode* pc = m >= 0 ? &groups[(size_t)m].code[j] : &scratch;
        if (!read_code(alphabet[j], pc)) return false;
        if (j >= 1 && j <= 3 && (m >= 0 || !libwebp_maps)) rba_single = rba_single && pc->single();
      }
    }
    // pixels
    const size_t total = (size_t)xsize * ysize;
    const uint32_t mask = huff_bits ? (1u << huff_bits) - 1 : ~0u;
    auto group_at = [&](int x, int y) -> const HTreeGroup& {
      if (!huff_bits) return groups[0];
      return groups[huff_image[(size_t)(y >> huff_bits) * huff_xsize + (x >> huff_bits)]];
    };
    if (level0) {
      if (pre_pixels && (pre_pixels_status = pre_pixels(pre_pixels_ctx)) != WG_STATUS_OK) return false;
      in_main_pixels = true;
      f->cache_bits = cache_bits;
      return decode_tokens(total, xsize, mask, cache_size, rba_single, f, group_at);
    }
    out->assign(total, 0u);
    uint32_t* data = out->data();
    std::vector<uint32_t> cache((size_t)std::max(cache_size, 1), 0u);
    const int cache_shift = 32 - cache_bits;
    auto insert = [&](uint32_t argb) {  // VP8LColorCacheInsert (color_cache.go:50-55)
      if (cache_bits) cache[(argb * 0x1e35a7bdu) >> cache_shift] = argb;
    };
    size_t pos = 0;
    int x = 0, y = 0;
    const HTreeGroup* hg = &group_at(0, 0);
    while (pos < total) {
      if ((x & mask) == 0) hg = &group_at(x, y);
      const int code = hg->code[0].read(br);
      if (code < kNumLiteralCodes) {
        const uint32_t r = (uint32_t)hg->code[1].read(br);
        const uint32_t b = (uint32_t)hg->code[2].read(br);
        const uint32_t a = (uint32_t)hg->code[3].read(br);
        if (br.eos()) return fail(WG_STATUS_BITSTREAM_ERROR);
        const uint32_t argb = (a << 24) | (r << 16) | ((uint32_t)code << 8) | b;
        data[pos++] = argb;
        insert(argb);
        if (++x >= xsize) {
          x = 0;
          ++y;
        }
      } else if (code < kNumLiteralCodes + kNumLengthCodes) {
        const int length = copy_distance(code - kNumLiteralCodes, br);
        const int dist_sym = hg->code[4].read(br);
        const int dist = plane_code_to_distance(xsize, copy_distance(dist_sym, br));
        if (br.eos() || (size_t)dist > pos || total - pos < (size_t)length) return fail(WG_STATUS_BITSTREAM_ERROR);
        for (int i = 0; i < length; ++i) {
          const uint32_t argb = data[pos - dist];
          data[pos++] = argb;
          insert(argb);
        }
        x += length;
        while (x >= xsize) {
          x -= xsize;
          ++y;
        }
        if (pos < total && (x & mask)) hg = &group_at(x, y);
      } else {
        if (br.eos()) return fail(WG_STATUS_BITSTREAM_ERROR);
        const int key = code - (kNumLiteralCodes + kNumLengthCodes);
        if (key >= cache_size) return fail(WG_STATUS_BITSTREAM_ERROR);
        const uint32_t argb = cache[(size_t)key];  // VP8LColorCacheLookup (color_cache.go:57-63)
        data[pos++] = argb;
        insert(argb);
        if (++x >= xsize) {
          x = 0;
          ++y;
        }
      }
    }
    return true;
  }
};

}  // namespace

int vp8l_parse(const uint8_t* data, size_t size, VP8LFrame* out, int (*pre_pixels)(void*), void* ctx) {
  if (!data || size < 5 || !out) return WG_STATUS_NOT_ENOUGH_DATA;
  out->fail_pixel = SIZE_MAX;
  Decoder d(data, size);
  if (d.br.read(8) != 0x2f) return WG_STATUS_BITSTREAM_ERROR;
  out->width = (int)d.br.read(14) + 1;
  out->height = (int)d.br.read(14) + 1;
  out->has_alpha = (int)d.br.read(1);
  if (d.br.read(3) != 0) return WG_STATUS_BITSTREAM_ERROR;
  out->transforms.clear();
  out->coded_width = out->width;
  out->cache_bits = 0;
  d.pre_pixels = pre_pixels;
  d.pre_pixels_ctx = ctx;
  if (!d.decode_stream(out->width, out->height, true, out, nullptr)) {
    if (d.pre_pixels_status != WG_STATUS_OK) return d.pre_pixels_status;
    out->fail_pixel = d.fail_pos;
    return d.status;
  }
  return WG_STATUS_OK;
}

// The ALPH chunk's lossless stream: a VP8L image stream without the 5-byte header, sized
// by the frame (VP8LDecodeAlphaHeader / VP8LDecodeAlphaImageStream, vp8l_dec.c.go:1493-1556).
// Status as WebPDecode reports it: a failure while reading the stream's transforms and
// codes leaves the alpha decoder without a VP8L decoder, which VP8DecompressAlphaRows
// reports as OUT_OF_MEMORY (alpha_dec.go:177-182); a failure in the pixel data is
// "Could not decode alpha data" = BITSTREAM_ERROR, seen only once the rows it lies in are
// requested (out->fail_pixel).
int vp8l_parse_alpha(const uint8_t* data, size_t size, int width, int height, VP8LFrame* out) {
  out->width = width;
  out->height = height;
  out->has_alpha = 0;
  out->transforms.clear();
  out->coded_width = width;
  out->cache_bits = 0;
  out->fail_pixel = SIZE_MAX;
  Decoder d(data, size);
  d.alpha_stream = true;
  if (!d.decode_stream(width, height, true, out, nullptr)) {
    if (!d.in_main_pixels) return WG_STATUS_OUT_OF_MEMORY;
    out->fail_pixel = d.fail_pos;
    return WG_STATUS_BITSTREAM_ERROR;
  }
  return WG_STATUS_OK;
}

}  // namespace wg
