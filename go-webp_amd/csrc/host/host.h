// Host-side stages of the WebP decode path: container parsing and the VP8 entropy
// stage (modes + residual tokens).  Their output is the batched per-macroblock
// record / coefficient stream consumed by the device kernels (device_format.h).
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#include "../../../include/gowebp_amd.h"
#include "../device_format.h"

namespace wg {

// Result of ParseHeadersInternal (pkg/libwebp/decoder/webp.go:300-440) with
// have_all_data = 1.
struct Container {
  int format = 0;  // 1 lossy, 2 lossless
  int width = 0, height = 0;
  int has_alpha = 0, has_animation = 0;
  size_t payload_off = 0, payload_size = 0;  // VP8 / VP8L bitstream
  size_t alpha_off = 0, alpha_size = 0;      // ALPH chunk payload (0 size = none)
  int is_lossless = 0;
};

// Bytes per pixel of an RGB-family WEBP_CSP_MODE (0..10): 3, 4 or 2; 0 for any other mode
// (K6, emit.hip, produces exactly these).
int output_bpp(int mode);

// have_all_data: 1 = DecodeInto's header pass, 0 = WebPGetFeatures' (see container.cpp).
int parse_container(const uint8_t* data, size_t size, Container* c, wg_features* feat, bool have_all_data = true);

// Growable buffer of trivially copyable T without zero-filling on growth (the entropy
// stage writes every element it keeps).
template <class T>
struct PodBuf {
  std::unique_ptr<T[]> p;
  size_t n = 0, cap = 0;
  T* data() { return p.get(); }
  const T* data() const { return p.get(); }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  void clear() { n = 0; }
  void release() {
    p.reset();
    n = cap = 0;
  }
  T* reserve_more(size_t k) {  // room for k more elements; returns the end
    if (n + k > cap) {
      const size_t nc = n + k > 2 * cap ? n + k : 2 * cap;
      T* q = new T[nc];
      if (n) std::memcpy(q, p.get(), n * sizeof(T));
      p.reset(q);
      cap = nc;
    }
    return p.get() + n;
  }
};

// Where the entropy stage writes one lossy frame's device layout (device_format.h): the
// batch hands out pinned staging memory, tools a SparseFrame's vectors.
struct SparseSink {
  MbRec* mbs = nullptr;            // mb_w * mb_h, raster order
  uint32_t* row_block0 = nullptr;  // mb_h: first coefficient block of each MB row
  int16_t* blocks = nullptr;       // room for sparse_max_blocks(mb_w, rows) blocks of 16 int16
};
// Upper bound on the coefficient blocks of `rows` MB rows: Y2 + 16 Y + 8 chroma per MB.
inline size_t sparse_max_blocks(int mb_w, int rows) { return (size_t)mb_w * (size_t)rows * 25; }
// Called once the headers are known: provide a sink for a frame of inf.mb_w x inf.mb_h MBs
// of which `rows` MB rows are parsed; false = out of memory.
using SparseAllocFn = bool (*)(void* ctx, const wg_vp8_info& inf, int rows, SparseSink* sink);
struct SparseResult {
  wg_vp8_info info{};
  size_t n_blocks = 0;  // blocks written
  size_t n_y2 = 0;      // of which Y2 blocks (one per i16 MB that has one)
  int br_mb_y = 0;      // MB rows parsed (VP8EnterCritical's br_mb_y_)
  int fail_row = -1;    // MB row whose parse failed (-1: none, or the headers)
};

// Entropy-decode one lossy frame into the device layout.  crop_bottom >= 0 bounds the MB
// rows parsed as WebPDecode does for a crop window (br_mb_y_ = (crop_bottom + 15 +
// kFilterExtraRows[filter_type]) >> 4, frame_dec.c.go); rows below it (and below a failing
// row) read as empty MBs, and a corrupt token stream there is not seen.
int vp8_parse_sparse(const uint8_t* data, size_t size, int flags, int crop_bottom, SparseAllocFn alloc, void* actx,
                     SparseResult* res);

// The same into vectors (tools, tests).
struct SparseFrame {
  wg_vp8_info info{};
  std::vector<MbRec> mbs;
  std::vector<uint32_t> row_block0;
  PodBuf<int16_t> blocks;  // 16 int16 per kept block
  int br_mb_y = 0, fail_row = -1;
};
int vp8_parse(const uint8_t* data, size_t size, int flags, SparseFrame* sf, int crop_bottom = -1);

// Entropy-decode one lossy frame into libwebp's data model (the CPU checker's input);
// `dense` (mb_w*mb_h) may be null to parse the headers only.
int vp8_parse(const uint8_t* data, size_t size, int flags, wg_vp8_info* info, wg_vp8_mb* dense,
              int crop_bottom = -1);

// VP8L (lossless) after the host entropy stage: the entropy-coded ARGB image and the
// transforms in bitstream (read) order; the device applies them in reverse.
enum : int { kVP8LPredictor = 0, kVP8LCrossColor = 1, kVP8LSubtractGreen = 2, kVP8LColorIndexing = 3 };

struct VP8LTransform {
  int type = 0;
  int bits = 0;               // tile bits (predictor / cross-color) or pixel-packing bits (color indexing)
  int xsize = 0, ysize = 0;   // image size the transform's output has
  std::vector<uint32_t> data; // tile image, or the expanded palette (1 << (8 >> bits) entries)
};

struct VP8LFrame {
  int width = 0, height = 0, has_alpha = 0;
  int coded_width = 0;                    // width of the coded image (reduced by color-index packing)
  std::vector<VP8LTransform> transforms;  // read order
  // The coded image before its color cache and back-references are resolved: one token per
  // pixel (coded_width * height, device_format.h kTok*), the literals they index, and the
  // stream's color cache bits (0 = no cache).
  std::vector<uint32_t> tokens;
  std::vector<uint32_t> lits;
  int cache_bits = 0;
  // After a failure in the pixel data: the first coded pixel whose symbol failed (SIZE_MAX:
  // the failure was in the header, transforms or codes).  A decode bounded to image rows
  // [0, r) -- a crop window, or the alpha rows requested so far -- fails iff
  // r * coded_width > fail_pixel.
  size_t fail_pixel = SIZE_MAX;
};

// Entropy-decode a VP8L bitstream (the VP8L chunk payload).  `pre_pixels` (optional) runs
// after the header, transforms and prefix codes, before the pixels; its non-OK status is
// returned as is (fail_pixel stays SIZE_MAX).
int vp8l_parse(const uint8_t* data, size_t size, VP8LFrame* out, int (*pre_pixels)(void*) = nullptr,
               void* ctx = nullptr);

// Animation demux (demux/demux.go): canvas + frames in display order.  A still image is a
// one-frame animation.  Status: OK, NOT_ENOUGH_DATA (truncated), BITSTREAM_ERROR (invalid).
struct AnimInfo {
  int canvas_width = 0, canvas_height = 0, loop_count = 0, frame_count = 0;
  uint32_t bgcolor = 0;
};
struct AnimFrame {
  int x_offset = 0, y_offset = 0, width = 0, height = 0, duration = 0;
  int dispose_bg = 0, no_blend = 0, has_alpha = 0;
  size_t off = 0, size = 0;  // the frame's fragment (ALPH + image chunk, or the whole bitstream)
};
int anim_demux(const uint8_t* data, size_t size, AnimInfo* info, std::vector<AnimFrame>* frames);

// ALPH chunk (alpha_dec.go:47-105): header byte = method (bits 0-1: 0 raw, 1 lossless),
// filter (2-3: none, horizontal, vertical, gradient), pre-processing (4-5), reserved (6-7).
struct AlphaHeader {
  int method = 0, filter = 0, pre_processing = 0;
};
// Validates the header as ALPHInit does; false -> WebPDecode's OUT_OF_MEMORY.
bool parse_alpha_header(const uint8_t* data, size_t size, int width, int height, AlphaHeader* out);
// The lossless alpha stream (headerless VP8L, green channel = alpha).
int vp8l_parse_alpha(const uint8_t* data, size_t size, int width, int height, VP8LFrame* out);

}  // namespace wg
