// Host stages of one decode batch (no HIP here): every frame's container, headers, output
// options and entropy stage, in WebPDecode's order, with its device inputs written into the
// staging arena.  capi.cpp lays the regions out in HBM and launches the kernels.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "host.h"
#include "staging.h"

namespace wg {

// One lossless stream (a VP8L frame or a lossless ALPH stream) after the host stage: the
// entropy-coded image and its transform data in staging, the transforms in READ order.
struct LLMeta {
  int width = 0, height = 0, coded_width = 0, n_transforms = 0;
  int type[4] = {0, 0, 0, 0}, bits[4] = {0, 0, 0, 0}, xsize[4] = {0, 0, 0, 0};
  int cache_bits = 0;
  Region tokens, lits, tdata[4];  // coded-image tokens (resolved by K7), literals, transform data
  size_t off_coded = 0;           // capi.cpp: K7's output (the coded ARGB image) in the plane buffer
  size_t n_px() const { return (size_t)coded_width * (size_t)height; }
  size_t fail_pixel = SIZE_MAX;  // see VP8LFrame::fail_pixel
  bool two_pass() const {        // predictor and color indexing both present
    int cores = 0;
    for (int t = 0; t < n_transforms; ++t) cores += (type[t] == kVP8LPredictor || type[t] == kVP8LColorIndexing);
    return cores > 1;
  }
};

struct FrameParse {
  int status = WG_STATUS_OK;
  bool lossless = false;
  int width = 0, height = 0;
  // lossy: the device layout in one staging region (MbRec[mb_h][mb_w] | row_block0[mb_h] |
  // blocks[n_blocks][16]), offsets within it
  wg_vp8_info info{};
  Region input;
  size_t off_rows = 0, off_blocks = 0, n_blocks = 0, n_y2 = 0;  // n_y2: i16 MBs with a Y2 block
  int br_mb_y = 0, fail_row = -1;
  // lossless
  LLMeta ll;
  // ALPH plane of a lossy frame (f2): raw bytes in staging, or a lossless stream K3 decodes
  bool alpha = false;
  AlphaHeader ah;
  LLMeta al;
  Region araw;
  bool alpha_direct = false;  // capi.cpp: K4 reads the alpha stream's coded image itself (no K3)
  bool alpha_k7 = false;      // capi.cpp: K7 writes the stream's filtered bytes (LLTokDesc::afilt)
  bool emit_direct = false;   // capi.cpp: K1's tail / K2 write the output colorspace itself (no K6)
  // output (cropping, f4): out_w x out_h, taken at (win_x, win_y) of the frame's RGBA buffer
  // (rgba_w x rgba_h: the window itself for lossy frames, the whole frame for lossless)
  int out_w = 0, out_h = 0, win_x = 0, win_y = 0, rgba_w = 0, rgba_h = 0;
  bool cropped = false;
  // device layout (capi.cpp): offsets within the batch's plane and RGBA buffers
  size_t off_y = 0, off_u = 0, off_v = 0, off_cols = 0, off_gprog = 0, off_scratch = 0, off_rgba = 0;
  size_t off_ascratch = 0, off_argba = 0, off_aplane = 0, off_atile = 0;
  size_t off_yc = 0, off_uc = 0, off_vc = 0;
  int yc_stride = 0, uvc_stride = 0;
  bool wide = false;
};

// Output options (WebPIoInitFromOptions / WebPAllocateDecBuffer, webp.go): colorspace,
// scaling, cropping -> the frame's output window, or INVALID_PARAM / UNSUPPORTED_FEATURE.
// Needs f->width, f->height, f->lossless.
int apply_output_options(const wg_decoder_options& opt, FrameParse* f);

// One frame's host stages and its WebPDecode status (webp.go:483-556 order).  Device inputs
// go to the arena at `cur`.
int parse_one(const uint8_t* data, size_t size, const wg_decoder_options& opt, StagingArena* arena,
              StagingArena::Cursor* cur, FrameParse* fp);

// parse_one with its failure handling: a failed frame keeps only its status (nothing throws).
void parse_frame(const uint8_t* data, size_t size, const wg_decoder_options& opt, StagingArena* arena,
                 StagingArena::Cursor* cur, FrameParse* f);

// parse_one over n frames on the pool (one frame per task).  A failed frame keeps only its
// status; nothing throws.
void parse_all(const uint8_t* const* data, const size_t* sizes, int n, const wg_decoder_options& opt,
               WorkerPool* pool, StagingArena* arena, std::vector<FrameParse>& out);

}  // namespace wg
