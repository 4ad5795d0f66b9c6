// Layout of the batched, device-resident decode inputs/outputs (shared host/device).
//
// One lossy frame in HBM:
//   MbRec[mb_h][mb_w]          16 B per macroblock (modes, non-zero block mask,
//                              filter strengths) -- what the reference keeps in
//                              VP8MBData + VP8FInfo (pkg/vp8/models.go:66-107)
//   row_block0[mb_h]           index of the first coefficient block of each MB row
//   blocks[n_nonzero][16]      int16 coefficients of every non-zero 4x4 block in MB
//                              raster order: the i16 MB's Y2 block first (kY2Bit; its
//                              Walsh-Hadamard transform runs on the device), then Y
//                              0..15 (AC only for i16 MBs: their DC comes from Y2),
//                              U 16..19, V 20..23; stored column-major
//                              (blocks[4*c + k] = coeff[4*k + c]) so lane c of the
//                              IDCT / WHT reads its column with one load
//   Y/U/V planes               16*mb_w x 16*mb_h and 8*mb_w x 8*mb_h (MB padded)
//   RGBA                       width x height x 4
#pragma once
#include <stdint.h>

namespace wg {

#if defined(__HIPCC__)
// Pointers read out of a FrameDesc are generic; re-qualified as global, loads/stores
// become global_* (vmcnt only) instead of flat_* (vmcnt AND lgkmcnt, which every LDS
// wait would then also drain).  Scalar element types only (copying structs across
// address spaces is not allowed in C++).
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
template <typename T>
__host__ __device__ __forceinline__ gptr<T> as_global(T* p) {
  return (gptr<T>)p;
}
#endif

// MbRec.flags bit fields
constexpr uint32_t kNzMask = 0x00ffffffu;  // bit b set: 4x4 block b has coefficients
constexpr int kI4Shift = 24;                // is_i4x4
constexpr int kYModeShift = 25;             // i16 mode (B_DC/TM/VE/HE = 0..3)
constexpr int kUVModeShift = 27;            // chroma mode (0..3)
constexpr uint32_t kY2Bit = 1u << 29;       // i16 MB with a non-zero Y2 block (stored first)

struct MbRec {
  uint32_t flags;
  uint32_t imodes_lo;  // 4 bits per i4x4 block, blocks 0..7
  uint32_t imodes_hi;  // blocks 8..15
  uint32_t finfo;      // f_limit | f_ilevel << 8 | f_inner << 16 | hev_thresh << 24
};
static_assert(sizeof(MbRec) == 16, "MbRec must be 16 bytes");

// FrameDesc.flags: WG_FLAG_BYPASS_FILTERING (1) and WG_FLAG_NO_FANCY_UPSAMPLING (2) of the
// decode, plus kFrameEmitRgba: K1 itself converts the frame to RGBA in its tail (no K2).
constexpr int32_t kFrameNoFancy = 2;
constexpr int32_t kFrameEmitRgba = 1 << 8;
// K1: the frame's column store is too wide for LDS (vp8_recon_max_mb_w): the global-column
// instantiation runs it.
constexpr int32_t kFrameGlobalCols = 1 << 9;
// K1 split kernel: bytes of per-frame part-boundary progress flags (FrameDesc::gprog), one
// flag per 128-B line, for up to kMaxSplitParts parts
constexpr int kMaxSplitParts = 4;
constexpr int kGProgBytes = 128 * kMaxSplitParts;

struct FrameDesc {
  const MbRec* mbs;
  const uint32_t* row_block0;
  const int16_t* blocks;
  uint8_t* y;
  uint8_t* u;
  uint8_t* v;
  uint8_t* rgba;
  uint8_t* cols;  // K1 column store in global memory (mb_w * 160 B): used by wide frames
                  // (kFrameGlobalCols) and by the split kernel, which runs every frame from it
  int32_t width, height, mb_w, mb_h;
  int32_t y_stride, uv_stride, rgba_stride, filter_type;
  int32_t flags, valid, blocks_bytes;  // blocks_bytes: size of `blocks` (K1 bounds)
  // alpha-first batches (K4 before K1): the frame's unfiltered alpha plane (width-byte rows) at
  // y + 16 * alpha_off16, which the YUV -> RGBA strips take A from; 0: none (A = 255)
  int32_t alpha_off16;
  uint32_t* gprog;  // split kernel: one progress flag per part boundary, 128 B apart (kGProgBytes)
  // K1's tail / K2 output: 0 RGBA at `rgba`; else 1 + the WEBP_CSP_MODE written straight into
  // `rgba` (the frame's output slot, rgba_stride = bpp * width), rows bottom-up if emit_flip
  int32_t emit, emit_flip;
};
static_assert(sizeof(FrameDesc) == 128, "FrameDesc must be 128 bytes");

// VP8L coded-image tokens (host entropy stage -> K7, vp8l_resolve.hip): bits 31..30 the kind,
// bits 29..0 its payload.
constexpr uint32_t kTokLiteral = 0u << 30;  // payload: index into the stream's literal array
constexpr uint32_t kTokCache = 1u << 30;    // payload: color-cache key (< 1 << cache_bits)
constexpr uint32_t kTokCopy = 2u << 30;     // payload: backward distance in pixels (>= 1)
constexpr uint32_t kTokUnset = 3u << 30;    // after a failed symbol: value 0, no cache insert
constexpr uint32_t kTokPayload = (1u << 30) - 1;

// One lossless stream for K7: its tokens + literals in, the coded ARGB image out (K3's input).
struct LLTokDesc {
  const uint32_t* tokens;  // n_px tokens
  const uint32_t* lits;    // n_lits literal ARGB values
  uint32_t* coded;         // n_px resolved pixels
  int32_t n_px, n_lits, cache_bits, valid;
  int32_t trusted;  // tokens from the host entropy stage, which keeps them in bounds (no device check)
  int32_t a_cw;     // afilt: the coded image's width (coded pixels per row)
  // An 8-bit alpha stream (libwebp's ALPH: a colour map of at most 16 entries, bundled, or no
  // transform): K7 also writes its FILTERED alpha bytes -- green through the map -- into `afilt`
  // (a_width-byte rows, a_height rows), so K4 reads 1 B/px instead of the coded image (and, for
  // filter none or vertical / gradient, finds them already in its plane).  Null: not written.
  uint8_t* afilt;
  int32_t a_width, a_height, a_cbits, a_pal;  // a_pal: the map's green bytes in a_pg (else the green itself)
  uint32_t a_pg[4];                           // entry 4j + i in byte i of a_pg[j]
  uint32_t a_cw_m;                            // p / a_cw = (p * a_cw_m) >> (28 + a_cw_s) for p < 2^28
  int32_t a_cw_s;
  // gradient-filtered planes: rows 1.. go to `atile` instead, as K4's wavefront reads them -- per
  // 64-row band b (rows 1 + 64 b ..) and 16-column block c, a 1 KiB tile of 64 rows x 16 bytes,
  // tile (b, c) at ((b * ceil(a_width / 16) + c) << 10), row r at r << 4.  Row 0 stays in afilt.
  uint8_t* atile;
  uint64_t pad2;
};
static_assert(sizeof(LLTokDesc) == 112, "LLTokDesc must be 112 bytes");

// One lossless (VP8L) frame for K3.  `coded` is the entropy-coded ARGB image from the host
// stage; `stages` are its transforms in APPLICATION order (the reverse of bitstream order).
// Transform types: 0 predictor, 1 cross-color, 2 add-green (subtract-green undone),
// 3 color indexing.
struct LLStage {
  int32_t type, bits, xsize, tiles_per_row;
  const uint32_t* data;  // tile image (predictor / cross-color) or expanded palette
};
static_assert(sizeof(LLStage) == 24, "LLStage must be 24 bytes");

struct LLDesc {
  const uint32_t* coded;
  uint32_t* scratch;  // width*height words, used when the transforms need two passes
  uint8_t* rgba;
  uint64_t pad0;
  int32_t width, height, coded_width, n_stages;
  int32_t valid, rgba_stride, coded_bytes, scratch_bytes;
  LLStage stages[4];
  uint64_t pad1[4];
};
static_assert(sizeof(LLDesc) == 192, "LLDesc must be 192 bytes");

// One ALPH plane for K4 (alpha.hip).  Exactly one of green / raw / coded is set.
struct AlphaDesc {
  const uint8_t* green;  // K3's RGBA output of the lossless alpha stream: byte 1 of each pixel
  const uint8_t* raw;    // method 0: the filtered bytes, width*height
  uint8_t* plane;        // width*height scratch: filtered -> unfiltered alpha (vertical / gradient)
  uint8_t* rgba;         // the frame's RGBA output; K4 writes its A bytes
  int32_t width, height, rgba_stride, filter;  // plane size; filter: 0 none, 1 horizontal, 2 vertical, 3 gradient
  int32_t valid, win_x, win_y, win_w;           // the output window of the plane (cropping)
  int32_t win_h, cbits, coded_width;
  int32_t to_plane;  // alpha-first: the unfiltered bytes into `plane` (width-byte rows), not the A bytes
  // a lossless alpha stream whose only transform is color indexing (or that has none), filter
  // none / horizontal: K7's coded image read directly (K3 skipped) -- green of pal[index of
  // pixel x in coded[x >> cbits]], or of the coded pixel itself when pal is null
  const uint32_t* coded;
  const uint32_t* pal;   // 1 << (8 >> cbits) ARGB entries (ExpandColorMap's padded map)
  // gradient: the filtered rows 1.. in K7's band tiles (LLTokDesc::atile), or null (in `raw` /
  // the plane, width-byte rows)
  const uint8_t* tiles;
  uint64_t pad0;
};
static_assert(sizeof(AlphaDesc) == 112, "AlphaDesc must be 112 bytes");

// One frame's YUV output for K8 (emit_yuva.hip, MODE_YUV / MODE_YUVA): compact planes of the
// output window -- Y (width x height), U and V ((width + 1) / 2 x (height + 1) / 2), A (width x
// height, MODE_YUVA) -- from the lossy frame's reconstructed planes or the lossless frame's RGBA.
struct YuvaDesc {
  const uint8_t* y;      // lossy: the planes at the window origin (even x, y)
  const uint8_t* u;
  const uint8_t* v;
  const uint8_t* rgba;   // lossless: the RGBA window origin
  const uint8_t* a;      // lossy with ALPH: the unfiltered alpha plane at the window origin; else null (0xff)
  uint8_t* oy;           // outputs, rows of width / (width + 1) / 2 bytes, row 0 at the top
  uint8_t* ou;
  uint8_t* ov;
  uint8_t* oa;           // null: MODE_YUV
  int32_t y_stride, uv_stride, rgba_stride, a_stride;
  int32_t width, height, flip, lossless;
  int32_t valid, pad0, pad1, pad2, pad3, pad4;
};
static_assert(sizeof(YuvaDesc) == 128, "YuvaDesc must be 128 bytes");

// One frame's output conversion for K6 (emit.hip): RGBA window -> WEBP_CSP_MODE bytes.
struct EmitDesc {
  const uint8_t* src;  // RGBA, first pixel of the window
  uint8_t* dst;        // output rows (stride dst_stride), row 0 at the top
  int32_t src_stride, dst_stride, width, height;
  int32_t mode, flip, valid, pad0;
};
static_assert(sizeof(EmitDesc) == 48, "EmitDesc must be 48 bytes");

// One frame of an animation for K5 (anim.hip), in display order.
struct AnimFrameDesc {
  const uint8_t* rgba;     // the frame's decoded RGBA (width x height, stride 4*width)
  int32_t x, y, width, height;
  int32_t key;             // IsKeyFrame: start from a transparent canvas
  int32_t blend;           // frame > 1, blend method BLEND and not a key frame
  int32_t prev_dispose_bg; // the previous frame disposes to background: no blend inside its rectangle
  int32_t dispose_bg;      // this frame disposes to background
  int32_t px, py, pw, ph;  // the previous frame's rectangle
};
static_assert(sizeof(AnimFrameDesc) == 56, "AnimFrameDesc must be 56 bytes");

}  // namespace wg
