// RIFF / VP8X / optional-chunk parsing.
//
// Follows ParseHeadersInternal and its helpers in the reference
// (pkg/libwebp/decoder/webp.go: ParseRIFF :85-120, ParseVP8X :122-175,
// ParseOptionalChunks :177-237, ParseVP8Header :247-295, ParseHeadersInternal
// :300-440), plus VP8GetInfo (pkg/vp8/vp8_dec.go:189-228) and VP8LGetInfo for the frame
// size.  have_all_data = 1 is DecodeInto's pass (whole files: a chunk running past the end
// is NOT_ENOUGH_DATA); have_all_data = 0 is WebPGetFeatures' (headers == NULL: truncated
// chunks pass, and a VP8X file short of its image header still reports its features).
#include <cstring>

#include "host.h"

namespace wg {
namespace {

constexpr size_t kTag = 4, kChunkHdr = 8, kRiffHdr = 12, kVp8xChunk = 10;
constexpr uint64_t kMaxChunkPayload = ~0u - kChunkHdr - 1;
constexpr uint64_t kMaxImageArea = 1ull << 32;
constexpr size_t kVp8FrameHdr = 10, kVp8lFrameHdr = 5;
constexpr uint32_t kAlphaFlag = 0x10, kAnimFlag = 0x02;

inline uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
inline uint32_t le24(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16); }
inline bool tag_is(const uint8_t* p, const char* t) { return std::memcmp(p, t, 4) == 0; }

// VP8GetInfo (vp8_dec.go:189-228) with the integer promotions the Go lost restored.
bool vp8_get_info(const uint8_t* d, size_t size, size_t chunk_size, int* w, int* h) {
  if (size < kVp8FrameHdr) return false;
  if (!(d[3] == 0x9d && d[4] == 0x01 && d[5] == 0x2a)) return false;  // VP8CheckSignature
  const uint32_t bits = d[0] | (d[1] << 8) | (d[2] << 16);
  const bool key_frame = !(bits & 1);
  const int ww = ((d[7] << 8) | d[6]) & 0x3fff;
  const int hh = ((d[9] << 8) | d[8]) & 0x3fff;
  if (!key_frame) return false;
  if (((bits >> 1) & 7) > 3) return false;  // unknown profile
  if (!((bits >> 4) & 1)) return false;     // first frame invisible
  if ((bits >> 5) >= chunk_size) return false;
  if (ww == 0 || hh == 0) return false;
  *w = ww;
  *h = hh;
  return true;
}

// VP8LCheckSignature + ReadImageInfo (LSB-first bits).
bool vp8l_check_signature(const uint8_t* d, size_t size) {
  return size >= kVp8lFrameHdr && d[0] == 0x2f && (d[4] >> 5) == 0;
}
bool vp8l_get_info(const uint8_t* d, size_t size, int* w, int* h, int* a) {
  if (!vp8l_check_signature(d, size)) return false;
  uint64_t v = 0;
  for (int i = 0; i < 5; ++i) v |= (uint64_t)d[i] << (8 * i);
  if ((v & 0xff) != 0x2f) return false;
  *w = (int)((v >> 8) & 0x3fff) + 1;
  *h = (int)((v >> 22) & 0x3fff) + 1;
  *a = (int)((v >> 36) & 1);
  if (((v >> 37) & 7) != 0) return false;
  return true;
}

}  // namespace

int parse_container(const uint8_t* data, size_t data_size, Container* c, wg_features* feat, bool have_all_data) {
  *c = Container{};
  if (data == nullptr || data_size < kRiffHdr) return WG_STATUS_NOT_ENOUGH_DATA;
  const uint8_t* p = data;
  size_t left = data_size;
  uint64_t riff_size = 0;
  // ParseRIFF
  if (tag_is(p, "RIFF")) {
    if (!tag_is(p + 8, "WEBP")) return WG_STATUS_BITSTREAM_ERROR;
    const uint32_t size = le32(p + kTag);
    if (size < kTag + kChunkHdr) return WG_STATUS_BITSTREAM_ERROR;
    if (size > kMaxChunkPayload) return WG_STATUS_BITSTREAM_ERROR;
    if (have_all_data && size > left - kChunkHdr) return WG_STATUS_NOT_ENOUGH_DATA;
    riff_size = size;
    p += kRiffHdr;
    left -= kRiffHdr;
  }
  const bool found_riff = riff_size > 0;
  // ParseVP8X
  bool found_vp8x = false;
  int canvas_w = 0, canvas_h = 0;
  uint32_t vflags = 0;
  if (left < kChunkHdr) return WG_STATUS_NOT_ENOUGH_DATA;
  if (tag_is(p, "VP8X")) {
    if (le32(p + kTag) != kVp8xChunk) return WG_STATUS_BITSTREAM_ERROR;
    if (left < kChunkHdr + kVp8xChunk) return WG_STATUS_NOT_ENOUGH_DATA;
    vflags = le32(p + 8);
    canvas_w = 1 + (int)le24(p + 12);
    canvas_h = 1 + (int)le24(p + 15);
    if ((uint64_t)canvas_w * (uint64_t)canvas_h >= kMaxImageArea) return WG_STATUS_BITSTREAM_ERROR;
    p += kChunkHdr + kVp8xChunk;
    left -= kChunkHdr + kVp8xChunk;
    found_vp8x = true;
  }
  if (!found_riff && found_vp8x) return WG_STATUS_BITSTREAM_ERROR;
  c->has_alpha = !!(vflags & kAlphaFlag);
  c->has_animation = !!(vflags & kAnimFlag);
  int image_w = canvas_w, image_h = canvas_h;
  auto finish = [&](int status) {
    // ParseHeadersInternal's ReturnWidthHeight: GetFeatures on a VP8X file short of data
    // still succeeds with the canvas size
    if (status == WG_STATUS_NOT_ENOUGH_DATA && found_vp8x && !have_all_data) status = WG_STATUS_OK;
    if (status != WG_STATUS_OK) return status;
    if (feat) {
      feat->width = image_w;
      feat->height = image_h;
      feat->has_alpha = c->has_alpha | (c->alpha_size > 0);
      feat->has_animation = c->has_animation;
      feat->format = c->format;
    }
    c->width = image_w;
    c->height = image_h;
    return status;
  };
  if (found_vp8x && c->has_animation) {
    // WebPDecode does not decode animations; features come from VP8X only.
    finish(WG_STATUS_OK);
    return have_all_data ? WG_STATUS_UNSUPPORTED_FEATURE : WG_STATUS_OK;
  }
  if (left < kTag) return finish(WG_STATUS_NOT_ENOUGH_DATA);
  // ParseOptionalChunks
  if ((found_riff && found_vp8x) || (!found_riff && !found_vp8x && tag_is(p, "ALPH"))) {
    uint64_t total = kTag + kChunkHdr + kVp8xChunk;
    for (;;) {
      if (left < kChunkHdr) return finish(WG_STATUS_NOT_ENOUGH_DATA);
      const uint32_t csize = le32(p + kTag);
      if (csize > kMaxChunkPayload) return WG_STATUS_BITSTREAM_ERROR;
      const uint64_t disk = (kChunkHdr + (uint64_t)csize + 1) & ~1ull;
      total += disk;
      if (riff_size > 0 && total > riff_size) return WG_STATUS_BITSTREAM_ERROR;
      if (tag_is(p, "VP8 ") || tag_is(p, "VP8L")) break;
      if (left < disk) return finish(WG_STATUS_NOT_ENOUGH_DATA);
      if (tag_is(p, "ALPH")) {
        c->alpha_off = (size_t)(p + kChunkHdr - data);
        c->alpha_size = csize;
      }
      p += disk;
      left -= disk;
    }
  }
  // ParseVP8Header
  if (left < kChunkHdr) return finish(WG_STATUS_NOT_ENOUGH_DATA);
  const bool is_vp8 = tag_is(p, "VP8 "), is_vp8l = tag_is(p, "VP8L");
  size_t chunk_size;
  if (is_vp8 || is_vp8l) {
    const uint32_t size = le32(p + kTag);
    const uint64_t minimal = kTag + kChunkHdr;
    if (riff_size >= minimal && size > riff_size - minimal) return WG_STATUS_BITSTREAM_ERROR;
    if (have_all_data && size > left - kChunkHdr) return finish(WG_STATUS_NOT_ENOUGH_DATA);
    chunk_size = size;
    p += kChunkHdr;
    left -= kChunkHdr;
    c->is_lossless = is_vp8l;
  } else {
    c->is_lossless = vp8l_check_signature(p, left);
    chunk_size = left;
  }
  if (chunk_size > kMaxChunkPayload) return WG_STATUS_BITSTREAM_ERROR;
  c->format = c->is_lossless ? 2 : 1;
  if (!c->is_lossless) {
    if (left < kVp8FrameHdr) return finish(WG_STATUS_NOT_ENOUGH_DATA);
    if (!vp8_get_info(p, left, chunk_size, &image_w, &image_h)) return WG_STATUS_BITSTREAM_ERROR;
  } else {
    if (left < kVp8lFrameHdr) return finish(WG_STATUS_NOT_ENOUGH_DATA);
    int a = 0;
    if (!vp8l_get_info(p, left, &image_w, &image_h, &a)) return WG_STATUS_BITSTREAM_ERROR;
    if (!found_vp8x) c->has_alpha = a;
  }
  if (found_vp8x && (canvas_w != image_w || canvas_h != image_h)) return WG_STATUS_BITSTREAM_ERROR;
  c->payload_off = (size_t)(p - data);
  c->payload_size = left;  // io.data_size = headers.data_size - headers.offset
  return finish(WG_STATUS_OK);
}

}  // namespace wg

namespace wg {

// ALPHInit's header checks (alpha_dec.go:57-101): ALPHA_HEADER_LEN = 1, method 0/1,
// any of the four filters, pre-processing 0/1, reserved bits 0; raw alpha must hold
// width * height bytes.
bool parse_alpha_header(const uint8_t* data, size_t size, int width, int height, AlphaHeader* out) {
  if (data == nullptr || size <= 1) return false;
  out->method = data[0] & 3;
  out->filter = (data[0] >> 2) & 3;
  out->pre_processing = (data[0] >> 4) & 3;
  if (out->method > 1 || out->pre_processing > 1 || (data[0] >> 6) != 0) return false;
  if (out->method == 0 && size - 1 < (size_t)width * (size_t)height) return false;
  return true;
}

int output_bpp(int mode) {
  switch (mode) {
    case 0:
    case 2: return 3;
    case 5:
    case 6:
    case 10: return 2;
    case 1:
    case 3:
    case 4:
    case 7:
    case 8:
    case 9: return 4;
    default: return 0;
  }
}

}  // namespace wg
