// Animation demux (ANIM / ANMF) for the animated-decode entry point.
//
// Follows the reference's demuxer (pkg/libwebp/demux/demux.go) with whole data
// (WebPDemux, allow_partial = 0):
//   ReadHeader :346-372, ParseSingleImage :374-412, ParseVP8XChunks :414-492 (ANIM first, then
//   ANMF frames; ICCP/EXIF/XMP/unknown chunks skipped), ParseVP8X :494-520,
//   ParseAnimationFrame :243-282 and StoreFrame :135-222 (first ALPH, then the first VP8/VP8L
//   chunk; its features give the frame's size; VP8L after ALPH is an error),
//   IsValidSimpleFormat / CheckFrameBounds / IsValidExtendedFormat :524-603 (as libwebp's C:
//   the Go translation advances the frame pointer before using it),
//   CreateRawImageDemuxer :617-641 (a bare VP8/VP8L bitstream is a one-frame image),
//   GetFramePayload :752-770 (a frame's fragment runs from its ALPH to the end of its image).
#include <cstring>

#include "host.h"

namespace wg {
namespace {

constexpr uint32_t kChunkHdr = 8, kRiffHdr = 12, kVp8xChunk = 10, kAnmfChunk = 16, kAnimChunk = 6;
constexpr uint32_t kMaxChunkPayload = ~0u - kChunkHdr - 1;
constexpr uint64_t kMaxImageArea = 1ull << 32;
constexpr uint32_t kAlphaFlag = 0x10, kAnimFlag = 0x02, kAllValidFlags = 0x3e;

inline uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
inline uint32_t le24(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16); }
inline uint32_t le16(const uint8_t* p) { return p[0] | (p[1] << 8); }
inline bool tag_is(const uint8_t* p, const char* t) { return std::memcmp(p, t, 4) == 0; }

struct Frame {
  AnimFrame f;
  size_t alpha_off = 0, alpha_size = 0;  // chunk header + payload available
  size_t image_off = 0, image_size = 0;
  int frame_num = 0;
  bool complete = false;
};

struct Demux {
  const uint8_t* buf = nullptr;
  size_t start = 0, end = 0, riff_end = 0;
  uint32_t flags = 0;
  int canvas_w = -1, canvas_h = -1, loop_count = 1;
  uint32_t bgcolor = 0xffffffffu;  // white by default (InitDemux)
  bool is_ext = false;
  std::vector<Frame> frames;

  size_t avail() const { return end - start; }
  bool size_invalid(uint64_t size) const { return size > riff_end - start; }

  // StoreFrame: ALPH (first), then the first VP8/VP8L image chunk; stops at anything else.
  bool store_frame(int frame_num, uint32_t min_size, Frame* fr) {
    if (avail() < kChunkHdr || avail() < min_size) return false;  // NEED_MORE_DATA: an error with whole data
    int alpha_chunks = 0, image_chunks = 0;
    for (;;) {
      const size_t chunk_start = start;
      const uint8_t* p = buf + start;
      const uint32_t payload = le32(p + 4);
      if (payload > kMaxChunkPayload) return false;
      const uint32_t padded = payload + (payload & 1);
      start += kChunkHdr;
      if (size_invalid(padded)) return false;
      const size_t available = padded > avail() ? avail() : padded;
      const size_t chunk_size = kChunkHdr + available;
      const bool full = padded <= avail();
      bool done = false;
      if (tag_is(p, "ALPH") && alpha_chunks == 0) {
        ++alpha_chunks;
        fr->alpha_off = chunk_start;
        fr->alpha_size = chunk_size;
        fr->f.has_alpha = 1;
        fr->frame_num = frame_num;
        start += available;
      } else if ((tag_is(p, "VP8L") || tag_is(p, "VP8 ")) && image_chunks == 0) {
        if (tag_is(p, "VP8L") && alpha_chunks > 0) return false;  // VP8L has its own alpha
        Container c;
        wg_features feat{};
        if (parse_container(buf + chunk_start, chunk_size, &c, &feat) != WG_STATUS_OK || !full) return false;
        ++image_chunks;
        fr->image_off = chunk_start;
        fr->image_size = chunk_size;
        fr->f.width = feat.width;
        fr->f.height = feat.height;
        fr->f.has_alpha |= feat.has_alpha;
        fr->frame_num = frame_num;
        fr->complete = true;
        start += available;
      } else {
        start -= kChunkHdr;  // rewind: the chunk belongs to the parent level
        done = true;
      }
      if (start == riff_end) done = true;
      else if (avail() < kChunkHdr) return false;
      if (done) return true;
    }
  }

  bool add_frame(const Frame& fr) {
    if (!frames.empty() && !frames.back().complete) return false;
    frames.push_back(fr);
    return true;
  }

  bool parse_single_image() {
    if (!frames.empty() || size_invalid(kChunkHdr) || avail() < kChunkHdr) return false;
    Frame fr;
    if (!store_frame(1, 0, &fr)) return false;
    if (!(flags & kAlphaFlag) && fr.alpha_size > 0) {  // alpha flag missing: drop the ALPH
      fr.alpha_off = fr.alpha_size = 0;
      fr.f.has_alpha = 0;
    }
    if (!is_ext && fr.f.width > 0 && fr.f.height > 0) {
      canvas_w = fr.f.width;
      canvas_h = fr.f.height;
      flags |= fr.f.has_alpha ? kAlphaFlag : 0;
    }
    return add_frame(fr);
  }

  bool parse_animation_frame(uint32_t frame_chunk_size) {
    const uint32_t anmf_payload = frame_chunk_size - kAnmfChunk;
    if (size_invalid(kAnmfChunk) || frame_chunk_size < kAnmfChunk || avail() < kAnmfChunk) return false;
    const uint8_t* h = buf + start;
    Frame fr;
    fr.f.x_offset = 2 * (int)le24(h);
    fr.f.y_offset = 2 * (int)le24(h + 3);
    fr.f.width = 1 + (int)le24(h + 6);
    fr.f.height = 1 + (int)le24(h + 9);
    fr.f.duration = (int)le24(h + 12);
    fr.f.dispose_bg = h[15] & 1;
    fr.f.no_blend = (h[15] >> 1) & 1;
    start += kAnmfChunk;
    if ((uint64_t)fr.f.width * (uint64_t)fr.f.height >= kMaxImageArea) return false;
    const size_t s0 = start;
    if (!store_frame((int)frames.size() + 1, anmf_payload, &fr)) return false;
    if (start - s0 > anmf_payload) return false;
    if ((flags & kAnimFlag) && fr.frame_num > 0) return add_frame(fr);
    return true;  // an ANMF without image data adds no frame
  }

  bool parse_vp8x_chunks() {
    const bool is_anim = flags & kAnimFlag;
    int anim_chunks = 0;
    for (;;) {
      if (avail() < kChunkHdr) return false;
      const size_t chunk_start = start;
      const uint8_t* p = buf + start;
      const uint32_t csize = le32(p + 4);
      if (csize > kMaxChunkPayload) return false;
      const uint32_t padded = csize + (csize & 1);
      start += kChunkHdr;
      if (size_invalid(padded)) return false;
      if (tag_is(p, "VP8X")) return false;
      if (tag_is(p, "ALPH") || tag_is(p, "VP8 ") || tag_is(p, "VP8L")) {
        if (anim_chunks > 0 || is_anim) return false;  // all frames of an animation are in ANMF
        start = chunk_start;
        if (!parse_single_image()) return false;
      } else if (tag_is(p, "ANIM")) {
        if (padded < kAnimChunk || avail() < padded) return false;
        if (anim_chunks == 0) {
          ++anim_chunks;
          bgcolor = le32(buf + start);
          loop_count = (int)le16(buf + start + 4);
        }
        start += padded;
      } else if (tag_is(p, "ANMF")) {
        if (anim_chunks == 0) return false;  // ANIM precedes frames
        if (!parse_animation_frame(padded)) return false;
      } else {
        if (padded > avail()) return false;
        start += padded;
      }
      if (start == riff_end) return true;
    }
  }

  bool valid_extended() const {
    const bool is_anim = flags & kAnimFlag;
    if (canvas_w <= 0 || canvas_h <= 0 || loop_count < 0 || frames.empty()) return false;
    if (flags & ~kAllValidFlags) return false;
    for (const Frame& fr : frames) {
      if (!is_anim && fr.frame_num > 1) return false;
      if (!fr.complete) return false;  // no partial frames in complete data
      if (fr.alpha_size == 0 && fr.image_size == 0) return false;
      if (fr.alpha_size > 0 && fr.alpha_off > fr.image_off) return false;
      if (fr.f.width <= 0 || fr.f.height <= 0) return false;
      if (!is_anim) {
        if (fr.f.x_offset != 0 || fr.f.y_offset != 0 || fr.f.width != canvas_w || fr.f.height != canvas_h)
          return false;
      } else if (fr.f.x_offset < 0 || fr.f.y_offset < 0 || fr.f.width + fr.f.x_offset > canvas_w ||
                 fr.f.height + fr.f.y_offset > canvas_h) {
        return false;
      }
    }
    return true;
  }
};

}  // namespace

int anim_demux(const uint8_t* data, size_t size, AnimInfo* info, std::vector<AnimFrame>* out) {
  out->clear();
  *info = AnimInfo{};
  if (data == nullptr || size == 0) return WG_STATUS_INVALID_PARAM;
  Demux d;
  d.buf = data;
  d.end = size;
  if (size < kRiffHdr + kChunkHdr) return WG_STATUS_NOT_ENOUGH_DATA;  // ReadHeader: need more data
  const uint32_t riff_size = le32(data + 4);
  if (!tag_is(data, "RIFF") || !tag_is(data + 8, "WEBP") || riff_size < kChunkHdr || riff_size > kMaxChunkPayload) {
    // ReadHeader's PARSE_ERROR -> CreateRawImageDemuxer: a bare VP8/VP8L bitstream
    Container c;
    wg_features feat{};
    const int st = parse_container(data, size, &c, &feat);
    if (st != WG_STATUS_OK) return WG_STATUS_BITSTREAM_ERROR;
    AnimFrame f;
    f.width = feat.width;
    f.height = feat.height;
    f.has_alpha = feat.has_alpha;
    f.off = 0;
    f.size = size;
    out->push_back(f);
    info->canvas_width = f.width;
    info->canvas_height = f.height;
    info->loop_count = 1;
    info->bgcolor = 0xffffffffu;
    info->frame_count = 1;
    return WG_STATUS_OK;
  }
  d.riff_end = (size_t)riff_size + kChunkHdr;
  if (d.end > d.riff_end) d.end = d.riff_end;
  if (size < d.riff_end) return WG_STATUS_NOT_ENOUGH_DATA;  // partial data is not accepted
  d.start = kRiffHdr;
  const uint8_t* p = data + d.start;
  bool ok;
  if (tag_is(p, "VP8 ") || tag_is(p, "VP8L")) {
    ok = d.parse_single_image() && d.canvas_w > 0 && d.canvas_h > 0 && !d.frames.empty() &&
         d.frames[0].f.width > 0 && d.frames[0].f.height > 0;
  } else if (tag_is(p, "VP8X")) {
    d.is_ext = true;
    const uint32_t vsize = le32(p + 4);
    ok = vsize <= kMaxChunkPayload && vsize >= kVp8xChunk;
    if (ok) {
      const uint32_t vpad = vsize + (vsize & 1);
      d.start += kChunkHdr;
      ok = !d.size_invalid(vpad) && d.avail() >= vpad;
      if (ok) {
        d.flags = data[d.start];
        d.canvas_w = 1 + (int)le24(data + d.start + 4);
        d.canvas_h = 1 + (int)le24(data + d.start + 7);
        ok = (uint64_t)d.canvas_w * (uint64_t)d.canvas_h < kMaxImageArea;
        d.start += vpad;
        ok = ok && !d.size_invalid(kChunkHdr) && d.avail() >= kChunkHdr && d.parse_vp8x_chunks() &&
             d.valid_extended();
      }
    }
  } else {
    ok = false;
  }
  if (!ok) return WG_STATUS_BITSTREAM_ERROR;
  info->canvas_width = d.canvas_w;
  info->canvas_height = d.canvas_h;
  info->loop_count = d.loop_count;
  info->bgcolor = d.bgcolor;
  info->frame_count = (int)d.frames.size();
  for (const Frame& fr : d.frames) {
    AnimFrame f = fr.f;
    // GetFramePayload: from the ALPH (if any) to the end of the image chunk
    f.off = fr.alpha_size > 0 ? fr.alpha_off : fr.image_off;
    f.size = fr.image_off + fr.image_size - f.off;
    out->push_back(f);
  }
  return WG_STATUS_OK;
}

}  // namespace wg
