// VP8 entropy stage on the host: frame header, intra modes and residual tokens.
//
// This is the "host stage" of the north star: it stays on CPU and feeds the
// device kernels.  It restates, with the libwebp 1.6.0 semantics behind the
// reference's `// C:` lines and the SURVEY §2.3 trap fixes:
//   VP8GetHeaders            pkg/vp8/vp8_dec.go:362-484 (+ParseSegmentHeader :241,
//                            ParseFilterHeader :328, ParsePartitions :293)
//   VP8ParseQuant            pkg/libwebp/decoder/quant_dec.c.go:31-76
//   VP8ParseProba            pkg/libwebp/decoder/tree_dec.c.go:111-131
//   ParseIntraMode           pkg/libwebp/decoder/tree_dec.c.go:46-101
//   GetLargeValue/GetCoeffs  pkg/vp8/vp8_dec.go:489-547 (cat3-6 loop and the
//                            `out[kZigzag[n]] = ...` store restored)
//   ParseResiduals           pkg/vp8/vp8_dec.go:600-705 (incl. the WHT of
//                            dsp/dec.c.go:142-167 and its DC-only shortcut :622-628)
//   VP8DecodeMB / ParseFrame pkg/vp8/vp8_dec.go:709-774
//   PrecomputeFilterStrengths pkg/libwebp/decoder/frame_dec.c.go:266-315
// Output: the libwebp MB model (wg_vp8_mb, for the CPU checker) and/or the sparse
// device layout of device_format.h.
#include <algorithm>
#include <cstring>
#include <memory>

#include "bool_reader.h"
#include "host.h"

namespace wg {
namespace {

#include "vp8_tables.inc"

constexpr uint8_t kZigzag[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
constexpr uint8_t kBands[17] = {0, 1, 2, 3, 6, 4, 5, 6, 6, 6, 6, 6, 6, 6, 6, 7, 0};
constexpr uint8_t kCat3[] = {173, 148, 140, 0};
constexpr uint8_t kCat4[] = {176, 155, 140, 135, 0};
constexpr uint8_t kCat5[] = {180, 157, 141, 134, 130, 0};
constexpr uint8_t kCat6[] = {254, 254, 243, 230, 196, 177, 153, 140, 133, 130, 129, 0};
constexpr const uint8_t* kCat3456[4] = {kCat3, kCat4, kCat5, kCat6};
// kYModesIntra4 (tree_dec.c.go:20-22): negative = leaf -mode, positive = next node.
constexpr int8_t kYModesIntra4[18] = {-0, 1, -1, 2, -2, 3, 4, 6, -3, 5, -4, -5, -6, 7, -7, 8, -8, -9};

constexpr int kNumParts = 8;

struct BandProbas { uint8_t p[3][11]; };

struct Decoder {
  // headers
  int width = 0, height = 0, mb_w = 0, mb_h = 0;
  int use_segment = 0, update_map = 0, absolute_delta = 1;
  int8_t quantizer[4] = {0, 0, 0, 0}, filter_strength[4] = {0, 0, 0, 0};
  int simple = 0, level = 0, sharpness = 0, use_lf_delta = 0;
  int ref_lf_delta[4] = {0, 0, 0, 0}, mode_lf_delta[4] = {0, 0, 0, 0};
  int filter_type = 0;
  int num_parts_minus_one = 0;
  uint8_t segments_proba[3] = {255, 255, 255};
  BandProbas bands[4][8];
  int use_skip_proba = 0, skip_p = 0;
  int dq_y1[4][2], dq_y2[4][2], dq_uv[4][2];
  uint8_t fstr[4][2][4];  // [segment][i4x4] -> f_limit, f_ilevel, f_inner, hev_thresh
  BoolReader br;
  BoolReader parts[kNumParts];
};

inline int clip(int v, int M) { return v < 0 ? 0 : v > M ? M : v; }

int parse_segment_header(Decoder* d) {  // vp8_dec.go:241-282
  BoolReader& br = d->br;
  d->use_segment = br.get_bit(0x80);
  if (d->use_segment) {
    d->update_map = br.get_bit(0x80);
    if (br.get_bit(0x80)) {  // update data
      d->absolute_delta = br.get_bit(0x80);
      for (int s = 0; s < 4; ++s) d->quantizer[s] = br.get_bit(0x80) ? br.get_signed_value(7) : 0;
      for (int s = 0; s < 4; ++s) d->filter_strength[s] = br.get_bit(0x80) ? br.get_signed_value(6) : 0;
    }
    if (d->update_map) {
      for (int s = 0; s < 3; ++s) d->segments_proba[s] = br.get_bit(0x80) ? br.get_value(8) : 255;
    }
  } else {
    d->update_map = 0;
  }
  return !br.eof;
}

int parse_filter_header(Decoder* d) {  // vp8_dec.go:328-358
  BoolReader& br = d->br;
  d->simple = br.get_bit(0x80);
  d->level = br.get_value(6);
  d->sharpness = br.get_value(3);
  d->use_lf_delta = br.get_bit(0x80);
  if (d->use_lf_delta) {
    if (br.get_bit(0x80)) {
      for (int i = 0; i < 4; ++i)
        if (br.get_bit(0x80)) d->ref_lf_delta[i] = br.get_signed_value(6);
      for (int i = 0; i < 4; ++i)
        if (br.get_bit(0x80)) d->mode_lf_delta[i] = br.get_signed_value(6);
    }
  }
  d->filter_type = (d->level == 0) ? 0 : d->simple ? 1 : 2;
  return !br.eof;
}

int parse_partitions(Decoder* d, const uint8_t* buf, size_t size) {  // vp8_dec.go:293-325 (C lines)
  const uint8_t* sz = buf;
  const uint8_t* buf_end = buf + size;
  d->num_parts_minus_one = (1 << d->br.get_value(2)) - 1;
  const size_t last_part = (size_t)d->num_parts_minus_one;
  if (size < 3 * last_part) return WG_STATUS_NOT_ENOUGH_DATA;
  const uint8_t* part_start = buf + last_part * 3;
  size_t size_left = size - last_part * 3;
  for (size_t p = 0; p < last_part; ++p) {
    size_t psize = sz[0] | (sz[1] << 8) | (sz[2] << 16);
    if (psize > size_left) psize = size_left;
    d->parts[p].init(part_start, psize);
    part_start += psize;
    size_left -= psize;
    sz += 3;
  }
  d->parts[last_part].init(part_start, size_left);
  return part_start < buf_end ? WG_STATUS_OK : WG_STATUS_NOT_ENOUGH_DATA;
}

void parse_quant(Decoder* d) {  // quant_dec.c.go:31-76
  BoolReader& br = d->br;
  const int base_q0 = br.get_value(7);
  const int dqy1_dc = br.get_bit(0x80) ? br.get_signed_value(4) : 0;
  const int dqy2_dc = br.get_bit(0x80) ? br.get_signed_value(4) : 0;
  const int dqy2_ac = br.get_bit(0x80) ? br.get_signed_value(4) : 0;
  const int dquv_dc = br.get_bit(0x80) ? br.get_signed_value(4) : 0;
  const int dquv_ac = br.get_bit(0x80) ? br.get_signed_value(4) : 0;
  for (int i = 0; i < 4; ++i) {
    int q;
    if (d->use_segment) {
      q = d->quantizer[i];
      if (!d->absolute_delta) q += base_q0;
    } else {
      if (i > 0) {
        std::memcpy(d->dq_y1[i], d->dq_y1[0], sizeof(d->dq_y1[0]));
        std::memcpy(d->dq_y2[i], d->dq_y2[0], sizeof(d->dq_y2[0]));
        std::memcpy(d->dq_uv[i], d->dq_uv[0], sizeof(d->dq_uv[0]));
        continue;
      }
      q = base_q0;
    }
    d->dq_y1[i][0] = kDcQ[clip(q + dqy1_dc, 127)];
    d->dq_y1[i][1] = kAcQ[clip(q + 0, 127)];
    d->dq_y2[i][0] = kDcQ[clip(q + dqy2_dc, 127)] * 2;
    // x*155/100 == (x*101581) >> 16 for x in [0..284]
    d->dq_y2[i][1] = (kAcQ[clip(q + dqy2_ac, 127)] * 101581) >> 16;
    if (d->dq_y2[i][1] < 8) d->dq_y2[i][1] = 8;
    d->dq_uv[i][0] = kDcQ[clip(q + dquv_dc, 117)];
    d->dq_uv[i][1] = kAcQ[clip(q + dquv_ac, 127)];
  }
}

void parse_proba(Decoder* d) {  // tree_dec.c.go:111-131
  BoolReader& br = d->br;
  for (int t = 0; t < 4; ++t)
    for (int b = 0; b < 8; ++b)
      for (int c = 0; c < 3; ++c)
        for (int p = 0; p < 11; ++p) {
          const int idx = ((t * 8 + b) * 3 + c) * 11 + p;
          d->bands[t][b].p[c][p] = br.get_bit(kProbaUpdate[idx]) ? br.get_value(8) : kProba0[idx];
        }
  d->use_skip_proba = br.get_bit(0x80);
  if (d->use_skip_proba) d->skip_p = br.get_value(8);
}

void precompute_filter_strengths(Decoder* d) {  // frame_dec.c.go:266-315
  std::memset(d->fstr, 0, sizeof(d->fstr));
  if (d->filter_type == 0) return;
  for (int s = 0; s < 4; ++s) {
    int base_level;
    if (d->use_segment) {
      base_level = d->filter_strength[s];
      if (!d->absolute_delta) base_level += d->level;
    } else {
      base_level = d->level;
    }
    for (int i4x4 = 0; i4x4 <= 1; ++i4x4) {
      uint8_t* info = d->fstr[s][i4x4];
      int level = base_level;
      if (d->use_lf_delta) {
        level += d->ref_lf_delta[0];
        if (i4x4) level += d->mode_lf_delta[0];
      }
      level = level < 0 ? 0 : level > 63 ? 63 : level;
      if (level > 0) {
        int ilevel = level;
        if (d->sharpness > 0) {
          ilevel >>= (d->sharpness > 4) ? 2 : 1;
          if (ilevel > 9 - d->sharpness) ilevel = 9 - d->sharpness;
        }
        if (ilevel < 1) ilevel = 1;
        info[1] = (uint8_t)ilevel;
        info[0] = (uint8_t)(2 * level + ilevel);
        info[3] = level >= 40 ? 2 : level >= 15 ? 1 : 0;
      } else {
        info[0] = 0;  // no filtering
      }
      info[2] = (uint8_t)i4x4;
    }
  }
}

int get_large_value(BoolReader* br, const uint8_t* p) {  // vp8_dec.go:489-519
  int v;
  if (!br->get_bit(p[3])) {
    if (!br->get_bit(p[4])) {
      v = 2;
    } else {
      v = 3 + br->get_bit(p[5]);
    }
  } else {
    if (!br->get_bit(p[6])) {
      if (!br->get_bit(p[7])) {
        v = 5 + br->get_bit(159);
      } else {
        v = 7 + 2 * br->get_bit(165);
        v += br->get_bit(145);
      }
    } else {
      const int bit1 = br->get_bit(p[8]);
      const int bit0 = br->get_bit(p[9 + bit1]);
      const int cat = 2 * bit1 + bit0;
      v = 0;
      for (const uint8_t* tab = kCat3456[cat]; *tab; ++tab) v += v + br->get_bit(*tab);
      v += 3 + (8 << cat);
    }
  }
  return v;
}

// GetCoeffs (vp8_dec.go:522-547).  `prob[n]` = band probas of coefficient n.
// kZigzag composed with the raster -> column-major transpose of the device block layout
// (device_format.h): the sparse path writes coefficients where the kernel reads them.
constexpr uint8_t kZigzagColMajor[16] = {0, 4, 1, 2, 5, 8, 12, 9, 6, 3, 7, 10, 13, 14, 11, 15};

template <bool kColMajor>
int get_coeffs_t(BoolReader* br, const BandProbas* const* prob, int ctx, const int* dq, int n, int16_t* out) {
  const uint8_t* p = prob[n]->p[ctx];
  for (; n < 16; ++n) {
    if (!br->get_bit(p[0])) return n;  // previous coeff was last non-zero coeff
    while (!br->get_bit(p[1])) {       // sequence of zero coeffs
      p = prob[++n]->p[0];
      if (n == 16) return 16;
    }
    const BandProbas* const p_ctx = prob[n + 1];
    int v;
    if (!br->get_bit(p[2])) {
      v = 1;
      p = p_ctx->p[1];
    } else {
      v = get_large_value(br, p);
      p = p_ctx->p[2];
    }
    out[kColMajor ? kZigzagColMajor[n] : kZigzag[n]] = (int16_t)(br->get_signed(v) * dq[n > 0]);  // wraps
  }
  return 16;
}

int get_coeffs(BoolReader* br, const BandProbas* const* prob, int ctx, const int* dq, int n, int16_t* out) {
  return get_coeffs_t<false>(br, prob, ctx, dq, n, out);
}

// GetCoeffs entered after its first "not the last coefficient" bit (p[0] of coefficient n
// read as 1): the same token walk as get_coeffs_t from the zero-run loop on.  The sparse path
// reads that first bit itself, so a block whose first token is EOB (two thirds of c3's
// blocks) costs one bit -- no call, no zeroing of its slot.
int get_coeffs_after_first(BoolReader* br, const BandProbas* const* prob, const uint8_t* p, const int* dq, int n,
                           int16_t* out) {
  for (;;) {
    while (!br->get_bit(p[1])) {  // sequence of zero coeffs
      p = prob[++n]->p[0];
      if (n == 16) return 16;
    }
    const BandProbas* const p_ctx = prob[n + 1];
    int v;
    if (!br->get_bit(p[2])) {
      v = 1;
      p = p_ctx->p[1];
    } else {
      v = get_large_value(br, p);
      p = p_ctx->p[2];
    }
    out[kZigzagColMajor[n]] = (int16_t)(br->get_signed(v) * dq[n > 0]);  // wraps
    if (++n == 16 || !br->get_bit(p[0])) return n;  // previous coeff was last non-zero coeff
  }
}

inline uint32_t nz_code_bits(uint32_t nz_coeffs, int nz, int dc_nz) {  // vp8_dec.go:588-598
  nz_coeffs <<= 2;
  nz_coeffs |= (nz > 3) ? 3 : (nz > 1) ? 2 : dc_nz;
  return nz_coeffs;
}

// TransformWHT_C (dsp/dec.c.go:142-167): int16 in, DC of each Y block out.
void transform_wht(const int16_t* in, int16_t* out) {
  int tmp[16];
  for (int i = 0; i < 4; ++i) {
    const int a0 = in[0 + i] + in[12 + i];
    const int a1 = in[4 + i] + in[8 + i];
    const int a2 = in[4 + i] - in[8 + i];
    const int a3 = in[0 + i] - in[12 + i];
    tmp[0 + i] = a0 + a1;
    tmp[8 + i] = a0 - a1;
    tmp[4 + i] = a3 + a2;
    tmp[12 + i] = a3 - a2;
  }
  for (int i = 0; i < 4; ++i) {
    const int dc = tmp[0 + i * 4] + 3;
    const int a0 = dc + tmp[3 + i * 4];
    const int a1 = tmp[1 + i * 4] + tmp[2 + i * 4];
    const int a2 = tmp[1 + i * 4] - tmp[2 + i * 4];
    const int a3 = dc - tmp[3 + i * 4];
    out[0] = (int16_t)((a0 + a1) >> 3);
    out[16] = (int16_t)((a3 + a2) >> 3);
    out[32] = (int16_t)((a0 - a1) >> 3);
    out[48] = (int16_t)((a3 - a2) >> 3);
    out += 64;
  }
}

struct MBCtx { uint8_t nz = 0, nz_dc = 0; };

struct MBOut {
  int16_t coeffs[384];
  uint32_t non_zero_y = 0, non_zero_uv = 0;
  uint8_t is_i4x4 = 0, uvmode = 0, segment = 0, skip = 0;
  uint8_t imodes[16];
};

// ParseIntraMode (tree_dec.c.go:46-101)
void parse_intra_mode(Decoder* d, uint8_t* top, uint8_t* left, MBOut* b) {
  BoolReader& br = d->br;
  if (d->update_map) {
    b->segment = !br.get_bit(d->segments_proba[0]) ? br.get_bit(d->segments_proba[1])
                                                  : br.get_bit(d->segments_proba[2]) + 2;
  } else {
    b->segment = 0;
  }
  b->skip = d->use_skip_proba ? br.get_bit(d->skip_p) : 0;
  b->is_i4x4 = !br.get_bit(145);
  if (!b->is_i4x4) {
    const int ymode = br.get_bit(156) ? (br.get_bit(128) ? 1 /*TM*/ : 3 /*H*/)
                                      : (br.get_bit(163) ? 2 /*V*/ : 0 /*DC*/);
    b->imodes[0] = (uint8_t)ymode;
    std::memset(top, ymode, 4);
    std::memset(left, ymode, 4);
  } else {
    uint8_t* modes = b->imodes;
    for (int y = 0; y < 4; ++y) {
      int ymode = left[y];
      for (int x = 0; x < 4; ++x) {
        const uint8_t* prob = kBModeProba + (top[x] * 10 + ymode) * 9;
        int i = kYModesIntra4[br.get_bit(prob[0])];
        while (i > 0) i = kYModesIntra4[2 * i + br.get_bit(prob[i])];
        ymode = -i;
        top[x] = (uint8_t)ymode;
      }
      std::memcpy(modes, top, 4);
      modes += 4;
      left[y] = (uint8_t)ymode;
    }
  }
  if (!br.get_bit(142)) b->uvmode = 0;       // DC
  else if (!br.get_bit(114)) b->uvmode = 2;  // V
  else if (br.get_bit(183)) b->uvmode = 1;   // TM
  else b->uvmode = 3;                        // H
}

// ParseResiduals (vp8_dec.go:600-705).  Returns 1 when the MB has no coefficient.
int parse_residuals(Decoder* d, MBCtx* mb, MBCtx* left_mb, BoolReader* token_br, MBOut* block,
                    const BandProbas* const (*bands)[17]) {
  const int seg = block->segment;
  int16_t* dst = block->coeffs;
  uint8_t tnz, lnz;
  uint32_t non_zero_y = 0, non_zero_uv = 0;
  uint32_t out_t_nz, out_l_nz;
  int first;
  const BandProbas* const* ac_proba;
  std::memset(dst, 0, 384 * sizeof(*dst));
  if (!block->is_i4x4) {  // parse DC
    int16_t dc[16] = {0};
    const int ctx = mb->nz_dc + left_mb->nz_dc;
    const int nz = get_coeffs(token_br, bands[1], ctx, d->dq_y2[seg], 0, dc);
    mb->nz_dc = left_mb->nz_dc = (nz > 0);
    if (nz > 1) {
      transform_wht(dc, dst);
    } else {
      const int dc0 = (dc[0] + 3) >> 3;
      for (int i = 0; i < 16 * 16; i += 16) dst[i] = (int16_t)dc0;
    }
    first = 1;
    ac_proba = bands[0];
  } else {
    first = 0;
    ac_proba = bands[3];
  }
  tnz = mb->nz & 0x0f;
  lnz = left_mb->nz & 0x0f;
  for (int y = 0; y < 4; ++y) {
    int l = lnz & 1;
    uint32_t nz_coeffs = 0;
    for (int x = 0; x < 4; ++x) {
      const int ctx = l + (tnz & 1);
      const int nz = get_coeffs(token_br, ac_proba, ctx, d->dq_y1[seg], first, dst);
      l = (nz > first);
      tnz = (uint8_t)((tnz >> 1) | (l << 7));
      nz_coeffs = nz_code_bits(nz_coeffs, nz, dst[0] != 0);
      dst += 16;
    }
    tnz >>= 4;
    lnz = (uint8_t)((lnz >> 1) | (l << 7));
    non_zero_y = (non_zero_y << 8) | nz_coeffs;
  }
  out_t_nz = tnz;
  out_l_nz = lnz >> 4;
  for (int ch = 0; ch < 4; ch += 2) {
    uint32_t nz_coeffs = 0;
    tnz = (uint8_t)(mb->nz >> (4 + ch));
    lnz = (uint8_t)(left_mb->nz >> (4 + ch));
    for (int y = 0; y < 2; ++y) {
      int l = lnz & 1;
      for (int x = 0; x < 2; ++x) {
        const int ctx = l + (tnz & 1);
        const int nz = get_coeffs(token_br, bands[2], ctx, d->dq_uv[seg], 0, dst);
        l = (nz > 0);
        tnz = (uint8_t)((tnz >> 1) | (l << 3));
        nz_coeffs = nz_code_bits(nz_coeffs, nz, dst[0] != 0);
        dst += 16;
      }
      tnz >>= 2;
      lnz = (uint8_t)((lnz >> 1) | (l << 5));
    }
    non_zero_uv |= nz_coeffs << (4 * ch);
    out_t_nz |= (uint32_t)(tnz << 4) << ch;
    out_l_nz |= (uint32_t)(lnz & 0xf0) << ch;
  }
  mb->nz = (uint8_t)out_t_nz;
  left_mb->nz = (uint8_t)out_l_nz;
  block->non_zero_y = non_zero_y;
  block->non_zero_uv = non_zero_uv;
  return !(non_zero_y | non_zero_uv);
}

// TransformWHT_C (dsp/dec.c.go:142-167) of a column-major Y2 block (the device layout):
// the 16 Y DC values, raster block order.  The device runs the same transform (K1); the
// host needs only which outputs are non-zero (NzCodeBits' dc_nz and through it f_inner).
void transform_wht_colmajor(const int16_t* cm, int16_t* dcs) {
  int tmp[16];
  for (int i = 0; i < 4; ++i) {  // column i: in[4r + i] = cm[4i + r]
    const int16_t* c = cm + 4 * i;
    const int a0 = c[0] + c[3], a1 = c[1] + c[2], a2 = c[1] - c[2], a3 = c[0] - c[3];
    tmp[0 + i] = a0 + a1;
    tmp[8 + i] = a0 - a1;
    tmp[4 + i] = a3 + a2;
    tmp[12 + i] = a3 - a2;
  }
  for (int i = 0; i < 4; ++i) {
    const int dc = tmp[0 + i * 4] + 3;
    const int a0 = dc + tmp[3 + i * 4];
    const int a1 = tmp[1 + i * 4] + tmp[2 + i * 4];
    const int a2 = tmp[1 + i * 4] - tmp[2 + i * 4];
    const int a3 = dc - tmp[3 + i * 4];
    dcs[4 * i + 0] = (int16_t)((a0 + a1) >> 3);
    dcs[4 * i + 1] = (int16_t)((a3 + a2) >> 3);
    dcs[4 * i + 2] = (int16_t)((a0 - a1) >> 3);
    dcs[4 * i + 3] = (int16_t)((a3 - a2) >> 3);
  }
}

inline bool block_nonzero(const int16_t* ob) {
  uint64_t w[4];
  std::memcpy(w, ob, 32);
  return (w[0] | w[1] | w[2] | w[3]) != 0;
}

// ParseResiduals for the sparse device layout: the same token walk and contexts as
// parse_residuals, but each 4x4 block is decoded straight into the next free slot of
// `out` (column-major, kZigzagColMajor) and kept only if some coefficient is non-zero.
// An i16 MB ships its Y2 block itself (first slot, kY2Bit) instead of 16 DC-filled Y
// blocks: its Y blocks hold only their AC coefficients and the device adds the WHT's DC.
// Returns the flags' block bits (bit b = block b kept, blocks 0..15 Y raster, 16..19 U,
// 20..23 V, plus kY2Bit) and sets *n_kept and block->non_zero_*.
uint32_t parse_residuals_sparse(Decoder* d, MBCtx* mb, MBCtx* left_mb, BoolReader* token_br, MBOut* block,
                                const BandProbas* const (*bands)[17], int16_t* out, int* n_kept) {
  const int seg = block->segment;
  uint32_t non_zero_y = 0, non_zero_uv = 0, mask = 0;
  int nb = 0;
  int16_t dcs[16];
  const BandProbas* const* ac_proba;
  int first;
  if (!block->is_i4x4) {  // parse DC (Y2)
    int16_t* y2 = out;
    std::memset(y2, 0, 32);
    const int ctx = mb->nz_dc + left_mb->nz_dc;
    const int nz = get_coeffs_t<true>(token_br, bands[1], ctx, d->dq_y2[seg], 0, y2);
    mb->nz_dc = left_mb->nz_dc = (nz > 0);
    if (block_nonzero(y2)) {
      // nz <= 1: libwebp's shortcut (dc[0] + 3) >> 3 for all 16, which is what the full
      // transform gives for a DC-only input (vp8_dec.go:620-628) -- taken here too when only the
      // DC is non-zero (the common case), the full transform otherwise
      uint64_t w[4];
      std::memcpy(w, y2, 32);
      if ((w[0] & ~0xffffull) == 0 && (w[1] | w[2] | w[3]) == 0) {
        const int16_t dc0 = (int16_t)((y2[0] + 3) >> 3);
        for (int i = 0; i < 16; ++i) dcs[i] = dc0;
      } else {
        transform_wht_colmajor(y2, dcs);
      }
      mask |= kY2Bit;
      nb = 1;
    } else {
      std::memset(dcs, 0, sizeof(dcs));
    }
    first = 1;
    ac_proba = bands[0];
  } else {
    std::memset(dcs, 0, sizeof(dcs));
    first = 0;
    ac_proba = bands[3];
  }
  uint8_t tnz = mb->nz & 0x0f, lnz = left_mb->nz & 0x0f;
  for (int y = 0; y < 4; ++y) {
    int l = lnz & 1;
    uint32_t nz_coeffs = 0;
    for (int x = 0; x < 4; ++x) {
      int16_t* ob = out + 16 * nb;
      const int ctx = l + (tnz & 1);
      const uint8_t* p0 = ac_proba[first]->p[ctx];
      int nz = first;
      if (token_br->get_bit(p0[0])) {
        std::memset(ob, 0, 32);
        nz = get_coeffs_after_first(token_br, ac_proba, p0, d->dq_y1[seg], first, ob);
      }
      l = (nz > first);
      tnz = (uint8_t)((tnz >> 1) | (l << 7));
      nz_coeffs = nz_code_bits(nz_coeffs, nz, (first ? dcs[4 * y + x] : nz > 0 ? ob[0] : 0) != 0);
      // (nz == first: no coefficient was decoded; past it one may still wrap to 0 in int16)
      if (nz > first && block_nonzero(ob)) {
        mask |= 1u << (4 * y + x);
        ++nb;
      }
    }
    tnz >>= 4;
    lnz = (uint8_t)((lnz >> 1) | (l << 7));
    non_zero_y = (non_zero_y << 8) | nz_coeffs;
  }
  uint32_t out_t_nz = tnz, out_l_nz = lnz >> 4;
  for (int ch = 0; ch < 4; ch += 2) {
    uint32_t nz_coeffs = 0;
    tnz = (uint8_t)(mb->nz >> (4 + ch));
    lnz = (uint8_t)(left_mb->nz >> (4 + ch));
    for (int y = 0; y < 2; ++y) {
      int l = lnz & 1;
      for (int x = 0; x < 2; ++x) {
        int16_t* ob = out + 16 * nb;
        const int ctx = l + (tnz & 1);
        const uint8_t* p0 = bands[2][0]->p[ctx];
        int nz = 0;
        if (token_br->get_bit(p0[0])) {
          std::memset(ob, 0, 32);
          nz = get_coeffs_after_first(token_br, bands[2], p0, d->dq_uv[seg], 0, ob);
        }
        l = (nz > 0);
        tnz = (uint8_t)((tnz >> 1) | (l << 3));
        nz_coeffs = nz_code_bits(nz_coeffs, nz, nz > 0 && ob[0] != 0);
        if (nz > 0 && block_nonzero(ob)) {
          mask |= 1u << (16 + 2 * ch + 2 * y + x);
          ++nb;
        }
      }
      tnz >>= 2;
      lnz = (uint8_t)((lnz >> 1) | (l << 5));
    }
    non_zero_uv |= nz_coeffs << (4 * ch);
    out_t_nz |= (uint32_t)(tnz << 4) << ch;
    out_l_nz |= (uint32_t)(lnz & 0xf0) << ch;
  }
  mb->nz = (uint8_t)out_t_nz;
  left_mb->nz = (uint8_t)out_l_nz;
  block->non_zero_y = non_zero_y;
  block->non_zero_uv = non_zero_uv;
  *n_kept = nb;
  return mask;
}

int get_headers(Decoder* d, const uint8_t* buf, size_t buf_size) {  // vp8_dec.go:362-484
  if (buf_size < 4) return WG_STATUS_NOT_ENOUGH_DATA;
  const uint32_t bits = buf[0] | (buf[1] << 8) | (buf[2] << 16);
  const int key_frame = !(bits & 1);
  const int profile = (bits >> 1) & 7;
  const int show = (bits >> 4) & 1;
  const uint32_t partition_length = bits >> 5;
  if (profile > 3) return WG_STATUS_BITSTREAM_ERROR;
  if (!show) return WG_STATUS_UNSUPPORTED_FEATURE;
  buf += 3;
  buf_size -= 3;
  if (key_frame) {
    if (buf_size < 7) return WG_STATUS_NOT_ENOUGH_DATA;
    if (!(buf[0] == 0x9d && buf[1] == 0x01 && buf[2] == 0x2a)) return WG_STATUS_BITSTREAM_ERROR;
    d->width = ((buf[4] << 8) | buf[3]) & 0x3fff;
    d->height = ((buf[6] << 8) | buf[5]) & 0x3fff;
    buf += 7;
    buf_size -= 7;
    d->mb_w = (d->width + 15) >> 4;
    d->mb_h = (d->height + 15) >> 4;
  }
  if (partition_length > buf_size) return WG_STATUS_NOT_ENOUGH_DATA;
  d->br.init(buf, partition_length);
  buf += partition_length;
  buf_size -= partition_length;
  if (key_frame) {
    d->br.get_bit(0x80);  // colorspace
    d->br.get_bit(0x80);  // clamp_type
  }
  if (!parse_segment_header(d)) return WG_STATUS_BITSTREAM_ERROR;
  if (!parse_filter_header(d)) return WG_STATUS_BITSTREAM_ERROR;
  const int st = parse_partitions(d, buf, buf_size);
  if (st != WG_STATUS_OK) return st;
  parse_quant(d);
  if (!key_frame) return WG_STATUS_UNSUPPORTED_FEATURE;
  d->br.get_bit(0x80);  // ignore the value of update_proba
  parse_proba(d);
  return WG_STATUS_OK;
}

}  // namespace

namespace {

// VP8GetHeaders + PrecomputeFilterStrengths of a frame: fills *inf and the decoder state.
int begin_frame(const uint8_t* data, size_t size, int flags, Decoder* d, wg_vp8_info* inf) {
  Container c;
  int st = parse_container(data, size, &c, nullptr);
  if (st != WG_STATUS_OK) return st;
  if (c.is_lossless) return WG_STATUS_UNSUPPORTED_FEATURE;  // VP8L: not this entry point
  st = get_headers(d, data + c.payload_off, c.payload_size);
  if (st != WG_STATUS_OK) return st;
  if (flags & WG_FLAG_BYPASS_FILTERING) d->filter_type = 0;  // VP8EnterCritical
  precompute_filter_strengths(d);
  *inf = wg_vp8_info{};
  inf->width = d->width;
  inf->height = d->height;
  inf->mb_w = d->mb_w;
  inf->mb_h = d->mb_h;
  inf->filter_type = d->filter_type;
  inf->num_parts = d->num_parts_minus_one + 1;
  inf->use_segment = d->use_segment;
  inf->frame_offset = (int32_t)c.payload_off;
  return WG_STATUS_OK;
}

// The MB rows WebPDecode parses for a crop window (VP8EnterCritical's br_mb_y_).
int parsed_rows(const Decoder* d, int crop_bottom) {
  static const int kFilterExtraRows[3] = {0, 2, 8};  // frame_dec.c.go (VP8EnterCritical)
  return crop_bottom < 0 ? d->mb_h : std::min(d->mb_h, (crop_bottom + 15 + kFilterExtraRows[d->filter_type]) >> 4);
}

// ParseFrame (vp8_dec.go:750-774) over rows [0, rows): the libwebp MB model into `dense`,
// or the device layout into `sink`.  Returns the status and the failing row.
int parse_rows(Decoder* d, int rows, wg_vp8_mb* dense, const SparseSink* sink, size_t* n_blocks, int* fail_row) {
  const int mb_w = d->mb_w;
  // bands_ptr (tree_dec.c.go:127-129)
  const BandProbas* bands_ptr[4][17];
  for (int t = 0; t < 4; ++t)
    for (int b = 0; b < 17; ++b) bands_ptr[t][b] = &d->bands[t][kBands[b]];
  std::vector<uint8_t> intra_t(4 * (size_t)mb_w, 0);  // B_DC_PRED
  uint8_t intra_l[4];
  std::vector<MBCtx> mb_info((size_t)mb_w + 1);  // [0] = left
  MBCtx* left = &mb_info[0];
  MBOut blk;
  size_t nblocks = 0;
  int st = WG_STATUS_OK;
  *fail_row = -1;
  for (int mb_y = 0; mb_y < rows && st == WG_STATUS_OK; ++mb_y) {
    BoolReader* token_br = &d->parts[mb_y & d->num_parts_minus_one];
    std::memset(intra_l, 0, sizeof(intra_l));  // VP8InitScanline: B_DC_PRED
    left->nz = left->nz_dc = 0;
    if (sink) sink->row_block0[mb_y] = (uint32_t)nblocks;
    for (int mb_x = 0; mb_x < mb_w; ++mb_x) {
      // Modes come from partition 0.  libwebp parses the whole row of modes first
      // (VP8ParseIntraModeRow); partition 0 is independent of the token partitions,
      // so interleaving per MB reads the same bits.
      parse_intra_mode(d, &intra_t[4 * (size_t)mb_x], intra_l, &blk);
      MBCtx* mb = &mb_info[1 + mb_x];
      int skip = d->use_skip_proba ? blk.skip : 0;
      uint32_t mask = 0;
      int n_kept = 0;
      if (!skip) {
        if (dense) {
          skip = parse_residuals(d, mb, left, token_br, &blk, bands_ptr);
        } else {
          mask = parse_residuals_sparse(d, mb, left, token_br, &blk, bands_ptr, sink->blocks + 16 * nblocks, &n_kept);
          skip = !(blk.non_zero_y | blk.non_zero_uv);
        }
      } else {
        left->nz = mb->nz = 0;
        if (!blk.is_i4x4) left->nz_dc = mb->nz_dc = 0;
        blk.non_zero_y = 0;
        blk.non_zero_uv = 0;
        if (dense) std::memset(blk.coeffs, 0, sizeof(blk.coeffs));
      }
      uint8_t fi[4] = {0, 0, 0, 0};
      if (d->filter_type > 0) {
        std::memcpy(fi, d->fstr[blk.segment][blk.is_i4x4], 4);
        fi[2] |= !skip;
      }
      if (token_br->eof) {
        st = WG_STATUS_NOT_ENOUGH_DATA;  // "Premature end-of-file encountered."
        *fail_row = mb_y;
        break;
      }
      const size_t idx = (size_t)mb_y * mb_w + mb_x;
      if (dense) {
        wg_vp8_mb& o = dense[idx];
        std::memcpy(o.coeffs, blk.coeffs, sizeof(o.coeffs));
        o.non_zero_y = blk.non_zero_y;
        o.non_zero_uv = blk.non_zero_uv;
        o.is_i4x4 = blk.is_i4x4;
        o.uvmode = blk.uvmode;
        o.segment = blk.segment;
        o.skip = (uint8_t)skip;
        if (blk.is_i4x4) std::memcpy(o.imodes, blk.imodes, 16);
        else { std::memset(o.imodes, 0, 16); o.imodes[0] = blk.imodes[0]; }
        o.f_limit = fi[0]; o.f_ilevel = fi[1]; o.f_inner = fi[2]; o.hev_thresh = fi[3];
      } else {
        nblocks += n_kept;
        MbRec r{0, 0, 0, 0};
        r.flags = mask | ((uint32_t)blk.is_i4x4 << kI4Shift) |
                  ((uint32_t)(blk.is_i4x4 ? 0 : blk.imodes[0]) << kYModeShift) |
                  ((uint32_t)blk.uvmode << kUVModeShift);
        if (blk.is_i4x4) {
          for (int n = 0; n < 8; ++n) r.imodes_lo |= (uint32_t)blk.imodes[n] << (4 * n);
          for (int n = 0; n < 8; ++n) r.imodes_hi |= (uint32_t)blk.imodes[8 + n] << (4 * n);
        }
        r.finfo = fi[0] | (fi[1] << 8) | (fi[2] << 16) | ((uint32_t)fi[3] << 24);
        sink->mbs[idx] = r;
      }
    }
    if (st == WG_STATUS_OK && d->br.eof) {  // partition 0 exhausted
      st = WG_STATUS_NOT_ENOUGH_DATA;
      *fail_row = mb_y;
    }
  }
  *n_blocks = nblocks;
  return st;
}

}  // namespace

int vp8_parse(const uint8_t* data, size_t size, int flags, wg_vp8_info* info, wg_vp8_mb* dense, int crop_bottom) {
  std::unique_ptr<Decoder> dp(new Decoder());
  wg_vp8_info inf;
  int st = begin_frame(data, size, flags, dp.get(), &inf);
  if (st != WG_STATUS_OK) return st;
  if (info) *info = inf;
  if (!dense) return WG_STATUS_OK;
  size_t nb = 0;
  int fail_row = -1;
  return parse_rows(dp.get(), parsed_rows(dp.get(), crop_bottom), dense, nullptr, &nb, &fail_row);
}

int vp8_parse_sparse(const uint8_t* data, size_t size, int flags, int crop_bottom, SparseAllocFn alloc, void* actx,
                     SparseResult* res) {
  std::unique_ptr<Decoder> dp(new Decoder());
  Decoder* d = dp.get();
  res->n_blocks = 0;
  res->n_y2 = 0;
  res->fail_row = -1;
  res->br_mb_y = 0;
  int st = begin_frame(data, size, flags, d, &res->info);
  if (st != WG_STATUS_OK) return st;
  const int rows = parsed_rows(d, crop_bottom);
  res->br_mb_y = rows;
  SparseSink sink{};
  if (!alloc(actx, res->info, rows, &sink)) return WG_STATUS_OUT_OF_MEMORY;
  st = parse_rows(d, rows, nullptr, &sink, &res->n_blocks, &res->fail_row);
  // rows not parsed (below a crop window's br_mb_y, or after a failure) read as empty
  const int done = st == WG_STATUS_OK ? rows : std::max(res->fail_row, 0);
  const size_t mb_w = (size_t)d->mb_w;
  std::memset(sink.mbs + (size_t)done * mb_w, 0, ((size_t)d->mb_h - done) * mb_w * sizeof(MbRec));
  for (int y = done; y < d->mb_h; ++y) sink.row_block0[y] = (uint32_t)res->n_blocks;
  for (size_t i = 0; i < (size_t)done * mb_w; ++i) res->n_y2 += (sink.mbs[i].flags & kY2Bit) != 0;
  return st;
}

int vp8_parse(const uint8_t* data, size_t size, int flags, SparseFrame* sf, int crop_bottom) {
  auto alloc = [](void* p, const wg_vp8_info& inf, int rows, SparseSink* sink) {
    SparseFrame* f = static_cast<SparseFrame*>(p);
    f->mbs.resize((size_t)inf.mb_w * inf.mb_h);
    f->row_block0.resize((size_t)inf.mb_h);
    f->blocks.clear();
    sink->mbs = f->mbs.data();
    sink->row_block0 = f->row_block0.data();
    sink->blocks = f->blocks.reserve_more(16 * sparse_max_blocks(inf.mb_w, rows));
    return true;
  };
  SparseResult r;
  const int st = vp8_parse_sparse(data, size, flags, crop_bottom, alloc, sf, &r);
  sf->info = r.info;
  sf->blocks.n = 16 * r.n_blocks;
  sf->br_mb_y = r.br_mb_y;
  sf->fail_row = r.fail_row;
  return st;
}

}  // namespace wg
