/*
 * vp8l_oracle.c -- CPU restatement of the VP8L (lossless) inverse transforms and the
 * BGRA->RGBA emit.
 *
 * TEST INFRASTRUCTURE ONLY: the checker for the device transform kernel (K3) and the
 * CPU baseline of the C5 workload.  Nothing in the product library links or calls it.
 *
 * Input is the host entropy stage's output (wg_vp8l_parse: one token per coded pixel, the
 * literals, and the transforms in read order); oracle_vp8l_resolve first restates the value
 * half of the symbol loop -- the color cache and the back-references -- serially, exactly as
 * the reference orders it.  Pinning: libwebp 1.6.0 RGBA of the lossless
 * fixtures and the C5 bench frame's SHA-256 (tests/test_vp8l.py); the reference's own
 * VP8L decoder is an unimplemented stub (pkg/vp8/vp8l_dec.c.go DecodeImageStream).
 * Semantics follow (file:line in /root/reference/pkg/libwebp/dsp):
 *   Average2/3/4, Clip255, ClampedAddSubtract{Full,Half}, Select   lossless.go:31-89
 *   VP8LPredictor0..13                                              lossless.go:91-148
 *   PredictorInverseTransform (row 0 = L, column 0 = T, tile mode,
 *     rightmost top-right = first pixel of the current row)         lossless.go:290-333
 *   VP8LAddGreenToBlueAndRed                                        lossless.go:337-347
 *   ColorTransformDelta, TransformColorInverse                      lossless.go:349-374
 *   ColorSpaceInverseTransform (per-tile multipliers)               lossless.go:377-413
 *   ColorIndexInverseTransform (pixel unpacking, palette)           lossless.go:428-459
 *   VP8LInverseTransform (reverse order)                            lossless.go:511-547
 *   VP8LConvertBGRAToRGBA                                           lossless.go:561-573
 *   VP8LAddPixels                                                   lossless_common.go:110-114
 * and (/root/reference/pkg/vp8):
 *   DecodeImageData pixel loop: literal / CopyBlock32b / cache       vp8l_dec.c.go:1038-1189
 *     (every decoded pixel inserted in scan order :1105-1109,
 *      lookup :1141-1153)
 *   VP8LHashPix (0x1e35a7bd), Insert, Lookup                         color_cache.go:16, 46-63
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/gowebp_amd.h"

/* The coded image from its tokens (device_format.h kTok*: 0 literal index, 1 cache key, 2 copy
 * distance, 3 unset): one pixel at a time, every pixel inserted into the color cache in scan
 * order (a never-written slot reads as 0, calloc'd like VP8LColorCacheInit's).  Returns 0, or
 * -1 for a token the host stage cannot produce. */
int oracle_vp8l_resolve(const uint32_t* tokens, const uint32_t* lits, int n_lits, int n_px, int cache_bits,
                        uint32_t* argb) {
  uint32_t cache[2048];
  memset(cache, 0, sizeof(cache));
  if (cache_bits < 0 || cache_bits > 11) return -1;
  for (int i = 0; i < n_px; ++i) {
    const uint32_t t = tokens[i], kind = t >> 30, pl = t & 0x3fffffffu;
    uint32_t v = 0;
    if (kind == 0) {
      if (pl >= (uint32_t)n_lits) return -1;
      v = lits[pl];
    } else if (kind == 1) {
      if (pl >= (1u << cache_bits) || cache_bits == 0) return -1;
      v = cache[pl];                                  /* VP8LColorCacheLookup */
    } else if (kind == 2) {
      if (pl == 0 || pl > (uint32_t)i) return -1;
      v = argb[i - (int)pl];                          /* CopyBlock32b, one pixel at a time */
    }
    argb[i] = v;
    if (kind != 3 && cache_bits) cache[(v * 0x1e35a7bdu) >> (32 - cache_bits)] = v;  /* Insert */
  }
  return 0;
}

static uint32_t add_pixels(uint32_t a, uint32_t b) {
  const uint32_t ag = (a & 0xff00ff00u) + (b & 0xff00ff00u);
  const uint32_t rb = (a & 0x00ff00ffu) + (b & 0x00ff00ffu);
  return (ag & 0xff00ff00u) | (rb & 0x00ff00ffu);
}

static uint32_t avg2(uint32_t a, uint32_t b) { return (((a ^ b) & 0xfefefefeu) >> 1) + (a & b); }

static uint32_t clip255(uint32_t a) { return a < 256 ? a : (~a >> 24); }

static uint32_t add_sub_full(uint32_t c0, uint32_t c1, uint32_t c2) {
  uint32_t r = 0;
  for (int s = 0; s < 32; s += 8) {
    const int a = (int)((c0 >> s) & 0xff), b = (int)((c1 >> s) & 0xff), c = (int)((c2 >> s) & 0xff);
    r |= clip255((uint32_t)(a + b - c)) << s;
  }
  return r;
}

static uint32_t add_sub_half(uint32_t c0, uint32_t c1, uint32_t c2) {
  const uint32_t ave = avg2(c0, c1);
  uint32_t r = 0;
  for (int s = 0; s < 32; s += 8) {
    const int a = (int)((ave >> s) & 0xff), b = (int)((c2 >> s) & 0xff);
    r |= clip255((uint32_t)(a + (a - b) / 2)) << s;  /* C division truncates toward 0 */
  }
  return r;
}

static int sub3(int a, int b, int c) { return abs(b - c) - abs(a - c); }

static uint32_t select_px(uint32_t a, uint32_t b, uint32_t c) {
  int d = 0;
  for (int s = 0; s < 32; s += 8) d += sub3((int)((a >> s) & 0xff), (int)((b >> s) & 0xff), (int)((c >> s) & 0xff));
  return d <= 0 ? a : b;
}

/* top[0] = T, top[-1] = TL, top[1] = TR */
static uint32_t predict(int mode, uint32_t L, const uint32_t* top) {
  switch (mode) {
    case 1: return L;
    case 2: return top[0];
    case 3: return top[1];
    case 4: return top[-1];
    case 5: return avg2(avg2(L, top[1]), top[0]);
    case 6: return avg2(L, top[-1]);
    case 7: return avg2(L, top[0]);
    case 8: return avg2(top[-1], top[0]);
    case 9: return avg2(top[0], top[1]);
    case 10: return avg2(avg2(L, top[-1]), avg2(top[0], top[1]));
    case 11: return select_px(top[0], L, top[-1]);
    case 12: return add_sub_full(L, top[0], top[-1]);
    case 13: return add_sub_half(L, top[0], top[-1]);
    default: return 0xff000000u; /* 0, and the padding entries 14, 15 */
  }
}

static void inv_predictor(int bits, const uint32_t* modes, const uint32_t* in, uint32_t* out, int w, int h) {
  const int tpr = (w + (1 << bits) - 1) >> bits;
  out[0] = add_pixels(in[0], 0xff000000u);
  for (int x = 1; x < w; ++x) out[x] = add_pixels(in[x], out[x - 1]);
  for (int y = 1; y < h; ++y) {
    const uint32_t* src = in + (size_t)y * w;
    uint32_t* dst = out + (size_t)y * w;
    const uint32_t* mrow = modes + (size_t)(y >> bits) * tpr;
    dst[0] = add_pixels(src[0], dst[-w]);
    for (int x = 1; x < w; ++x) {
      const int mode = (int)((mrow[x >> bits] >> 8) & 0xf);
      /* contiguous buffer: at x = w-1, top + 1 is this row's first pixel */
      dst[x] = add_pixels(src[x], predict(mode, dst[x - 1], dst + x - w));
    }
  }
}

static int color_delta(int8_t t, int8_t c) { return ((int)t * (int)c) >> 5; }

static void inv_cross_color(int bits, const uint32_t* mult, const uint32_t* in, uint32_t* out, int w, int h) {
  const int tpr = (w + (1 << bits) - 1) >> bits;
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const uint32_t m = mult[(size_t)(y >> bits) * tpr + (x >> bits)];
      const int8_t g2r = (int8_t)(m & 0xff), g2b = (int8_t)((m >> 8) & 0xff), r2b = (int8_t)((m >> 16) & 0xff);
      const uint32_t argb = in[(size_t)y * w + x];
      const int8_t green = (int8_t)(argb >> 8);
      int r = (int)((argb >> 16) & 0xff), b = (int)(argb & 0xff);
      r = (r + color_delta(g2r, green)) & 0xff;
      b = (b + color_delta(g2b, green) + color_delta(r2b, (int8_t)r)) & 0xff;
      out[(size_t)y * w + x] = (argb & 0xff00ff00u) | ((uint32_t)r << 16) | (uint32_t)b;
    }
}

static void add_green(const uint32_t* in, uint32_t* out, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    const uint32_t argb = in[i];
    const uint32_t g = (argb >> 8) & 0xff;
    uint32_t rb = argb & 0x00ff00ffu;
    rb += (g << 16) | g;
    out[i] = (argb & 0xff00ff00u) | (rb & 0x00ff00ffu);
  }
}

static void inv_color_index(int bits, const uint32_t* pal, const uint32_t* in, int in_w, uint32_t* out, int w, int h) {
  const int bpp = 8 >> bits;
  for (int y = 0; y < h; ++y) {
    const uint32_t* src = in + (size_t)y * in_w;
    uint32_t* dst = out + (size_t)y * w;
    if (bits == 0) {
      for (int x = 0; x < w; ++x) dst[x] = pal[(src[x] >> 8) & 0xff];
    } else {
      const int count_mask = (1 << bits) - 1;
      const uint32_t bit_mask = (1u << bpp) - 1;
      uint32_t packed = 0;
      for (int x = 0; x < w; ++x) {
        if ((x & count_mask) == 0) packed = (*src++ >> 8) & 0xff;
        dst[x] = pal[packed & bit_mask];
        packed >>= bpp;
      }
    }
  }
}

/* Undo the transforms of `info` (reverse read order) on the entropy-coded image and
 * write RGBA (stride 4*width).  0 on success. */
int oracle_vp8l_decode(const wg_vp8l_info* info, const uint32_t* argb, const uint32_t* const* tdata,
                       uint8_t* rgba) {
  const int w = info->width, h = info->height;
  const size_t cap = (size_t)w * h;
  uint32_t* cur = (uint32_t*)malloc(cap * 4);
  uint32_t* tmp = (uint32_t*)malloc(cap * 4);
  if (!cur || !tmp) return -1;
  int cw = info->coded_width;
  memcpy(cur, argb, (size_t)cw * h * 4);
  for (int i = info->num_transforms - 1; i >= 0; --i) {
    const int type = info->transform_type[i], bits = info->transform_bits[i], xs = info->transform_xsize[i];
    switch (type) {
      case 0: inv_predictor(bits, tdata[i], cur, tmp, xs, h); break;
      case 1: inv_cross_color(bits, tdata[i], cur, tmp, xs, h); break;
      case 2: add_green(cur, tmp, (size_t)xs * h); break;
      case 3: inv_color_index(bits, tdata[i], cur, cw, tmp, xs, h); break;
      default: free(cur); free(tmp); return -1;
    }
    cw = xs;
    uint32_t* t = cur;
    cur = tmp;
    tmp = t;
  }
  for (size_t p = 0; p < cap; ++p) {
    const uint32_t c = cur[p];
    rgba[4 * p + 0] = (uint8_t)(c >> 16);
    rgba[4 * p + 1] = (uint8_t)(c >> 8);
    rgba[4 * p + 2] = (uint8_t)c;
    rgba[4 * p + 3] = (uint8_t)(c >> 24);
  }
  free(cur);
  free(tmp);
  return 0;
}
