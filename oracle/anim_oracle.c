/*
 * anim_oracle.c -- CPU restatement of the animation canvas logic (WebPAnimDecoderGetNext).
 *
 * TEST INFRASTRUCTURE ONLY: the checker for the device compositor (K5).  Nothing in the
 * product library links or calls it.
 *
 * Input: per frame, its decoded RGBA (from the oracle decoders of tests/oracle_lib.py) and its
 * demux description (rectangle, duration, disposal, blending, has_alpha).  Pinning: the
 * canvases WebPAnimDecoder (libwebp 1.6.0, MODE_RGBA) returns for tests/golden/anim
 * (tests/test_anim.py).  Semantics follow (file:line in /root/reference/pkg/libwebp/demux):
 *   IsFullFrame / IsKeyFrame                                anim_decode.go:143-197
 *   ZeroFillCanvas / ZeroFillFrameRect / CopyCanvas         anim_decode.go:148-181
 *   BlendChannelNonPremult / BlendPixelNonPremult /
 *     BlendPixelRowNonPremult                               anim_decode.go:199-258
 *   FindBlendRangeAtRow                                      anim_decode.go:263-289
 *   WebPAnimDecoderGetNext (canvas init, decode into the
 *     rectangle, blend, dispose, timestamps)                anim_decode.go:312-420
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  const uint8_t* rgba; /* width x height, stride 4 * width */
  int x, y, width, height, duration, dispose_bg, no_blend, has_alpha;
} oracle_anim_frame;

static int is_full(const oracle_anim_frame* f, int cw, int ch) { return f->width == cw && f->height == ch; }

static int is_key(const oracle_anim_frame* cur, const oracle_anim_frame* prev, int num, int prev_key, int cw,
                  int ch) {
  if (num == 1) return 1;
  if ((!cur->has_alpha || cur->no_blend) && is_full(cur, cw, ch)) return 1;
  return prev->dispose_bg && (is_full(prev, cw, ch) || prev_key);
}

static uint8_t blend_channel(uint32_t src, uint8_t src_a, uint32_t dst, uint8_t dst_a, uint32_t scale, int shift) {
  const uint32_t s = (src >> shift) & 0xff, d = (dst >> shift) & 0xff;
  const uint32_t unscaled = s * src_a + d * dst_a;
  return (uint8_t)((unscaled * scale) >> 24);
}

static uint32_t blend_pixel(uint32_t src, uint32_t dst) {
  const uint8_t src_a = (uint8_t)(src >> 24);
  if (src_a == 0) return dst;
  const uint8_t dst_a = (uint8_t)(dst >> 24);
  const uint8_t dst_factor_a = (uint8_t)((dst_a * (256 - src_a)) >> 8);
  const uint8_t blend_a = (uint8_t)(src_a + dst_factor_a);
  const uint32_t scale = (1u << 24) / blend_a;
  return (uint32_t)blend_channel(src, src_a, dst, dst_factor_a, scale, 0) |
         ((uint32_t)blend_channel(src, src_a, dst, dst_factor_a, scale, 8) << 8) |
         ((uint32_t)blend_channel(src, src_a, dst, dst_factor_a, scale, 16) << 16) | ((uint32_t)blend_a << 24);
}

static void blend_row(uint32_t* src, const uint32_t* dst, int n) {
  for (int i = 0; i < n; ++i)
    if ((src[i] >> 24) != 0xff) src[i] = blend_pixel(src[i], dst[i]);
}

/* canvases: n * ch * cw * 4 bytes; timestamps: n ints.  0 on success. */
int oracle_anim_compose(const oracle_anim_frame* frames, int n, int cw, int ch, uint8_t* canvases,
                        int32_t* timestamps) {
  const size_t npx = (size_t)cw * ch;
  uint32_t* cur = (uint32_t*)calloc(npx, 4);
  uint32_t* disposed = (uint32_t*)calloc(npx, 4);
  if (!cur || !disposed) return -1;
  int ts = 0, prev_key = 0;
  for (int i = 0; i < n; ++i) {
    const oracle_anim_frame* f = &frames[i];
    const oracle_anim_frame* p = i > 0 ? &frames[i - 1] : NULL;
    const int key = is_key(f, p, i + 1, prev_key, cw, ch);
    ts += f->duration;
    if (key) memset(cur, 0, npx * 4);
    else memcpy(cur, disposed, npx * 4);
    for (int y = 0; y < f->height; ++y)  /* WebPDecode into the rectangle */
      memcpy(cur + (size_t)(f->y + y) * cw + f->x, f->rgba + (size_t)y * f->width * 4, (size_t)f->width * 4);
    if (i > 0 && !f->no_blend && !key) {
      for (int y = 0; y < f->height; ++y) {
        const int cy = f->y + y;
        const size_t row = (size_t)cy * cw;
        if (!p->dispose_bg) {
          blend_row(cur + row + f->x, disposed + row + f->x, f->width);
        } else {
          /* FindBlendRangeAtRow: only the parts of this row outside the previous rectangle */
          const int src_max_x = f->x + f->width, dst_max_x = p->x + p->width, dst_max_y = p->y + p->height;
          int l1 = -1, w1 = 0, l2 = -1, w2 = 0;
          if (cy < p->y || cy >= dst_max_y || f->x >= dst_max_x || src_max_x <= p->x) {
            l1 = f->x;
            w1 = f->width;
          } else {
            if (f->x < p->x) {
              l1 = f->x;
              w1 = p->x - f->x;
            }
            if (src_max_x > dst_max_x) {
              l2 = dst_max_x;
              w2 = src_max_x - dst_max_x;
            }
          }
          if (w1 > 0) blend_row(cur + row + l1, disposed + row + l1, w1);
          if (w2 > 0) blend_row(cur + row + l2, disposed + row + l2, w2);
        }
      }
    }
    memcpy(canvases + (size_t)i * npx * 4, cur, npx * 4);
    timestamps[i] = ts;
    prev_key = key;
    memcpy(disposed, cur, npx * 4);
    if (f->dispose_bg)
      for (int y = 0; y < f->height; ++y) memset(disposed + (size_t)(f->y + y) * cw + f->x, 0, (size_t)f->width * 4);
  }
  free(cur);
  free(disposed);
  return 0;
}
