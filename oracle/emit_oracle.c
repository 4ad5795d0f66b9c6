/*
 * emit_oracle.c -- CPU restatement of the RGB-family output modes (and flip) from RGBA.
 *
 * TEST INFRASTRUCTURE ONLY: the checker for the device output stage (K6).  Nothing in the
 * product library links or calls it.
 *
 * Pinning: libwebp 1.6.0 WebPDecode outputs for every mode x crop x flip in
 * tests/golden/modes (tests/test_modes.py).  Semantics follow (file:line in
 * /root/reference/pkg/libwebp):
 *   VP8YuvToRgb / Bgr / Argb / Rgba4444 / Rgb565 (per-pixel packings of the 8-bit R,G,B)
 *                                                           dsp/yuv.go, dsp/upsampling.c.go:107-114
 *   VP8LConvertBGRAToRGB / BGR / RGBA4444 / RGB565          dsp/lossless.go:561-666
 *   EmitAlphaRGB / EmitAlphaRGB4444 (alpha into A / the low nibble of the second byte)
 *                                                           decoder/io_dec.c.go:175-230
 *   ApplyAlphaMultiply_C: c = (c * a * 32897) >> 23 for a != 255
 *   ApplyAlphaMultiply4444_C: nibbles dithered, * (a * 0x1111) >> 16
 *                                                           dsp/alpha_processing.go:96-150
 *   options.flip (negative stride)                          decoder/buffer_dec.c.go
 */
#include <stdint.h>
#include <stddef.h>

static uint32_t premul(uint32_t c, uint32_t a) { return (c * (a * 32897u)) >> 23; }

static void premul4444(uint8_t* rg, uint8_t* ba) {
  const uint32_t a = *ba & 0x0f, mult = a * 0x1111u;
  const uint8_t dh_rg = (uint8_t)((*rg & 0xf0) | (*rg >> 4)), dl_rg = (uint8_t)((*rg & 0x0f) | (*rg << 4));
  const uint8_t dh_ba = (uint8_t)((*ba & 0xf0) | (*ba >> 4));
  const uint8_t r = (uint8_t)((dh_rg * mult) >> 16), g = (uint8_t)((dl_rg * mult) >> 16);
  const uint8_t b = (uint8_t)((dh_ba * mult) >> 16);
  *rg = (uint8_t)((r & 0xf0) | ((g >> 4) & 0x0f));
  *ba = (uint8_t)((b & 0xf0) | a);
}

/* rgba: w x h, row stride `stride`; out rows of `out_stride`.  mode 0..10.  0 on success. */
int oracle_emit(const uint8_t* rgba, int w, int h, int stride, int mode, int flip, uint8_t* out, int out_stride) {
  if (mode < 0 || mode > 10) return -1;
  for (int y = 0; y < h; ++y) {
    const uint8_t* s = rgba + (size_t)y * stride;
    uint8_t* d = out + (size_t)(flip ? h - 1 - y : y) * out_stride;
    for (int x = 0; x < w; ++x) {
      uint32_t r = s[4 * x], g = s[4 * x + 1], b = s[4 * x + 2];
      const uint32_t a = s[4 * x + 3];
      if ((mode == 7 || mode == 8 || mode == 9) && a != 0xff) {
        r = premul(r, a);
        g = premul(g, a);
        b = premul(b, a);
      }
      switch (mode) {
        case 0: d[3 * x] = (uint8_t)r; d[3 * x + 1] = (uint8_t)g; d[3 * x + 2] = (uint8_t)b; break;
        case 2: d[3 * x] = (uint8_t)b; d[3 * x + 1] = (uint8_t)g; d[3 * x + 2] = (uint8_t)r; break;
        case 1:
        case 7: d[4 * x] = (uint8_t)r; d[4 * x + 1] = (uint8_t)g; d[4 * x + 2] = (uint8_t)b; d[4 * x + 3] = (uint8_t)a; break;
        case 3:
        case 8: d[4 * x] = (uint8_t)b; d[4 * x + 1] = (uint8_t)g; d[4 * x + 2] = (uint8_t)r; d[4 * x + 3] = (uint8_t)a; break;
        case 4:
        case 9: d[4 * x] = (uint8_t)a; d[4 * x + 1] = (uint8_t)r; d[4 * x + 2] = (uint8_t)g; d[4 * x + 3] = (uint8_t)b; break;
        case 5:
        case 10: {
          uint8_t rg = (uint8_t)((r & 0xf0) | (g >> 4)), ba = (uint8_t)((b & 0xf0) | (a >> 4));
          if (mode == 10) premul4444(&rg, &ba);
          d[2 * x] = rg;
          d[2 * x + 1] = ba;
          break;
        }
        default:
          d[2 * x] = (uint8_t)((r & 0xf8) | (g >> 5));
          d[2 * x + 1] = (uint8_t)(((g << 3) & 0xe0) | (b >> 3));
          break;
      }
    }
  }
  return 0;
}
