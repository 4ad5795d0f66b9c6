/*
 * yuva_oracle.c -- CPU restatement of libwebp's ARGB -> YUV(A) conversion for the YUV output modes
 * of lossless frames (MODE_YUV / MODE_YUVA).
 *
 * TEST INFRASTRUCTURE ONLY: the checker for the device kernel K8 (device/argb_to_yuva.hip).
 * Nothing in the product library links or calls it.
 *
 * Pinning: libwebp 1.6.0 WebPDecode outputs in MODE_YUV / MODE_YUVA for every lossless source x
 * crop x flip in tests/golden/yuv (tests/test_yuv.py).  libwebp 1.6.0 converts each output row of a
 * lossless frame with ConvertToYUVA (file:line in /root/reference/pkg):
 *   ConvertToYUVA: Y of the row, U / V stored on even output rows and averaged into on odd ones,
 *   A = the alpha bytes (MODE_YUVA)                     vp8/vp8l_dec.c.go:544-563
 *   WebPConvertARGBToY                                  libwebp/dsp/yuv.go:74-80
 *   WebPConvertARGBToUV (pairs of pixels at 2x, the odd last pixel at 4x; the odd row's
 *   "approximated average-of-four" (u + tmp + 1) >> 1)  libwebp/dsp/yuv.go:82-125
 *   RGBToY / RGBToU / RGBToV / ClipUV                   color/yuv/conversion.go:50-70
 * Output rows count from the crop window's top (dec.last_out_row), so the row pairs are aligned
 * to it.  (The reference's EmitRowsYUVA, vp8l_dec.c.go:606-650, restates a later libwebp's
 * gamma-corrected WebPImportYUVAFromRGBA instead; libwebp 1.6.0 -- the version the reference pins,
 * pkg/vp8/constants.go:18-20 -- and its goldens use ConvertToYUVA: 2-5 % of the chroma samples
 * differ by one between the two.)
 */
#include <stdint.h>
#include <stddef.h>

static int clip_uv(int uv) {
  uv = (uv + (1 << 17) + (128 << 18)) >> 18;  /* rounding YUV_HALF << 2, YUV_FIX + 2 */
  return (uv & ~0xff) == 0 ? uv : (uv < 0 ? 0 : 255);
}

static int rgb_to_y(int r, int g, int b) { return (16839 * r + 33059 * g + 6420 * b + (1 << 15) + (16 << 16)) >> 16; }

/* rgba: w x h window (RGBA bytes), row stride `stride`.  Outputs: y (w x h, y_stride), u / v
 * ((w + 1) / 2 x (h + 1) / 2, uv_stride), a (w x h, a_stride) or NULL for MODE_YUV.  Rows are
 * written bottom-up with flip (WebPFlipBuffer).  Returns 0. */
int oracle_rgba_to_yuva(const uint8_t* rgba, int w, int h, int stride, uint8_t* y, int y_stride, uint8_t* u,
                        uint8_t* v, int uv_stride, uint8_t* a, int a_stride, int flip) {
  const int uw = (w + 1) >> 1, uh = (h + 1) >> 1;
  for (int r = 0; r < h; ++r) {
    const uint8_t* s = rgba + (size_t)r * stride;
    uint8_t* dy = y + (size_t)(flip ? h - 1 - r : r) * y_stride;
    for (int x = 0; x < w; ++x) dy[x] = (uint8_t)rgb_to_y(s[4 * x], s[4 * x + 1], s[4 * x + 2]);
    if (a) {
      uint8_t* da = a + (size_t)(flip ? h - 1 - r : r) * a_stride;
      for (int x = 0; x < w; ++x) da[x] = s[4 * x + 3];
    }
    const int cy = r >> 1;
    uint8_t* du = u + (size_t)(flip ? uh - 1 - cy : cy) * uv_stride;
    uint8_t* dv = v + (size_t)(flip ? uh - 1 - cy : cy) * uv_stride;
    for (int cx = 0; cx < uw; ++cx) {
      const uint8_t* p0 = s + 8 * cx;
      const uint8_t* p1 = 2 * cx + 1 < w ? p0 + 4 : p0;  /* (the odd last pixel counts twice: 4x) */
      const int rr = 2 * (p0[0] + p1[0]), gg = 2 * (p0[1] + p1[1]), bb = 2 * (p0[2] + p1[2]);
      const int tu = clip_uv(-9719 * rr - 19081 * gg + 28800 * bb);
      const int tv = clip_uv(28800 * rr - 24116 * gg - 4684 * bb);
      if ((r & 1) == 0) {
        du[cx] = (uint8_t)tu;
        dv[cx] = (uint8_t)tv;
      } else {
        du[cx] = (uint8_t)((du[cx] + tu + 1) >> 1);
        dv[cx] = (uint8_t)((dv[cx] + tv + 1) >> 1);
      }
    }
  }
  return 0;
}
