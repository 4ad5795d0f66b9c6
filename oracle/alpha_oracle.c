/*
 * alpha_oracle.c -- CPU restatement of the ALPH plane unfilters.
 *
 * TEST INFRASTRUCTURE ONLY: the checker for the device alpha kernel (K4).  Nothing in the
 * product library links or calls it.
 *
 * Input is the plane's filtered bytes: the raw ALPH payload (method 0), or the green channel
 * of the alpha stream after its inverse transforms (method 1; tests get it from
 * oracle_vp8l_decode of the host entropy stage, wg_alpha_parse).  Pinning: the A channel of
 * libwebp 1.6.0's RGBA decode of the tests/golden/alpha fixtures (tests/test_alpha.py).
 * Semantics follow (file:line in /root/reference/pkg/libwebp):
 *   HorizontalUnfilter_C (pred = prev[0], or 0 for row 0)     dsp/filters.go:137-144
 *   VerticalUnfilter_C (row 0: horizontal with pred 0)        dsp/filters.go:146-154
 *   GradientUnfilter_C (row 0: horizontal with pred 0)        dsp/filters.go:156-171
 *   GradientPredictor_C = clip(a + b - c) to [0, 255]         dsp/filters.go:83-86
 *     (the Go computes a + b - c in uint8 and wraps; libwebp's C promotes to int, which is
 *     what the fixtures pin, so the sum is taken in int here)
 *   row-by-row application with the previous output row      decoder/alpha_dec.go:118-130,
 *                                                             pkg/vp8/vp8l_dec.c.go:802-814
 * WebPDequantizeLevels runs only with alpha dithering > 0 (alpha_dec.go:199-206), which
 * WebPDecode's default options leave at 0: not restated.
 */
#include <stdint.h>
#include <string.h>

static int clip255(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

static void horizontal(const uint8_t* prev, const uint8_t* in, uint8_t* out, int width) {
  uint8_t pred = prev == NULL ? 0 : prev[0];
  for (int i = 0; i < width; ++i) {
    out[i] = (uint8_t)(pred + in[i]);
    pred = out[i];
  }
}

static void vertical(const uint8_t* prev, const uint8_t* in, uint8_t* out, int width) {
  if (prev == NULL) {
    horizontal(NULL, in, out, width);
  } else {
    for (int i = 0; i < width; ++i) out[i] = (uint8_t)(prev[i] + in[i]);
  }
}

static void gradient(const uint8_t* prev, const uint8_t* in, uint8_t* out, int width) {
  if (prev == NULL) {
    horizontal(NULL, in, out, width);
    return;
  }
  uint8_t top = prev[0], top_left = top, left = top;
  for (int i = 0; i < width; ++i) {
    top = prev[i];
    left = (uint8_t)(in[i] + clip255(left + top - top_left));
    top_left = top;
    out[i] = left;
  }
}

/* filter: 0 none, 1 horizontal, 2 vertical, 3 gradient.  out may not alias filtered. */
int oracle_alpha_unfilter(int filter, int width, int height, const uint8_t* filtered, uint8_t* out) {
  if (filter < 0 || filter > 3 || width <= 0 || height <= 0) return -1;
  const uint8_t* prev = NULL;
  for (int y = 0; y < height; ++y) {
    const uint8_t* in = filtered + (size_t)y * width;
    uint8_t* dst = out + (size_t)y * width;
    switch (filter) {
      case 0: memcpy(dst, in, (size_t)width); break;
      case 1: horizontal(prev, in, dst, width); break;
      case 2: vertical(prev, in, dst, width); break;
      default: gradient(prev, in, dst, width); break;
    }
    prev = dst;
  }
  return 0;
}
