// One RGBA pixel in a WEBP_CSP_MODE: the per-pixel output functions shared by K6 (emit.hip) and
// the YUV -> RGB strips (yuv_rgba_strip.h: K1's tail and K2 emitting lossy frames without alpha
// straight into the output colorspace).
//
// Every mode is a per-pixel function of the final non-premultiplied RGBA (R in byte 0): the
// 565 / 4444 packings take the same 8-bit R, G, B as the RGBA path (VP8YuvToRgb565,
// VP8YuvToRgba4444, pkg/libwebp/dsp/yuv.go; VP8LConvertBGRAToRGB565 / ...4444,
// dsp/lossless.go:561-666), premultiplication (WebPApplyAlphaMultiply / ...4444,
// dsp/alpha_processing.go:96-150) is (c * a * 32897) >> 23 for a < 255 and a * 0x1111 on the
// dithered nibbles.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wg {

__device__ __forceinline__ uint32_t premul(uint32_t c, uint32_t a) { return (c * (a * 32897u)) >> 23; }

// ApplyAlphaMultiply4444_C on one packed pixel (rg = byte 0, ba = byte 1)
__device__ __forceinline__ void premul4444(uint32_t& rg, uint32_t& ba) {
  const uint32_t a = ba & 0x0f, mult = a * 0x1111u;
  const uint32_t r = (((rg & 0xf0) | (rg >> 4)) * mult) >> 16;
  const uint32_t g = ((((rg & 0x0f) | (rg << 4)) & 0xff) * mult) >> 16;
  const uint32_t b = (((ba & 0xf0) | (ba >> 4)) * mult) >> 16;
  rg = (r & 0xf0) | ((g >> 4) & 0x0f);
  ba = (b & 0xf0) | a;
}

// Bytes per output pixel of WEBP_CSP_MODE m (0..10).
__host__ __device__ constexpr int bpp_of(int m) { return (m == 0 || m == 2) ? 3 : (m == 5 || m == 6 || m == 10) ? 2 : 4; }

// One pixel (RGBA dword, R in byte 0) in mode M: the low bpp_of(M) bytes of the result, first
// output byte lowest.
template <int M>
__device__ __forceinline__ uint32_t emit_px(uint32_t p) {
  uint32_t r = p & 0xff, g = (p >> 8) & 0xff, b = (p >> 16) & 0xff;
  const uint32_t a = p >> 24;
  if ((M == 7 || M == 8 || M == 9) && a != 0xff) {  // rgbA, bgrA, Argb
    r = premul(r, a);
    g = premul(g, a);
    b = premul(b, a);
  }
  if (M == 0) return r | (g << 8) | (b << 16);             // RGB
  if (M == 2) return b | (g << 8) | (r << 16);             // BGR
  if (M == 1 || M == 7) return r | (g << 8) | (b << 16) | (a << 24);  // RGBA, rgbA
  if (M == 3 || M == 8) return b | (g << 8) | (r << 16) | (a << 24);  // BGRA, bgrA
  if (M == 4 || M == 9) return a | (r << 8) | (g << 16) | (b << 24);  // ARGB, Argb
  if (M == 5 || M == 10) {  // RGBA_4444, rgbA_4444
    uint32_t rg = (r & 0xf0) | (g >> 4), ba = (b & 0xf0) | (a >> 4);
    if (M == 10) premul4444(rg, ba);
    return rg | (ba << 8);
  }
  return ((r & 0xf8) | (g >> 5)) | ((((g << 3) & 0xe0) | (b >> 3)) << 8);  // RGB_565
}

}  // namespace wg
