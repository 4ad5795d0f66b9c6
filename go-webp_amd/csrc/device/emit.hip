// K6: output colorspaces, cropping window and flip -- RGBA -> WEBP_CSP_MODE bytes.
//
// Replaces the per-mode output stage of the reference: the RGB-family upsampler / sampler
// variants (pkg/libwebp/dsp/upsampling.c.go:107-114, yuv.go VP8YuvToRgb/Bgr/Argb/Rgba4444/
// Rgb565), the lossless VP8LConvertFromBGRA (dsp/lossless.go:561-666), the alpha emission
// EmitAlphaRGB / EmitAlphaRGB4444 (io_dec.c.go:175-230) and the premultiplied modes
// (WebPApplyAlphaMultiply / WebPApplyAlphaMultiply4444, dsp/alpha_processing.go:96-150), and
// options.flip (rows emitted bottom-up).  Every mode is a per-pixel function of the final
// non-premultiplied RGBA: the 565 / 4444 packings take the same 8-bit R, G, B the RGBA path
// has (VP8YuvToRgb565: (r & 0xf8) | (g >> 5), ((g << 3) & 0xe0) | (b >> 3); 4444: (r & 0xf0) |
// (g >> 4), (b & 0xf0) | (a >> 4)), and premultiplication is (c * a * 32897) >> 23 for a < 255
// (4444: a * 0x1111 on the dithered nibbles).  K6 only runs when the output is not plain
// full-frame RGBA.  One thread per pixel, grid.y = frame.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../device_format.h"
#include "kernels.h"

namespace wg {
namespace {

constexpr int kThreads = 256;

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

__global__ void __launch_bounds__(kThreads) emit_kernel(const EmitDesc* __restrict__ frames) {
  const EmitDesc& F = frames[blockIdx.y];
  if (!F.valid) return;
  const int n = F.width * F.height;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
    const int y = i / F.width, x = i - y * F.width;
    const uint32_t p = *reinterpret_cast<const uint32_t*>(F.src + (size_t)y * F.src_stride + 4 * (size_t)x);
    uint32_t r = p & 0xff, g = (p >> 8) & 0xff, b = (p >> 16) & 0xff;
    const uint32_t a = p >> 24;
    const int mode = F.mode;
    if ((mode == 7 || mode == 8 || mode == 9) && a != 0xff) {  // rgbA, bgrA, Argb
      r = premul(r, a);
      g = premul(g, a);
      b = premul(b, a);
    }
    uint8_t* d = F.dst + (size_t)(F.flip ? F.height - 1 - y : y) * F.dst_stride;
    switch (mode) {
      case 0:  // RGB
        d += 3 * x;
        d[0] = (uint8_t)r, d[1] = (uint8_t)g, d[2] = (uint8_t)b;
        break;
      case 2:  // BGR
        d += 3 * x;
        d[0] = (uint8_t)b, d[1] = (uint8_t)g, d[2] = (uint8_t)r;
        break;
      case 1:
      case 7:  // RGBA, rgbA
        *reinterpret_cast<uint32_t*>(d + 4 * x) = r | (g << 8) | (b << 16) | (a << 24);
        break;
      case 3:
      case 8:  // BGRA, bgrA
        *reinterpret_cast<uint32_t*>(d + 4 * x) = b | (g << 8) | (r << 16) | (a << 24);
        break;
      case 4:
      case 9:  // ARGB, Argb
        *reinterpret_cast<uint32_t*>(d + 4 * x) = a | (r << 8) | (g << 16) | (b << 24);
        break;
      case 5:
      case 10: {  // RGBA_4444, rgbA_4444
        uint32_t rg = (r & 0xf0) | (g >> 4), ba = (b & 0xf0) | (a >> 4);
        if (mode == 10) premul4444(rg, ba);
        d += 2 * x;
        d[0] = (uint8_t)rg, d[1] = (uint8_t)ba;
        break;
      }
      default: {  // 6: RGB_565
        d += 2 * x;
        d[0] = (uint8_t)((r & 0xf8) | (g >> 5));
        d[1] = (uint8_t)(((g << 3) & 0xe0) | (b >> 3));
        break;
      }
    }
  }
}

}  // namespace

hipError_t launch_emit(const EmitDesc* d_frames, int n_frames, int max_pixels, hipStream_t stream) {
  if (n_frames <= 0) return hipSuccess;
  const int blocks = std::min(1024, std::max(1, (max_pixels + kThreads - 1) / kThreads));
  hipLaunchKernelGGL(emit_kernel, dim3(blocks, n_frames), dim3(kThreads), 0, stream, d_frames);
  return hipGetLastError();
}

}  // namespace wg
