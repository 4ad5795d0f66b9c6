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
// full-frame RGBA.  grid.y = frame; a wave converts 256 pixels of a row per unit (emit_frame).
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

// Bytes per output pixel of WEBP_CSP_MODE m (0..10).
constexpr int bpp_of(int m) { return (m == 0 || m == 2) ? 3 : (m == 5 || m == 6 || m == 10) ? 2 : 4; }

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

// One frame in mode M.  Work unit = 256 pixels of a row for one wave: lane l converts the 4-pixel
// group x = 256 s + 4 l with one 16-byte RGBA load and one 4 * bpp-byte store (8 B for the 2-byte
// modes, three dwords for RGB / BGR, 16 B for the 4-byte ones), so each wave instruction reads
// 1 KB and writes a contiguous run; the row of a unit comes from a scalar division.  Groups at the
// right edge, and frames whose rows are not aligned for the vector accesses (lossless crop windows
// at odd origins), take a per-pixel path.
template <int M>
__device__ __forceinline__ void emit_frame(const EmitDesc& F) {
  constexpr int bpp = bpp_of(M);
  const int W = F.width, H = F.height;
  const int groups = (W + 3) >> 2;
  const int segs = (groups + 63) >> 6;  // 256-pixel units per row
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const bool vec = ((reinterpret_cast<uintptr_t>(F.src) | (uintptr_t)F.src_stride) & 15) == 0 &&
                   ((reinterpret_cast<uintptr_t>(F.dst) | (uintptr_t)F.dst_stride) & (bpp == 3 ? 3 : 4 * bpp - 1)) == 0;
  const int units = H * segs, step = (int)gridDim.x * (kThreads / 64);
  for (int u = (int)blockIdx.x * (kThreads / 64) + wave; u < units; u += step) {
    const int y = u / segs, x = 4 * ((u - y * segs) * 64 + lane);
    if (x >= W) continue;
    const uint8_t* sp = F.src + (size_t)y * F.src_stride + 4 * (size_t)x;
    uint8_t* dp = F.dst + (size_t)(F.flip ? H - 1 - y : y) * F.dst_stride + (size_t)bpp * x;
    if (vec && x + 4 <= W) {
      const uint4 q = *reinterpret_cast<const uint4*>(sp);
      const uint32_t o0 = emit_px<M>(q.x), o1 = emit_px<M>(q.y), o2 = emit_px<M>(q.z), o3 = emit_px<M>(q.w);
      if (bpp == 4) {
        *reinterpret_cast<uint4*>(dp) = make_uint4(o0, o1, o2, o3);
      } else if (bpp == 2) {
        *reinterpret_cast<uint2*>(dp) = make_uint2(o0 | (o1 << 16), o2 | (o3 << 16));
      } else {  // 3 bytes per pixel: 12 bytes as three dwords
        uint32_t* d = reinterpret_cast<uint32_t*>(dp);
        d[0] = o0 | (o1 << 24);
        d[1] = (o1 >> 8) | (o2 << 16);
        d[2] = (o2 >> 16) | (o3 << 8);
      }
    } else {
      for (int k = 0; k < 4 && x + k < W; ++k) {
        const uint32_t o = emit_px<M>(*reinterpret_cast<const uint32_t*>(sp + 4 * k));
#pragma unroll
        for (int c = 0; c < bpp; ++c) dp[bpp * k + c] = (uint8_t)(o >> (8 * c));
      }
    }
  }
}

__global__ void __launch_bounds__(kThreads) emit_kernel(const EmitDesc* __restrict__ frames) {
  const EmitDesc& F = frames[blockIdx.y];
  if (!F.valid) return;
  switch (F.mode) {  // (uniform per frame: one instantiation per mode)
    case 0: emit_frame<0>(F); break;
    case 1: emit_frame<1>(F); break;
    case 2: emit_frame<2>(F); break;
    case 3: emit_frame<3>(F); break;
    case 4: emit_frame<4>(F); break;
    case 5: emit_frame<5>(F); break;
    case 6: emit_frame<6>(F); break;
    case 7: emit_frame<7>(F); break;
    case 8: emit_frame<8>(F); break;
    case 9: emit_frame<9>(F); break;
    case 10: emit_frame<10>(F); break;
    default: break;
  }
}

}  // namespace

hipError_t launch_emit(const EmitDesc* d_frames, int n_frames, int max_pixels, hipStream_t stream) {
  if (n_frames <= 0) return hipSuccess;
  // (a block's four waves take 1,024 pixels per round: enough blocks for a few rounds per frame,
  // and the grid's frames fill the CUs)
  const int blocks = std::min(256, std::max(1, (max_pixels + 4 * 1024 - 1) / (4 * 1024)));
  hipLaunchKernelGGL(emit_kernel, dim3(blocks, n_frames), dim3(kThreads), 0, stream, d_frames);
  return hipGetLastError();
}

}  // namespace wg
