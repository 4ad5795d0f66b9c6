// K8: the YUV output modes (MODE_YUV / MODE_YUVA) -- every frame's output window as compact Y, U, V
// (and A) planes.
//
// Replaces the reference's YUV emitters:
//   EmitYUV (lossy: the reconstructed planes' window, WebPCopyPlane)
//                                                   pkg/libwebp/decoder/io_dec.c.go:36-50
//   EmitAlphaYUV (the alpha plane, or 0xff when the frame has none)      io_dec.c.go:128-150
//   ConvertToYUVA (lossless, per output row: WebPConvertARGBToY, WebPConvertARGBToUV with the odd
//   row averaged into the even one's chroma, WebPExtractAlpha)          pkg/vp8/vp8l_dec.c.go:544-563
//     WebPConvertARGBToY / ToUV                                         pkg/libwebp/dsp/yuv.go:74-125
//     RGBToY / RGBToU / RGBToV                                          pkg/color/yuv/conversion.go:50-70
//   options.flip (WebPFlipBuffer: every plane bottom-up)                decoder/buffer_dec.c.go
// libwebp 1.6.0's lossless path (tests/golden/yuv pin it; the reference's EmitRowsYUVA restates a
// later libwebp's gamma-corrected import, see oracle/yuva_oracle.c).
//
// Work unit: one chroma row (two output rows) x 64 chroma columns for a wave; lane l owns chroma
// column 64 s + l, i.e. output columns 2 cx, 2 cx + 1: one 8-byte RGBA load per row (a wave reads
// 512 contiguous bytes per row), byte stores.  grid.y = frame.  HBM-bound, a next-row output stage:
// algorithmic bytes = (lossless) 4 B/px in + Y/U/V/A out, (lossy) the window's planes in and out.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../device_format.h"
#include "kernels.h"

namespace wg {
namespace {

constexpr int kThreads = 256;

// ClipUV (rounding YUV_HALF << 2 at YUV_FIX + 2) of a chroma sum of two pixels at 2x (conversion.go:50-70)
__device__ __forceinline__ int clip_uv(int uv) { return min(max((uv + (1 << 17) + (128 << 18)) >> 18, 0), 255); }
__device__ __forceinline__ int rgb_to_y(uint32_t p) {  // p = R | G << 8 | B << 16 (RGBA bytes)
  return (16839 * (int)(p & 0xff) + 33059 * (int)((p >> 8) & 0xff) + 6420 * (int)((p >> 16) & 0xff) + (1 << 15) +
          (16 << 16)) >> 16;
}
// WebPConvertARGBToUV's value of one pixel pair (p1 = p0 for the odd last pixel: 4x)
__device__ __forceinline__ void pair_uv(uint32_t p0, uint32_t p1, int& u, int& v) {
  const int r = 2 * (int)((p0 & 0xff) + (p1 & 0xff)), g = 2 * (int)(((p0 >> 8) & 0xff) + ((p1 >> 8) & 0xff)),
            b = 2 * (int)(((p0 >> 16) & 0xff) + ((p1 >> 16) & 0xff));
  u = clip_uv(-9719 * r - 19081 * g + 28800 * b);
  v = clip_uv(28800 * r - 24116 * g - 4684 * b);
}

__global__ void __launch_bounds__(kThreads) emit_yuva_kernel(const YuvaDesc* __restrict__ frames) {
  const YuvaDesc& F = frames[blockIdx.y];
  if (!F.valid) return;
  const int W = F.width, H = F.height, uw = (W + 1) >> 1, uh = (H + 1) >> 1;
  const int segs = (uw + 63) >> 6;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int units = uh * segs, step = (int)gridDim.x * (kThreads / 64);
  for (int un = (int)blockIdx.x * (kThreads / 64) + wave; un < units; un += step) {
    const int cy = un / segs, cx = (un - cy * segs) * 64 + lane;
    if (cx >= uw) continue;
    const int x0 = 2 * cx, y0 = 2 * cy;
    const bool two_c = x0 + 1 < W, two_r = y0 + 1 < H;
    const int r0 = F.flip ? H - 1 - y0 : y0, r1 = F.flip ? H - 2 - y0 : y0 + 1;
    const int rc = F.flip ? uh - 1 - cy : cy;
    uint8_t* oy0 = F.oy + (size_t)r0 * W + x0;
    uint8_t* oy1 = F.oy + (size_t)r1 * W + x0;
    if (F.lossless) {
      const uint8_t* s0 = F.rgba + (size_t)y0 * F.rgba_stride + 4 * (size_t)x0;
      const uint8_t* s1 = s0 + F.rgba_stride;
      const uint32_t p00 = *reinterpret_cast<const uint32_t*>(s0);
      const uint32_t p01 = two_c ? *reinterpret_cast<const uint32_t*>(s0 + 4) : p00;
      const uint32_t p10 = two_r ? *reinterpret_cast<const uint32_t*>(s1) : 0u;
      const uint32_t p11 = two_r && two_c ? *reinterpret_cast<const uint32_t*>(s1 + 4) : p10;
      int u0, v0;
      pair_uv(p00, p01, u0, v0);
      oy0[0] = (uint8_t)rgb_to_y(p00);
      if (two_c) oy0[1] = (uint8_t)rgb_to_y(p01);
      if (two_r) {  // the odd row: "approximated average-of-four" (u + tmp + 1) >> 1
        int u1, v1;
        pair_uv(p10, p11, u1, v1);
        u0 = (u0 + u1 + 1) >> 1;
        v0 = (v0 + v1 + 1) >> 1;
        oy1[0] = (uint8_t)rgb_to_y(p10);
        if (two_c) oy1[1] = (uint8_t)rgb_to_y(p11);
      }
      F.ou[(size_t)rc * uw + cx] = (uint8_t)u0;
      F.ov[(size_t)rc * uw + cx] = (uint8_t)v0;
      if (F.oa) {
        uint8_t* oa0 = F.oa + (size_t)r0 * W + x0;
        uint8_t* oa1 = F.oa + (size_t)r1 * W + x0;
        oa0[0] = (uint8_t)(p00 >> 24);
        if (two_c) oa0[1] = (uint8_t)(p01 >> 24);
        if (two_r) {
          oa1[0] = (uint8_t)(p10 >> 24);
          if (two_c) oa1[1] = (uint8_t)(p11 >> 24);
        }
      }
    } else {
      const uint8_t* s0 = F.y + (size_t)y0 * F.y_stride + x0;
      oy0[0] = s0[0];
      if (two_c) oy0[1] = s0[1];
      if (two_r) {
        oy1[0] = s0[F.y_stride];
        if (two_c) oy1[1] = s0[F.y_stride + 1];
      }
      F.ou[(size_t)rc * uw + cx] = F.u[(size_t)cy * F.uv_stride + cx];
      F.ov[(size_t)rc * uw + cx] = F.v[(size_t)cy * F.uv_stride + cx];
      if (F.oa) {
        uint8_t* oa0 = F.oa + (size_t)r0 * W + x0;
        uint8_t* oa1 = F.oa + (size_t)r1 * W + x0;
        const uint8_t* a0 = F.a ? F.a + (size_t)y0 * F.a_stride + x0 : nullptr;
        oa0[0] = a0 ? a0[0] : 0xff;
        if (two_c) oa0[1] = a0 ? a0[1] : 0xff;
        if (two_r) {
          oa1[0] = a0 ? a0[F.a_stride] : 0xff;
          if (two_c) oa1[1] = a0 ? a0[F.a_stride + 1] : 0xff;
        }
      }
    }
  }
}

}  // namespace

hipError_t launch_emit_yuva(const YuvaDesc* d_frames, int n_frames, int max_uw, int max_uh, hipStream_t stream) {
  if (n_frames <= 0) return hipSuccess;
  // (a block's four waves take four 64-column units per round: enough blocks for a few rounds per
  // frame, and the grid's frames fill the CUs)
  const int units = std::max(1, max_uh * ((max_uw + 63) / 64));
  const int blocks = std::min(256, std::max(1, (units + 15) / 16));
  hipLaunchKernelGGL(emit_yuva_kernel, dim3(blocks, n_frames), dim3(kThreads), 0, stream, d_frames);
  return hipGetLastError();
}

}  // namespace wg
