// K6: output colorspaces, cropping window and flip -- RGBA -> WEBP_CSP_MODE bytes.
//
// Replaces the per-mode output stage of the reference: the RGB-family upsampler / sampler
// variants (pkg/libwebp/dsp/upsampling.c.go:107-114, yuv.go VP8YuvToRgb/Bgr/Argb/Rgba4444/
// Rgb565), the lossless VP8LConvertFromBGRA (dsp/lossless.go:561-666), the alpha emission
// EmitAlphaRGB / EmitAlphaRGB4444 (io_dec.c.go:175-230) and the premultiplied modes
// (WebPApplyAlphaMultiply / WebPApplyAlphaMultiply4444, dsp/alpha_processing.go:96-150), and
// options.flip (rows emitted bottom-up); the per-pixel functions are emit_px.h's.  K6 runs for
// the frames of a non-RGBA or flipped batch that the YUV -> RGB strips do not emit directly
// (lossless frames, frames with alpha, crop windows).  grid.y = frame; a wave converts 256
// pixels of a row per unit (emit_frame).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../device_format.h"
#include "emit_px.h"
#include "kernels.h"

namespace wg {
namespace {

constexpr int kThreads = 256;

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
