// K2: YUV420 -> RGBA for a batch of frames (the headline HBM-roofline stage), one wave per
// 1024-px x 32-row strip.  The conversion itself (EmitFancyRGB / EmitSampledRGB +
// VP8YuvToRgba, io_dec.c.go:53-115, upsampling.c.go:43-107, conversion.go:28-49) is
// strip::convert_strip (yuv_rgba_strip.h), shared with K1's tail.  K2 runs when the RGBA
// is not emitted by K1 itself: cropped batches (the crop windows are upsampled as standalone
// images), and the stage-alone entries (wg_batch_run_emit, wg_yuv420_to_rgba_device).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device_format.h"
#include "kernels.h"
#include "yuv_rgba_strip.h"

namespace wg {
namespace {

constexpr int kWavesPerWG = 4;

// kModes: strip::kModesRgba (no frame of the launch is emitted directly: the plain RGBA stores) or
// kModesAll (frames written straight in their output colorspace, FrameDesc::emit)
template <bool kFancy, int kModes>
__global__ void __launch_bounds__(64 * kWavesPerWG) yuv_to_rgba_kernel(const FrameDesc* __restrict__ frames,
                                                                       FrameDesc single, int use_single) {
  const FrameDesc& F = use_single ? single : frames[blockIdx.y];
  if (!F.valid) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sx = strip::strips_x(F.width);
  const int tx = blockIdx.x % sx, ty = blockIdx.x / sx;
  if (__builtin_amdgcn_readfirstlane(F.alpha_off16) != 0)  // (an alpha-first frame: RGBA, A from its plane)
    strip::convert_strip<kFancy, strip::kAuxNt, strip::kModesRgba, true>(F, tx, ty * kWavesPerWG + wave, lane);
  else
    strip::convert_strip<kFancy, strip::kAuxNt, kModes>(F, tx, ty * kWavesPerWG + wave, lane);
}

}  // namespace

hipError_t launch_yuv_to_rgba(const FrameDesc* d_frames, const FrameDesc* single, int n_frames, int max_w,
                              int max_h, int fancy, hipStream_t stream, bool modes) {
  const int strips_x = (max_w + strip::kStripPx - 1) / strip::kStripPx;
  const int npairs = (max_h >> 1) + 1;
  const int strips_y = (npairs + strip::kPairs * kWavesPerWG - 1) / (strip::kPairs * kWavesPerWG);
  const dim3 grid(strips_x * strips_y, single ? 1 : n_frames);
  FrameDesc s{};
  if (single) s = *single;
  const dim3 block(64 * kWavesPerWG);
  const int us = single ? 1 : 0;
  if (modes) {
    if (fancy) hipLaunchKernelGGL((yuv_to_rgba_kernel<true, strip::kModesAll>), grid, block, 0, stream, d_frames, s, us);
    else hipLaunchKernelGGL((yuv_to_rgba_kernel<false, strip::kModesAll>), grid, block, 0, stream, d_frames, s, us);
  } else {
    if (fancy) hipLaunchKernelGGL((yuv_to_rgba_kernel<true, strip::kModesRgba>), grid, block, 0, stream, d_frames, s, us);
    else hipLaunchKernelGGL((yuv_to_rgba_kernel<false, strip::kModesRgba>), grid, block, 0, stream, d_frames, s, us);
  }
  return hipGetLastError();
}

}  // namespace wg
