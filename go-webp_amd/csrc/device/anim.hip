// K5: animation compositing (ANMF frames already decoded by K1..K4) -> one full canvas per frame.
//
// Replaces the canvas logic of WebPAnimDecoderGetNext (pkg/libwebp/demux/anim_decode.go:312-433):
//   a key frame (IsKeyFrame :183-197) starts from a transparent canvas, any other frame from
//   the previous canvas after its disposal (ZeroFillFrameRect :164-172 for dispose-to-
//   background); the frame's pixels replace its rectangle; with blend method BLEND on a
//   non-key frame, pixels with alpha < 255 are blended over the disposed previous canvas by
//   BlendPixelNonPremult (:201-247) -- except inside the previous rectangle when that frame
//   disposed to background (FindBlendRangeAtRow :263-289: blending with transparent is
//   skipped, the decoded pixel is kept).  Output mode RGBA (non-premultiplied, the
//   WebPAnimDecoder default).
//
// The canvas recurrence is per pixel, so the kernel is data-parallel over the canvas: each
// thread owns four horizontally adjacent pixels (one 16-byte store per frame) and walks the
// frames in order with the current and the disposed value in registers, loading four frames'
// pixels ahead.  The per-frame
// descriptors are wave-uniform.  Bytes per frame: the canvas write (4 B/px) + the frame's
// rectangle read -- HBM-bound.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device_format.h"
#include "kernels.h"

namespace wg {
namespace {

constexpr int kThreads = 256;

// BlendChannelNonPremult: (src_c * src_a + dst_c * dst_factor_a) * scale >> 24, uint32
__device__ __forceinline__ uint32_t blend_channel(uint32_t src, uint32_t sa, uint32_t dst, uint32_t dfa,
                                                  uint32_t scale, int shift) {
  const uint32_t s = (src >> shift) & 0xff, d = (dst >> shift) & 0xff;
  return ((s * sa + d * dfa) * scale) >> 24;
}

// BlendPixelNonPremult (with BlendPixelRowNonPremult's alpha == 255 shortcut); RGBA bytes
// in a little-endian word: R bits 0-7 ... A bits 24-31 (CHANNEL_SHIFT(i) = 8 i).
__device__ __forceinline__ uint32_t blend_px(uint32_t src, uint32_t dst, const uint32_t* scale_tab) {
  const uint32_t sa = src >> 24;
  if (sa == 0xff) return src;
  if (sa == 0) return dst;
  const uint32_t da = dst >> 24;
  const uint32_t dfa = (da * (256 - sa)) >> 8;
  const uint32_t ba = sa + dfa;
  const uint32_t scale = scale_tab[ba];  // (1 << 24) / ba, exact
  return blend_channel(src, sa, dst, dfa, scale, 0) | (blend_channel(src, sa, dst, dfa, scale, 8) << 8) |
         (blend_channel(src, sa, dst, dfa, scale, 16) << 16) | (ba << 24);
}

__global__ void __launch_bounds__(kThreads) anim_compose_kernel(const AnimFrameDesc* __restrict__ frames,
                                                                 int n_frames, uint8_t* __restrict__ canvases,
                                                                 int cw, int ch) {
  __shared__ uint32_t scale_tab[256];
  scale_tab[threadIdx.x] = threadIdx.x ? (1u << 24) / threadIdx.x : 0u;
  __syncthreads();
  const int qw = (cw + 3) >> 2;  // 4-pixel groups per canvas row
  const int g = blockIdx.x * kThreads + threadIdx.x;
  if (g >= qw * ch) return;
  const int cy = g / qw, cx0 = (g - cy * qw) * 4;
  const int npx = min(4, cw - cx0);
  const size_t canvas_bytes = (size_t)cw * ch * 4;
  uint32_t cur[4], disp[4] = {0, 0, 0, 0};
  // the frames' pixels kAhead frames at a time: all their loads issued before the first is used
  // (the recurrence is serial in f, its loads are not: one frame at a time left each wave waiting
  // out a load per frame)
  constexpr int kAhead = 4;
  for (int f0 = 0; f0 < n_frames; f0 += kAhead) {
    uint32_t src[kAhead][4];
#pragma unroll
    for (int j = 0; j < kAhead; ++j) {
      const int f = min(f0 + j, n_frames - 1);
      const AnimFrameDesc& F = frames[f];
      const bool row_in = cy >= F.y && cy < F.y + F.height;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int cx = cx0 + k;
        const bool in = row_in && cx >= F.x && cx < F.x + F.width && k < npx;
        src[j][k] = in ? *reinterpret_cast<const uint32_t*>(F.rgba + ((size_t)(cy - F.y) * F.width + (cx - F.x)) * 4) : 0u;
      }
    }
#pragma unroll
    for (int j = 0; j < kAhead; ++j) {
      const int f = f0 + j;
      if (f >= n_frames) break;
      const AnimFrameDesc& F = frames[f];
      const bool row_in = cy >= F.y && cy < F.y + F.height;
      const bool prow_in = cy >= F.py && cy < F.py + F.ph;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int cx = cx0 + k;
        uint32_t c = F.key ? 0u : disp[k];
        const bool in = row_in && cx >= F.x && cx < F.x + F.width && k < npx;
        if (in) {
          const bool in_prev = prow_in && cx >= F.px && cx < F.px + F.pw;
          c = (F.blend && !(F.prev_dispose_bg && in_prev)) ? blend_px(src[j][k], disp[k], scale_tab) : src[j][k];
        }
        cur[k] = c;
        disp[k] = (F.dispose_bg && in) ? 0u : c;
      }
      uint8_t* out = canvases + (size_t)f * canvas_bytes + ((size_t)cy * cw + cx0) * 4;
      if (npx == 4 && (cw & 3) == 0) {
        *reinterpret_cast<uint4*>(out) = make_uint4(cur[0], cur[1], cur[2], cur[3]);
      } else {
        for (int k = 0; k < npx; ++k) reinterpret_cast<uint32_t*>(out)[k] = cur[k];
      }
    }
  }
}

}  // namespace

hipError_t launch_anim_compose(const AnimFrameDesc* d_frames, int n_frames, uint8_t* d_canvases, int canvas_w,
                               int canvas_h, hipStream_t stream) {
  if (n_frames <= 0) return hipSuccess;
  const int groups = ((canvas_w + 3) / 4) * canvas_h;
  hipLaunchKernelGGL(anim_compose_kernel, dim3((groups + kThreads - 1) / kThreads), dim3(kThreads), 0, stream,
                     d_frames, n_frames, d_canvases, canvas_w, canvas_h);
  return hipGetLastError();
}

}  // namespace wg
