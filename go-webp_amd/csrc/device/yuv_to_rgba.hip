// K2: YUV420 -> RGBA for a batch of frames (the headline HBM-roofline stage).
//
// Replaces the reference's output emitters:
//   EmitFancyRGB           pkg/libwebp/decoder/io_dec.c.go:65-115
//   UpsampleRgbaLinePair_C pkg/libwebp/dsp/upsampling.c.go:43-107
//   EmitSampledRGB         pkg/libwebp/decoder/io_dec.c.go:53-59, dsp/yuv.go:19-58
//   VP8YuvToRgba           R,G,B = YUVToR/G/B (pkg/color/yuv/conversion.go:28-49), A=0xff
//
// The line-pair upsampler with its packed-u/v "diagonal" trick is exactly the
// separable 9-3-3-1 filter (9a + 3b + 3c + d + 8) >> 4 with edge replication
// (tests/test_oracle.py::test_upsampler_closed_form), where for output pixel
// (x, y): near chroma = (y>>1, x>>1), far row/col = near -/+ 1 toward the pixel,
// clamped to the plane.  So every output pixel is independent: one thread makes an
// 8-pixel x 2-row block (output rows 2p-1 and 2p share chroma rows p-1 and p),
// reading 2 x 8 luma bytes and 2 x 2 x 6 chroma bytes and writing 64 RGBA bytes
// with 16-byte stores.  Algorithmic traffic: W*H + 2*ceil(W/2)*ceil(H/2) bytes in,
// 4*W*H bytes out.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device_format.h"
#include "kernels.h"

namespace wg {
namespace {

constexpr int kTileX = 64;  // 8-pixel groups per workgroup row (512 px)
constexpr int kTileY = 4;   // row pairs per workgroup

// clamp(v, 0, 255) as an opaque v_med3_i32.  Written in asm on purpose: ROCm 7.2 fuses
// two `clamp(x >> 6)` + byte-pack sequences into gfx950's v_ashr_pk_u8_i32 and then
// assumes its upper 16 bits are zero, which corrupted the B byte whenever G saturated
// low (caught by tests/test_gpu_parity.py).
__device__ __forceinline__ uint32_t clamp_u8(int v) {
  int r;
  asm("v_med3_i32 %0, %1, 0, %2" : "=v"(r) : "v"(v), "s"(255));
  return (uint32_t)r;
}

__device__ __forceinline__ uint32_t yuv_to_rgba(int y, int u, int v) {
  // MultHi(a, c) = (a*c) >> 8; Clip8(v) = clamp(v >> 6, 0, 255) (YUV_FIX2 = 6)
  const int y1 = __mul24(y, 19077) >> 8;
  const int r = (y1 + (__mul24(v, 26149) >> 8) - 14234) >> 6;
  const int g = (y1 - (__mul24(u, 6419) >> 8) - (__mul24(v, 13320) >> 8) + 8708) >> 6;
  const int b = (y1 + (__mul24(u, 33050) >> 8) - 17685) >> 6;
  return clamp_u8(r) | (clamp_u8(g) << 8) | (clamp_u8(b) << 16) | 0xff000000u;
}

__device__ __forceinline__ int bsel(uint32_t w, int i) { return (w >> (8 * i)) & 0xff; }

// Chroma samples c0-1 .. c0+4 of one row as an array s[0..5] (clamped at the edges).
struct Row6 { int s[6]; };

__device__ __forceinline__ Row6 load_row6(const uint8_t* row, int c0, int uv_w) {
  Row6 r;
  const uint32_t w = *reinterpret_cast<const uint32_t*>(row + c0);
  const int last = uv_w - 1;
  r.s[0] = row[max(c0 - 1, 0)];
  r.s[1] = bsel(w, 0);
  r.s[2] = c0 + 1 <= last ? bsel(w, 1) : r.s[1];
  r.s[3] = c0 + 2 <= last ? bsel(w, 2) : r.s[2];
  r.s[4] = c0 + 3 <= last ? bsel(w, 3) : r.s[3];
  r.s[5] = c0 + 4 <= last ? row[c0 + 4] : r.s[4];
  return r;
}

// Upsampled chroma for the 8 pixels x0..x0+7 (x0 = 2*c0) of one output row.
__device__ __forceinline__ void upsample8(const Row6& n, const Row6& f, int out[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int nc = 1 + (i >> 1);
    const int fc = (i & 1) ? nc + 1 : nc - 1;
    out[i] = (9 * n.s[nc] + 3 * n.s[fc] + 3 * f.s[nc] + f.s[fc] + 8) >> 4;
  }
}

__device__ __forceinline__ void store8(uint8_t* dst, const uint32_t px[8], int nvalid, bool aligned) {
  if (aligned && nvalid == 8) {
    reinterpret_cast<uint4*>(dst)[0] = make_uint4(px[0], px[1], px[2], px[3]);
    reinterpret_cast<uint4*>(dst)[1] = make_uint4(px[4], px[5], px[6], px[7]);
  } else {
    for (int i = 0; i < 8; ++i)
      if (i < nvalid) reinterpret_cast<uint32_t*>(dst)[i] = px[i];
  }
}

template <bool kFancy>
__global__ void __launch_bounds__(256) yuv_to_rgba_kernel(const FrameDesc* __restrict__ frames, FrameDesc single,
                                                          int use_single) {
  const FrameDesc& F = use_single ? single : frames[blockIdx.y];
  if (!F.valid) return;
  const int W = F.width, H = F.height;
  const int uv_w = (W + 1) >> 1, uv_h = (H + 1) >> 1;
  const int groups = (W + 7) >> 3;
  const int gx_tiles = (groups + kTileX - 1) / kTileX;
  const int tile = blockIdx.x;
  const int tx = tile % gx_tiles, ty = tile / gx_tiles;
  const int g = tx * kTileX + (threadIdx.x & (kTileX - 1));
  const int p = ty * kTileY + (threadIdx.x / kTileX);
  const int npairs = kFancy ? (H >> 1) + 1 : (H + 1) >> 1;
  if (g >= groups || p >= npairs) return;
  const int x0 = 8 * g, c0 = 4 * g;
  const int nvalid = min(8, W - x0);
  const bool aligned = ((F.rgba_stride & 15) == 0) && ((reinterpret_cast<uintptr_t>(F.rgba) & 15) == 0);
  const uint8_t* Y = F.y;
  const uint8_t* U = F.u;
  const uint8_t* V = F.v;
  if (kFancy) {
    // output rows ya = 2p-1 (odd) and yb = 2p (even); chroma rows r0 = p-1, r1 = p (clamped)
    const int ya = 2 * p - 1, yb = 2 * p;
    const int r0 = max(p - 1, 0), r1 = min(p, uv_h - 1);
    const Row6 u0 = load_row6(U + (size_t)r0 * F.uv_stride, c0, uv_w);
    const Row6 u1 = load_row6(U + (size_t)r1 * F.uv_stride, c0, uv_w);
    const Row6 v0 = load_row6(V + (size_t)r0 * F.uv_stride, c0, uv_w);
    const Row6 v1 = load_row6(V + (size_t)r1 * F.uv_stride, c0, uv_w);
    if (ya >= 0) {  // near = r0, far = r1
      const uint2 yy = *reinterpret_cast<const uint2*>(Y + (size_t)ya * F.y_stride + x0);
      int uu[8], vv[8];
      upsample8(u0, u1, uu);
      upsample8(v0, v1, vv);
      uint32_t px[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) px[i] = yuv_to_rgba(bsel(i < 4 ? yy.x : yy.y, i & 3), uu[i], vv[i]);
      store8(F.rgba + (size_t)ya * F.rgba_stride + 4 * x0, px, nvalid, aligned);
    }
    if (yb < H) {  // near = r1, far = r0
      const uint2 yy = *reinterpret_cast<const uint2*>(Y + (size_t)yb * F.y_stride + x0);
      int uu[8], vv[8];
      upsample8(u1, u0, uu);
      upsample8(v1, v0, vv);
      uint32_t px[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) px[i] = yuv_to_rgba(bsel(i < 4 ? yy.x : yy.y, i & 3), uu[i], vv[i]);
      store8(F.rgba + (size_t)yb * F.rgba_stride + 4 * x0, px, nvalid, aligned);
    }
  } else {
    // point sampling: rows 2p and 2p+1 both use chroma row p (WebPSamplerProcessPlane)
    const uint32_t uw = *reinterpret_cast<const uint32_t*>(U + (size_t)p * F.uv_stride + c0);
    const uint32_t vw = *reinterpret_cast<const uint32_t*>(V + (size_t)p * F.uv_stride + c0);
    for (int k = 0; k < 2; ++k) {
      const int yr = 2 * p + k;
      if (yr >= H) break;
      const uint2 yy = *reinterpret_cast<const uint2*>(Y + (size_t)yr * F.y_stride + x0);
      uint32_t px[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        px[i] = yuv_to_rgba(bsel(i < 4 ? yy.x : yy.y, i & 3), bsel(uw, i >> 1), bsel(vw, i >> 1));
      store8(F.rgba + (size_t)yr * F.rgba_stride + 4 * x0, px, nvalid, aligned);
    }
  }
}

}  // namespace

hipError_t launch_yuv_to_rgba(const FrameDesc* d_frames, const FrameDesc* single, int n_frames, int max_w,
                              int max_h, int fancy, hipStream_t stream) {
  const int groups = (max_w + 7) >> 3;
  const int gx = (groups + kTileX - 1) / kTileX;
  const int npairs = (max_h >> 1) + 1;
  const int gy = (npairs + kTileY - 1) / kTileY;
  const dim3 grid(gx * gy, single ? 1 : n_frames);
  FrameDesc s{};
  if (single) s = *single;
  if (fancy)
    hipLaunchKernelGGL(yuv_to_rgba_kernel<true>, grid, dim3(256), 0, stream, d_frames, s, single ? 1 : 0);
  else
    hipLaunchKernelGGL(yuv_to_rgba_kernel<false>, grid, dim3(256), 0, stream, d_frames, s, single ? 1 : 0);
  return hipGetLastError();
}

}  // namespace wg
