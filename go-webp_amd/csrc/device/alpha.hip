// K4: ALPH alpha planes of lossy frames -> the A channel of their RGBA output.
//
// Replaces the reference's alpha stage (pkg/libwebp/decoder/alpha_dec.go:47-213):
//   ALPHDecode / ExtractAlphaRows (vp8l_dec.c.go:1462-1489): alpha = green channel of the
//     lossless stream after its inverse transforms (here: K3's RGBA output, byte 1), or the
//     raw bytes for method 0;
//   WebPUnfilters (dsp/filters.go:130-171): HorizontalUnfilter_C, VerticalUnfilter_C,
//     GradientUnfilter_C, row by row with the previous output row as `prev` (none for row 0);
//   EmitAlphaRGB (io_dec.c.go:175-195): A bytes of the (non-premultiplied) RGBA output.
// WebPDequantizeLevels only runs with alpha dithering > 0 (alpha_dec.go:199-206); the
// decode options here keep it 0, as WebPDecode's defaults do, so pre-processed (level
// quantized) planes are emitted as decoded.
//
// After K2 / K1's tail (which wrote A = 255).  Filters none and horizontal -- what libwebp's
// encoder picks for most planes -- go straight from the filtered bytes to the A bytes, rows in
// parallel (alpha_rows_direct): out[y][x] = c[y-1] + sum_{i<=x} in[y][i] with c the column-0
// prefix sums (one block scan), then a wave scan per row.  Vertical and gradient keep one
// 1024-thread workgroup per plane and a scratch plane:
//   1. gather the filtered bytes into `plane` (green extraction or a copy);
//   2. unfilter in place:
//        vertical    row 0 as horizontal, then out[y][x] = out[y-1][x] + in[y][x]
//                    -> a running sum per column (threads across columns);
//        gradient    row 0 as horizontal, then out = in + clip(L + T - TL): a wavefront
//                    over 1024-row bands (thread = row, one column per step, T from the
//                    thread above via DPP / LDS, the band's top row from LDS);
//   3. write the plane (its output window when cropping) into the A bytes (dword
//      read-modify-write, coalesced).
// The gradient wavefront is latency-bound (one barrier per column step) and is the slow case.
//
// Alpha-first batches (AlphaDesc::to_plane; capi.cpp decides): K4 runs before K1 and leaves the
// unfiltered plane in `plane` (width-byte rows, the whole plane: no crop window) for the YUV -> RGBA
// strips to take A from, instead of read-modify-writing the RGBA's A bytes afterwards -- 1 B/px
// written here and read there instead of 8 B/px.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../device_format.h"
#include "kernels.h"

namespace wg {
namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;
constexpr int kMaxDim = 16384;

// Inclusive scan over the wave in DPP moves (no LDS traffic): row_shr 1 / 2 / 4 / 8 within each
// 16-lane row (lanes without a source add 0, the `old` operand), then row_bcast:15 adds row r's
// total to row r + 1 (rows 1, 3) and row_bcast:31 lane 31's to rows 2 and 3.
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

__device__ __forceinline__ int lane63(int v) { return __builtin_amdgcn_readlane(v, 63); }

// Exclusive scan of one int per thread over the block; `tot` gets the block total.
__device__ __forceinline__ int block_excl_scan(int v, int* wsum, int* tot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int inc = wave_incl_scan(v);
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  if (wave == 0) {
    const int w = lane < kWaves ? wsum[lane] : 0;
    const int wi = wave_incl_scan(w);
    if (lane < kWaves) wsum[lane] = wi - w;
    if (lane == kWaves - 1) *tot = wi;
  }
  __syncthreads();
  return wsum[wave] + inc - v;
}

// One row as HorizontalUnfilter_C with `pred` for its first byte, by wave `wave` (all
// lanes of that wave call it): 64-byte chunks, wave scan + running carry.
__device__ __forceinline__ void scan_row(uint8_t* row, int W, uint32_t pred) {
  const int lane = threadIdx.x & 63;
  uint32_t carry = pred;
  for (int x0 = 0; x0 < W; x0 += 64) {
    const int x = x0 + lane;
    const int v = x < W ? row[x] : 0;
    const int inc = wave_incl_scan(v);
    if (x < W) row[x] = (uint8_t)(carry + (uint32_t)inc);
    carry += (uint32_t)lane63(inc);
  }
}

__device__ __forceinline__ uint32_t shr1(uint32_t old, uint32_t v) {  // lane i <- lane i-1; lane 0 <- old
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

// Filtered byte x of row y: green = byte 1 of K3's pixel; raw = the ALPH payload; coded = K7's
// coded image of an 8-bit alpha stream (ColorIndexInverseTransform, lossless.go:428-459: index
// of pixel x in the green of coded[x >> cbits], its palette entry's green from `palg`, the
// palette's green bytes in LDS; no palette: the coded pixel's green).
__device__ __forceinline__ uint32_t coded_green(const AlphaDesc& F, const uint8_t* palg, uint32_t v, int x) {
  const uint32_t g = (v >> 8) & 0xff;
  if (!F.pal) return g;
  const int cb = F.cbits, bpp = 8 >> cb;
  return palg[(g >> ((x & ((1 << cb) - 1)) * bpp)) & ((1u << bpp) - 1)];
}

__device__ __forceinline__ uint32_t src_byte(const AlphaDesc& F, const uint8_t* palg, int y, int x) {
  if (F.coded) return coded_green(F, palg, F.coded[(size_t)y * F.coded_width + (x >> F.cbits)], x);
  const size_t i = (size_t)y * F.width + x;
  return F.green ? (reinterpret_cast<const uint32_t*>(F.green)[i] >> 8) & 0xff : F.raw[i];
}

// Four filtered bytes x .. x+3 of row y (x % 4 == 0, x + 3 < W), packed little-endian: green as
// one 16-byte load when the row's pixels are 16-byte aligned (`vec`); coded as one load per
// coded pixel the four share (1, 2 or 4); raw per byte.
__device__ __forceinline__ uint32_t src_quad(const AlphaDesc& F, const uint8_t* palg, int y, int x, bool vec) {
  if (F.coded) {
    const uint32_t* c = F.coded + (size_t)y * F.coded_width;
    uint32_t v0, v1, v2, v3;
    if (F.cbits >= 2) {
      v0 = v1 = v2 = v3 = c[x >> F.cbits];
    } else if (F.cbits == 1) {
      v0 = v1 = c[x >> 1];
      v2 = v3 = c[(x >> 1) + 1];
    } else {
      v0 = c[x], v1 = c[x + 1], v2 = c[x + 2], v3 = c[x + 3];
    }
    return coded_green(F, palg, v0, x) | coded_green(F, palg, v1, x + 1) << 8 | coded_green(F, palg, v2, x + 2) << 16 |
           coded_green(F, palg, v3, x + 3) << 24;
  }
  const size_t i = (size_t)y * F.width + x;
  if (F.green && vec) {
    const uint4 g = *reinterpret_cast<const uint4*>(F.green + 4 * i);
    return __builtin_amdgcn_perm(__builtin_amdgcn_perm(g.w, g.z, 0x0c0c0501u), __builtin_amdgcn_perm(g.y, g.x, 0x0c0c0501u),
                                 0x05040100u);
  }
  return src_byte(F, palg, y, x) | src_byte(F, palg, y, x + 1) << 8 | src_byte(F, palg, y, x + 2) << 16 |
         src_byte(F, palg, y, x + 3) << 24;
}

// An 8-bit alpha stream with a map of at most 16 colours (bits >= 1): the four pixels' filtered
// bytes straight from the map's green bytes held in four uniform dwords `pg` (entries 4j .. 4j + 3
// in pg[j]), by v_perm on the four indices at once instead of four LDS reads.
__device__ __forceinline__ uint32_t pal_quad(const AlphaDesc& F, const uint32_t pg[4], int y, int x) {
  const uint32_t* c = F.coded + (size_t)y * F.coded_width;
  uint32_t i4;
  if (F.cbits == 1) {
    const uint32_t a = (c[x >> 1] >> 8) & 0xff, b = (c[(x >> 1) + 1] >> 8) & 0xff;
    i4 = (a & 15) | (a >> 4) << 8 | (b & 15) << 16 | (b >> 4) << 24;
  } else if (F.cbits == 2) {
    const uint32_t g = (c[x >> 2] >> 8) & 0xff;
    i4 = (g & 3) | ((g >> 2) & 3) << 8 | ((g >> 4) & 3) << 16 | (g >> 6) << 24;
  } else {
    const uint32_t t = ((c[x >> 3] >> 8) & 0xff) >> (x & 7);
    i4 = (t & 1) | ((t >> 1) & 1) << 8 | ((t >> 2) & 1) << 16 | ((t >> 3) & 1) << 24;
  }
  const uint32_t sel = i4 & 0x07070707u;
  const uint32_t lo = __builtin_amdgcn_perm(pg[1], pg[0], sel), hi = __builtin_amdgcn_perm(pg[3], pg[2], sel);
  const uint32_t m = ((i4 >> 3) & 0x01010101u) * 0xffu;
  return (hi & m) | (lo & ~m);
}

// Filters none / horizontal straight from the filtered bytes into the A bytes, one wave per
// output row, no plane: HorizontalUnfilter_C (filters.go:130-140) is out[y][x] = out[y-1][0] +
// sum_{i<=x} in[y][i] (mod 256), and out[y-1][0] is the column-0 prefix c[y-1], so the rows are
// independent once c (one block scan of column 0, `rowbuf`) is known.  A lane owns 4 adjacent
// pixels: 4 filtered bytes in, an in-lane prefix, one wave scan of the 4-sums, a running carry
// per 256 pixels, and the RGBA window's 16 bytes read-modify-written (4 dwords where the window
// is not 16-byte aligned).  Workgroup `part` of `parts` takes output rows part, part + parts, ...
// (each computes c itself: H strided bytes).  12 B/px (green) at most: 4 in + 8 RMW.
__device__ void alpha_rows_direct(const AlphaDesc& F, int part, int parts, uint8_t* rowbuf, uint8_t* palg, int* wsum,
                                  int* total) {
  const int W = F.width, H = F.height, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const bool horiz = F.filter == 1;
  if (F.coded && F.pal) {
    if (tid < (1 << (8 >> F.cbits))) palg[tid] = (uint8_t)(F.pal[tid] >> 8);
    __syncthreads();
  }
  if (horiz) {
    const int per = (H + kThreads - 1) / kThreads, y0 = tid * per, y1 = min(H, y0 + per);
    int s = 0;
    for (int y = y0; y < y1; ++y) s += src_byte(F, palg, y, 0);
    int run = block_excl_scan(s, wsum, total);
    for (int y = y0; y < y1; ++y) {
      run += src_byte(F, palg, y, 0);
      rowbuf[y] = (uint8_t)run;
    }
    __syncthreads();
  }
  const bool ppal = F.coded && F.pal && F.cbits >= 1;  // (pal_quad)
  uint32_t pg[4] = {0u, 0u, 0u, 0u};
  if (ppal) {
    const int ne = 1 << (8 >> F.cbits);
#pragma unroll
    for (int e = 0; e < 16; ++e)
      if (e < ne) pg[e >> 2] |= ((F.pal[e] >> 8) & 0xffu) << (8 * (e & 3));
  }
  const bool gvec = F.green && (reinterpret_cast<uintptr_t>(F.green) & 15) == 0 && (W & 3) == 0;
  const bool ovec = ((reinterpret_cast<uintptr_t>(F.rgba) | (uintptr_t)F.rgba_stride) & 15) == 0 && (F.win_x & 3) == 0;
  const bool pvec = (W & 3) == 0;  // to_plane: the rows' dwords are aligned (the plane is)
  const int xe = F.win_x + F.win_w;  // window columns [win_x, xe)
  for (int yo = part * kWaves + wave; yo < F.win_h; yo += parts * kWaves) {
    const int y = yo + F.win_y;
    uint8_t* orow = F.rgba + (size_t)yo * F.rgba_stride - 4 * (size_t)F.win_x;  // (pixel x at orow + 4x)
    uint8_t* prow = F.plane + (size_t)y * W;  // (to_plane: the whole plane, window = plane)
    uint32_t carry = horiz && y > 0 ? rowbuf[y - 1] : 0u;
    // (horizontal: every chunk from x = 0, the prefix needs it; none: the window's chunks)
    for (int x0 = horiz ? 0 : (F.win_x & ~255); x0 < xe; x0 += 256) {
      const int x = x0 + 4 * lane;
      uint32_t q = 0;
      if (x + 3 < W) q = ppal ? pal_quad(F, pg, y, x) : src_quad(F, palg, y, x, gvec);
      else
        for (int k = 0; k < 4 && x + k < W; ++k) q |= src_byte(F, palg, y, x + k) << (8 * k);
      uint32_t o = q;
      if (horiz) {  // in-lane prefix of the 4 bytes (mod 256 per byte), then the wave scan
        const uint32_t b0 = q & 0xff, b1 = b0 + ((q >> 8) & 0xff), b2 = b1 + ((q >> 16) & 0xff), b3 = b2 + (q >> 24);
        const uint32_t incl = (uint32_t)wave_incl_scan((int)(b3 & 0xff));
        const uint32_t base = carry + incl - (b3 & 0xff);
        o = ((base + b0) & 0xff) | ((base + b1) & 0xff) << 8 | ((base + b2) & 0xff) << 16 | (base + b3) << 24;
        carry += (uint32_t)lane63((int)incl);
      }
      if (x0 + 256 <= F.win_x) continue;
      if (F.to_plane) {
        if (pvec && x + 3 < W) {
          *reinterpret_cast<uint32_t*>(prow + x) = o;
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (x + k < W) prow[x + k] = (uint8_t)(o >> (8 * k));
        }
      } else if (ovec && x >= F.win_x && x + 3 < xe) {
        uint4* d = reinterpret_cast<uint4*>(orow + 4 * (size_t)x);
        uint4 v = *d;
        v.x = (v.x & 0x00ffffffu) | o << 24;
        v.y = (v.y & 0x00ffffffu) | (o >> 8) << 24;
        v.z = (v.z & 0x00ffffffu) | (o >> 16) << 24;
        v.w = (v.w & 0x00ffffffu) | (o >> 24) << 24;
        *d = v;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (x + k < F.win_x || x + k >= xe) continue;
          uint32_t* d = reinterpret_cast<uint32_t*>(orow + 4 * (size_t)(x + k));
          *d = (*d & 0x00ffffffu) | ((o >> (8 * k)) & 0xff) << 24;
        }
      }
    }
  }
}

__global__ void __launch_bounds__(kThreads) alpha_kernel(const AlphaDesc* __restrict__ frames) {
  __shared__ uint8_t rowbuf[kMaxDim];  // horizontal: column-0 prefix; gradient: the band's top row
  __shared__ int wsum[kWaves];
  __shared__ int total;
  __shared__ uint32_t edge[2][kWaves];  // gradient: each wave's lane-63 output of the last step
  __shared__ uint8_t palg[256];         // an 8-bit alpha stream's palette (green bytes)
  const AlphaDesc& F = frames[blockIdx.x];
  if (!F.valid) return;
  if (F.filter <= 1) {
    alpha_rows_direct(F, blockIdx.y, gridDim.y, rowbuf, palg, wsum, &total);
    return;
  }
  if (blockIdx.y > 0) return;  // (vertical / gradient: the whole plane in one workgroup)
  const int W = F.width, H = F.height, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const size_t n = (size_t)W * H;
  uint8_t* plane = F.plane;

  // ---- 1. filtered bytes into the plane (4 px per thread step)
  if (F.green) {
    const uint32_t* g = reinterpret_cast<const uint32_t*>(F.green);
    uint32_t* p4 = reinterpret_cast<uint32_t*>(plane);
    const size_t n4 = n / 4;
    for (size_t i = tid; i < n4; i += kThreads) {
      const uint32_t a = g[4 * i], b = g[4 * i + 1], c = g[4 * i + 2], d = g[4 * i + 3];
      p4[i] = ((a >> 8) & 0xff) | (b & 0xff00) | ((c << 8) & 0xff0000) | ((d << 16) & 0xff000000u);
    }
    for (size_t i = n4 * 4 + tid; i < n; i += kThreads) plane[i] = (uint8_t)(g[i] >> 8);
  } else {
    const uint32_t* r4 = reinterpret_cast<const uint32_t*>(F.raw);
    uint32_t* p4 = reinterpret_cast<uint32_t*>(plane);
    const size_t n4 = (reinterpret_cast<uintptr_t>(F.raw) & 3) ? 0 : n / 4;
    for (size_t i = tid; i < n4; i += kThreads) p4[i] = r4[i];
    for (size_t i = n4 * 4 + tid; i < n; i += kThreads) plane[i] = F.raw[i];
  }
  __syncthreads();

  // ---- 2. unfilter in place
  if (F.filter == 1) {  // horizontal
    // column-0 prefix sums c[y] (mod 256) into rowbuf
    const int per = (H + kThreads - 1) / kThreads, y0 = tid * per, y1 = min(H, y0 + per);
    int s = 0;
    for (int y = y0; y < y1; ++y) s += plane[(size_t)y * W];
    int run = block_excl_scan(s, wsum, &total);
    for (int y = y0; y < y1; ++y) {
      run += plane[(size_t)y * W];
      rowbuf[y] = (uint8_t)run;
    }
    __syncthreads();
    for (int y = wave; y < H; y += kWaves) scan_row(plane + (size_t)y * W, W, y == 0 ? 0u : rowbuf[y - 1]);
  } else if (F.filter == 2) {  // vertical
    if (wave == 0) scan_row(plane, W, 0u);
    __syncthreads();
    for (int x = tid; x < W; x += kThreads) {
      uint32_t acc = plane[x];
      int y = 1;
      for (; y + 8 <= H; y += 8) {  // eight rows of loads in flight per step
        uint8_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = plane[(size_t)(y + k) * W + x];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          acc += v[k];
          plane[(size_t)(y + k) * W + x] = (uint8_t)acc;
        }
      }
      for (; y < H; ++y) {
        acc += plane[(size_t)y * W + x];
        plane[(size_t)y * W + x] = (uint8_t)acc;
      }
    }
  } else if (F.filter == 3) {  // gradient
    if (wave == 0) scan_row(plane, W, 0u);
    __syncthreads();
    for (int x = tid; x < W; x += kThreads) rowbuf[x] = plane[x];
    __syncthreads();
    for (int yb = 1; yb < H; yb += kThreads) {
      const int rows = min(kThreads, H - yb);
      const int y = yb + tid;
      const bool row_ok = tid < rows;
      uint8_t* prow = plane + (size_t)min(y, H - 1) * W;
      // inputs eight steps ahead (a shift register of loaded bytes)
      constexpr int kAhead = 8;
      uint32_t q[kAhead];
#pragma unroll
      for (int k = 0; k < kAhead; ++k) {
        const int x = k - tid;
        q[k] = (row_ok && x >= 0 && x < W) ? prow[x] : 0u;
      }
      uint32_t L = 0, TL = 0;
      const int steps = W + rows - 1;
      for (int s = 0; s < steps; ++s) {
        const int x = s - tid;
        const bool ok = row_ok && x >= 0 && x < W;
        // T = out[y-1][x]: the thread above's output of step s-1 (DPP within the wave;
        // across waves through `edge`; the band's top row from rowbuf)
        uint32_t up = 0;
        if (wave > 0) up = edge[(s + 1) & 1][wave - 1];
        else if (s < W) up = rowbuf[s];
        uint32_t T = shr1(up, L) & 0xff;
        const uint32_t v = q[0];
#pragma unroll
        for (int k = 0; k + 1 < kAhead; ++k) q[k] = q[k + 1];
        {
          const int xa = x + kAhead;
          q[kAhead - 1] = (row_ok && xa >= 0 && xa < W) ? prow[xa] : 0u;
        }
        uint32_t l = L, tl = TL;
        if (x == 0) l = tl = T;  // leftmost: predicted from above
        const int g = (int)l + (int)T - (int)tl;
        const uint32_t o = (v + (uint32_t)min(max(g, 0), 255)) & 0xff;
        if (ok) {
          prow[x] = (uint8_t)o;
          L = o;
          if (tid == rows - 1) rowbuf[x] = (uint8_t)o;  // the next band's top row
        }
        TL = T;
        if (lane == 63) edge[s & 1][wave] = L;
        __syncthreads();
      }
      __syncthreads();
    }
  }
  __syncthreads();

  // ---- 3. plane window -> A bytes (the RGBA holds the window: the whole plane unless cropping)
  if (F.to_plane) return;  // (alpha-first: the strips read the plane)
  for (int y = wave; y < F.win_h; y += kWaves) {
    uint32_t* dst = reinterpret_cast<uint32_t*>(F.rgba + (size_t)y * F.rgba_stride);
    const uint8_t* src = plane + (size_t)(y + F.win_y) * W + F.win_x;
    for (int x = lane; x < F.win_w; x += 64) dst[x] = (dst[x] & 0x00ffffffu) | ((uint32_t)src[x] << 24);
  }
}

}  // namespace

hipError_t launch_alpha(const AlphaDesc* d_frames, int n_frames, hipStream_t stream) {
  if (n_frames <= 0) return hipSuccess;
  // filters none / horizontal run rows on `parts` workgroups per plane (the chip holds two
  // 1024-thread workgroups per CU); vertical / gradient planes use the first only
  const int parts = std::max(1, std::min(8, 512 / n_frames));
  hipLaunchKernelGGL(alpha_kernel, dim3(n_frames, parts), dim3(kThreads), 0, stream, d_frames);
  return hipGetLastError();
}

}  // namespace wg
