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
// prefix sums (one block scan), then a wave scan per row.  Vertical and gradient run one
// 1024-thread workgroup per plane, reading the filtered bytes straight from their source (K3's
// green, the raw payload) and writing the unfiltered plane (round 6; no gather pass):
//   1. row 0 as horizontal (one wave scan);
//   2. vertical    out[y][x] = out[y-1][x] + in[y][x]: a running sum per column, four columns per
//                  thread as one dword (bytewise adds without carries), rows loaded 8 ahead;
//      gradient    out = in + clip(L + T - TL): a wavefront in 64-row bands, one band per wave at
//                  a time (lane = row, one column per step, T from the lane above by DPP, the top
//                  row of the band from the plane behind the band above's LDS progress counter --
//                  no workgroup barrier per step), bands b = w, w + 16, ... on wave w;
//   3. write the plane (its output window when cropping) into the A bytes (dword
//      read-modify-write, coalesced) -- or leave it there (alpha-first).
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
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

// kWave = false: planes with filter none / horizontal (alpha_rows_direct, `parts` workgroups each);
// true: vertical / gradient (one workgroup per plane).  Two instantiations, so the direct path keeps
// its own registers and code, and only the second holds the gradient's LDS ring.
template <bool kWave>
__global__ void __launch_bounds__(kThreads) alpha_kernel(const AlphaDesc* __restrict__ frames) {
  __shared__ int wsum[kWaves];
  __shared__ int total;
  __shared__ uint8_t palg[256];         // an 8-bit alpha stream's palette (green bytes)
  const AlphaDesc& F = frames[blockIdx.x];
  if (!F.valid || (F.filter >= 2) != kWave) return;
  if constexpr (!kWave) {
    __shared__ uint8_t rowbuf[kMaxDim];  // horizontal: column-0 prefix
    alpha_rows_direct(F, blockIdx.y, gridDim.y, rowbuf, palg, wsum, &total);
    return;
  } else {
  __shared__ uint32_t gprog[kWaves];    // gradient: each band's last row's columns done (tag: band << 16)
  // gradient: per wave, its band's outputs (a 32-column ring per row) on their way to 16-byte stores
  __shared__ __attribute__((aligned(16))) uint8_t ring[kWaves][64][32];
  const int W = F.width, H = F.height, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const gptr<uint8_t> plane = as_global(F.plane);
  if (F.coded && F.pal) {  // (an 8-bit stream's palette: only with filters none / horizontal in practice)
    if (tid < (1 << (8 >> F.cbits))) palg[tid] = (uint8_t)(F.pal[tid] >> 8);
  }
  if (tid < kWaves) gprog[tid] = 0;
  __syncthreads();
  const bool gvec = F.green && (reinterpret_cast<uintptr_t>(F.green) & 15) == 0 && (W & 3) == 0;

  // ---- 1. the filtered bytes into the plane (coalesced: four per thread and step; K7's coded
  //         image through the palette, K3's green, or the raw payload), then row 0 as
  //         HorizontalUnfilter_C with no row above (filters.go:130-140)
  {
    const bool dw = (W & 3) == 0;
    const size_t n4 = dw ? (size_t)W * H / 4 : 0;
    const int q4 = W >> 2;
    for (size_t i = tid; i < n4; i += kThreads) {
      const int y = (int)(i / (size_t)q4), x = 4 * (int)(i - (size_t)y * q4);
      *reinterpret_cast<gptr<uint32_t>>(plane + 4 * i) = src_quad(F, palg, y, x, gvec);
    }
    for (size_t i = n4 * 4 + tid; i < (size_t)W * H; i += kThreads) {
      const int y = (int)(i / (size_t)W), x = (int)(i - (size_t)y * W);
      plane[i] = (uint8_t)src_byte(F, palg, y, x);
    }
  }
  __syncthreads();
  if (wave == 0) {
    uint32_t carry = 0;
    for (int x0 = 0; x0 < W; x0 += 64) {
      const int x = x0 + lane;
      const int v = x < W ? (int)plane[x] : 0;
      const int inc = wave_incl_scan(v);
      if (x < W) plane[x] = (uint8_t)(carry + (uint32_t)inc);
      carry += (uint32_t)lane63(inc);
    }
  }
  __syncthreads();

  // ---- 2. rows 1 .. H-1
  if (F.filter == 2) {  // VerticalUnfilter_C (filters.go:146-155): a running sum per column
    const bool dw = (W & 3) == 0;  // (dword rows: four columns per thread)
    const int cols = dw ? W >> 2 : W;
    for (int c = tid; c < cols; c += kThreads) {
      if (dw) {
        const int x = 4 * c;
        uint32_t acc = *reinterpret_cast<gptr<const uint32_t>>(plane + x);
        int y = 1;
        // bytewise a + b mod 256 per byte (no carry between the four columns)
        auto badd = [](uint32_t a, uint32_t b) {
          return ((a & 0x7f7f7f7fu) + (b & 0x7f7f7f7fu)) ^ ((a ^ b) & 0x80808080u);
        };
        for (; y + 8 <= H; y += 8) {  // eight rows of loads in flight
          uint32_t v[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<gptr<const uint32_t>>(plane + (size_t)(y + k) * W + x);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            acc = badd(acc, v[k]);
            *reinterpret_cast<gptr<uint32_t>>(plane + (size_t)(y + k) * W + x) = acc;
          }
        }
        for (; y < H; ++y) {
          acc = badd(acc, *reinterpret_cast<gptr<const uint32_t>>(plane + (size_t)y * W + x));
          *reinterpret_cast<gptr<uint32_t>>(plane + (size_t)y * W + x) = acc;
        }
      } else {
        uint32_t acc = plane[c];
        for (int y = 1; y < H; ++y) {
          acc += plane[(size_t)y * W + c];
          plane[(size_t)y * W + c] = (uint8_t)acc;
        }
      }
    }
  } else if (F.filter == 3) {  // GradientUnfilter_C (filters.go:157-171)
    // Band b = rows [1 + 64 b, 1 + 64 b + 64): lane l owns row y = 1 + 64 b + l and at step s
    // works on column x = s - l.  T = out[y-1][x] is what the lane above produced at step s - 1
    // (DPP row shift); lane 0's comes from the band above's last row, read back from the plane in
    // chunks of 64 columns (one per lane, then v_readlane per step) once that band's progress
    // counter covers them; TL = the previous step's T; L = the lane's previous output.  The
    // leftmost column predicts from above (L = TL = T).
    // Memory: a lane's filtered bytes arrive 16 steps at a time (K3's green: four 16-byte loads of
    // its row, a group ahead), and its outputs go into its row of the wave's LDS ring (32 columns),
    // from which each group stores the one 16-column block of the row that has become complete --
    // 16-byte stores instead of a byte store per lane and step (64 rows touched per instruction).
    // Every 64 steps the band publishes how many columns of its last row are in the plane
    // (gprog[b & 15], tag b << 16: a later band's value on the same slot implies this one is done).
    const int nb = (H - 1 + 63) / 64;
    // (the filtered bytes are in the plane since step 1: read in place, ahead of the outputs)
    const __amdgpu_buffer_rsrc_t psrc = __builtin_amdgcn_make_buffer_rsrc(F.plane, 0, W * H, 0x00020000);
    const bool st16 = (W & 15) == 0 && (reinterpret_cast<uintptr_t>(F.plane) & 15) == 0;
    uint8_t* myring = &ring[wave][lane][0];
#ifdef WG_ABL_GRAD_1BAND  // (measurement only: one band per wave, output wrong)
    for (int bnd = wave; bnd < min(nb, kWaves); bnd += kWaves) {
#else
    for (int bnd = wave; bnd < nb; bnd += kWaves) {
#endif
      const int y0 = 1 + 64 * bnd, rows = min(64, H - y0);
      const int y = y0 + min(lane, rows - 1);
      const bool row_ok = lane < rows;
      // (global address space: flat accesses would make every LDS-ring access wait for them too)
      const gptr<const uint8_t> above = plane + (size_t)(y0 - 1) * W;
      const gptr<uint8_t> prow = as_global(plane) + (size_t)y * W;
      uint32_t L = 0, T = 0, TL = 0;
      int stored = 0;   // columns [0, stored) of the lane's row are in the plane
      // the 16 filtered bytes of steps sg .. sg + 15 (columns sg - lane ..): the five aligned dwords
      // around them as loaded, shifted into place (v_alignbyte) where used, so the loads stay in
      // flight a group ahead
      struct Grp {
        u32x4 w;
        uint32_t w4, sh;
      };
      auto load_group = [&](int sg, Grp& q) {
        // (columns before the row's start, x0 < 0 -- possible only for W < 64 -- and rows past the
        // band read 0 through the buffer range: their values are never used)
        const int e = y * W + (sg - lane);
        const uint32_t off = row_ok && e >= 0 ? (uint32_t)e : 0x20000000u;
        q.w = __builtin_amdgcn_raw_buffer_load_b128(psrc, (int)(off & ~3u), 0, 0);
        q.w4 = __builtin_amdgcn_raw_buffer_load_b32(psrc, (int)((off & ~3u) + 16), 0, 0);
        q.sh = off & 3u;
      };
      // store the lane's complete 16-column blocks below `upto` (exclusive) from the ring: during
      // the band at most one per group (the lane's columns advance 16 per group), a fixed number of
      // vector-memory operations -- a store loop of varying trip count would make the compiler wait
      // for vmcnt(0), i.e. for the group loads just issued, at the next group
      auto flush_one = [&](int upto) {
        if (row_ok && stored + 16 <= upto) {
          const uint4 v = *reinterpret_cast<const uint4*>(myring + (stored & 31));
          if (st16) {
            *reinterpret_cast<gptr<u32x4>>(prow + stored) = u32x4{v.x, v.y, v.z, v.w};
          } else {
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 16; ++k) prow[stored + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
          }
          stored += 16;
        }
      };
      auto flush_rest = [&] {  // (the row's remaining columns, after the band's last group)
        for (int m = stored; row_ok && m < W; ++m) prow[m] = myring[m & 31];
        stored = W;
      };
      Grp qa, qb;
      const int steps = W + rows - 1;
      load_group(0, qa);
      // Groups of 16 steps.  Lane j < 16 holds column 16 g + j of the row above for group g (t0),
      // loaded one group ahead (tn) once the band above's last row has stored 16 g + 32 columns;
      // the band publishes its own last row's stored columns after every group.
      auto wait_above = [&](int cols) {
#ifdef WG_ABL_GRAD_NOWAIT  // (measurement only: output wrong)
        return;
#endif
        if (bnd == 0) return;  // (row 0 is complete)
        const uint32_t need = ((uint32_t)(bnd - 1) << 16) | (uint32_t)min(W, cols);
        uint32_t* pg = gprog + ((bnd - 1) & (kWaves - 1));
        if (__hip_atomic_load(pg, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
          const uint64_t t_0 = __builtin_amdgcn_s_memrealtime();
          while (__hip_atomic_load(pg, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t_0 > 200000000ull) break;  // (2 s: never reached)
          }
        }
      };
      // (straight-line steps: no break at the band's end and no test on s < W -- steps past the
      // band's end have x >= W on every row (no output) and lane 0's T past the row's end feeds
      // nothing; a branch around each v_readlane of t0 made the waitcnt pass wait vmcnt(0) before
      // every one of them, i.e. for the group loads in flight)
      auto run_group = [&](int sg, const Grp& q, uint32_t t0) {
        const uint32_t b[4] = {__builtin_amdgcn_alignbyte(q.w.y, q.w.x, q.sh), __builtin_amdgcn_alignbyte(q.w.z, q.w.y, q.sh),
                               __builtin_amdgcn_alignbyte(q.w.w, q.w.z, q.sh), __builtin_amdgcn_alignbyte(q.w4, q.w.w, q.sh)};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int s = sg + k;
          const int x = s - lane;
          const bool ok = row_ok && x >= 0 && x < W;
          const uint32_t up = (uint32_t)__builtin_amdgcn_readlane((int)t0, k);
          T = shr1(up, L) & 0xffu;
          const uint32_t l = x == 0 ? T : L, tl = x == 0 ? T : TL;
          const int g = (int)l + (int)T - (int)tl;
          const uint32_t o = (((b[k >> 2] >> (8 * (k & 3))) & 0xffu) + (uint32_t)min(max(g, 0), 255)) & 0xffu;
          if (ok) {
#ifndef WG_ABL_GRAD_NOLDS  // (measurement only: output wrong)
            myring[x & 31] = (uint8_t)o;
#endif
            L = o;
          }
          TL = T;
        }
      };
      auto publish = [&] {  // (release: the row's plane stores before the counter; lane rows - 1 has the fewest)
        const uint32_t done = (uint32_t)__builtin_amdgcn_readlane(stored, rows - 1);
        if (lane == 0)
          __hip_atomic_store(gprog + (bnd & (kWaves - 1)), ((uint32_t)bnd << 16) | done, __ATOMIC_RELEASE,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      };
      wait_above(16);
      uint32_t ta = above[min(lane & 15, W - 1)], tb = 0;
      for (int sg = 0; sg < steps; sg += 32) {
        // group sg (qa, ta), then group sg + 16 (qb, tb)
        load_group(sg + 16, qb);
        if (sg + 16 < W) {
          wait_above(sg + 32);
          tb = above[min(sg + 16 + (lane & 15), W - 1)];
        }
        run_group(sg, qa, ta);
        flush_one(min(W, max(0, sg + 16 - lane)));
        publish();
        if (sg + 16 >= steps) break;
        load_group(sg + 32, qa);
        if (sg + 32 < W) {
          wait_above(sg + 48);
          ta = above[min(sg + 32 + (lane & 15), W - 1)];
        }
        run_group(sg + 16, qb, tb);
        flush_one(min(W, max(0, sg + 32 - lane)));
        publish();
      }
      flush_rest();
      const uint32_t done = (uint32_t)__builtin_amdgcn_readlane(stored, rows - 1);
      if (lane == 0)
        __hip_atomic_store(gprog + (bnd & (kWaves - 1)), ((uint32_t)bnd << 16) | done, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();

  // ---- 3. plane window -> A bytes (the RGBA holds the window: the whole plane unless cropping)
  if (F.to_plane) return;  // (alpha-first: the strips read the plane)
  for (int y = wave; y < F.win_h; y += kWaves) {
    uint32_t* dst = reinterpret_cast<uint32_t*>(F.rgba + (size_t)y * F.rgba_stride);
    const gptr<const uint8_t> src = plane + (size_t)(y + F.win_y) * W + F.win_x;
    for (int x = lane; x < F.win_w; x += 64) dst[x] = (dst[x] & 0x00ffffffu) | ((uint32_t)src[x] << 24);
  }
  }  // (kWave)
}

}  // namespace

hipError_t launch_alpha(const AlphaDesc* d_frames, int n_frames, hipStream_t stream, int n_wave) {
  if (n_frames <= 0) return hipSuccess;
  // filters none / horizontal run rows on `parts` workgroups per plane (the chip holds two
  // 1024-thread workgroups per CU); vertical / gradient planes one workgroup each, in a second
  // launch over the same descriptors (each instantiation skips the other's planes)
  if (n_wave < n_frames) {
    const int parts = std::max(1, std::min(8, 512 / n_frames));
    hipLaunchKernelGGL(alpha_kernel<false>, dim3(n_frames, parts), dim3(kThreads), 0, stream, d_frames);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (n_wave > 0) hipLaunchKernelGGL(alpha_kernel<true>, dim3(n_frames, 1), dim3(kThreads), 0, stream, d_frames);
  return hipGetLastError();
}

}  // namespace wg
