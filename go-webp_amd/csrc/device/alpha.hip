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
// 1024-thread workgroup per plane on a scratch plane (width-byte rows):
//   1. the filtered bytes into it (a wave per row: K3's green, the raw payload, K7's coded image
//      through its map) -- unless K7 wrote them there itself (8-bit streams, LLTokDesc::afilt) --
//      then row 0 as horizontal (one wave scan);
//   2. vertical    out[y][x] = out[y-1][x] + in[y][x]: a running sum per column, four columns per
//                  thread as one dword (bytewise adds without carries), rows loaded 8 ahead;
//      gradient    out = in + clip(L + T - TL): a wavefront in 64-row bands, one band per wave at
//                  a time (lane = row, one column per step, T from the lane above by DPP, the top
//                  row of the band through an LDS ring written by the band above, behind its LDS
//                  progress counter -- no workgroup barrier per step), bands b = w, w + 16, ... on
//                  wave w; the filtered bytes arrive 16 columns per lane by LDS-DMA three groups
//                  ahead, from K7's band tiles (64 rows x 16 columns per KiB) when K7 wrote them;
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

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
// LDS byte address of a __shared__ object (M0 / ds address form)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// The gradient's LDS-DMA loads: 16 bytes per lane from buffer `rs` (bounds-checked: out-of-range
// offsets read 0) at `off` into LDS at `lds` + 16 lane.  Invisible to the compiler's vmcnt
// bookkeeping: the consumer waits with its own counted s_waitcnt.  M0 is written and restored in
// the same statement (compiler-reserved); s_nop 4 covers a descriptor fresh from v_readfirstlane,
// s_nop 0 the M0 write before the load.
__device__ __forceinline__ void dma_load_b128(i32x4 rs, uint32_t off, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(off), "s"(lds), "s"(rs)
      : "memory");
}

// Bytes [4 q + r, 4 q + r + 16) of the 32 in d0..d7 (zeros past them), q in 0..4, r in 0..3,
// per-lane values: a binary mux on q's bits (18 v_cndmask), then v_alignbyte.  (Scalars, no
// array: a select chain over an array becomes an indexed access, i.e. a private array in scratch.)
__device__ __forceinline__ void window16(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t d4, uint32_t d5,
                                         uint32_t d6, uint32_t d7, int q, int r, uint32_t o[4]) {
  const bool b1 = (q & 1) != 0, b2 = (q & 2) != 0, b4 = (q & 4) != 0;
  const uint32_t e0 = b1 ? d1 : d0, e1 = b1 ? d2 : d1, e2 = b1 ? d3 : d2, e3 = b1 ? d4 : d3, e4 = b1 ? d5 : d4,
                 e5 = b1 ? d6 : d5, e6 = b1 ? d7 : d6, e7 = b1 ? 0u : d7;
  const uint32_t f0 = b2 ? e2 : e0, f1 = b2 ? e3 : e1, f2 = b2 ? e4 : e2, f3 = b2 ? e5 : e3, f4 = b2 ? e6 : e4;
  (void)e7;
  const uint32_t g0 = b4 ? d4 : f0, g1 = b4 ? d5 : f1, g2 = b4 ? d6 : f2, g3 = b4 ? d7 : f3, g4 = b4 ? 0u : f4;
  o[0] = __builtin_amdgcn_alignbyte(g1, g0, r);
  o[1] = __builtin_amdgcn_alignbyte(g2, g1, r);
  o[2] = __builtin_amdgcn_alignbyte(g3, g2, r);
  o[3] = __builtin_amdgcn_alignbyte(g4, g3, r);
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
  if (F.raw && ((reinterpret_cast<uintptr_t>(F.raw) | (uintptr_t)F.width) & 3) == 0)
    return *reinterpret_cast<const uint32_t*>(F.raw + i);
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
  // (filter none, alpha-first, K7 wrote the bytes into the plane: they are the output already)
  if (!horiz && F.to_plane && F.raw == F.plane) return;
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
  const int W = F.width, H = F.height, tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // (uniform: the band loop and its exits stay scalar)
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
  //         (a wave per row, a lane per four columns; maps of at most 16 colours by v_perm)
  //         (K7 wrote an 8-bit stream's filtered bytes into the plane itself: nothing to gather)
  if (F.raw != F.plane) {
    const bool dw = (W & 3) == 0;
    const bool ppal = F.coded && F.pal && F.cbits >= 1;
    uint32_t pg[4] = {0u, 0u, 0u, 0u};
    if (ppal) {
      const int ne = 1 << (8 >> F.cbits);
#pragma unroll
      for (int e = 0; e < 16; ++e)
        if (e < ne) pg[e >> 2] |= ((F.pal[e] >> 8) & 0xffu) << (8 * (e & 3));
    }
    for (int y = wave; y < H; y += kWaves) {
      const gptr<uint8_t> prow = plane + (size_t)y * W;
      for (int x = 4 * lane; x < W; x += 256) {
        if (x + 3 < W) {
          const uint32_t q = ppal ? pal_quad(F, pg, y, x) : src_quad(F, palg, y, x, gvec);
          if (dw) {
            *reinterpret_cast<gptr<uint32_t>>(prow + x) = q;
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) prow[x + k] = (uint8_t)(q >> (8 * k));
          }
        } else {
          for (int k = 0; x + k < W; ++k) prow[x + k] = (uint8_t)src_byte(F, palg, y, x + k);
        }
      }
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
#ifdef WG_ABL_GRAD_SKIP  // (measurement only: output wrong)
    if (F.width != 12345) goto grad_done;
#endif
    // Band b = rows [1 + 64 b, 1 + 64 b + 64): lane l owns row y = 1 + 64 b + l and at step s
    // works on column x = s - l.  T = out[y-1][x] is what the lane above produced at step s - 1
    // (DPP wave shift); TL = the previous step's T; L = the lane's previous output; the leftmost
    // column predicts from above (L = TL = T).  Lane 0's T is the band above's last row: that band
    // writes the row's outputs into an LDS ring (`tring`, one per band slot b & 15, 512 columns)
    // as it stores them, and publishes how many columns are there (gprog[b & 15], tag b << 16: a
    // later band's value on the slot implies this one is done); band 0's T is row 0 (`row0`).  The
    // band below reports the columns it has read (cprog) so the ring is not overwritten early.
    // Steps go in groups of 16 (column x0 = 16 g - lane .. x0 + 15 for the lane in group g).
    // Inputs: a group's 16 filtered bytes span two aligned 16-byte blocks of the row, the second
    // being the first of the next group: each group loads ONE aligned block -- A lane is a row, so
    // every load or store touches 64 lines, and that line rate bounds the wavefront (an unaligned
    // 16 + 4-byte pair per group, plus a global T load, cost 0.6 ms more on c3ag).  The blocks go
    // by LDS-DMA (buffer_load ... lds: no VGPR destination, so nothing the compiler could copy
    // before the data lands) into the wave's four 1 KiB slots, three groups ahead; the wave waits
    // for them with a counted vmcnt (hidden from the compiler: its own count fell back to waiting
    // for nearly every load at the loop's back edge).  Blocks start at or after x0: none holds an
    // output yet; a neighbouring row's bytes in a block feed only columns outside the row.
    // Outputs: a group's 16 outputs sit in `cur` (static byte positions); after the group the lane
    // stores the aligned 16-column block of its row that has just become complete, shifted out of
    // prv|cur (the shift is the same for every group of the lane).
    const int nb = (H - 1 + 63) / 64;
    constexpr int kRing = 512;
    __shared__ __attribute__((aligned(16))) uint8_t tring[kWaves][kRing];
    __shared__ __attribute__((aligned(16))) uint8_t row0[kMaxDim];
    __shared__ __attribute__((aligned(16))) uint32_t dma[kWaves][4][256];  // (1 KiB per slot: 16 B per lane)
    __shared__ uint32_t cprog[kWaves];
    if (tid < kWaves) cprog[tid] = 0;
    for (int x = tid; x < W; x += kThreads) row0[x] = plane[x];
    __syncthreads();
    const __amdgpu_buffer_rsrc_t psrc = __builtin_amdgcn_make_buffer_rsrc(F.plane, 0, W * H, 0x00020000);
    // the group loads' source: K7's band tiles (rows 1..: tile (b, c) = 64 rows x 16 columns, 1 KiB,
    // LLTokDesc::atile) -- a group's loads then read four 256-byte runs instead of 64 rows -- or the
    // plane itself (width-byte rows)
    const bool tl = F.tiles != nullptr;
    const int ncb = (W + 15) >> 4;
    const uint64_t pa = reinterpret_cast<uintptr_t>(tl ? F.tiles : F.plane);
    const i32x4 prs = {__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)pa),
                       __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)(pa >> 32) & 0xffff),
                       __builtin_amdgcn_readfirstlane(tl ? nb * ncb * 1024 : W * H), 0x00020000};
    const bool st16 = (W & 15) == 0 && (reinterpret_cast<uintptr_t>(F.plane) & 15) == 0;
    uint32_t dslot[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) dslot[k] = lds_addr(&dma[wave][k][0]);
    auto spin = [&](const uint32_t* ctr, uint32_t need) {  // (acquire; 2 s bound: never reached)
#ifdef WG_ABL_GRAD_NOWAIT  // (measurement only: output wrong)
      return;
#endif
      if (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
        const uint64_t t_0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t_0 > 200000000ull) break;
        }
      }
    };
#ifdef WG_ABL_GRAD_1BAND  // (measurement only: output wrong)
    for (int bnd = wave; bnd < min(nb, kWaves); bnd += kWaves) {
#else
    for (int bnd = wave; bnd < nb; bnd += kWaves) {
#endif
      const int y0 = 1 + 64 * bnd, rows = min(64, H - y0);
      const int y = y0 + min(lane, rows - 1);
      const bool row_ok = lane < rows;
#ifdef WG_ABL_GRAD_1BAND
      const bool produce = bnd + 1 < min(nb, kWaves);
#else
      const bool produce = bnd + 1 < nb;
#endif  // (a band below reads this one's last row, lane 63)
      const int slot = bnd & (kWaves - 1), aslot = (bnd - 1) & (kWaves - 1);
      // (global address space: flat accesses would make every LDS access wait for them too)
      const gptr<uint8_t> prow = as_global(plane) + (size_t)y * W;
      uint32_t L = 0, T = 0, TL = 0;
      int stored = 0;   // columns [0, stored) of the lane's row are in the plane
      // Group g's new block: the plane's aligned block c = ceil(A / 16) at A = y W + x0, taken from
      // (previous | new) at ls = 16 - (-A mod 16); or, in tiles, the row's block g - lane / 16 of
      // the band (x0 = 16 g - lane: ls = 16 - lane mod 16), one tile (1 KiB) further per group.
      // Group 0's previous block: tiles -- only columns x < 0, unused; plane -- a plain counted load.
      const int A0 = tl ? -lane : y * W - lane;
      const int ls = 16 - ((-A0) & 15), lq = ls >> 2, lr = ls & 3;
      const uint32_t blk0 = !row_ok ? 0x80000000u
                            : tl    ? (uint32_t)(((bnd * ncb - (lane >> 4)) << 10) + (lane << 4))
                                    : (uint32_t)(A0 + ((-A0) & 15));
      const uint32_t gstep = tl ? 64u : 1u;  // (offset per step: a tile per 16 steps)
      u32x4 prevw = {0u, 0u, 0u, 0u};
      if (!tl) prevw = __builtin_amdgcn_raw_buffer_load_b128(psrc, (int)(blk0 - 16u), 0, 0);
#ifdef WG_ABL_GRAD_NOLOAD  // (measurement only: output wrong)
      auto load_group = [&](int sg, int k) { if (F.width == 12345) dma_load_b128(prs, blk0 + gstep * (uint32_t)sg, dslot[k]); };
#else
      auto load_group = [&](int sg, int k) { dma_load_b128(prs, blk0 + gstep * (uint32_t)sg, dslot[k]); };
#endif
      const int sh = 16 - ((-lane) & 15), sq = sh >> 2, sr = sh & 3;
      uint32_t prv[4] = {0u, 0u, 0u, 0u}, cur[4] = {0u, 0u, 0u, 0u};
      // A group's 16 outputs as the aligned block [B, B + 16) of the lane's row (B = x0 rounded down
      // to 16, x0 = 16 g - lane), kept in slot g mod 4 (static: the loop's four stages); when B is
      // 48 mod 64 the 64-byte segment [B - 48, B + 16) is complete and leaves as four 16-byte stores
      // back to back -- whole 64-byte pieces of lines, 16 lanes a group -- instead of one 16-byte
      // piece per row and group (c3ag: the L2 wrote the part-written lines back at 2.9x the bytes).
      // Every lane issues the four stores (lanes without a due, whole block store past the buffer:
      // dropped), so each stage has a fixed count of vector-memory operations for the counted vmcnt.
      // Blocks after a lane's last segment go out after the loop (flush); row ends byte by byte.
      uint32_t os[4][4];
      const int cl = (lane + 15) >> 4;  // B(g) = 16 (g - cl)
      auto block_whole = [&](int Bb) { return row_ok && Bb >= 0 && Bb + 16 <= W && st16; };
      auto block_bytes = [&](int Bb, const uint32_t* o) {  // (a block not stored whole: its bytes in the row)
        if (row_ok && Bb >= 0 && Bb < W && !block_whole(Bb)) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (Bb + i < W) prow[Bb + i] = (uint8_t)(o[i >> 2] >> (8 * (i & 3)));
        }
      };
      auto emit = [&](int sg, int k) {
        const int x0 = sg - lane, B = x0 - (x0 & 15);
        window16(prv[0], prv[1], prv[2], prv[3], cur[0], cur[1], cur[2], cur[3], sq, sr, os[k]);
        const bool due = (B & 63) == 48;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int Bi = B - 48 + 16 * i;
          const uint32_t* o = os[(k + 1 + i) & 3];
#ifdef WG_ABL_GRAD_NOSTORE  // (measurement only: output wrong)
          const uint32_t voff = 0x80000000u;
#else
          const uint32_t voff = due && block_whole(Bi) ? (uint32_t)(y * W + Bi) : 0x80000000u;
#endif
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{o[0], o[1], o[2], o[3]}, psrc, voff, 0, 0);
        }
        if (due) {
#pragma unroll
          for (int i = 0; i < 4; ++i) block_bytes(B - 48 + 16 * i, os[(k + 1 + i) & 3]);
        }
        stored = row_ok ? max(0, min(W, B + 16)) : W;
        // the last row's block into the ring, once the band below has read what it replaces
        const int Bl = sg - 63 - ((sg - 63) & 15);  // (lane 63's B)
        if (produce && Bl >= 0 && Bl < W) {
          const uint32_t need = Bl < kRing ? (((uint32_t)(bnd - 15) << 16) | 0xffffu)
                                           : (((uint32_t)(bnd + 1) << 16) | (uint32_t)(Bl - kRing + 16));
          // (the slot's previous reader, band b - 15, exists from b = 16 on: band 0 reads row0)
          if (bnd >= 16 || Bl >= kRing) spin(cprog + slot, need);
          if (lane == 63)
            *reinterpret_cast<u32x4*>(&tring[slot][Bl & (kRing - 1)]) = u32x4{os[k][0], os[k][1], os[k][2], os[k][3]};
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) prv[j] = cur[j];
      };
      // after the loop (gf = the last group emitted): slot j holds group g_j, the latest g <= gf with
      // g = j mod 4; its block went out with a segment iff a due group (g - cl = 3 mod 4) lies in
      // [g_j, g_j + 3] at or before gf -- else it goes out now
      auto flush = [&](int gf) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int gj = gf - ((gf - j) & 3);
          const int tj = gj + ((cl + 3 - gj) & 3);
          if (gj >= 0 && tj > gf) {
            const int Bj = 16 * (gj - cl);
            if (block_whole(Bj))
              __builtin_amdgcn_raw_buffer_store_b128(u32x4{os[j][0], os[j][1], os[j][2], os[j][3]}, psrc,
                                                     (uint32_t)(y * W + Bj), 0, 0);
            block_bytes(Bj, os[j]);
          }
        }
      };
      // lane 0's T for group sg (lanes j < 16: column sg + j of the row above; past the row's end
      // a clamped column, unused), once the band above has it in its ring
      auto read_t = [&](int sg) -> uint32_t {
        const int c = min(sg + (lane & 15), W - 1);
        if (bnd == 0) return row0[c];
        if (sg < W) spin(gprog + aslot, ((uint32_t)(bnd - 1) << 16) | (uint32_t)min(W, sg + 16));
        const uint32_t t = tring[aslot][c & (kRing - 1)];
        // (the read stays before the report in program order -- LDS serves a wave's accesses in
        // order, so the producer's overwrite, issued after it sees the report, comes after it)
        asm volatile("" ::: "memory");
        if (lane == 0) __hip_atomic_store(cprog + aslot, ((uint32_t)bnd << 16) | (uint32_t)min(W, sg + 16),
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return t;
      };
      auto run_group = [&](int sg, const u32x4& q, uint32_t t0) {
        uint32_t b[4];
        {
          window16(prevw.x, prevw.y, prevw.z, prevw.w, q.x, q.y, q.z, q.w, lq, lr, b);
          prevw = q;
        }
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
          cur[k >> 2] = (k & 3) == 0 ? o : cur[k >> 2] | (o << (8 * (k & 3)));
          L = ok ? o : L;
          TL = T;
        }
      };
      auto publish = [&] {  // (release: the ring and the row's plane stores before the counter)
        const uint32_t done = (uint32_t)__builtin_amdgcn_readlane(stored, rows - 1);
        if (lane == 0)
          __hip_atomic_store(gprog + slot, ((uint32_t)bnd << 16) | done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      };
      const int steps = W + rows - 1;
      load_group(0, 0);
      load_group(16, 1);
      load_group(32, 2);
      int last = 0;  // the last group's first step
      // stage: issue group sg + 48's block, read T, wait for group sg's block, the 16 steps, the
      // stores.  Issued after group sg's block: its stage's four stores, then a block and four stores
      // per stage since, and this stage's block -- vmcnt(15) (the first three stages: 3, fewer
      // stores behind them) leaves exactly those in flight.  (Byte stores at row ends only add
      // younger operations: the wait then covers a few more, never fewer.)  The stage past the last
      // group emits the row's tail only (its last group's bytes) and ends the loop.
      auto stage = [&](int sg, int k) -> bool {
        const bool work = sg < steps;
        if (work) {
          load_group(sg + 48, (k + 3) & 3);
          const uint32_t t = read_t(sg);
          if (sg < 48)
            asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
          else
            asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
          const u32x4 q = *reinterpret_cast<const u32x4*>(&dma[wave][k][4 * lane]);
          run_group(sg, q, t);
        }
        emit(sg, k);
        if (work) publish();
        last = sg;
        return !work;
      };
      for (int sg = 0;; sg += 64) {
        if (stage(sg, 0)) break;
        if (stage(sg + 16, 1)) break;
        if (stage(sg + 32, 2)) break;
        if (stage(sg + 48, 3)) break;
      }
      flush(last >> 4);
      const uint32_t done = (uint32_t)__builtin_amdgcn_readlane(stored, rows - 1);
      if (lane == 0) {
        __hip_atomic_store(gprog + slot, ((uint32_t)bnd << 16) | done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (bnd > 0)  // (this band has read all of the band above's ring)
          __hip_atomic_store(cprog + aslot, ((uint32_t)bnd << 16) | 0xffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      // (the blocks loaded past the end land before their slots are reused)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
#ifdef WG_ABL_GRAD_SKIP
grad_done:
#endif
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
