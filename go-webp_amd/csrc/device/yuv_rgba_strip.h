// YUV420 -> RGBA of one wave strip (1024 px wide, kPairs row pairs): the conversion shared by
// K2 (yuv_to_rgba.hip, one wave per strip) and K1's tail (vp8_recon_filter.hip, waves whose
// reconstruction work is done convert finished bands of their own frame).
//
// Replaces the reference's output emitters:
//   EmitFancyRGB           pkg/libwebp/decoder/io_dec.c.go:65-115
//   UpsampleRgbaLinePair_C pkg/libwebp/dsp/upsampling.c.go:43-107
//   EmitSampledRGB         pkg/libwebp/decoder/io_dec.c.go:53-59, dsp/yuv.go:19-58
//   VP8YuvToRgba           R,G,B = YUVToR/G/B (pkg/color/yuv/conversion.go:28-49), A=0xff
//
// The line-pair upsampler with its packed-u/v "diagonal" trick is exactly the separable
// 9-3-3-1 filter (9a + 3b + 3c + d + 8) >> 4 with edge replication
// (tests/test_oracle.py::test_upsampler_closed_form): for output pixel (x, y) the near
// chroma sample is (y>>1, x>>1), the far row/column is near -/+ 1 toward the pixel,
// clamped to the plane.  Written separably: v = 3*near_row + far_row per chroma column,
// then pixel = (3*v[near_col] + v[far_col] + 8) >> 4.
//
// Work split: output rows 2p-1 and 2p ("pair p") both read chroma rows p-1 and p.  A wave
// covers a 1024-pixel-wide strip and walks kPairs pairs down it, carrying chroma row p
// into pair p+1 (each chroma row is loaded once per strip).  Lane l owns the four
// 4-pixel groups x = x0 + 256k + 4l (k = 0..3), so every load and every 16-byte RGBA
// store instruction of the wave touches one contiguous run (256 B of luma, 128 B per
// chroma plane, 1 KB of RGBA): full cache lines, no partial-line write amplification.
// A group needs chroma columns cb-1 .. cb+2 (cb = x/2); the outer two come from the
// neighbouring lanes as one packed U/V dword through ds_bpermute, and only the wave's
// edge lanes load them.  Algorithmic traffic: W*H + 2*ceil(W/2)*ceil(H/2) bytes in,
// 4*W*H bytes out.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device_format.h"

namespace wg {
namespace strip {

constexpr int kGroups = 4;                   // 4-pixel groups per lane per row
constexpr int kStripPx = 64 * 4 * kGroups;   // pixels per wave row (1024)
constexpr int kPairs = 16;                   // row pairs per wave strip (32 output rows)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Packed 16-bit arithmetic: two pixels per VALU instruction (v_pk_mad_u16, v_pk_sub_u16
// with clamp, v_pk_min_u16, v_pk_lshrrev_b16).  Every VP8YuvToRgba term fits 16 bits once
// MultHi(a, c) = (a*c) >> 8 is split at the multiplier's high byte, c = 256*h + l:
// MultHi(a, c) = h*a + ((l*a) >> 8) exactly (a <= 255, l*a < 2^16).  The signed
// `(sum - k) >> 6` followed by Clip8 is min(sat_sub(sum, k) >> 6, 255): a negative sum
// clips to 0 either way.  Exhaustively checked over all (y, u, v) against the reference
// formulas (tests/test_oracle.py::test_packed_yuv_formulas).
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t w) { return __builtin_bit_cast(u16x2, w); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ u16x2 splat(unsigned short c) { return u16x2{c, c}; }
__device__ __forceinline__ u16x2 sat_sub(u16x2 a, unsigned short c) { return __builtin_elementwise_sub_sat(a, splat(c)); }
__device__ __forceinline__ u16x2 sat_sub(u16x2 a, u16x2 b) { return __builtin_elementwise_sub_sat(a, b); }

// (a * 4) saturated at 0xffff, two 16-bit lanes in one v_pk_mad_u16 with clamp: its HIGH byte is
// min(a >> 6, 255) -- the final `>> 6` + Clip8 in one instruction instead of a shift and a min
// (tests/test_oracle.py::test_packed_yuv_formulas; on the device over all 2^24 (y, u, v):
// tests/test_gpu_parity.py::test_yuv_to_rgba_device_every_yuv_triple).
__device__ __forceinline__ uint32_t sat_x4(u16x2 a) {
  uint32_t r;
  asm("v_pk_mad_u16 %0, %1, %2, 0 clamp" : "=v"(r) : "v"(as_u32(a)), "s"(0x00040004u));
  return r;
}

// VP8YuvToRgba (conversion.go:28-49, A = 0xff) of two pixels; y, u, v hold one 8-bit
// sample per 16-bit half.  Returns the two RGBA dwords.
__device__ __forceinline__ uint2 yuv_to_rgba2(u16x2 y, u16x2 u, u16x2 v) {
  const u16x2 y1 = y * splat(74) + ((y * splat(133)) >> 8);                            // MultHi(y, 19077)
  const uint32_t r = sat_x4(sat_sub(y1 + v * splat(102) + ((v * splat(37)) >> 8), 14234));  // + MultHi(v, 26149)
  const u16x2 gu = u * splat(25) + ((u * splat(19)) >> 8);                             // MultHi(u, 6419)
  const u16x2 gv = v * splat(52) + (v >> 5);                                           // MultHi(v, 13320)
  const uint32_t g = sat_x4(sat_sub(sat_sub(y1 + splat(8708), gu), gv));
  const uint32_t b = sat_x4(sat_sub(y1 + u * splat(129) + ((u * splat(26)) >> 8), 17685));  // + MultHi(u, 33050)
  // the channel values are the high bytes of the 16-bit lanes: t = R0 G0 R1 G1; px = R G B 0xff
  // (perm selector 0x0d = 0xff)
  const uint32_t t = __builtin_amdgcn_perm(g, r, 0x07030501u);
  return make_uint2(__builtin_amdgcn_perm(b, t, 0x0d050100u), __builtin_amdgcn_perm(b, t, 0x0d070302u));
}

// bytes i and j of w as the two 16-bit halves
__device__ __forceinline__ u16x2 bytes2(uint32_t w, int i, int j) {
  return as_u16x2(__builtin_amdgcn_perm(0u, w, 0x0c000c00u | (uint32_t)i | ((uint32_t)j << 16)));
}

__device__ __forceinline__ uint32_t bperm(uint32_t v, int src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}

// One chroma row as loaded by a lane: per group k the packed dword
// U[cb] | U[cb+1] << 8 | V[cb] << 16 | V[cb+1] << 24 (cb = group's first chroma column,
// cb+1 already replicated at the right edge), plus the wave-edge bytes: lane 0 holds
// the column left of its group 0, lane 63 the column right of its group 3 (same packing,
// U in byte 0, V in byte 2).
struct ChromaRaw {
  uint32_t p[kGroups];
  uint32_t edge;
};

// Per group, the 4 chroma columns cb-1 .. cb+2 with edge replication:
// u = U[cb-1] | U[cb] << 8 | U[cb+1] << 16 | U[cb+2] << 24, v likewise.
struct ChromaWin {
  uint32_t u[kGroups], v[kGroups];
};

__device__ __forceinline__ ChromaRaw load_chroma(gptr<const uint8_t> ur, gptr<const uint8_t> vr, int cb0, int uv_w,
                                                 int lane, bool row_ok) {
  ChromaRaw r;
#pragma unroll
  for (int k = 0; k < kGroups; ++k) {
    const int cb = cb0 + 128 * k;
    uint32_t u = 0, v = 0;
    if (row_ok && cb < uv_w) {
      u = *reinterpret_cast<gptr<const uint16_t>>(ur + cb);
      v = *reinterpret_cast<gptr<const uint16_t>>(vr + cb);
      if (cb + 1 >= uv_w) {  // odd width: column cb+1 replicates cb
        u = (u & 0xff) * 0x101u;
        v = (v & 0xff) * 0x101u;
      }
    }
    r.p[k] = u | (v << 16);
  }
  r.edge = 0;
  if (row_ok) {
    const int ce = lane == 0 ? cb0 - 1 : cb0 + 128 * (kGroups - 1) + 2;
    if ((lane == 0 && ce >= 0) || (lane == 63 && ce < uv_w)) r.edge = ur[ce] | ((uint32_t)vr[ce] << 16);
  }
  return r;
}

__device__ __forceinline__ ChromaWin make_win(const ChromaRaw& r, int cb0, int uv_w, int lane) {
  ChromaWin w;
  const int from_l = (lane + 63) & 63, from_r = (lane + 1) & 63;
#pragma unroll
  for (int k = 0; k < kGroups; ++k) {
    const int cb = cb0 + 128 * k;
    // neighbour lanes' packed dwords; lane 63 / lane 0 forward the adjacent group's so the
    // rotation across the wave boundary lands on the right column.
    uint32_t lp = bperm(lane == 63 && k > 0 ? r.p[k - 1] : r.p[k], from_l) >> 8;  // U[cb-1] b0, V[cb-1] b2
    uint32_t rp = bperm(lane == 0 && k + 1 < kGroups ? r.p[k + 1] : r.p[k], from_r);  // U[cb+2] b0, V b2
    if (lane == 0 && k == 0) lp = r.edge;
    if (lane == 63 && k == kGroups - 1) rp = r.edge;
    const uint32_t s = r.p[k];
    uint32_t ul = lp & 0xff, vl = (lp >> 16) & 0xff;
    uint32_t ur = rp & 0xff, vr = (rp >> 16) & 0xff;
    if (cb == 0) {
      ul = s & 0xff;
      vl = (s >> 16) & 0xff;
    }
    if (cb + 2 >= uv_w) {
      ur = (s >> 8) & 0xff;
      vr = s >> 24;
    }
    w.u[k] = ul | ((s & 0xffff) << 8) | (ur << 24);
    w.v[k] = vl | ((s >> 16) << 8) | (vr << 24);
  }
  return w;
}

// 4 pixels of group k: near/far chroma windows (n, f), luma dword.  Per chroma plane the
// vertical blend a[j] = 3*n[j] + f[j] is computed as two packed pairs (a0, a2), (a1, a3);
// pixel 2c takes (3*a[near] + a[far] + 8) >> 4 with far = c-1, pixel 2c+1 far = c+1.
__device__ __forceinline__ void upsample4(uint32_t n, uint32_t f, u16x2& p01, u16x2& p23) {
  const u16x2 a02 = as_u16x2(n & 0x00ff00ffu) * splat(3) + as_u16x2(f & 0x00ff00ffu);
  const u16x2 a13 = bytes2(n, 1, 3) * splat(3) + bytes2(f, 1, 3);
  p01 = (a13.xx * splat(3) + (a02 + splat(8))) >> 4;  // (3a1 + a0 + 8, 3a1 + a2 + 8) >> 4
  p23 = (a02.yy * splat(3) + (a13 + splat(8))) >> 4;  // (3a2 + a1 + 8, 3a2 + a3 + 8) >> 4
}

__device__ __forceinline__ u32x4 convert_group(uint32_t nu, uint32_t fu, uint32_t nv, uint32_t fv, uint32_t yw) {
  u16x2 u01, u23, v01, v23;
  upsample4(nu, fu, u01, u23);
  upsample4(nv, fv, v01, v23);
  const uint2 a = yuv_to_rgba2(bytes2(yw, 0, 1), u01, v01), b = yuv_to_rgba2(bytes2(yw, 2, 3), u23, v23);
  return u32x4{a.x, a.y, b.x, b.y};
}

// RGBA stores go through a buffer descriptor over the frame's RGBA (32-bit offsets: no 64-bit
// address arithmetic per store).  kAux = cache policy of the full 16-byte stores (buffer aux
// bits): K2 streams them non-temporally (2 = nt; sc1 measured 2.43 vs 2.36 ms on c3), K1's
// tail writes them through (16 = sc1: the lines leave the L2 at once instead of competing
// with the reconstruction's working set; c3 K1 7.71 vs 7.77 ms, same call).
constexpr int kAuxNt = 2, kAuxSc1 = 16;
template <int kAux>
__device__ __forceinline__ void store_group(__amdgpu_buffer_rsrc_t o, uint32_t off, u32x4 px, int nvalid, bool aligned) {
  if (aligned && nvalid >= 4) {
    __builtin_amdgcn_raw_buffer_store_b128(px, o, off, 0, kAux);
  } else {
    if (nvalid > 0) __builtin_amdgcn_raw_buffer_store_b32(px.x, o, off, 0, 0);
    if (nvalid > 1) __builtin_amdgcn_raw_buffer_store_b32(px.y, o, off + 4, 0, 0);
    if (nvalid > 2) __builtin_amdgcn_raw_buffer_store_b32(px.z, o, off + 8, 0, 0);
    if (nvalid > 3) __builtin_amdgcn_raw_buffer_store_b32(px.w, o, off + 12, 0, 0);
  }
}

// Strips and bands of a frame: strip tx covers x in [1024 tx, 1024 tx + 1024), band j the
// row pairs [kPairs j, kPairs j + kPairs) (fancy: pair p = output rows 2p-1, 2p; point:
// rows 2p, 2p+1).
__device__ __forceinline__ int strips_x(int W) { return (W + kStripPx - 1) / kStripPx; }
__device__ __forceinline__ int n_bands(int H, bool fancy) {
  const int npairs = fancy ? (H >> 1) + 1 : (H + 1) >> 1;
  return (npairs + kPairs - 1) / kPairs;
}

template <bool kFancy, int kAux>
__device__ __forceinline__ void convert_strip(const FrameDesc& F, int tx, int band, int lane) {
  const int W = F.width, H = F.height;
  const int uv_w = (W + 1) >> 1, uv_h = (H + 1) >> 1;
  const int xl = tx * kStripPx + 4 * lane;  // group k pixel x = xl + 256k
  const int cb0 = xl >> 1;
  const bool aligned = ((F.rgba_stride & 15) == 0) && ((reinterpret_cast<uintptr_t>(F.rgba) & 15) == 0);
  const gptr<const uint8_t> Y = as_global(static_cast<const uint8_t*>(F.y));
  const gptr<const uint8_t> U = as_global(static_cast<const uint8_t*>(F.u));
  const gptr<const uint8_t> V = as_global(static_cast<const uint8_t*>(F.v));
  const int ys = F.y_stride, uvs = F.uv_stride, os = F.rgba_stride;
  // (the descriptor from readfirstlane'd values: F is one frame per workgroup, but where the
  // compiler cannot prove it uniform (K2 picks `single` or frames[y]) a VGPR descriptor
  // would wrap every store in a readfirstlane waterfall loop)
  const uint64_t ob = reinterpret_cast<uint64_t>(F.rgba);
  const uint32_t ob_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(ob >> 32));
  const uint32_t ob_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)ob);  // (unsigned: no sign extension)
  uint8_t* const obase = reinterpret_cast<uint8_t*>(((uint64_t)ob_hi << 32) | ob_lo);
  const __amdgpu_buffer_rsrc_t out =
      __builtin_amdgcn_make_buffer_rsrc(obase, 0, __builtin_amdgcn_readfirstlane(os * H), 0x00020000);

  auto load_luma = [&](int row, uint32_t yw[kGroups]) {
#pragma unroll
    for (int k = 0; k < kGroups; ++k) {
      const int x = xl + 256 * k;
      yw[k] = (row >= 0 && row < H && x < W) ? *reinterpret_cast<gptr<const uint32_t>>(Y + (size_t)row * ys + x) : 0u;
    }
  };

  if (kFancy) {
    const int npairs = (H >> 1) + 1;  // pair p: output rows 2p-1, 2p
    const int p0 = band * kPairs;
    if (p0 >= npairs) return;
    const int p1 = min(p0 + kPairs, npairs);
    const int rp = max(p0 - 1, 0), rc = min(p0, uv_h - 1);
    const ChromaRaw raw_prev = load_chroma(U + (size_t)rp * uvs, V + (size_t)rp * uvs, cb0, uv_w, lane, true);
    ChromaRaw raw_cur = load_chroma(U + (size_t)rc * uvs, V + (size_t)rc * uvs, cb0, uv_w, lane, true);
    ChromaWin wp = make_win(raw_prev, cb0, uv_w, lane);
    for (int p = p0; p < p1; ++p) {
      const int ya = 2 * p - 1, yb = 2 * p;
      uint32_t yA[kGroups], yB[kGroups];
      load_luma(ya, yA);
      load_luma(yb, yB);
      const int rn = min(p + 1, uv_h - 1);  // chroma row for the next pair
      const ChromaRaw raw_next = load_chroma(U + (size_t)rn * uvs, V + (size_t)rn * uvs, cb0, uv_w, lane, p + 1 < p1);
      const ChromaWin wc = make_win(raw_cur, cb0, uv_w, lane);
#pragma unroll
      for (int k = 0; k < kGroups; ++k) {
        const int x = xl + 256 * k;
        const int nvalid = W - x;
        if (nvalid <= 0) continue;
        if (ya >= 0)  // near = chroma row p-1, far = row p
          store_group<kAux>(out, (uint32_t)(ya * os + 4 * x), convert_group(wp.u[k], wc.u[k], wp.v[k], wc.v[k], yA[k]), nvalid,
                      aligned);
        if (yb < H)  // near = chroma row p, far = row p-1
          store_group<kAux>(out, (uint32_t)(yb * os + 4 * x), convert_group(wc.u[k], wp.u[k], wc.v[k], wp.v[k], yB[k]), nvalid,
                      aligned);
      }
      wp = wc;
      raw_cur = raw_next;
    }
  } else {
    // point sampling: rows 2p and 2p+1 both use chroma row p (WebPSamplerProcessPlane)
    const int npairs = (H + 1) >> 1;
    const int p0 = band * kPairs;
    if (p0 >= npairs) return;
    const int p1 = min(p0 + kPairs, npairs);
    for (int p = p0; p < p1; ++p) {
      uint32_t yA[kGroups], yB[kGroups];
      load_luma(2 * p, yA);
      load_luma(2 * p + 1, yB);
      const ChromaRaw c = load_chroma(U + (size_t)p * uvs, V + (size_t)p * uvs, cb0, uv_w, lane, true);
#pragma unroll
      for (int k = 0; k < kGroups; ++k) {
        const int x = xl + 256 * k;
        const int nvalid = W - x;
        if (nvalid <= 0) continue;
        // pixels 0,1 take chroma column cb, pixels 2,3 column cb+1
        const uint32_t cp = c.p[k];
        const u16x2 u0 = bytes2(cp, 0, 0), u1 = bytes2(cp, 1, 1), v0 = bytes2(cp, 2, 2), v1 = bytes2(cp, 3, 3);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const int yr = 2 * p + r;
          if (yr >= H) break;
          const uint32_t yw = r ? yB[k] : yA[k];
          const uint2 a = yuv_to_rgba2(bytes2(yw, 0, 1), u0, v0), b = yuv_to_rgba2(bytes2(yw, 2, 3), u1, v1);
          const u32x4 px{a.x, a.y, b.x, b.y};
          store_group<kAux>(out, (uint32_t)(yr * os + 4 * x), px, nvalid, aligned);
        }
      }
    }
  }
}

}  // namespace strip
}  // namespace wg
