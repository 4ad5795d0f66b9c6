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
// edge lanes load them.  Each chroma row's taps are built once (make_cols) and serve two
// pairs, as the far row of the first and the near row of the second.  Algorithmic traffic: W*H + 2*ceil(W/2)*ceil(H/2) bytes in,
// 4*W*H bytes out.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device_format.h"
#include "emit_px.h"

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

// VP8YuvToRgba (conversion.go:28-49, A = 0xff) of two pixels; yl holds y + 32000 per 16-bit
// half (luma_lanes), u and v one 8-bit sample each.  Returns the two RGBA dwords.
//
// y1g = MultHi(y, 19077) + 8708 -- G's constant, folded into R's and B's subtrahends -- costs
// no add: two wrapping v_pk_mad_u16 on the biased lane, (133 yl + 4864) mod 2^16 = 133 y + 1024
// (so t4 = ((133 y) >> 8) + 4) and 74 yl mod 2^16 = 74 y + 8704.  y1g + MultHi(v, 26149) and
// y1g + MultHi(u, 33050) stay below 2^16 (tests/test_oracle.py::test_packed_yuv_formulas).
//
// kAlpha (alpha-first frames): A from `a` instead of 0xff -- the B bytes and the two pixels' A bytes
// (`asel`: a's bytes 0, 1 or 2, 3) packed into one dword first, so the pixels stay one v_perm each.
template <bool kAlpha = false>
__device__ __forceinline__ uint2 yuv_to_rgba2(u16x2 yl, u16x2 u, u16x2 v, uint32_t a = 0, uint32_t asel = 0) {
  const u16x2 y1g = yl * splat(74) + ((yl * splat(133) + splat(4864)) >> 8);  // MultHi(y, 19077) + 8708
  const uint32_t r = sat_x4(sat_sub(y1g + v * splat(102) + ((v * splat(37)) >> 8), 14234 + 8708));  // + MultHi(v, 26149)
  const u16x2 gu = u * splat(25) + ((u * splat(19)) >> 8);                                 // MultHi(u, 6419)
  const u16x2 gv = v * splat(52) + (v >> 5);                                               // MultHi(v, 13320)
  const uint32_t g = sat_x4(sat_sub(sat_sub(y1g, gu), gv));
  const uint32_t b = sat_x4(sat_sub(y1g + u * splat(129) + ((u * splat(26)) >> 8), 17685 + 8708));  // + MultHi(u, 33050)
  // the channel values are the high bytes of the 16-bit lanes: t = R0 G0 R1 G1; px = R G B 0xff
  // (perm selector 0x0d = 0xff)
  const uint32_t t = __builtin_amdgcn_perm(g, r, 0x07030501u);
  if constexpr (kAlpha) {
    const uint32_t ba = __builtin_amdgcn_perm(a, b, asel);  // B0 A0 B1 A1
    return make_uint2(__builtin_amdgcn_perm(ba, t, 0x05040100u), __builtin_amdgcn_perm(ba, t, 0x07060302u));
  }
  return make_uint2(__builtin_amdgcn_perm(b, t, 0x0d050100u), __builtin_amdgcn_perm(b, t, 0x0d070302u));
}
// yuv_to_rgba2's asel for pixels 0, 1 and 2, 3 of a group's alpha dword
constexpr uint32_t kASel01 = 0x05030401u, kASel23 = 0x07030601u;

// bytes i and j of w as the two 16-bit halves
__device__ __forceinline__ u16x2 bytes2(uint32_t w, int i, int j) {
  return as_u16x2(__builtin_amdgcn_perm(0u, w, 0x0c000c00u | (uint32_t)i | ((uint32_t)j << 16)));
}

// luma bytes i and j of w as yuv_to_rgba2's lanes y + 32000: the high byte 0x7d comes from
// v_perm's other source (selector 4 = its byte 0), so the bias costs nothing
__device__ __forceinline__ u16x2 luma_lanes(uint32_t w, int i, int j) {
  return as_u16x2(__builtin_amdgcn_perm(0x7d7d7d7du, w, 0x04000400u | (uint32_t)i | ((uint32_t)j << 16)));
}

__device__ __forceinline__ uint32_t bperm(uint32_t v, int src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}

// One chroma row as loaded by a lane: per group k the packed dword
// U[cb] | U[cb+1] << 8 | V[cb] << 16 | V[cb+1] << 24 (cb = group's first chroma column,
// cb+1 already replicated at the right edge), plus the wave-edge bytes: lane 0 holds
// the column left of its group 0 as U << 8 | V << 24 (the bytes a left neighbour's dword
// has them in), lane 63 the column right of its group 3 as U | V << 16.
struct ChromaRaw {
  uint32_t p[kGroups];
  uint32_t edge;
};

// One chroma row's taps per group k, the four columns cb-1 .. cb+2 (edge-replicated) of U and
// V as 16-bit pairs (cb-1, cb+1) and (cb, cb+2): plain, for the row's turn as the NEAR row,
// and plus 2, for its turn as the FAR row (upsample4's rounding term).  A row is built once,
// when it is the current row, and carried into the next pair as the previous row.
struct ChromaCols {
  u16x2 u02[kGroups], u13[kGroups], v02[kGroups], v13[kGroups];
  u16x2 u02f[kGroups], u13f[kGroups], v02f[kGroups], v13f[kGroups];
};

// A plane as a buffer resource (readfirstlane'd base: the planes are per frame, uniform, but
// where the compiler cannot prove it a VGPR descriptor would wrap every access in a
// readfirstlane waterfall loop).  Loads past num_records read 0: rows outside the frame are
// loaded at kOffDrop instead of being branched around, and no load needs 64-bit addresses.
constexpr uint32_t kOffDrop = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const void* base, int bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// Chroma row `row` (row_ok false: zeros) for the lane's groups: one 16-bit load per plane and
// group at voffset cb0 + row * uvs + 128 k.  Columns at or past uv_w hold other bytes (never
// used: make_cols replicates the edge, and pixels past the width are not stored), except the
// replicated U[cb+1] of an odd width's last group.
__device__ __forceinline__ ChromaRaw load_chroma(__amdgpu_buffer_rsrc_t ud, __amdgpu_buffer_rsrc_t vd,
                                                 gptr<const uint8_t> U, gptr<const uint8_t> V, int row, int uvs,
                                                 int cb0, int uv_w, int lane, bool row_ok) {
  ChromaRaw r;
  const uint32_t off = row_ok ? (uint32_t)(cb0 + row * uvs) : kOffDrop;
#pragma unroll
  for (int k = 0; k < kGroups; ++k) {
    const int cb = cb0 + 128 * k;
    uint32_t u = __builtin_amdgcn_raw_buffer_load_b16(ud, off + 128 * k, 0, 0);
    uint32_t v = __builtin_amdgcn_raw_buffer_load_b16(vd, off + 128 * k, 0, 0);
    if (cb + 1 == uv_w) {  // odd width: column cb+1 replicates cb
      u = (u & 0xff) * 0x101u;
      v = (v & 0xff) * 0x101u;
    }
    r.p[k] = u | (v << 16);
  }
  r.edge = 0;
  if (row_ok) {
    const int ce = lane == 0 ? cb0 - 1 : cb0 + 128 * (kGroups - 1) + 2;
    if ((lane == 0 && ce >= 0) || (lane == 63 && ce < uv_w)) {
      const size_t o = (size_t)row * uvs + ce;
      r.edge = (U[o] | ((uint32_t)V[o] << 16)) << (lane == 0 ? 8 : 0);
    }
  }
  return r;
}

// The taps straight from the packed dwords by v_perm: s = this group's dword, L = the left
// neighbour's (U[cb-1] in byte 1, V[cb-1] in byte 3), R = the right neighbour's (U[cb+2] in
// byte 0, V[cb+2] in byte 2) -- neighbour lanes through ds_bpermute, lane 63 / lane 0
// forwarding the adjacent group's dword so the rotation across the wave boundary lands on
// the right column; the frame's edges replicate s's own columns.
__device__ __forceinline__ ChromaCols make_cols(const ChromaRaw& r, int cb0, int uv_w, int lane) {
  ChromaCols c;
  const int from_l = (lane + 63) & 63, from_r = (lane + 1) & 63;
#pragma unroll
  for (int k = 0; k < kGroups; ++k) {
    const int cb = cb0 + 128 * k;
    const uint32_t s = r.p[k];
    uint32_t L = bperm(lane == 63 && k > 0 ? r.p[k - 1] : s, from_l);
    uint32_t R = bperm(lane == 0 && k + 1 < kGroups ? r.p[k + 1] : s, from_r);
    if (k == 0 && lane == 0) L = cb0 == 0 ? s << 8 : r.edge;  // (cb == 0: U[cb-1] := U[cb])
    if (k == kGroups - 1 && lane == 63) R = r.edge;
    if (cb + 2 >= uv_w) R = s >> 8;  // U[cb+2] := U[cb+1]
    c.u02[k] = as_u16x2(__builtin_amdgcn_perm(s, L, 0x0c050c01u));  // U[cb-1], U[cb+1]
    c.u13[k] = as_u16x2(__builtin_amdgcn_perm(R, s, 0x0c040c00u));  // U[cb],   U[cb+2]
    c.v02[k] = as_u16x2(__builtin_amdgcn_perm(s, L, 0x0c070c03u));  // V[cb-1], V[cb+1]
    c.v13[k] = as_u16x2(__builtin_amdgcn_perm(R, s, 0x0c060c02u));  // V[cb],   V[cb+2]
    c.u02f[k] = c.u02[k] + splat(2);
    c.u13f[k] = c.u13[k] + splat(2);
    c.v02f[k] = c.v02[k] + splat(2);
    c.v13f[k] = c.v13[k] + splat(2);
  }
  return c;
}

// 4 pixels of one plane from the near row's taps (n02, n13) and the far row's plus 2 (f02, f13):
// the vertical blend a[j] = 3*n[j] + f[j] + 2 as two packed pairs (a0, a2), (a1, a3); pixel 2c
// takes (3*a[near] + a[far]) >> 4 with far = c-1, pixel 2c+1 far = c+1 -- the 2s make its
// rounding 8.
// (The horizontal taps as one v_pk_mad_u16 each, the broadcast half by op_sel: written as vector
// code the compiler splits them into a multiply and an add.)
__device__ __forceinline__ void upsample4(u16x2 n02, u16x2 n13, u16x2 f02, u16x2 f13, u16x2& p01, u16x2& p23) {
  const u16x2 a02 = n02 * splat(3) + f02;
  const u16x2 a13 = n13 * splat(3) + f13;
  uint32_t h01, h23;
  asm("v_pk_mad_u16 %0, %1, 3, %2 op_sel_hi:[0,0,1]" : "=v"(h01) : "v"(as_u32(a13)), "v"(as_u32(a02)));  // a1 * 3 + (a0, a2)
  asm("v_pk_mad_u16 %0, %1, 3, %2 op_sel:[1,0,0] op_sel_hi:[1,0,1]" : "=v"(h23) : "v"(as_u32(a02)), "v"(as_u32(a13)));  // a2 * 3 + (a1, a3)
  p01 = as_u16x2(h01) >> 4;  // (3a1 + a0 + 8, 3a1 + a2 + 8) >> 4
  p23 = as_u16x2(h23) >> 4;  // (3a2 + a1 + 8, 3a2 + a3 + 8) >> 4
}

// group k of a row: n = the near row's taps, f = the far row's; kAlpha: A from the dword aw
template <bool kAlpha = false>
__device__ __forceinline__ u32x4 convert_group(const ChromaCols& n, const ChromaCols& f, int k, uint32_t yw,
                                               uint32_t aw = 0) {
  u16x2 u01, u23, v01, v23;
  upsample4(n.u02[k], n.u13[k], f.u02f[k], f.u13f[k], u01, u23);
  upsample4(n.v02[k], n.v13[k], f.v02f[k], f.v13f[k], v01, v23);
  const uint2 a = yuv_to_rgba2<kAlpha>(luma_lanes(yw, 0, 1), u01, v01, aw, kASel01),
              b = yuv_to_rgba2<kAlpha>(luma_lanes(yw, 2, 3), u23, v23, aw, kASel23);
  return u32x4{a.x, a.y, b.x, b.y};
}

// RGBA stores go through a buffer descriptor over the frame's RGBA (32-bit offsets: no 64-bit
// address arithmetic per store).  kAux = cache policy of the full 16-byte stores (buffer aux
// bits): K2 streams them non-temporally (2 = nt; sc1 measured 2.43 vs 2.36 ms on c3), K1's
// tail writes them through (16 = sc1: the lines leave the L2 at once instead of competing
// with the reconstruction's working set; c3 K1 7.71 vs 7.77 ms, same call).
constexpr int kAuxNt = 2, kAuxSc1 = 16;
template <int kAux>
__device__ __forceinline__ void store_group(__amdgpu_buffer_rsrc_t o, uint32_t off, u32x4 px, int nvalid, bool full) {
  if (full) {  // (wave-uniform: every lane's group is whole and the rows 16-byte aligned)
    __builtin_amdgcn_raw_buffer_store_b128(px, o, off, 0, kAux);
  } else {  // dword stores, those past the width dropped through the buffer range
    // (nvalid made opaque here: the lane masks of the four compares would otherwise be hoisted out
    // of the pair loop for every group, 32 SGPRs live across it, and spilled)
    asm volatile("" : "+v"(nvalid));
    __builtin_amdgcn_raw_buffer_store_b32(px.x, o, nvalid > 0 ? off : kOffDrop, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(px.y, o, nvalid > 1 ? off + 4 : kOffDrop, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(px.z, o, nvalid > 2 ? off + 8 : kOffDrop, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(px.w, o, nvalid > 3 ? off + 12 : kOffDrop, 0, 0);
  }
}

// Direct emission (FrameDesc::emit = 1 + WEBP_CSP_MODE, emit_flip): a lossy frame without alpha
// leaves the strips in its output colorspace, so no RGBA copy is written and read back (K6).  The
// group's four pixels in the mode (emit_px.h), bpp bytes each, at byte offset roff + bpp * x: one
// 16 / 12 / 8-byte store for a whole group, per-pixel stores (dropped past the width through the
// buffer range) otherwise.  The frames emitted directly are opaque (a = 255), where each
// premultiplied mode equals its plain form (emit_px: no premultiply at a = 255; the 4444 one is
// the identity at a = 0xf).  Only the conversion is switched on the mode: the store code is shared.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
template <int M>
__device__ __forceinline__ u32x4 conv4(u32x4 p) {
  return u32x4{emit_px<M>(p.x), emit_px<M>(p.y), emit_px<M>(p.z), emit_px<M>(p.w)};
}

// em = FrameDesc::emit (wave-uniform): 0 RGBA, else 1 + the mode.  kModes: kModesRgba = RGBA only,
// unflipped (K2 over batches without direct emission: no per-store mode or flip test in the stage
// the metric names),
// kModesTail = RGBA, rgbA and RGB_565 (K1's tail, whose code size is kept down: the switch sits at
// each of its eight unrolled store sites; capi.cpp sends batches in the other modes through K2),
// kModesAll = every mode (K2).
constexpr int kModesRgba = 0, kModesTail = 1, kModesAll = 2;
template <int kAux, int kModes>
__device__ __forceinline__ void store_out(__amdgpu_buffer_rsrc_t o, int em, uint32_t roff, int x, u32x4 px, int nvalid,
                                          bool full) {
  if (kModes == kModesRgba) {
    store_group<kAux>(o, roff + 4u * (uint32_t)x, px, nvalid, full);
    return;
  }
  int bpp = 4;
  u32x4 c = px;
  if (kModes == kModesAll) {
    switch (em) {
      case 1: c = conv4<0>(px), bpp = 3; break;            // RGB
      case 3: c = conv4<2>(px), bpp = 3; break;            // BGR
      case 4: case 9: c = conv4<3>(px); break;             // BGRA, bgrA
      case 5: case 10: c = conv4<4>(px); break;            // ARGB, Argb
      case 6: case 11: c = conv4<5>(px), bpp = 2; break;   // RGBA_4444, rgbA_4444
      case 7: c = conv4<6>(px), bpp = 2; break;            // RGB_565
      default: break;                                      // RGBA, rgbA
    }
  } else if (em == 7) {
    c = conv4<6>(px), bpp = 2;
  }
  if (bpp == 4) {
    store_group<kAux>(o, roff + 4u * (uint32_t)x, c, nvalid, full);
    return;
  }
  const uint32_t off = roff + (uint32_t)(bpp * x);
  asm volatile("" : "+v"(nvalid));  // (as in store_group: no hoisted per-group lane masks)
  if (full) {
    if (bpp == 2) __builtin_amdgcn_raw_buffer_store_b64(u32x2{c.x | c.y << 16, c.z | c.w << 16}, o, off, 0, kAux);
    else __builtin_amdgcn_raw_buffer_store_b96(u32x3{c.x | c.y << 24, c.y >> 8 | c.z << 16, c.z >> 16 | c.w << 8}, o, off, 0, kAux);
    return;
  }
  const uint32_t ov[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t a = nvalid > k ? off + (uint32_t)(bpp * k) : kOffDrop;
    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)ov[k], o, a, 0, 0);
    if (bpp == 3) __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(ov[k] >> 16), o, nvalid > k ? a + 2 : kOffDrop, 0, 0);
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

// kAlpha: an alpha-first frame (FrameDesc::alpha_off16 != 0, RGBA): A from its alpha plane.  A
// separate instantiation, chosen per frame by the callers, so the strips of frames without alpha
// keep their code (and K1's tail its I-cache footprint).
template <bool kFancy, int kAux, int kModes, bool kAlpha = false>
__device__ __forceinline__ void convert_strip(const FrameDesc& F, int tx, int band, int lane) {
  const int W = F.width, H = F.height;
  const int uv_w = (W + 1) >> 1, uv_h = (H + 1) >> 1;
  const int xl = tx * kStripPx + 4 * lane;  // group k pixel x = xl + 256k
  const int cb0 = xl >> 1;
  // output: RGBA, or (emit) the frame's mode, rows bottom-up with emit_flip
  int em = __builtin_amdgcn_readfirstlane(F.emit);
  const bool flip = kModes != kModesRgba && __builtin_amdgcn_readfirstlane(F.emit_flip) != 0;  // (K2's RGBA-only kernel: never)
  const int bpp = em ? bpp_of(em - 1) : 4;
  const bool aligned = ((F.rgba_stride & (bpp == 4 ? 15 : 3)) == 0) && ((reinterpret_cast<uintptr_t>(F.rgba) & 15) == 0);
  // per group k, from the wave's first pixel x0 (scalar): some lane's group lies in the frame
  // (else skipped), every lane's group is whole (one 16-byte store each)
  const int x0 = tx * kStripPx;
  // groups of the strip in the frame / whole (one 16-byte store each), as two scalar counts compared
  // per group: eight uniform booleans would be eight 64-bit lane masks held across the pair loop
  // (K1's tail spilled them).  refresh() makes the counts opaque at the top of each pair, so the
  // compares are not hoisted back out of it.
  // (wave-uniform: one frame per wave strip; readfirstlane where the compiler cannot prove it)
  int n_live = __builtin_amdgcn_readfirstlane((W - x0 + 255) >> 8);
  int n_full = __builtin_amdgcn_readfirstlane(aligned ? (W - x0) >> 8 : 0);
  auto refresh = [&] { asm volatile("" : "+s"(n_live), "+s"(n_full)); };
  auto live = [&](int k) { return k < n_live; };
  auto full = [&](int k) { return k < n_full; };
  const gptr<const uint8_t> U = as_global(static_cast<const uint8_t*>(F.u));
  const gptr<const uint8_t> V = as_global(static_cast<const uint8_t*>(F.v));
  const int ys = F.y_stride, uvs = F.uv_stride, os = F.rgba_stride;
  auto roff = [&](int y) { return (uint32_t)((flip ? H - 1 - y : y) * os); };
  // (the descriptor from readfirstlane'd values: F is one frame per workgroup, but where the
  // compiler cannot prove it uniform (K2 picks `single` or frames[y]) a VGPR descriptor
  // would wrap every store in a readfirstlane waterfall loop)
  const uint64_t ob = reinterpret_cast<uint64_t>(F.rgba);
  const uint32_t ob_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(ob >> 32));
  const uint32_t ob_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)ob);  // (unsigned: no sign extension)
  uint8_t* const obase = reinterpret_cast<uint8_t*>(((uint64_t)ob_hi << 32) | ob_lo);
  const __amdgpu_buffer_rsrc_t out =
      __builtin_amdgcn_make_buffer_rsrc(obase, 0, __builtin_amdgcn_readfirstlane(os * H), 0x00020000);

  const __amdgpu_buffer_rsrc_t yd = plane_rsrc(F.y, ys * H), ud = plane_rsrc(F.u, uvs * uv_h),
                               vd = plane_rsrc(F.v, uvs * uv_h);
  // (a group's bytes past the width are loaded but never stored)
  auto load_luma = [&](int row, uint32_t yw[kGroups]) {
    const uint32_t off = row >= 0 && row < H ? (uint32_t)(xl + row * ys) : kOffDrop;
#pragma unroll
    for (int k = 0; k < kGroups; ++k) yw[k] = __builtin_amdgcn_raw_buffer_load_b32(yd, off + 256 * k, 0, 0);
  };
  // kAlpha: the alpha plane's dwords of a row (W-byte rows).  The range check drops a whole dword
  // that crosses the end, so the range runs 3 bytes past the plane (inside its 256-byte-aligned
  // allocation): the last row's last group keeps its valid bytes.
  constexpr bool ha = kAlpha;
  const __amdgpu_buffer_rsrc_t ad = plane_rsrc(F.y + 16 * (ptrdiff_t)(kAlpha ? F.alpha_off16 : 0), W * H + 3);
  auto load_alpha = [&](int row, uint32_t aw[kGroups]) {
    const uint32_t off = row >= 0 && row < H ? (uint32_t)(xl + row * W) : kOffDrop;
#pragma unroll
    for (int k = 0; k < kGroups; ++k) aw[k] = __builtin_amdgcn_raw_buffer_load_b32(ad, off + 256 * k, 0, 0);
  };

  if (kFancy) {
    const int npairs = (H >> 1) + 1;  // pair p: output rows 2p-1, 2p
    const int p0 = band * kPairs;
    if (p0 >= npairs) return;
    const int p1 = min(p0 + kPairs, npairs);
    const int rp = max(p0 - 1, 0), rc = min(p0, uv_h - 1);
    const ChromaRaw raw_prev = load_chroma(ud, vd, U, V, rp, uvs, cb0, uv_w, lane, true);
    ChromaRaw raw_cur = load_chroma(ud, vd, U, V, rc, uvs, cb0, uv_w, lane, true);
    ChromaCols ca = make_cols(raw_prev, cb0, uv_w, lane);
    // one pair: rows 2p-1 (near = chroma row p-1, far = row p) and 2p (near = row p, far = row
    // p-1); returns row p's taps for the next pair.  (Unrolled by two, so the carried taps would
    // alternate between register sets instead of being copied, the loop measured no faster and
    // its code grew K1 by 8 KB: not kept.)
    auto pair_step = [&](int p, const ChromaCols& prv) __attribute__((always_inline)) {
      const int ya = 2 * p - 1, yb = 2 * p;
      asm volatile("" : "+s"(em));  // (no loop copy per output mode: only the conversion switches)
      refresh();
      uint32_t yA[kGroups], yB[kGroups], aA[kGroups] = {}, aB[kGroups] = {};
      load_luma(ya, yA);
      load_luma(yb, yB);
      if (ha) {
        load_alpha(ya, aA);
        load_alpha(yb, aB);
      }
      const int rn = min(p + 1, uv_h - 1);  // chroma row for the next pair
      const ChromaRaw raw_next = load_chroma(ud, vd, U, V, rn, uvs, cb0, uv_w, lane, p + 1 < p1);
      const ChromaCols cur = make_cols(raw_cur, cb0, uv_w, lane);
#pragma unroll
      for (int k = 0; k < kGroups; ++k) {
        const int x = xl + 256 * k;
        if (!live(k)) continue;
        if (ya >= 0) store_out<kAux, kModes>(out, em, roff(ya), x, convert_group<ha>(prv, cur, k, yA[k], aA[k]), W - x, full(k));
        if (yb < H) store_out<kAux, kModes>(out, em, roff(yb), x, convert_group<ha>(cur, prv, k, yB[k], aB[k]), W - x, full(k));
      }
      raw_cur = raw_next;
      // K1's tail yields the SIMD for a moment after each pair: its denser packed code otherwise
      // takes issue slots from the reconstructing waves, the frame's critical path (same-call
      // A/B, no sleep / sleep 4 / 16: c3 7.59 / 7.58 / 7.62 ms, c3s 8.24 / 8.22 / 8.19 ms)
      if (kAux == kAuxSc1) __builtin_amdgcn_s_sleep(4);
      return cur;
    };
    for (int p = p0; p < p1; ++p) ca = pair_step(p, ca);
  } else {
    // point sampling: rows 2p and 2p+1 both use chroma row p (WebPSamplerProcessPlane)
    const int npairs = (H + 1) >> 1;
    const int p0 = band * kPairs;
    if (p0 >= npairs) return;
    const int p1 = min(p0 + kPairs, npairs);
    for (int p = p0; p < p1; ++p) {
      asm volatile("" : "+s"(em));
      refresh();
      uint32_t yA[kGroups], yB[kGroups], aA[kGroups] = {}, aB[kGroups] = {};
      load_luma(2 * p, yA);
      load_luma(2 * p + 1, yB);
      if (ha) {
        load_alpha(2 * p, aA);
        load_alpha(2 * p + 1, aB);
      }
      const ChromaRaw c = load_chroma(ud, vd, U, V, p, uvs, cb0, uv_w, lane, true);
#pragma unroll
      for (int k = 0; k < kGroups; ++k) {
        const int x = xl + 256 * k;
        if (!live(k)) continue;
        // pixels 0,1 take chroma column cb, pixels 2,3 column cb+1
        const uint32_t cp = c.p[k];
        const u16x2 u0 = bytes2(cp, 0, 0), u1 = bytes2(cp, 1, 1), v0 = bytes2(cp, 2, 2), v1 = bytes2(cp, 3, 3);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const int yr = 2 * p + r;
          if (yr >= H) break;
          const uint32_t yw = r ? yB[k] : yA[k];
          const uint32_t aw = r ? aB[k] : aA[k];
          const uint2 a = yuv_to_rgba2<ha>(luma_lanes(yw, 0, 1), u0, v0, aw, kASel01),
                      b = yuv_to_rgba2<ha>(luma_lanes(yw, 2, 3), u1, v1, aw, kASel23);
          const u32x4 px{a.x, a.y, b.x, b.y};
          store_out<kAux, kModes>(out, em, roff(yr), x, px, W - x, full(k));
        }
      }
    }
  }
}

}  // namespace strip
}  // namespace wg
