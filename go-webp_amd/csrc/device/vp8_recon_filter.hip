// K1: VP8 macroblock reconstruction + in-loop deblocking, fused, for gfx950.
//
// Replaces the reference's per-MB DSP loop:
//   ReconstructRow       pkg/libwebp/decoder/frame_dec.c.go:69-197
//   DoFilter / FilterRow pkg/libwebp/decoder/frame_dec.c.go:204-261
//   transforms           pkg/libwebp/dsp/dec.c.go:49-134 (+DoTransform :43-67)
//   intra predictors     pkg/libwebp/dsp/dec.c.go:178-474 (indexed by mode enum)
//   loop filters         pkg/libwebp/dsp/dec.c.go:484-682
//
// Geometry: one 1024-thread workgroup per frame; wave w owns MB rows w, w+16, ...
// (16 rows in flight).  Row y at column x waits (LDS progress counter) until row
// y-1 has finished column min(x+1, mb_w-1): the classic t = x + 2y wavefront, since
// both intra prediction (top-right samples) and the loop filter (MB (x+1,y-1)'s
// left-edge writes) reach one MB up and to the right.
//
// One macroblock = one wave: lane l owns pixel row (l & 3) of 4x4 block (l >> 2)
// (a dword of the 16x16 luma block).  The IDCT's vertical pass runs per column
// lane, a quad DPP transpose hands rows to lanes, the horizontal pass produces the
// lane's 4 residuals.  Residuals are prediction-independent (STORE: dst + (v>>3)),
// so all 16 blocks are transformed at once; i4x4 prediction then walks its
// 10-step intra wavefront (block t = bx + 2*by) in the LDS workspace.
//
// A non-zero 4x4 block always goes through TransformOne: libwebp's TransformAC3 /
// TransformDC / TransformDCUV are exact special cases of it on their coefficient
// patterns (tests/test_oracle.py::test_transform_shortcuts_exact), and TransformOne
// of an all-zero block is the identity.
//
// Cross-wave data lives only in LDS (top samples `ytop`, filtered bottom rows
// `fbot`, progress counters); every HBM byte of the Y/U/V planes is written exactly
// once, when it is final.  Prediction uses UNFILTERED neighbours (ytop and the
// recon workspace), the filter works in a separate per-wave window, exactly as
// libwebp keeps yuv_t/yuv_b apart from its filtered cache rows.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device_format.h"
#include "kernels.h"

namespace wg {
namespace {

constexpr int kWaves = 16;
constexpr int BPS = 32;  // libwebp workspace stride
constexpr int Y_OFF = BPS * 1 + 8;
constexpr int U_OFF = Y_OFF + BPS * 16 + BPS;
constexpr int V_OFF = U_OFF + 16;
constexpr int kWsBytes = 832;  // YUV_SIZE = BPS*17 + BPS*9
// filter window: luma rows/cols -4..15 (stride 20), chroma rows/cols -4..7 (stride 12)
constexpr int FWY = 20, FWC = 12;
constexpr int kFwY = 0, kFwU = 400, kFwV = 544;
constexpr int kFwBytes = 704;
constexpr int kLeftBytes = 32;  // contiguous unfiltered left columns: Y 16, U 8, V 8
constexpr int kWaveBytes = kWsBytes + kFwBytes + kLeftBytes;  // 1568
constexpr int kProgBytes = 64;
constexpr int kColBytes = 32 + 128;  // ytop (y16 u8 v8) + fbot (Y 4x16, U 4x8, V 4x8)

__device__ __forceinline__ void lds_sync() {
  // LDS ops of one wave complete in order; this makes every lane's earlier LDS
  // write visible to every lane's later LDS read and stops compiler reordering.
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

__device__ __forceinline__ int clamp255(int v) { return min(max(v, 0), 255); }
__device__ __forceinline__ int avg3(int a, int b, int c) { return (a + 2 * b + c + 2) >> 2; }
__device__ __forceinline__ int avg2(int a, int b) { return (a + b + 1) >> 1; }
__device__ __forceinline__ uint32_t pack4(int a, int b, int c, int d) {
  return (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16) | ((uint32_t)d << 24);
}
__device__ __forceinline__ int byte_of(uint32_t w, int i) { return (w >> (8 * i)) & 0xff; }
// 4 bytes starting at byte offset o (0..7) of the 12-byte little-endian string w0|w1|w2
__device__ __forceinline__ uint32_t pick4(uint32_t w0, uint32_t w1, uint32_t w2, int o) {
  const uint32_t lo = o < 4 ? w0 : w1;
  const uint32_t hi = o < 4 ? w1 : w2;
  const int s = o & 3;
  return s ? ((lo >> (8 * s)) | (hi << (32 - 8 * s))) : lo;
}

// 32-bit wrapping MUL1/MUL2 (dsp.h.go WEBP_TRANSFORM_AC3_MUL1/2).  |a| < 2^23 for
// any int16 input, so the 24-bit multiplier gives the exact low 32 bits.
__device__ __forceinline__ int mul1(int a) { return (__mul24(a, 20091) >> 16) + a; }
__device__ __forceinline__ int mul2(int a) { return __mul24(a, 35468) >> 16; }

// quad transpose helpers (DPP quad_perm)
__device__ __forceinline__ int dpp_swap1(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true); }
__device__ __forceinline__ int dpp_swap2(int v) { return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true); }

// IDCT of one 4x4 block spread over a lane quad.  In: column q = lane&3 of the
// coefficients (c0..c3 = in[q], in[4+q], in[8+q], in[12+q]).  Out: residuals
// (v >> 3) of pixel row q, x = 0..3.  TransformOne (dec.c.go:49-88).
__device__ __forceinline__ void idct_quad(int q, int c0, int c1, int c2, int c3, int r[4]) {
  int t[4];
  {
    const int a = c0 + c2;
    const int b = c0 - c2;
    const int c = mul2(c1) - mul1(c3);
    const int d = mul1(c1) + mul2(c3);
    t[0] = a + d;  // tmp[4q + 0]
    t[1] = b + c;
    t[2] = b - c;
    t[3] = a - d;
  }
  // transpose: lane q ends with u[c] = tmp[4c + q]
  {
    const bool o1 = q & 1;
    int s = o1 ? t[0] : t[1];
    int g = dpp_swap1(s);
    if (o1) t[0] = g; else t[1] = g;
    s = o1 ? t[2] : t[3];
    g = dpp_swap1(s);
    if (o1) t[2] = g; else t[3] = g;
    const bool o2 = q & 2;
    s = o2 ? t[0] : t[2];
    g = dpp_swap2(s);
    if (o2) t[0] = g; else t[2] = g;
    s = o2 ? t[1] : t[3];
    g = dpp_swap2(s);
    if (o2) t[1] = g; else t[3] = g;
  }
  const int dc = t[0] + 4;
  const int a = dc + t[2];
  const int b = dc - t[2];
  const int c = mul2(t[1]) - mul1(t[3]);
  const int d = mul1(t[1]) + mul2(t[3]);
  r[0] = (a + d) >> 3;
  r[1] = (b + c) >> 3;
  r[2] = (b - c) >> 3;
  r[3] = (a - d) >> 3;
}

__device__ __forceinline__ uint32_t add_res(uint32_t pred, const int r[4]) {
  return pack4(clamp255(byte_of(pred, 0) + r[0]), clamp255(byte_of(pred, 1) + r[1]),
               clamp255(byte_of(pred, 2) + r[2]), clamp255(byte_of(pred, 3) + r[3]));
}

__device__ __forceinline__ int check_mode(int mb_x, int mb_y, int mode) {  // frame_dec.c.go:28-37
  if (mode == 0) {
    if (mb_x == 0) return mb_y == 0 ? 6 : 5;
    return mb_y == 0 ? 4 : 0;
  }
  return mode;
}

// Row `r` (0..3) of a 4x4 intra predictor (dec.c.go:261-410), mode = B_* enum.
// Edge samples: X = top-left, A..H = top row + top-right, I..L = left column.
__device__ uint32_t pred4_row(int mode, int r, uint32_t top_lo, uint32_t top_hi, int X, uint32_t left) {
  const int A = byte_of(top_lo, 0), B = byte_of(top_lo, 1), C = byte_of(top_lo, 2), D = byte_of(top_lo, 3);
  const int E = byte_of(top_hi, 0), F = byte_of(top_hi, 1), G = byte_of(top_hi, 2), H = byte_of(top_hi, 3);
  const int I = byte_of(left, 0), J = byte_of(left, 1), K = byte_of(left, 2), L = byte_of(left, 3);
  switch (mode) {
    case 0: {  // DC4
      const int dc = (A + B + C + D + I + J + K + L + 4) >> 3;
      return (uint32_t)dc * 0x01010101u;
    }
    case 1: {  // TM4
      const int ly = byte_of(left, r);
      return pack4(clamp255(A + ly - X), clamp255(B + ly - X), clamp255(C + ly - X), clamp255(D + ly - X));
    }
    case 2:  // VE4
      return pack4(avg3(X, A, B), avg3(A, B, C), avg3(B, C, D), avg3(C, D, E));
    case 3: {  // HE4
      const int lm = r == 0 ? X : byte_of(left, r - 1);
      const int lp = r == 3 ? L : byte_of(left, r + 1);
      return (uint32_t)avg3(lm, byte_of(left, r), lp) * 0x01010101u;
    }
    case 4: {  // RD4: row r = d[4-r .. 7-r], d[k] = avg3(Z[k-1], Z[k], Z[k+1]), Z = L K J I X A B C D
      const uint32_t w0 = pack4(avg3(L, K, J), avg3(K, J, I), avg3(J, I, X), avg3(I, X, A));
      const uint32_t w1 = pack4(avg3(X, A, B), avg3(A, B, C), avg3(B, C, D), 0);
      return pick4(w0, w1, 0, 3 - r);
    }
    case 5: {  // VR4
      uint32_t w0, w1;
      if (r & 1) {
        w0 = pack4(avg3(K, J, I), avg3(I, X, A), avg3(X, A, B), avg3(A, B, C));
        w1 = (uint32_t)avg3(B, C, D);
      } else {
        w0 = pack4(avg3(J, I, X), avg2(X, A), avg2(A, B), avg2(B, C));
        w1 = (uint32_t)avg2(C, D);
      }
      return pick4(w0, w1, 0, r < 2 ? 1 : 0);
    }
    case 6: {  // LD4: row r = d[r .. r+3], d[k] = avg3(T[k], T[k+1], T[k+2]), T[8] = H
      const uint32_t w0 = pack4(avg3(A, B, C), avg3(B, C, D), avg3(C, D, E), avg3(D, E, F));
      const uint32_t w1 = pack4(avg3(E, F, G), avg3(F, G, H), avg3(G, H, H), 0);
      return pick4(w0, w1, 0, r);
    }
    case 7: {  // VL4
      uint32_t w0, w1;
      if (r & 1) {
        w0 = pack4(avg3(A, B, C), avg3(B, C, D), avg3(C, D, E), avg3(D, E, F));
        w1 = (uint32_t)avg3(F, G, H);
      } else {
        w0 = pack4(avg2(A, B), avg2(B, C), avg2(C, D), avg2(D, E));
        w1 = (uint32_t)avg3(E, F, G);
      }
      return pick4(w0, w1, 0, r >> 1);
    }
    case 8: {  // HD4: row r = S[6-2r .. 9-2r]
      const uint32_t w0 = pack4(avg2(L, K), avg3(L, K, J), avg2(K, J), avg3(K, J, I));
      const uint32_t w1 = pack4(avg2(J, I), avg3(J, I, X), avg2(I, X), avg3(I, X, A));
      const uint32_t w2 = pack4(avg3(X, A, B), avg3(A, B, C), 0, 0);
      return pick4(w0, w1, w2, 6 - 2 * r);
    }
    default: {  // 9, HU4: row r = U[2r .. 2r+3]
      const uint32_t w0 = pack4(avg2(I, J), avg3(I, J, K), avg2(J, K), avg3(J, K, L));
      const uint32_t w1 = pack4(avg2(K, L), avg3(K, L, L), L, L);
      const uint32_t w2 = (uint32_t)L * 0x01010101u;
      return pick4(w0, w1, w2, 2 * r);
    }
  }
}

// ---------------------------------------------------------------- loop filter
struct Line { int p3, p2, p1, p0, q0, q1, q2, q3; };

__device__ __forceinline__ int sclip1(int v) { return min(max(v, -128), 127); }
__device__ __forceinline__ int sclip2(int v) { return min(max(v, -16), 15); }

__device__ __forceinline__ void do_filter2(Line& l) {  // DoFilter2_C (dec.c.go:484-491)
  const int a = 3 * (l.q0 - l.p0) + sclip1(l.p1 - l.q1);
  const int a1 = sclip2((a + 4) >> 3);
  const int a2 = sclip2((a + 3) >> 3);
  l.p0 = clamp255(l.p0 + a2);
  l.q0 = clamp255(l.q0 - a1);
}
__device__ __forceinline__ void do_filter4(Line& l) {  // DoFilter4_C (:494-504)
  const int a = 3 * (l.q0 - l.p0);
  const int a1 = sclip2((a + 4) >> 3);
  const int a2 = sclip2((a + 3) >> 3);
  const int a3 = (a1 + 1) >> 1;
  l.p1 = clamp255(l.p1 + a3);
  l.p0 = clamp255(l.p0 + a2);
  l.q0 = clamp255(l.q0 - a1);
  l.q1 = clamp255(l.q1 - a3);
}
__device__ __forceinline__ void do_filter6(Line& l) {  // DoFilter6_C (:507-521)
  const int a = sclip1(3 * (l.q0 - l.p0) + sclip1(l.p1 - l.q1));
  const int a1 = (27 * a + 63) >> 7;
  const int a2 = (18 * a + 63) >> 7;
  const int a3 = (9 * a + 63) >> 7;
  l.p2 = clamp255(l.p2 + a3);
  l.p1 = clamp255(l.p1 + a2);
  l.p0 = clamp255(l.p0 + a1);
  l.q0 = clamp255(l.q0 - a1);
  l.q1 = clamp255(l.q1 - a2);
  l.q2 = clamp255(l.q2 - a3);
}
__device__ __forceinline__ bool needs_filter(const Line& l, int t) {  // NeedsFilter_C (:530-533)
  return 4 * abs(l.p0 - l.q0) + abs(l.p1 - l.q1) <= t;
}
__device__ __forceinline__ bool needs_filter2(const Line& l, int t, int it) {  // NeedsFilter2_C (:537-545)
  if (4 * abs(l.p0 - l.q0) + abs(l.p1 - l.q1) > t) return false;
  return abs(l.p3 - l.p2) <= it && abs(l.p2 - l.p1) <= it && abs(l.p1 - l.p0) <= it &&
         abs(l.q3 - l.q2) <= it && abs(l.q2 - l.q1) <= it && abs(l.q1 - l.q0) <= it;
}
__device__ __forceinline__ bool hev(const Line& l, int thresh) {  // Hev (:523-526)
  return abs(l.p1 - l.p0) > thresh || abs(l.q1 - l.q0) > thresh;
}

// kind: 0 simple (NeedsFilter + DoFilter2), 1 complex MB edge (FilterLoop26),
// 2 complex inner edge (FilterLoop24).  thresh2 = 2*thresh + 1.
__device__ __forceinline__ void filter_line(Line& l, int kind, int thresh2, int ilevel, int hev_t) {
  if (kind == 0) {
    if (needs_filter(l, thresh2)) do_filter2(l);
  } else if (needs_filter2(l, thresh2, ilevel)) {
    if (hev(l, hev_t)) do_filter2(l);
    else if (kind == 1) do_filter6(l);
    else do_filter4(l);
  }
}

// Filter across a vertical edge at column e of a window row (horizontal step).
__device__ __forceinline__ void filter_row(uint8_t* row_at_e /* &win[row][e] */, int kind, int t2, int il, int ht) {
  const uint32_t lo = *reinterpret_cast<const uint32_t*>(row_at_e - 4);
  const uint32_t hi = *reinterpret_cast<const uint32_t*>(row_at_e);
  Line l{byte_of(lo, 0), byte_of(lo, 1), byte_of(lo, 2), byte_of(lo, 3),
         byte_of(hi, 0), byte_of(hi, 1), byte_of(hi, 2), byte_of(hi, 3)};
  filter_line(l, kind, t2, il, ht);
  *reinterpret_cast<uint32_t*>(row_at_e - 4) = pack4(l.p3, l.p2, l.p1, l.p0);
  *reinterpret_cast<uint32_t*>(row_at_e) = pack4(l.q0, l.q1, l.q2, l.q3);
}
// Filter across a horizontal edge (vertical step `s` = window stride).
__device__ __forceinline__ void filter_col(uint8_t* p /* &win[e][col] */, int s, int kind, int t2, int il, int ht) {
  Line l{p[-4 * s], p[-3 * s], p[-2 * s], p[-s], p[0], p[s], p[2 * s], p[3 * s]};
  filter_line(l, kind, t2, il, ht);
  p[-3 * s] = (uint8_t)l.p2;
  p[-2 * s] = (uint8_t)l.p1;
  p[-s] = (uint8_t)l.p0;
  p[0] = (uint8_t)l.q0;
  p[s] = (uint8_t)l.q1;
  p[2 * s] = (uint8_t)l.q2;
}

__device__ __forceinline__ uint32_t lds32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }
__device__ __forceinline__ void st32(uint8_t* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; }

}  // namespace

__global__ void __launch_bounds__(1024) vp8_recon_filter_kernel(const FrameDesc* __restrict__ frames) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const FrameDesc* F = frames + blockIdx.x;
  if (!F->valid) return;
  const int mb_w = F->mb_w, mb_h = F->mb_h;
  const int ftype = F->filter_type;
  const int ys = F->y_stride, uvs = F->uv_stride;
  const MbRec* __restrict__ mbs = F->mbs;
  const int16_t* __restrict__ blocks = F->blocks;
  uint8_t* __restrict__ Yp = F->y;
  uint8_t* __restrict__ Up = F->u;
  uint8_t* __restrict__ Vp = F->v;

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  volatile uint32_t* progress = reinterpret_cast<volatile uint32_t*>(lds);
  uint8_t* ws = lds + kProgBytes + wave * kWaveBytes;  // recon workspace (libwebp yuv_b)
  uint8_t* fw = ws + kWsBytes;                          // filter window
  uint8_t* left = fw + kFwBytes;                        // unfiltered left columns (contiguous)
  uint8_t* cols = lds + kProgBytes + kWaves * kWaveBytes;
  // per MB column c: cols + c*kColBytes: [0..15] ytop Y, [16..23] U, [24..31] V, [32..159] fbot
  if (threadIdx.x < kWaves) progress[threadIdx.x] = 0;
  __syncthreads();

  // lane roles
  const int lb = lane >> 2;       // luma block 0..15 (raster)
  const int lq = lane & 3;        // row within block / coefficient column
  const int lbx = lb & 3, lby = lb >> 2;
  const int crow = 4 * lby + lq;  // luma pixel row of this lane
  const int cpl = (lane >> 4) & 1;            // chroma plane (lanes 0..31)
  const int cb = (lane >> 2) & 3;             // chroma block
  const int cbx = cb & 1, cby = cb >> 1;
  const int ccrow = 4 * cby + lq;             // chroma pixel row
  const int coff = cpl ? V_OFF : U_OFF;

  for (int y = wave; y < mb_h; y += kWaves) {
    // ---- ReconstructRow prologue (frame_dec.c.go:79-98)
    if (lane < 16) ws[Y_OFF + lane * BPS - 1] = 129;
    else if (lane < 24) ws[U_OFF + (lane - 16) * BPS - 1] = 129;
    else if (lane < 32) ws[V_OFF + (lane - 24) * BPS - 1] = 129;
    if (lane < 32) left[lane] = 129;
    if (y > 0) {
      if (lane == 32) ws[Y_OFF - BPS - 1] = 129;
      if (lane == 33) ws[U_OFF - BPS - 1] = 129;
      if (lane == 34) ws[V_OFF - BPS - 1] = 129;
    } else {
      if (lane < 21) ws[Y_OFF - BPS - 1 + lane] = 127;
      else if (lane < 30) ws[U_OFF - BPS - 1 + (lane - 21)] = 127;
      else if (lane < 39) ws[V_OFF - BPS - 1 + (lane - 30)] = 127;
    }
    lds_sync();
    uint32_t blk = F->row_block0[y];  // running index of this MB's first coefficient block
    const int nrows_y = (y == mb_h - 1) ? 16 : 13;  // luma rows final after this row's pass
    const int nrows_c = (y == mb_h - 1) ? 8 : 5;

    for (int x = 0; x < mb_w; ++x) {
      const MbRec rec = mbs[(size_t)y * mb_w + x];
      const uint32_t flags = __builtin_amdgcn_readfirstlane(rec.flags);
      const uint32_t im_lo = __builtin_amdgcn_readfirstlane(rec.imodes_lo);
      const uint32_t im_hi = __builtin_amdgcn_readfirstlane(rec.imodes_hi);
      const uint32_t finfo = __builtin_amdgcn_readfirstlane(rec.finfo);
      const uint32_t nz = flags & kNzMask;
      const bool is_i4 = (flags >> kI4Shift) & 1;

      // ---- coefficient loads (one column of one block per lane)
      int yc[4] = {0, 0, 0, 0}, uc[4] = {0, 0, 0, 0};
      if ((nz >> lb) & 1) {
        const uint32_t bi = blk + __builtin_popcount(nz & ((1u << lb) - 1));
        const uint2 v = *reinterpret_cast<const uint2*>(blocks + (size_t)bi * 16 + 4 * lq);
        yc[0] = (int16_t)(v.x & 0xffff); yc[1] = (int16_t)(v.x >> 16);
        yc[2] = (int16_t)(v.y & 0xffff); yc[3] = (int16_t)(v.y >> 16);
      }
      const int cbi = 16 + cpl * 4 + cb;  // lanes 0..31: chroma blocks 16..23
      if (lane < 32 && ((nz >> cbi) & 1)) {
        const uint32_t bi = blk + __builtin_popcount(nz & ((1u << cbi) - 1));
        const uint2 v = *reinterpret_cast<const uint2*>(blocks + (size_t)bi * 16 + 4 * lq);
        uc[0] = (int16_t)(v.x & 0xffff); uc[1] = (int16_t)(v.x >> 16);
        uc[2] = (int16_t)(v.y & 0xffff); uc[3] = (int16_t)(v.y >> 16);
      }
      blk += __builtin_popcount(nz);

      // ---- wait for the row above (t = x + 2y wavefront)
      if (y > 0) {
        const uint32_t need = (uint32_t)(y - 1) * mb_w + min(x + 2, mb_w);
        volatile uint32_t* pr = progress + ((y - 1) & (kWaves - 1));
        while (*pr < need) __builtin_amdgcn_s_sleep(1);
      }
      uint8_t* col = cols + x * kColBytes;

      // ---- top samples (frame_dec.c.go:122-142)
      if (y > 0) {
        if (lane < 4) st32(ws + Y_OFF - BPS + 4 * lane, lds32(col + 4 * lane));
        else if (lane < 6) st32(ws + U_OFF - BPS + 4 * (lane - 4), lds32(col + 16 + 4 * (lane - 4)));
        else if (lane < 8) st32(ws + V_OFF - BPS + 4 * (lane - 6), lds32(col + 24 + 4 * (lane - 6)));
        else if (lane == 8 && is_i4) {
          const uint32_t tr = (x >= mb_w - 1) ? (uint32_t)col[15] * 0x01010101u : lds32(col + kColBytes);
          st32(ws + Y_OFF - BPS + 16, tr);
        }
      }
      lds_sync();
      if (is_i4 && lane < 3) st32(ws + Y_OFF + (3 + 4 * lane) * BPS + 16, lds32(ws + Y_OFF - BPS + 16));
      lds_sync();

      // ---- luma residuals (all 16 blocks at once)
      int ry[4];
      idct_quad(lq, yc[0], yc[1], yc[2], yc[3], ry);
      uint8_t* my = ws + Y_OFF + crow * BPS + 4 * lbx;
      if (!is_i4) {
        const int mode = check_mode(x, y, (flags >> kYModeShift) & 3);
        uint32_t pred;
        const uint32_t top = lds32(ws + Y_OFF - BPS + 4 * lbx);
        const int l = left[crow];
        if (mode == 2) {
          pred = top;
        } else if (mode == 3) {
          pred = (uint32_t)l * 0x01010101u;
        } else if (mode == 1) {
          const int tl = ws[Y_OFF - BPS - 1];
          pred = pack4(clamp255(byte_of(top, 0) + l - tl), clamp255(byte_of(top, 1) + l - tl),
                       clamp255(byte_of(top, 2) + l - tl), clamp255(byte_of(top, 3) + l - tl));
        } else {
          uint32_t st = 0, sl = 0;
          for (int k = 0; k < 4; ++k) {
            st = __builtin_amdgcn_sad_u8(lds32(ws + Y_OFF - BPS + 4 * k), 0, st);
            sl = __builtin_amdgcn_sad_u8(lds32(left + 4 * k), 0, sl);
          }
          int dc;
          if (mode == 0) dc = (int)(st + sl + 16) >> 5;
          else if (mode == 4) dc = (int)(sl + 8) >> 4;   // no top
          else if (mode == 5) dc = (int)(st + 8) >> 4;   // no left
          else dc = 0x80;
          pred = (uint32_t)dc * 0x01010101u;
        }
        lds_sync();
        st32(my, add_res(pred, ry));
      } else {
        const int mode = ((lb < 8 ? im_lo >> (4 * lb) : im_hi >> (4 * (lb - 8)))) & 0xf;
        const int tstep = lbx + 2 * lby;
        for (int t = 0; t < 10; ++t) {
          if (tstep == t) {
            const uint8_t* b0 = ws + Y_OFF + 4 * lby * BPS + 4 * lbx;  // block origin
            const uint32_t tlo = lds32(b0 - BPS);
            const uint32_t thi = lds32(b0 - BPS + 4);
            const int X = b0[-BPS - 1];
            const uint32_t lft = pack4(b0[-1], b0[BPS - 1], b0[2 * BPS - 1], b0[3 * BPS - 1]);
            const uint32_t pred = pred4_row(mode, lq, tlo, thi, X, lft);
            st32(my, add_res(pred, ry));
          }
          lds_sync();
        }
      }

      // ---- chroma (lanes 0..31)
      int rc[4];
      idct_quad(lq, uc[0], uc[1], uc[2], uc[3], rc);
      if (lane < 32) {
        const int mode = check_mode(x, y, (flags >> kUVModeShift) & 3);
        const uint8_t* base = ws + coff;
        const uint32_t top = lds32(base - BPS + 4 * cbx);
        const int l = left[16 + 8 * cpl + ccrow];
        uint32_t pred;
        if (mode == 2) {
          pred = top;
        } else if (mode == 3) {
          pred = (uint32_t)l * 0x01010101u;
        } else if (mode == 1) {
          const int tl = base[-BPS - 1];
          pred = pack4(clamp255(byte_of(top, 0) + l - tl), clamp255(byte_of(top, 1) + l - tl),
                       clamp255(byte_of(top, 2) + l - tl), clamp255(byte_of(top, 3) + l - tl));
        } else {
          uint32_t st = 0, sl = 0;
          for (int k = 0; k < 2; ++k) {
            st = __builtin_amdgcn_sad_u8(lds32(base - BPS + 4 * k), 0, st);
            sl = __builtin_amdgcn_sad_u8(lds32(left + 16 + 8 * cpl + 4 * k), 0, sl);
          }
          int dc;
          if (mode == 0) dc = (int)(st + sl + 8) >> 4;
          else if (mode == 4) dc = (int)(sl + 4) >> 3;
          else if (mode == 5) dc = (int)(st + 4) >> 3;
          else dc = 0x80;
          pred = (uint32_t)dc * 0x01010101u;
        }
        lds_sync();
        st32(ws + coff + ccrow * BPS + 4 * cbx, add_res(pred, rc));
      }
      lds_sync();

      // ---- stash top samples for the row below (frame_dec.c.go:175-179)
      if (y < mb_h - 1) {
        if (lane < 4) st32(col + 4 * lane, lds32(ws + Y_OFF + 15 * BPS + 4 * lane));
        else if (lane < 6) st32(col + 16 + 4 * (lane - 4), lds32(ws + U_OFF + 7 * BPS + 4 * (lane - 4)));
        else if (lane < 8) st32(col + 24 + 4 * (lane - 6), lds32(ws + V_OFF + 7 * BPS + 4 * (lane - 6)));
      }
      // ---- fill the filter window: MB body from the workspace, rows above from fbot
      {
        const int r = lane >> 2, d = lane & 3;
        st32(fw + kFwY + (r + 4) * FWY + 4 + 4 * d, lds32(ws + Y_OFF + r * BPS + 4 * d));
        if (lane < 32) {
          const int p = lane >> 4, rr = (lane >> 1) & 7, dd = lane & 1;
          st32(fw + (p ? kFwV : kFwU) + (rr + 4) * FWC + 4 + 4 * dd,
               lds32(ws + (p ? V_OFF : U_OFF) + rr * BPS + 4 * dd));
        } else if (y > 0) {
          const int k = lane - 32;  // 0..31
          if (k < 16) {             // luma rows -4..-1
            st32(fw + kFwY + (k >> 2) * FWY + 4 + 4 * (k & 3), lds32(col + 32 + 4 * k));
          } else {                  // chroma rows -4..-1
            const int p = (k - 16) >> 3, rr = ((k - 16) >> 1) & 3, dd = k & 1;
            st32(fw + (p ? kFwV : kFwU) + rr * FWC + 4 + 4 * dd, lds32(col + 96 + 32 * p + 8 * rr + 4 * dd));
          }
        }
      }
      lds_sync();

      // ---- loop filter (DoFilter, frame_dec.c.go:204-251) on the window
      const int limit = finfo & 0xff;
      if (ftype > 0 && limit > 0) {
        const int ilevel = (finfo >> 8) & 0xff;
        const int inner = (finfo >> 16) & 0xff;
        const int hev_t = (finfo >> 24) & 0xff;
        const int kmb = ftype == 1 ? 0 : 1, kin = ftype == 1 ? 0 : 2;
        const int t_mb = 2 * (limit + 4) + 1, t_in = 2 * limit + 1;
        // lanes 0..15: luma line; 16..23: U line; 24..31: V line (complex only)
        const bool luma = lane < 16;
        const bool chroma = lane >= 16 && lane < 32 && ftype == 2;
        const int li = lane & 15;
        const int cli = lane & 7;
        uint8_t* cwin = fw + ((lane >> 3) & 1 ? kFwV : kFwU);
        if (x > 0) {  // left MB edge (HFilter16 / HFilter8)
          if (luma) filter_row(fw + kFwY + (li + 4) * FWY + 4, kmb, t_mb, ilevel, hev_t);
          if (chroma) filter_row(cwin + (cli + 4) * FWC + 4, kmb, t_mb, ilevel, hev_t);
          lds_sync();
        }
        if (inner) {  // inner vertical edges (HFilter16i / HFilter8i)
          if (luma) filter_row(fw + kFwY + (li + 4) * FWY + 8, kin, t_in, ilevel, hev_t);
          if (chroma) filter_row(cwin + (cli + 4) * FWC + 8, kin, t_in, ilevel, hev_t);
          lds_sync();
          if (luma) filter_row(fw + kFwY + (li + 4) * FWY + 12, kin, t_in, ilevel, hev_t);
          lds_sync();
          if (luma) filter_row(fw + kFwY + (li + 4) * FWY + 16, kin, t_in, ilevel, hev_t);
          lds_sync();
        }
        if (y > 0) {  // top MB edge (VFilter16 / VFilter8)
          if (luma) filter_col(fw + kFwY + 4 * FWY + 4 + li, FWY, kmb, t_mb, ilevel, hev_t);
          if (chroma) filter_col(cwin + 4 * FWC + 4 + cli, FWC, kmb, t_mb, ilevel, hev_t);
          lds_sync();
        }
        if (inner) {  // inner horizontal edges (VFilter16i / VFilter8i)
          if (luma) filter_col(fw + kFwY + 8 * FWY + 4 + li, FWY, kin, t_in, ilevel, hev_t);
          if (chroma) filter_col(cwin + 8 * FWC + 4 + cli, FWC, kin, t_in, ilevel, hev_t);
          lds_sync();
          if (luma) filter_col(fw + kFwY + 12 * FWY + 4 + li, FWY, kin, t_in, ilevel, hev_t);
          lds_sync();
          if (luma) filter_col(fw + kFwY + 16 * FWY + 4 + li, FWY, kin, t_in, ilevel, hev_t);
          lds_sync();
        }
      }

      // ---- deposit this row's bottom samples for the row below (fbot)
      {
        const bool last_x = (x == mb_w - 1);
        if (lane < 16) {  // luma rows 12..15, dwords: cols -4..-1 -> col x-1, cols 0..11 / 12..15 -> col x
          const int rr = lane >> 2, d = lane & 3;  // d=0: cols -4..-1, d=1..3: cols 0..11
          if (d == 0) {
            if (x > 0) st32(col - kColBytes + 32 + rr * 16 + 12, lds32(fw + kFwY + (rr + 16) * FWY + 0));
          } else {
            st32(col + 32 + rr * 16 + 4 * (d - 1), lds32(fw + kFwY + (rr + 16) * FWY + 4 * d));
          }
          if (last_x && d == 0) st32(col + 32 + rr * 16 + 12, lds32(fw + kFwY + (rr + 16) * FWY + 16));
        } else if (lane < 32) {  // chroma rows 4..7
          const int k = lane - 16, p = k >> 3, rr = (k >> 1) & 3, d = k & 1;
          const uint8_t* cw = fw + (p ? kFwV : kFwU);
          uint8_t* cb0 = col + 96 + 32 * p + 8 * rr;
          if (d == 0) {
            if (x > 0) st32(cb0 - kColBytes + 4, lds32(cw + (rr + 8) * FWC + 0));
          } else {
            st32(cb0, lds32(cw + (rr + 8) * FWC + 4));
          }
          if (last_x && d == 0) st32(cb0 + 4, lds32(cw + (rr + 8) * FWC + 8));
        }
      }

      // ---- final pixels to HBM (each byte written once)
      {
        const bool last_x = (x == mb_w - 1);
        // luma: rows 0..nrows_y-1, window cols -4..11 (dword d = cols 4d-4..4d-1)
        {
          const int r = lane >> 2, d = lane & 3;
          if (r < nrows_y && (d > 0 || x > 0))
            *reinterpret_cast<uint32_t*>(Yp + (size_t)(16 * y + r) * ys + 16 * x - 4 + 4 * d) =
                lds32(fw + kFwY + (r + 4) * FWY + 4 * d);
        }
        // luma rows 13..15 of the last row: r = 16..15 handled above via nrows; extra lanes:
        if (lane < 16) {
          const int r = lane;  // rows -3..-1 (MB above) use lanes 0..11; last column cols 12..15
          if (y > 0 && r < 12) {
            const int rr = (r >> 2) - 3, d = r & 3;
            *reinterpret_cast<uint32_t*>(Yp + (size_t)(16 * y + rr) * ys + 16 * x + 4 * d) =
                lds32(fw + kFwY + (rr + 4) * FWY + 4 + 4 * d);
          }
          if (last_x && r < nrows_y)
            *reinterpret_cast<uint32_t*>(Yp + (size_t)(16 * y + r) * ys + 16 * x + 12) =
                lds32(fw + kFwY + (r + 4) * FWY + 16);
        } else if (lane < 48) {  // chroma: rows 0..nrows_c-1 cols -4..3, both planes
          const int k = lane - 16, p = k >> 4, r = (k >> 1) & 7, d = k & 1;
          const uint8_t* cw = fw + (p ? kFwV : kFwU);
          uint8_t* plane = p ? Vp : Up;
          if (r < nrows_c && (d > 0 || x > 0))
            *reinterpret_cast<uint32_t*>(plane + (size_t)(8 * y + r) * uvs + 8 * x - 4 + 4 * d) =
                lds32(cw + (r + 4) * FWC + 4 * d);
          if (last_x && d == 0 && r < nrows_c)
            *reinterpret_cast<uint32_t*>(plane + (size_t)(8 * y + r) * uvs + 8 * x + 4) =
                lds32(cw + (r + 4) * FWC + 8);
        } else if (y > 0) {  // chroma rows -3..-1 of the MB above, cols 0..7
          const int k = lane - 48;  // 0..15: p, row, d
          const int p = k >> 3, rr = ((k >> 1) & 3), d = k & 1;
          if (rr < 3) {
            const uint8_t* cw = fw + (p ? kFwV : kFwU);
            uint8_t* plane = p ? Vp : Up;
            const int row = rr - 3;
            *reinterpret_cast<uint32_t*>(plane + (size_t)(8 * y + row) * uvs + 8 * x + 4 * d) =
                lds32(cw + (row + 4) * FWC + 4 + 4 * d);
          }
        }
      }
      lds_sync();

      // ---- rotate for the next MB (frame_dec.c.go:106-114) + filter window
      if (lane < 17) {  // Y rows -1..15: cols 12..15 -> -4..-1
        const int r = lane - 1;
        const uint32_t v = lds32(ws + Y_OFF + r * BPS + 12);
        st32(ws + Y_OFF + r * BPS - 4, v);
        if (r >= 0) left[r] = (uint8_t)(v >> 24);
      } else if (lane < 35) {  // U/V rows -1..7: cols 4..7 -> -4..-1
        const int k = lane - 17, p = k / 9, r = k % 9 - 1;
        const int off = p ? V_OFF : U_OFF;
        const uint32_t v = lds32(ws + off + r * BPS + 4);
        st32(ws + off + r * BPS - 4, v);
        if (r >= 0) left[16 + 8 * p + r] = (uint8_t)(v >> 24);
      } else if (lane < 51) {  // window luma rows 0..15
        const int r = lane - 35;
        st32(fw + kFwY + (r + 4) * FWY, lds32(fw + kFwY + (r + 4) * FWY + 16));
      } else if (lane < 64) {  // window chroma rows 0..7 (13 lanes: U 0..7, V 0..4)
        const int k = lane - 51, p = k >> 3, r = k & 7;
        uint8_t* cw = fw + (p ? kFwV : kFwU);
        st32(cw + (r + 4) * FWC, lds32(cw + (r + 4) * FWC + 8));
      }
      if (lane < 3) {  // window V rows 5..7
        uint8_t* cw = fw + kFwV;
        const int r = 5 + lane;
        st32(cw + (r + 4) * FWC, lds32(cw + (r + 4) * FWC + 8));
      }
      lds_sync();
      if (lane == 0) progress[y & (kWaves - 1)] = (uint32_t)y * mb_w + x + 1;
    }
  }
}

size_t vp8_recon_lds_bytes(int mb_w) {
  return (size_t)kProgBytes + (size_t)kWaves * kWaveBytes + (size_t)mb_w * kColBytes;
}

int vp8_recon_max_mb_w() { return (int)((163840 - kProgBytes - kWaves * kWaveBytes) / kColBytes); }

hipError_t launch_vp8_recon_filter(const FrameDesc* d_frames, int n_frames, int max_mb_w, hipStream_t stream) {
  const size_t lds = vp8_recon_lds_bytes(max_mb_w);
  static size_t configured = 0;
  if (lds > 65536 && lds > configured) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&vp8_recon_filter_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    configured = lds;
  }
  hipLaunchKernelGGL(vp8_recon_filter_kernel, dim3(n_frames), dim3(1024), lds, stream, d_frames);
  return hipGetLastError();
}

}  // namespace wg
