// K1: VP8 macroblock reconstruction + in-loop deblocking, fused, for gfx950.
//
// Replaces the reference's per-MB DSP loop:
//   ReconstructRow       pkg/libwebp/decoder/frame_dec.c.go:69-197
//   DoFilter / FilterRow pkg/libwebp/decoder/frame_dec.c.go:204-261
//   transforms           pkg/libwebp/dsp/dec.c.go:49-134 (+DoTransform :43-67)
//   intra predictors     pkg/libwebp/dsp/dec.c.go:178-474 (indexed by mode enum)
//   loop filters         pkg/libwebp/dsp/dec.c.go:484-682
//
// Geometry.  One 1024-thread workgroup per frame.  Wave w < R owns MB-row QUADS
// k = w, w+R, ...: lane group g = lane >> 4 decodes row 4k+g, at column i-2g in step i --
// the t = x + 2y wavefront, since intra prediction (top-right samples) and the loop filter
// (MB (x+1,y-1)'s left-edge writes) both reach one MB up and to the right.  Inside a quad
// the lockstep skew satisfies the dependency; across quads an LDS progress counter does
// (4R MB rows in flight per frame).
//
// One macroblock = 16 lanes.  Lane m = lane & 15 plays two "roles" r = m + 16s (s = 0, 1;
// two unrolled passes per section) of a 32-role MB layout: role r owns column/row q = r&3
// of luma 4x4 blocks r>>2 and (r>>2)+8 and of chroma block 16+(r>>2).  IDCT (TransformOne,
// all blocks at once since the residual (v>>3) does not depend on the prediction):
// vertical pass per column lane, quad DPP transpose, horizontal pass.  i16/chroma
// prediction: one 4-pixel row per role.  i4x4 prediction walks the 16 blocks in the order
// t = bx + 2by (a block's left, top, top-left and top-right neighbours all have a smaller
// t) with ONE PIXEL PER LANE: each pixel of each predictor is a 3-tap recipe of edge
// samples (pred4_table.inc, generated from dec.c.go's DST() formulas), so no lane branches
// on the mode.  A non-zero block always goes through TransformOne: TransformAC3 /
// TransformDC / TransformDCUV are exact special cases of it
// (tests/test_oracle.py::test_transform_shortcuts_exact).
//
// Loop filter (per MB, libwebp edge order): lane m filters luma line m (4 edges), then
// chroma line m&7 of U (m < 8) or V (2 edges), of a per-MB LDS window: every vertical edge
// of a line in registers, then the same on columns (two LDS round trips per MB).
//
// Why four MBs per wave step.  The kernel is bound by instruction issue on the frame's CU
// (DESIGN.md §4).  With 32 lanes per MB the filter's chroma lanes sat out the two luma-only
// inner edges of each pass (8 edge slots per 2 MBs; here 12 per 4), and every per-step cost
// that does not scale with the lanes -- scalar control, branches, the wavefront wait, the
// LDS hand-off latency of the ~20 dependent sections -- is shared by twice the MBs.
//
// Memory.  Cross-MB state lives in LDS only: the unfiltered top samples `ytop`
// (VP8TopSamples), the final bottom rows `fbot` of each MB column for the next row's
// top-edge filter, progress counters.  Every HBM byte of the Y/U/V planes is written
// exactly once, when final.  MB records and coefficients are software-pipelined: record
// x+2 is loaded at the top of MB x's step, the coefficients of x+1 right after x's IDCT.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>
#include <stdlib.h>

#include "../device_format.h"
#include "kernels.h"
#include "yuv_rgba_strip.h"

namespace wg {
namespace {

#include "pred4_table.inc"

constexpr int kWaves = 16;
constexpr int kRows = 4;       // MB rows per wave (a quad); 16 lanes per MB
#ifndef WG_K1_MAX_RECON
#define WG_K1_MAX_RECON 12
#endif
constexpr int kMaxRecon = WG_K1_MAX_RECON;  // waves that may reconstruct: LDS slots for 4 x 12 MB rows
constexpr int BPS = 32;        // libwebp workspace stride (vp8/constants.go BPS)
constexpr int Y_OFF = BPS * 1 + 8;
constexpr int U_OFF = Y_OFF + BPS * 16 + BPS;
constexpr int V_OFF = U_OFF + 16;
constexpr int kWsBytes = 832;  // YUV_SIZE = BPS*17 + BPS*9
// filter window: luma rows/cols -4..15 (stride 20), chroma rows/cols -4..7 (stride 12)
constexpr int FWY = 20, FWC = 12;
constexpr int kFwY = 0, kFwU = 400, kFwV = 544;
constexpr int kFwBytes = 704;
constexpr int kLeftBytes = 32;   // contiguous unfiltered left columns: Y 16, U 8, V 8
constexpr int kResBytes = 512;   // i4x4 residuals, int16 [16 blocks][16 px]
constexpr int kSlotBytes = kWsBytes + kFwBytes + kLeftBytes + kResBytes;  // 2080 per MB row
constexpr int kProgBytes = 64;  // reserved (progress lives in a static __shared__ array)
constexpr int kTabBytes = 640;
constexpr int kHdrBytes = kProgBytes + kTabBytes;
constexpr int kColBytes = 32 + 128;  // ytop (y16 u8 v8) + fbot (Y 4x16, U 4x8, V 4x8)
constexpr uint32_t kDrop = 0x80000000u;  // buffer offset beyond any frame: store dropped
// i4x4 blocks in wavefront order t = bx + 2*by, and their t
constexpr int kI4Order[16] = {0, 1, 2, 4, 3, 5, 6, 8, 7, 9, 10, 12, 11, 13, 14, 15};
constexpr int kI4Step[16] = {0, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 9};

// Opt-in per-section cycle accounting (make VARIANT=timing -> libgowebp_amd_timing.so,
// read back by scripts/k1_sections.py): s_memtime deltas summed per loop section in
// SGPRs, added to a device array once per wave.  Compiled out of the product library.
#ifdef WG_K1_SECTION_TIMING
constexpr int kSections = 14;
__device__ unsigned long long g_k1_sections[kSections];
// timeline: per workgroup (frame) the start time and each wave's exit time (s_memrealtime)
constexpr int kTimelineFrames = 1024;
// [0] start, [1 + w] wave w leaves reconstruction, [1 + kWaves + w] wave w leaves the kernel
__device__ unsigned long long g_k1_timeline[kTimelineFrames][1 + 2 * kWaves];
#define K1_SECT_DECL() uint64_t sect_acc[kSections] = {}, sect_t = 0
#define K1_SECT_START() (sect_t = __builtin_amdgcn_s_memtime())
#define K1_SECT(id)                                       \
  do {                                                    \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();     \
    sect_acc[id] += t_ - sect_t;                          \
    sect_t = t_;                                          \
  } while (0)
#define K1_SECT_FLUSH()                                                        \
  do {                                                                         \
    if (lane == 0) {                                                           \
      for (int s_ = 0; s_ < kSections; ++s_) atomicAdd(&g_k1_sections[s_], sect_acc[s_]); \
      if (blockIdx.x < kTimelineFrames)                                        \
        g_k1_timeline[blockIdx.x][1 + wave] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                          \
  } while (0)
// per frame and quad: start and end of the quad's MB loop
constexpr int kTimelineQuads = 64;
__device__ unsigned long long g_k1_quads[kTimelineFrames][kTimelineQuads][2];
#define K1_QUAD_MARK(k, which)                                                 \
  do {                                                                         \
    if (lane == 0 && blockIdx.x < kTimelineFrames && (k) < kTimelineQuads)     \
      g_k1_quads[blockIdx.x][k][which] = __builtin_amdgcn_s_memrealtime();     \
  } while (0)
#define K1_TIMELINE_END()                                                      \
  do {                                                                         \
    if (lane == 0 && blockIdx.x < kTimelineFrames)                             \
      g_k1_timeline[blockIdx.x][1 + kWaves + wave] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define K1_TIMELINE_START()                                                    \
  do {                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < kTimelineFrames)                     \
      g_k1_timeline[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();         \
  } while (0)
#else
#define K1_SECT_DECL() (void)0
#define K1_SECT_START() (void)0
#define K1_SECT(id) (void)0
#define K1_SECT_FLUSH() (void)0
#define K1_TIMELINE_START() (void)0
#define K1_TIMELINE_END() (void)0
#define K1_QUAD_MARK(k, which) (void)0
#endif

__device__ __forceinline__ void lds_sync() {
  // Intra-wave LDS exchange.  A wave's DS instructions execute in order, so a later read
  // sees an earlier write of any lane (and a later write cannot overtake an earlier read)
  // with no s_waitcnt; only compiler reordering has to be stopped.  Wavefront-scope fences
  // emit no instruction.  Cross-wave hand-off goes through the release/acquire progress
  // counters instead.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}


__device__ __forceinline__ int clamp255(int v) { return min(max(v, 0), 255); }
// byte 0 of v in all four bytes: one v_perm_b32 (a multiply by 0x01010101 is a quarter-rate
// v_mul_lo_u32)
__device__ __forceinline__ uint32_t bcast(uint32_t v) { return __builtin_amdgcn_perm(v, v, 0u); }
__device__ __forceinline__ int byte_of(uint32_t w, int i) { return (w >> (8 * i)) & 0xff; }
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }
__device__ __forceinline__ void st32(uint8_t* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; }
// Column-store accesses (LDS, or global memory for wide frames and the split kernel, see
// vp8_recon_filter_kernel).  Those of the split kernel's part-boundary quads (kSplit): global_load /
// global_store with sc1 (relaxed agent-scope atomics lower to exactly that) -- the producer's
// lines written through, the consumer's read past its CU's L1 and its XCD's L2 state, the
// placement-independent hand-off of MI355X_MICROARCH.md §Workgroup dispatch (sc1 stores, vmcnt(0),
// sc1 flag; sc1 poll, sc1 loads).  `sc1` is wave-uniform.
__device__ __forceinline__ uint32_t col_ld(uint8_t* p, bool sc1) { return ld32(p); }
__device__ __forceinline__ void col_st(uint8_t* p, uint32_t v, bool sc1) { st32(p, v); }
__device__ __forceinline__ uint32_t col_ld(gptr<uint8_t> p, bool sc1) {
  if (sc1) return __hip_atomic_load((gptr<uint32_t>)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *(gptr<const uint32_t>)p;
}
__device__ __forceinline__ void col_st(gptr<uint8_t> p, uint32_t v, bool sc1) {
  if (sc1) __hip_atomic_store((gptr<uint32_t>)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *(gptr<uint32_t>)p = v;
}

// 32-bit wrapping MUL1/MUL2 (dsp.h.go WEBP_TRANSFORM_AC3_MUL1/2).  |a| < 2^23 for any
// int16 input, so the 24-bit multiplier gives the exact low 32 bits of a*c.
__device__ __forceinline__ int mul1(int a) { return (__mul24(a, 20091) >> 16) + a; }
__device__ __forceinline__ int mul2(int a) { return __mul24(a, 35468) >> 16; }


// 4x4 transpose across a lane quad (lane q holds row q in t[0..3], ends with column q):
// two DPP exchange stages, each pair as two v_cndmask_b32_dpp (the swapped operand through
// DPP, the kept one selected by a lane-parity mask in VCC) -- 8 VALU instead of 4 DPP moves
// plus 12 selects.  Hardware hazard: DPP reading a VGPR written by the previous VALU needs
// two wait states (the leading s_nop 1; the second stage's inputs are >= 2 instructions
// old).  Checked on the device by scripts/probes/quad_transpose.hip.
__device__ __forceinline__ void quad_transpose(int t[4]) {
  int n0, n1, n2, n3, m0, m1, m2, m3;
  asm volatile(
      "s_nop 1\n\t"
      "s_mov_b32 vcc_lo, 0xaaaaaaaa\n\ts_mov_b32 vcc_hi, 0xaaaaaaaa\n\t"
      "v_cndmask_b32_dpp %1, %8, %9, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %3, %10, %11, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "s_mov_b32 vcc_lo, 0x55555555\n\ts_mov_b32 vcc_hi, 0x55555555\n\t"
      "v_cndmask_b32_dpp %0, %9, %8, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %2, %11, %10, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "s_mov_b32 vcc_lo, 0xcccccccc\n\ts_mov_b32 vcc_hi, 0xcccccccc\n\t"
      "v_cndmask_b32_dpp %6, %0, %2, vcc quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %7, %1, %3, vcc quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "s_mov_b32 vcc_lo, 0x33333333\n\ts_mov_b32 vcc_hi, 0x33333333\n\t"
      "v_cndmask_b32_dpp %4, %2, %0, vcc quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %5, %3, %1, vcc quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf"
      : "=&v"(n0), "=&v"(n1), "=&v"(n2), "=&v"(n3), "=&v"(m0), "=&v"(m1), "=&v"(m2), "=&v"(m3)
      : "v"(t[0]), "v"(t[1]), "v"(t[2]), "v"(t[3])
      : "vcc");
  t[0] = m0;
  t[1] = m1;
  t[2] = m2;
  t[3] = m3;
}

// TransformOne (dec.c.go:49-88) of a 4x4 block spread over a lane quad.  In: column q of
// the coefficients (c0..c3 = in[q], in[4+q], in[8+q], in[12+q]) and `dadd`, the block's DC
// from the Y2 transform (0 unless i16 luma): in[0] enters the vertical pass of column 0 only
// as a common term of its four outputs, i.e. every row's tmp[0 + row], so it is added where
// the horizontal pass reads that term.  Out: residuals (v >> 3) of pixel row q, x = 0..3.
__device__ __forceinline__ void idct_quad(int q, uint2 cv, int dadd, int r[4]) {
  const int c0 = (int16_t)(cv.x & 0xffff), c1 = (int16_t)(cv.x >> 16);
  const int c2 = (int16_t)(cv.y & 0xffff), c3 = (int16_t)(cv.y >> 16);
  int t[4];
  {
    const int a = c0 + c2;
    const int b = c0 - c2;
    const int c = mul2(c1) - mul1(c3);
    const int d = mul1(c1) + mul2(c3);
    t[0] = a + d;
    t[1] = b + c;
    t[2] = b - c;
    t[3] = a - d;
  }
  quad_transpose(t);  // lane q ends with t[c] = tmp[4q + c]
  const int dc = t[0] + 4 + dadd;
  const int a = dc + t[2];
  const int b = dc - t[2];
  const int c = mul2(t[1]) - mul1(t[3]);
  const int d = mul1(t[1]) + mul2(t[3]);
  r[0] = (a + d) >> 3;
  r[1] = (b + c) >> 3;
  r[2] = (b - c) >> 3;
  r[3] = (a - d) >> 3;
}

// Residuals of one IDCT pass (6 per MB step: luma blocks b0, b0+8 and chroma, for both
// roles).  When every block in the pass (all four MBs) is zero or DC-only, TransformOne
// reduces to (in[0] + 4) >> 3 on every pixel (TransformDC, dec.c.go:112-118): broadcast
// the DC from the quad's column-0 lane instead of running both butterfly passes.  An i16
// block's stored in[0] is 0 (its DC is dadd, from Y2), any other block's dadd is 0.
__device__ __forceinline__ void idct_pass(int q, uint2 cv, int dadd, int r[4]) {
  const uint32_t ac = (q == 0 ? (cv.x & 0xffff0000u) : cv.x) | cv.y;
  if (__all(ac == 0)) {
    const int dc = __builtin_amdgcn_mov_dpp((int)(int16_t)(cv.x & 0xffff), 0x00, 0xF, 0xF, true) + dadd;
    r[0] = r[1] = r[2] = r[3] = (dc + 4) >> 3;
  } else {
    idct_quad(q, cv, dadd, r);
  }
}

// TransformWHT (dec.c.go:142-167; called from ParseResiduals, vp8_dec.go:615-634) of the
// MB's Y2 block, computed by every lane quad of the MB's 16 lanes: lane q holds column q of
// Y2 (the same layout as the IDCT).  Vertical pass, quad transpose, horizontal pass: lane q
// then holds row q of the 4x4 matrix of Y DCs (row = block row by, element = block column
// bx), stored as int16 like libwebp's.  Lane (p, q), p = m >> 2, keeps element p, and the
// quad broadcasts give every lane DC[by][p] for by = 0..3: its roles' luma blocks p + 4s
// (row s) and p + 4s + 8 (row s + 2) read dc[s] and dc[s + 2].
__device__ __forceinline__ void wht_quad(int p, uint2 cv, int dc[4]) {
  const int c0 = (int16_t)(cv.x & 0xffff), c1 = (int16_t)(cv.x >> 16);
  const int c2 = (int16_t)(cv.y & 0xffff), c3 = (int16_t)(cv.y >> 16);
  int t[4];
  {
    const int a0 = c0 + c3, a1 = c1 + c2, a2 = c1 - c2, a3 = c0 - c3;
    t[0] = a0 + a1;  // tmp[0 + q]
    t[1] = a3 + a2;  // tmp[4 + q]
    t[2] = a0 - a1;  // tmp[8 + q]
    t[3] = a3 - a2;  // tmp[12 + q]
  }
  quad_transpose(t);  // lane q: t[c] = tmp[4q + c]
  const int d0 = t[0] + 3;
  const int a0 = d0 + t[3], a1 = t[1] + t[2], a2 = t[1] - t[2], a3 = d0 - t[3];
  const int e = p == 0 ? a0 + a1 : p == 1 ? a3 + a2 : p == 2 ? a0 - a1 : a3 - a2;
  const int v = (int16_t)(e >> 3);
  dc[0] = __builtin_amdgcn_mov_dpp(v, 0x00, 0xF, 0xF, true);  // quad_perm [0,0,0,0]
  dc[1] = __builtin_amdgcn_mov_dpp(v, 0x55, 0xF, 0xF, true);  // [1,1,1,1]
  dc[2] = __builtin_amdgcn_mov_dpp(v, 0xAA, 0xF, 0xF, true);  // [2,2,2,2]
  dc[3] = __builtin_amdgcn_mov_dpp(v, 0xFF, 0xF, 0xF, true);  // [3,3,3,3]
}

// clamp(a..d, 0, 255) packed little-endian into one dword with gfx950's v_ashr_pk_u8_i32
// (D[15:0] = sat_u8(S1 >> S2) << 8 | sat_u8(S0 >> S2), D[31:16] kept; measured by
// scripts/probes/ashr_pk.hip): the high pair first, shifted up, then the low pair written
// under it -- three instructions instead of four v_med3 and three v_lshl_or.
__device__ __forceinline__ uint32_t pack_sat4(int a, int b, int c, int d) {
  uint32_t hi, out;
  asm("v_ashr_pk_u8_i32 %0, %1, %2, 0" : "=v"(hi) : "v"(c), "v"(d));
  out = hi << 16;
  asm("v_ashr_pk_u8_i32 %0, %1, %2, 0" : "+v"(out) : "v"(a), "v"(b));
  return out;
}

__device__ __forceinline__ uint32_t add_res(uint32_t pred, const int r[4]) {
  return pack_sat4(byte_of(pred, 0) + r[0], byte_of(pred, 1) + r[1], byte_of(pred, 2) + r[2],
                   byte_of(pred, 3) + r[3]);
}

__device__ __forceinline__ int check_mode(int mb_x, int mb_y, int mode) {  // frame_dec.c.go:28-37
  if (mode == 0) {
    if (mb_x == 0) return mb_y == 0 ? 6 : 5;
    return mb_y == 0 ? 4 : 0;
  }
  return mode;
}

// One pixel row of the 16x16 luma / 8x8 chroma predictors (DC*, TM, VE, HE;
// dec.c.go:178-249, 422-474) selected by bits of a one-hot mode mask (oh = 1 << mode): a
// chain of `mode == k` tests becomes a switch lowered to a branch tree, bit tests stay
// v_cndmask.  TrueMotion is only computed when some lane of the wave needs it.
__device__ __forceinline__ uint32_t pred_row(uint32_t oh, uint32_t top, int left, int tl, int dc) {
  uint32_t tm = 0;
  if (__any(oh & 0x2))
    tm = pack_sat4(byte_of(top, 0) + left - tl, byte_of(top, 1) + left - tl, byte_of(top, 2) + left - tl,
                   byte_of(top, 3) + left - tl);
  const uint32_t v = (oh & 0x4) ? top : bcast((uint32_t)dc);  // VE : DC variants
  const uint32_t w = (oh & 0x8) ? bcast((uint32_t)left) : tm;  // HE : TM
  return (oh & 0xA) ? w : v;
}

// DC value by one-hot mode: DC (0) both edges, DC_NOTOP (4) left only, DC_NOLEFT (5) top
// only, DC_NOTOPLEFT (6) 0x80.  `shift` = log2(edge length).
__device__ __forceinline__ int dc_value(uint32_t oh, uint32_t st, uint32_t sl, int shift) {
  const int both = (int)(st + sl + (1u << shift)) >> (shift + 1);
  const int lonly = (int)(sl + (1u << (shift - 1))) >> shift;
  const int tonly = (int)(st + (1u << (shift - 1))) >> shift;
  const int a = (oh & 0x10) ? lonly : tonly;
  const int b = (oh & 0x1) ? both : 0x80;
  return (oh & 0x30) ? a : b;
}

// ---------------------------------------------------------------- loop filter
struct Line { int p3, p2, p1, p0, q0, q1, q2, q3; };

__device__ __forceinline__ int sclip1(int v) { return min(max(v, -128), 127); }
__device__ __forceinline__ int sclip2(int v) { return min(max(v, -16), 15); }

// |a - b| (+ c) for byte values (0..255) in one v_sad_u8 (sub/neg/max otherwise); a builtin,
// not inline asm, so the hazard recognizer sees it (no conservative s_nop after each).
__device__ __forceinline__ int absd(int a, int b, int c = 0) {
  return (int)__builtin_amdgcn_sad_u8((uint32_t)a, (uint32_t)b, (uint32_t)c);
}

// KIND 0: simple (NeedsFilter + DoFilter2, dec.c.go:552-586);
// KIND 1: complex MB edge (FilterLoop26: hev ? DoFilter2 : DoFilter6, :592-606);
// KIND 2: complex inner edge (FilterLoop24: hev ? DoFilter2 : DoFilter4, :608-622).
// The masks are computed for every line; the complex kinds then update the samples under the
// lane mask of the lines that filter (see below).  t2 = 2*thresh + 1.
template <int KIND>
__device__ __forceinline__ void filter_line(Line& l, int t2, int it, int hev_t) {
  const int d0 = l.q0 - l.p0;
  const int sp = sclip1(l.p1 - l.q1);
  const bool edge_ok = absd(l.p1, l.q1, 4 * absd(l.p0, l.q0)) <= t2;
  // DoFilter2 (24-bit multiplies: a 32-bit 3*d0 + sp became a quarter-rate v_mad_u64_u32)
  const int a = __mul24(d0, 3) + sp;
  auto f2p0 = [&] { return clamp255(l.p0 + sclip2((a + 3) >> 3)); };
  auto f2q0 = [&] { return clamp255(l.q0 - sclip2((a + 4) >> 3)); };
  if (KIND == 0) {
    const int np0 = f2p0(), nq0 = f2q0();
    l.p0 = edge_ok ? np0 : l.p0;
    l.q0 = edge_ok ? nq0 : l.q0;
    return;
  }
  const int dp = absd(l.p1, l.p0), dq = absd(l.q1, l.q0);
  const int in_p = max(max(absd(l.p3, l.p2), absd(l.p2, l.p1)), dp);
  const int in_q = max(max(absd(l.q3, l.q2), absd(l.q2, l.q1)), dq);
  const bool on = edge_ok & (max(in_p, in_q) <= it);  // & not &&: no short-circuit branch
  const bool hv = max(dp, dq) > hev_t;
  const bool f2 = on & hv, fx = on & !hv;
#ifndef WG_FILTER_SELECT  // (measurement build: the round-3 select form)
  // Exec-masked updates instead of selects: the new values are written under the lane mask of
  // the lines that filter, so no v_cndmask per sample (a "complex" op: twice the issue cost of
  // a plain one) -- the mask costs a few scalar instructions per region instead.  The empty asm
  // keeps each region a branch (the compiler would flatten it back into selects).
  if (KIND == 1) {  // DoFilter6, or DoFilter2 on hev lines
    if (on) {
      asm volatile("");
      if (hv) {  // (DoFilter2 computed only where some line of the wave needs it)
        asm volatile("");
        const int np0 = f2p0(), nq0 = f2q0();
        l.p0 = np0;
        l.q0 = nq0;
      } else {
        asm volatile("");
        const int w = sclip1(a);
        const int a1 = (__mul24(w, 27) + 63) >> 7, a2 = (__mul24(w, 18) + 63) >> 7, a3 = (__mul24(w, 9) + 63) >> 7;
        l.p2 = clamp255(l.p2 + a3);
        l.p1 = clamp255(l.p1 + a2);
        l.p0 = clamp255(l.p0 + a1);
        l.q0 = clamp255(l.q0 - a1);
        l.q1 = clamp255(l.q1 - a2);
        l.q2 = clamp255(l.q2 - a3);
      }
    }
  } else {
    if (on) {
      asm volatile("");
      int a = __mul24(d0, 3);
      if (hv) {  // (the hev term added under the lane mask: no select)
        asm volatile("");
        a += sp;
      }
      const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3), a3 = (a1 + 1) >> 1;
      l.p0 = clamp255(l.p0 + a2);
      l.q0 = clamp255(l.q0 - a1);
      if (!hv) {
        asm volatile("");
        l.p1 = clamp255(l.p1 + a3);
        l.q1 = clamp255(l.q1 - a3);
      }
    }
  }
  (void)f2;
  (void)fx;
#else
  if (KIND == 1) {  // DoFilter6
    const int w = sclip1(a);
    const int a1 = (__mul24(w, 27) + 63) >> 7, a2 = (__mul24(w, 18) + 63) >> 7, a3 = (__mul24(w, 9) + 63) >> 7;
    const int np2 = clamp255(l.p2 + a3), np1 = clamp255(l.p1 + a2), np0 = clamp255(l.p0 + a1);
    const int nq0 = clamp255(l.q0 - a1), nq1 = clamp255(l.q1 - a2), nq2 = clamp255(l.q2 - a3);
    l.p2 = fx ? np2 : l.p2;
    l.p1 = fx ? np1 : l.p1;
    l.q1 = fx ? nq1 : l.q1;
    l.q2 = fx ? nq2 : l.q2;
    const int g0 = f2p0(), h0 = f2q0();
    l.p0 = fx ? np0 : (f2 ? g0 : l.p0);
    l.q0 = fx ? nq0 : (f2 ? h0 : l.q0);
  } else {  // DoFilter4, or DoFilter2 on hev lines: both are p0 += sclip2((a+3)>>3),
            // q0 -= sclip2((a+4)>>3) with a = 3*(q0-p0) [+ sclip1(p1-q1) when hev]
    const int a = __mul24(d0, 3) + (hv ? sp : 0);
    const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3), a3 = (a1 + 1) >> 1;
    const int np0 = clamp255(l.p0 + a2), nq0 = clamp255(l.q0 - a1);
    const int np1 = clamp255(l.p1 + a3), nq1 = clamp255(l.q1 - a3);
    l.p1 = fx ? np1 : l.p1;
    l.q1 = fx ? nq1 : l.q1;
    l.p0 = on ? np0 : l.p0;
    l.q0 = on ? nq0 : l.q0;
  }
#endif
}

// One edge on eight consecutive samples v[0..7] = p3..q3 held in registers.
template <int KIND>
__device__ __forceinline__ void filter_at(int* v, int t2, int it, int ht) {
  Line l{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
  filter_line<KIND>(l, t2, it, ht);
  v[1] = l.p2;
  v[2] = l.p1;
  v[3] = l.p0;
  v[4] = l.q0;
  v[5] = l.q1;
  v[6] = l.q2;
}

// One line of DoFilter (frame_dec.c.go:204-251): the lane's window row (vertical edges,
// the left MB edge first) or column (kCol: horizontal edges, the top MB edge first) of
// luma (-4..15, edges at 0, 4, 8, 12) or chroma (-4..7, edges at 0, 4), loaded once, every
// edge in registers, stored back.  Single-byte LDS accesses: the LDS unit zero-extends and
// narrows, so the (issue-bound) wave spends no instructions unpacking and repacking.
template <bool kComplex, bool kLuma, bool kCol>
__device__ __forceinline__ void filter_line_pass(uint8_t* win, int li, bool f_mb, bool fin, int limit, int ilevel,
                                                 int hev_t) {
  constexpr int KMB = kComplex ? 1 : 0, KIN = kComplex ? 2 : 0;
  constexpr int st = kLuma ? FWY : FWC;
  constexpr int n = kLuma ? 20 : 12;
  constexpr int step = kCol ? st : 1;
  const int t_mb = 2 * (limit + 4) + 1, t_in = 2 * limit + 1;
  // volatile: kept as single-byte accesses, not merged back into dwords + shifts
  volatile __attribute__((address_space(3))) uint8_t* p =
      (__attribute__((address_space(3))) uint8_t*)(kCol ? win + 4 + li : win + (li + 4) * st);
  int v[n];
#pragma unroll
  for (int k = 0; k < n; ++k) v[k] = p[k * step];
  if (f_mb) filter_at<KMB>(v + 0, t_mb, ilevel, hev_t);  // {H,V}Filter16 / {H,V}Filter8 / Simple{H,V}Filter16
  if (fin) {
    filter_at<KIN>(v + 4, t_in, ilevel, hev_t);  // {H,V}Filter16i / {H,V}Filter8i
    if (kLuma) {
      filter_at<KIN>(v + 8, t_in, ilevel, hev_t);
      filter_at<KIN>(v + 12, t_in, ilevel, hev_t);
    }
  }
#pragma unroll
  for (int k = 1; k < n - 1; ++k) p[k * step] = (uint8_t)v[k];
}

// DoFilter (frame_dec.c.go:204-251) for the lane group's MB, libwebp edge order (left MB
// edge, inner vertical edges, top MB edge, inner horizontal edges): lane m filters luma line
// m and -- complex filter only -- chroma line m & 7 of U (m < 8) / V (m >= 8).
template <bool kComplex>
__device__ __forceinline__ void filter_mb(uint8_t* fw, int m, bool on, bool fx, bool fy, bool fin, int limit,
                                          int ilevel, int hev_t) {
  uint8_t* wy = fw + kFwY;
  uint8_t* wc = fw + (m >= 8 ? kFwV : kFwU);
  const int mc = m & 7;
  if (on) {
    filter_line_pass<kComplex, true, false>(wy, m, fx, fin, limit, ilevel, hev_t);
    if (kComplex) filter_line_pass<true, false, false>(wc, mc, fx, fin, limit, ilevel, hev_t);
  }
  lds_sync();
  if (on) {
    filter_line_pass<kComplex, true, true>(wy, m, fy, fin, limit, ilevel, hev_t);
    if (kComplex) filter_line_pass<true, false, true>(wc, mc, fy, fin, limit, ilevel, hev_t);
  }
  lds_sync();
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// MB record of (x, y); out-of-frame positions read as all-zero through the buffer range
// check (no branch, 32-bit offsets instead of 64-bit address arithmetic).
__device__ __forceinline__ MbRec load_rec(__amdgpu_buffer_rsrc_t recs, int mb_w, int y, bool row_ok, int x) {
  const bool ok = row_ok && x >= 0 && x < mb_w;
  const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(recs, ok ? (y * mb_w + x) * 16 : (int)kDrop, 0, 0);
  return MbRec{r.x, r.y, r.z, r.w};
}

struct Coefs { uint2 y0, y1, c; };

// Column q of non-zero block `bi` (16 int16 = 32 B per block, column-major); a zero block
// reads as zeros through the range check.
__device__ __forceinline__ uint2 ld_blockcol(__amdgpu_buffer_rsrc_t blks, bool nz, uint32_t bi, int q) {
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(blks, nz ? (int)(bi * 32 + 8 * q) : (int)kDrop, 0, 0);
  return make_uint2(v.x, v.y);
}

// The MB's blocks start at `blk`: its Y2 block first when kY2Bit is set, then the kept
// Y / U / V blocks in order (device_format.h).
__device__ __forceinline__ Coefs load_coefs(__amdgpu_buffer_rsrc_t blks, uint32_t flags, uint32_t blk, int b0, int cb,
                                            int q) {
  const uint32_t nz = flags & kNzMask;
  const uint32_t base = blk + ((flags & kY2Bit) ? 1u : 0u);
  Coefs c;
  c.y0 = ld_blockcol(blks, (nz >> b0) & 1, base + __builtin_popcount(nz & ((1u << b0) - 1)), q);
  c.y1 = ld_blockcol(blks, (nz >> (b0 + 8)) & 1, base + __builtin_popcount(nz & ((1u << (b0 + 8)) - 1)), q);
  c.c = ld_blockcol(blks, (nz >> cb) & 1, base + __builtin_popcount(nz & ((1u << cb) - 1)), q);
  return c;
}

// Bounded LDS spin (workgroup-scope acquire) until *p >= need; false after 2 s.  Used by the
// converting waves only: the longest sleep (127 x 64 cycles) leaves the most issue slots to
// the reconstructing waves (s_sleep 2 / 8 / 32 / 127 measured 9.44 / 9.27 / 9.26 / 9.22 ms).
__device__ __forceinline__ bool wait_at_least(uint32_t* p, uint32_t need) {
  if (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= need) return true;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
    __builtin_amdgcn_s_sleep(127);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) return false;
  }
  return true;
}

// K1's tail: the frame's YUV420 -> RGBA (K2's strip conversion, yuv_rgba_strip.h) done by
// the waves whose reconstruction work is over, while the last MB-row quads are still being
// decoded.  Units = (band, strip), claimed top-down from an LDS counter.  A band needs luma
// rows <= L and chroma rows <= C final: MB row m has published luma rows <= 16m + 12 and
// chroma rows <= 8m + 4 once its quad's progress reaches mb_w (rows 13-15 / 5-7 are written
// by the row below; the last MB row writes all).  One MB row of margin beyond that.  The
// last quad publishes no progress (no quad waits on it): its rows wait for every wave.
template <bool kFancy>
__device__ __forceinline__ void emit_tail(const FrameDesc& F, uint32_t* progress, uint32_t* recon_done,
                                          uint32_t* next_unit, int lane, int* err) {
  const int W = F.width, H = F.height, uv_h = (H + 1) >> 1, mb_w = F.mb_w, mb_h = F.mb_h;
  const int nquads = (mb_h + kRows - 1) / kRows;
  const int sx = strip::strips_x(W);
  const int npairs = kFancy ? (H >> 1) + 1 : (H + 1) >> 1;
  const int n_units = sx * ((npairs + strip::kPairs - 1) / strip::kPairs);
  for (;;) {
    uint32_t u = 0;
    if (lane == 0) u = __hip_atomic_fetch_add(next_unit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    u = __builtin_amdgcn_readfirstlane(u);
    if (u >= (uint32_t)n_units) return;
    const int band = (int)u / sx, tx = (int)u - band * sx;
    const int p1 = min((band + 1) * strip::kPairs, npairs);
    const int L = min(2 * p1 - 1, H - 1), C = min(p1 - 1, uv_h - 1);
    const int m = max(max((L + 3) >> 4, (C + 3) >> 3), 0) + 1;  // ceil((L-12)/16), ceil((C-4)/8), + margin
    const int qm = m / kRows;
    bool ok;
    if (m >= mb_h - 1 || qm >= nquads - 1) ok = wait_at_least(recon_done, kWaves);
    else ok = wait_at_least(progress + (qm & (kWaves - 1)), ((uint32_t)qm << 16) | (uint32_t)mb_w);
    if (!ok) {
      if (lane == 0) atomicOr(err, 1);
      return;
    }
    if (__builtin_amdgcn_readfirstlane(F.alpha_off16) != 0)  // (an alpha-first frame: RGBA, A from its plane)
      strip::convert_strip<kFancy, strip::kAuxSc1, strip::kModesRgba, true>(F, tx, band, lane);
    else
      strip::convert_strip<kFancy, strip::kAuxSc1, strip::kModesTail>(F, tx, band, lane);  // (RGBA / RGB_565 only)
  }
}

}  // namespace

// kGlobalCols: the per-MB-column store (kColBytes per column) lives in LDS when the frame's
// columns fit next to the workspaces (mb_w <= vp8_recon_max_mb_w()), else in a per-frame
// global buffer (FrameDesc::cols, wide frames up to VP8's 16383 px).  Each variant skips the
// other's frames.  The hand-offs through the store keep their ordering: within a wave (row
// 4k+g -> 4k+g+1) by the fences of lds_sync, across waves by the release/acquire progress
// counters -- at workgroup scope the AMDGPU memory model orders global accesses of one CU
// the same way (its L1 is shared by the workgroup), no extra s_waitcnt needed.
//
// kSplit (implies kGlobalCols): nparts workgroups per frame for batches of fewer frames than CUs.
// Part p reconstructs the quads [pR, pR + R) -- one quad per reconstructing wave, the frame in
// nparts horizontal slabs of 4R MB rows -- so a frame's wavefront runs on nparts CUs instead of
// one (a lone 4K frame: 34 quads on 3 CUs).  Inside a part everything is as in the unsplit kernel;
// across a slab boundary the part's first quad waits on a progress flag the previous part's last
// quad publishes in global memory (FrameDesc::gprog, tagged with the launch's epoch), and both
// quads access the column store with sc1 (col_ld / col_st).  Dependencies only run from part p - 1
// to part p, and part p - 1's workgroup has the lower index (blocks are dispatched in order), so
// no part waits on a part that cannot be running.  No RGBA tail: a split batch converts in K2.
// A frame taller than nparts * R quads runs on part 0 alone.
template <bool kGlobalCols, bool kSplit>
__global__ void __launch_bounds__(1024) vp8_recon_filter_kernel(const FrameDesc* __restrict__ frames, int* err,
                                                                int lead_arg, int recon_waves_arg, int n_frames,
                                                                int nparts, uint32_t epoch) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  // Progress counters as a typed __shared__ array + relaxed workgroup atomics, so the spin
  // is a ds_read (lgkmcnt) -- a volatile generic pointer became a flat load whose
  // vmcnt(0) drained the record/coefficient prefetch every MB.
  __shared__ uint32_t progress[kWaves];
  __shared__ uint32_t recon_done, next_unit;  // K1 tail (emit_tail): waves done, units claimed
  static_assert(!kSplit || kGlobalCols, "the split kernel keeps the column store in global memory");
  int fidx = blockIdx.x, part = 0;
  if constexpr (kSplit) {
    // blocks b and b + 8 -- one XCD under the observed round-robin dealing, a matter of speed only
    // (the hand-off is placement independent) -- are parts of one frame
    const int b = blockIdx.x;
    fidx = (b / (8 * nparts)) * 8 + (b & 7);
    part = (b >> 3) % nparts;
    if (fidx >= n_frames) return;
  }
  const FrameDesc* F = frames + fidx;
  if (!F->valid) return;
  if constexpr (!kSplit)
    if (((F->flags & kFrameGlobalCols) != 0) != kGlobalCols) return;
  const int mb_w = F->mb_w, mb_h = F->mb_h;
  const int ftype = F->filter_type;
  const int ys = F->y_stride, uvs = F->uv_stride;
  const gptr<const uint32_t> row_block0 = as_global(F->row_block0);
  // Buffer descriptors: out-of-range loads return 0 and out-of-range stores are dropped.
  const __amdgpu_buffer_rsrc_t recs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<MbRec*>(F->mbs), 0, mb_w * mb_h * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t blks =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t*>(F->blocks), 0, F->blocks_bytes, 0x00020000);
  // One buffer descriptor over the frame's planes: the batch allocates Y, U, V of a frame
  // back to back (capi.cpp), so U and V are 32-bit offsets from Y.
  const uint32_t uoff = (uint32_t)(F->u - F->y), voff = (uint32_t)(F->v - F->y);
  const __amdgpu_buffer_rsrc_t planes =
      __builtin_amdgcn_make_buffer_rsrc(F->y, 0, (int)(voff + (uint32_t)(8 * mb_h * uvs)), 0x00020000);

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // SGPR: k and the quad loop stay uniform
  const int lane = threadIdx.x & 63;
  K1_SECT_DECL();
  // Required lead of the previous quad's last row, in MB columns: 2 (top-right samples and
  // the left-edge filter of MB (x+1, y-1) reach one MB up-right).  Larger leads were
  // measured slower (round 1, pairs): waves held back at start-up idle while the running
  // ones gain nothing.
  const int lead = max(2, lead_arg);
  const int g = lane >> 4;  // MB row of the quad this lane decodes
  uint32_t* tab = reinterpret_cast<uint32_t*>(lds + kProgBytes);
  using ColPtr = std::conditional_t<kGlobalCols, gptr<uint8_t>, uint8_t*>;
  ColPtr cols;
  if constexpr (kGlobalCols) cols = as_global(F->cols);
  else cols = lds + kHdrBytes + kMaxRecon * kRows * kSlotBytes;
  // per MB column c: cols + c*kColBytes: [0..15] ytop Y, [16..23] U, [24..31] V, [32..159] fbot
  if (threadIdx.x < kWaves) progress[threadIdx.x] = 0;
  if (threadIdx.x == 0) recon_done = next_unit = 0;
  const bool emit = !kSplit && (F->flags & kFrameEmitRgba);
  if (emit) __builtin_amdgcn_s_setprio(2);  // reconstruction is the critical path; the tail's conversion yields
  const int nquads = (mb_h + kRows - 1) / kRows;
  // Waves that reconstruct (quads k = wave, wave + R, ...); with the RGBA tail the others
  // convert bands from the start.  R <= kMaxRecon (the LDS slots) also keeps the progress
  // ring safe: quad k + 16 only starts on a wave that has completed a quad > k, so quad k
  // is complete whenever its slot holds a later quad's value.
  const int R = recon_waves_arg > 0 ? min(recon_waves_arg, kMaxRecon) : kMaxRecon;
  // split: the frame in slabs (one quad per reconstructing wave) when it has at most nparts * R
  // quads; parts without quads, and every part but 0 of a taller frame, leave (whole workgroups,
  // before any barrier)
  bool slabs = false;
  if constexpr (kSplit) {
    slabs = nquads <= nparts * R;
    if (slabs ? part * R >= nquads : part > 0) return;
  }
  const gptr<uint32_t> gprog = as_global(F->gprog);
  for (int t = threadIdx.x; t < 160; t += blockDim.x) tab[t] = kPred4Table[t];
  K1_TIMELINE_START();
  __syncthreads();

  bool aborted = false;  // a progress wait timed out (error flagged): stop waiting
  const int k0 = slabs ? part * R + wave : wave;
  const int kend = slabs ? min(nquads, part * R + R) : nquads;
  for (int k = k0; wave < R && k < kend; k += R) {
    const int y = kRows * k + g;
    const bool row_ok = y < mb_h;
    const bool has_next = kRows * (k + 1) < mb_h;  // a later quad waits on this one's last row
    const bool last_row = y == mb_h - 1;
    // split slabs: the part's first quad waits on the previous part's last, which publishes its
    // progress to global memory; both access the column store agent-coherently (sc1)
    const bool g_wait = kSplit && slabs && part > 0 && k == part * R;
    const bool g_pub = kSplit && slabs && k == part * R + R - 1 && has_next;
    const bool csc1 = g_wait || g_pub;
    uint32_t gseen = 0;  // the previous part's published progress last read (g_wait)
    uint32_t blk = row_ok ? row_block0[y] : 0u;
    MbRec rc = load_rec(recs, mb_w, y, row_ok, -2 * g);
    MbRec rn = load_rec(recs, mb_w, y, row_ok, -2 * g + 1);
    Coefs cc[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int r = (lane & 15) + 16 * s;
      cc[s] = load_coefs(blks, rc.flags, blk, r >> 2, 16 + (r >> 2), r & 3);
    }
    uint2 y2c = ld_blockcol(blks, (rc.flags & kY2Bit) != 0, blk, lane & 3);  // Y2 column (i16 MBs)
    // Retire the prologue loads here (visible to the waitcnt pass: 0x0F70 = vmcnt(0)), so the
    // loop header has no pending loads on cc/rc/rn and the in-loop uses of cc do not
    // conservatively drain the NEXT MB's prefetch with a vmcnt(0).
    __builtin_amdgcn_s_waitcnt(0x0F70);
    uint32_t top_carry = 0;  // see "top samples"
    // Plane offsets (at MB column 0) of the lane's two row-segment stores, once per quad (see
    // "final pixels to HBM"); per MB only `x << 4` / `x << 3` is added.  Luma: lanes 0..12
    // row m, cols -4..11; lanes 13..15 rows 13..15 of the MB above, cols 0..15.  Chroma
    // (U lanes 0..7, V 8..15): rows 0..4 cols -4..3; lanes 5..7 rows 5..7 above, cols 0..7.
    // Rows above exist for y > 0 only: kDrop + 16x stays beyond the planes.
    uint32_t sb_y, sb_c;
    {
      int lid0;  // (opaque, like the loop's lane roles: lane-constant terms hoisted out of the quad loop spilled)
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid0));
      const int m0 = lid0 & 15, rc = m0 & 7;
      // (minus 4: the per-MB offset adds the segment's window column, 0 or 4)
      sb_y = m0 >= 13 ? (y > 0 ? (uint32_t)__mul24(16 * y - 16 + m0, ys) - 4u : kDrop)
                      : (uint32_t)__mul24(16 * y + m0, ys) - 4u;
      const uint32_t cp = m0 >= 8 ? voff : uoff;
      sb_c = rc >= 5 ? (y > 0 ? cp + (uint32_t)__mul24(8 * y - 8 + rc, uvs) - 4u : kDrop)
                     : cp + (uint32_t)__mul24(8 * y + rc, uvs) - 4u;
    }

    K1_SECT_START();
    K1_QUAD_MARK(k, 0);
    uint32_t seen = 0;  // progress of quad k - 1 last read (wave-uniform)

    for (int i = 0; i < mb_w + 2 * (kRows - 1); ++i) {
      // Lane roles, recomputed every iteration from an opaque lane id: hoisted out of the
      // loop, the lane-constant LDS addresses derived from them spill (rule from
      // cdna_hip_programming.md: recompute per block with v_mbcnt).
      int lid;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
      const int m = lid & 15;
      const int gg = lid >> 4;
      uint8_t* ws = lds + kHdrBytes + __mul24(wave * kRows + gg, kSlotBytes);  // recon workspace (libwebp yuv_b)
      uint8_t* fw = ws + kWsBytes;                                        // filter window
      uint8_t* left = fw + kFwBytes;                                      // unfiltered left columns
      int16_t* res = reinterpret_cast<int16_t*>(left + kLeftBytes);        // i4x4 residuals
      const int q = m & 3;
      const int x = i - 2 * gg;
      const bool act = row_ok && x >= 0 && x < mb_w;
      const bool last_x = x == mb_w - 1;
      K1_SECT(13);
      // ---- software pipeline: record x+2 in flight during MB x; the coefficients of x+1 are
      //      loaded into cc as soon as the IDCT has consumed x's (below)
      const MbRec rnn = load_rec(recs, mb_w, y, row_ok, x + 2);
      const uint32_t blk_next = blk + __builtin_popcount(rc.flags & (kNzMask | kY2Bit));

      K1_SECT(0);
      // ---- wait for the previous quad's last row (t = x + 2y wavefront)
      //      The counter is read into an SGPR (readfirstlane) so the spin is a scalar branch,
      //      and the timeout does not leave the loop: any path reaching the loop latch without
      //      this iteration's plane stores makes the waitcnt pass extend the latch's prefetch
      //      wait over those stores (a vmcnt that waits for store acks every MB).
      if (g_wait && i < mb_w) {
        // the flag: epoch << 16 | columns the previous part's last row has completed (sc1 poll;
        // a flag of an earlier launch reads as 0)
        const uint32_t gneed = (uint32_t)min(i + lead, mb_w);
        const gptr<uint32_t> gf = gprog + 32 * (part - 1);
        auto gcur = [&] {
          const uint32_t v =
              __builtin_amdgcn_readfirstlane(__hip_atomic_load(gf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          return (v >> 16) == (epoch & 0xffffu) ? (v & 0xffffu) : 0u;
        };
        if (!aborted && gseen < gneed && (gseen = gcur()) < gneed) {
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          for (;;) {
            __builtin_amdgcn_s_sleep(8);
            if ((gseen = gcur()) >= gneed) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s: give up, flag
              if (lane == 0) atomicOr(err, 1);
              aborted = true;
              break;
            }
          }
        }
        // Compiler barrier: the relaxed sc1 column-store loads below must not be moved above the
        // relaxed poll (the hardware orders them: the poll's value is waited for and branched on
        // before they issue).  tests/test_k1_isa.py checks the machine code at this marker.
        asm volatile("; wg-gprog-polled" ::: "memory");
      } else if (k > 0 && i < mb_w) {
        const uint32_t need = ((uint32_t)(k - 1) << 16) | (uint32_t)min(i + lead, mb_w);
        uint32_t* pr = progress + ((k - 1) & (kWaves - 1));
        auto cur = [&] {
          return __builtin_amdgcn_readfirstlane(__hip_atomic_load(pr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
        };
        // (the last value read, kept in an SGPR: while the previous quad is further ahead than this
        // step needs, no LDS read and no wait for it -- the acquire that returned it already
        // ordered the data of every column it covers)
        if (!aborted && seen < need && (seen = cur()) < need) {
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          for (;;) {
            __builtin_amdgcn_s_sleep(4);
            if ((seen = cur()) >= need) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s: give up, flag
              // no exit from the loop here (an exit path skipping the stores would reach the
              // latch too): the wave runs on without waiting and the batch reports the error
              if (lane == 0) atomicOr(err, 1);
              aborted = true;
              break;
            }
          }
        }
      }
      const uint32_t fl = rc.flags;
      const bool i4 = (fl >> kI4Shift) & 1;
      const ColPtr col = cols + __mul24(x, kColBytes);

      K1_SECT(1);
      // ---- ReconstructRow prologue at the row's first MB (frame_dec.c.go:79-98)
      if (act && x == 0) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int l = m + 16 * s;
          if (l < 16) ws[Y_OFF + l * BPS - 1] = 129;
          else if (l < 24) ws[U_OFF + (l - 16) * BPS - 1] = 129;
          else ws[V_OFF + (l - 24) * BPS - 1] = 129;
          left[l] = 129;
          if (y > 0) {
            if (l == 0) ws[Y_OFF - BPS - 1] = 129;
            if (l == 1) ws[U_OFF - BPS - 1] = 129;
            if (l == 2) ws[V_OFF - BPS - 1] = 129;
          } else {
            if (l < 21) ws[Y_OFF - BPS - 1 + l] = 127;
            if (l < 18) ws[(l < 9 ? U_OFF - BPS - 1 + l : V_OFF - BPS - 1 + (l - 9))] = 127;
            // row 0's top-right samples (127) replicated to rows 3, 7, 11 for i4 blocks;
            // nothing else writes those workspace bytes, so they hold for the whole MB row
            if (l >= 21 && l < 24) st32(ws + Y_OFF + (3 + 4 * (l - 21)) * BPS + 16, 0x7f7f7f7fu);
          }
        }
      }
      lds_sync();
      K1_SECT(2);
      // ---- top samples (frame_dec.c.go:122-142), lanes m < 9.  The top-left sample (row -1,
      //      col -1) is the previous column's top byte 15 (chroma: 7), which the current row
      //      has already overwritten in `cols`: lanes 3, 5, 7 carry it over from their
      //      previous load.
      if (act && y > 0) {
        if (m < 8) {
          const uint32_t tv = col_ld(col + 4 * m, csc1);
          st32(ws + (m < 4 ? Y_OFF - BPS + 4 * m : m < 6 ? U_OFF - BPS + 4 * (m - 4) : V_OFF - BPS + 4 * (m - 6)), tv);
          if (x > 0 && (m == 3 || m == 5 || m == 7))
            ws[(m == 3 ? Y_OFF : m == 5 ? U_OFF : V_OFF) - BPS - 1] = (uint8_t)(top_carry >> 24);
          top_carry = tv;
        } else if (m == 8 && i4) {
          // top-right samples, replicated down to rows 3, 7, 11 by the same lane (no read-back)
          const uint32_t tr = last_x ? bcast(col_ld(col + 12, csc1) >> 24) : col_ld(col + kColBytes, csc1);
          st32(ws + Y_OFF - BPS + 16, tr);
          st32(ws + Y_OFF + 3 * BPS + 16, tr);
          st32(ws + Y_OFF + 7 * BPS + 16, tr);
          st32(ws + Y_OFF + 11 * BPS + 16, tr);
        }
      }
      lds_sync();

      K1_SECT(3);
      // ---- residuals of all blocks (prediction-independent); i16 luma DCs from the Y2 WHT
      int ydc[4] = {0, 0, 0, 0};
      if (__any((fl & kY2Bit) != 0)) wht_quad(m >> 2, y2c, ydc);  // Y2 of i4 / no-Y2 MBs reads as 0: DCs 0
      int ry0[2][4], ry1[2][4], rcr[2][4];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#ifndef WG_ABL_IDCT
        idct_pass(q, cc[s].y0, ydc[s], ry0[s]);
        idct_pass(q, cc[s].y1, ydc[s + 2], ry1[s]);
        idct_pass(q, cc[s].c, 0, rcr[s]);
#else
        for (int t = 0; t < 4; ++t) ry0[s][t] = ry1[s][t] = rcr[s][t] = (int)(cc[s].y0.x + cc[s].y1.y + cc[s].c.x) >> 20;
#endif
      }

      // coefficients of x+1 into the registers the IDCT just freed: no rotation copies at the loop
      // latch (which waited there for these loads), and the loads are issued ahead of this step's
      // plane stores -- gfx950's single in-order vmcnt makes a load complete only after every
      // store issued before it, so issuing them here gives the previous step's stores more slack
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int r = m + 16 * s;
        cc[s] = load_coefs(blks, rn.flags, blk_next, r >> 2, 16 + (r >> 2), q);
      }
      y2c = ld_blockcol(blks, (rn.flags & kY2Bit) != 0, blk_next, q);
      K1_SECT(4);
      // ---- luma prediction + residual (role r: block column (r>>2)&3, pixel rows
      //      4*((r>>2)>>2)+q and that + 8)
#ifndef WG_ABL_PRED
      if (act && !i4) {
        const uint32_t oh = 1u << check_mode(x, y, (fl >> kYModeShift) & 3);
        const int tl = ws[Y_OFF - BPS - 1];
        uint32_t st = 0, sl = 0;
        if (__any(oh & 0x31)) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            st = __builtin_amdgcn_sad_u8(ld32(ws + Y_OFF - BPS + 4 * j), 0, st);
            sl = __builtin_amdgcn_sad_u8(ld32(left + 4 * j), 0, sl);
          }
        }
        const int dc = dc_value(oh, st, sl, 4);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int b0 = (m + 16 * s) >> 2, lbx = b0 & 3, lby = b0 >> 2;
          const int row_a = 4 * lby + q, row_b = row_a + 8;
          const uint32_t top = ld32(ws + Y_OFF - BPS + 4 * lbx);
          const uint32_t va = add_res(pred_row(oh, top, left[row_a], tl, dc), ry0[s]);
          const uint32_t vb = add_res(pred_row(oh, top, left[row_b], tl, dc), ry1[s]);
          st32(ws + Y_OFF + row_a * BPS + 4 * lbx, va);
          st32(ws + Y_OFF + row_b * BPS + 4 * lbx, vb);
          // (and straight into the filter window: no copy section)
          st32(fw + kFwY + (row_a + 4) * FWY + 4 + 4 * lbx, va);
          st32(fw + kFwY + (row_b + 4) * FWY + 4 + 4 * lbx, vb);
        }
      }
      if (act && i4) {  // stage residuals for the pixel-per-lane block walk
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int b0 = (m + 16 * s) >> 2;
          *reinterpret_cast<uint2*>(res + b0 * 16 + q * 4) =
              make_uint2((ry0[s][0] & 0xffff) | (ry0[s][1] << 16), (ry0[s][2] & 0xffff) | (ry0[s][3] << 16));
          *reinterpret_cast<uint2*>(res + (b0 + 8) * 16 + q * 4) =
              make_uint2((ry1[s][0] & 0xffff) | (ry1[s][1] << 16), (ry1[s][2] & 0xffff) | (ry1[s][3] << 16));
        }
      }
      // ---- chroma prediction + residual (role m + 16s: plane U for s = 0, V for s = 1; one
      //      pixel row of one 4x4 block); independent of the luma blocks, so it shares their
      //      section (one LDS hand-off less per MB)
      if (act) {
        const uint32_t oh = 1u << check_mode(x, y, (fl >> kUVModeShift) & 3);
        const int cbk = (m >> 2) & 3, cbx = cbk & 1, cby = cbk >> 1;
        const int row = 4 * cby + q;
        const bool any_dc = __any(oh & 0x31);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int coff = s ? V_OFF : U_OFF;
          const uint8_t* base = ws + coff;
          const uint8_t* cleft = left + 16 + 8 * s;
          uint32_t st = 0, sl = 0;
          if (any_dc) {
            st = __builtin_amdgcn_sad_u8(ld32(base - BPS), 0, 0);
            st = __builtin_amdgcn_sad_u8(ld32(base - BPS + 4), 0, st);
            sl = __builtin_amdgcn_sad_u8(ld32(cleft), 0, 0);
            sl = __builtin_amdgcn_sad_u8(ld32(cleft + 4), 0, sl);
          }
          const uint32_t pred =
              pred_row(oh, ld32(base - BPS + 4 * cbx), cleft[row], base[-BPS - 1], dc_value(oh, st, sl, 3));
          const uint32_t v = add_res(pred, rcr[s]);
          st32(ws + coff + row * BPS + 4 * cbx, v);
          st32(fw + (s ? kFwV : kFwU) + (row + 4) * FWC + 4 + 4 * cbx, v);
        }
      }
#endif
      lds_sync();
      K1_SECT(5);
#ifndef WG_ABL_I4
      if (__any(act && i4)) {
        // recipe words and residuals of all sixteen blocks fetched up front (independent loads)
        const uint32_t im_lo = rc.imodes_lo, im_hi = rc.imodes_hi;
        const int ppx = m & 3, ppy = m >> 2;
        uint32_t e[16];
        int rs[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int bi = kI4Order[j];
          const int mode = (bi < 8 ? im_lo >> (4 * bi) : im_hi >> (4 * (bi - 8))) & 0xf;
          e[j] = tab[mode * 16 + m];
          rs[j] = res[bi * 16 + m];
        }
        // blocks of equal t are independent: one LDS hand-off per t.  The lane mask is set once
        // for the whole walk (one exec save/restore instead of one per block: the chain is paced
        // by each wave's instruction count, SALU included)
        if (act && i4) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int bi = kI4Order[j], bx = bi & 3, by = bi >> 2;
          {
            uint8_t* org = ws + Y_OFF + 4 * by * BPS + 4 * bx;
            const uint32_t ew = e[j];
            int v;
            if (ew == 0xC0000000u) {  // DC4 (pred4_table.inc: the one DC word)
              const uint32_t s = __builtin_amdgcn_sad_u8(ld32(org - BPS), 0, 0);
              v = (int)(s + org[-1] + org[BPS - 1] + org[2 * BPS - 1] + org[3 * BPS - 1] + 4) >> 3;
            } else {
              const int a = org[(int8_t)(ew & 0xff)];
              const int b = org[(int8_t)((ew >> 8) & 0xff)];
              const int c = org[(int8_t)((ew >> 16) & 0xff)];
              // v_lerp_u8 averages bytes, rounding up where its third operand's bit is set:
              // AVG3 = (a + 2b + c + 2) >> 2 = (((a + c) >> 1) + b + 1) >> 1 in two instructions
              // (exact: tests/test_oracle.py::test_avg3_lerp_identity); AVG2(a, b) is stored as
              // AVG3(a, b, a).  TM words are the negative ones.
              const int avg3 = (int)__builtin_amdgcn_lerp(__builtin_amdgcn_lerp(a, c, 0u), b, 1u);
              const int tm = clamp255(a + b - c);
              v = (int)ew < 0 ? tm : avg3;
            }
            const uint8_t px = (uint8_t)clamp255(v + rs[j]);
            org[ppy * BPS + ppx] = px;
            fw[kFwY + (4 * by + ppy + 4) * FWY + 4 + 4 * bx + ppx] = px;  // (the filter window too)
          }
          if (j == 15 || kI4Step[j + 1] != kI4Step[j]) lds_sync();
        }
        }
      }
#endif

      K1_SECT(6);
      K1_SECT(7);
      if (act) {
        // ---- stash unfiltered bottom samples for the row below (frame_dec.c.go:175-179)
        //      (lanes 0..3 luma, 4..5 U, 6..7 V: the column store's dword m either way)
        if (!last_row && m < 8) {
          const int so = m < 4 ? Y_OFF + 15 * BPS + 4 * m : (m < 6 ? U_OFF - 16 : V_OFF - 24) + 7 * BPS + 4 * m;
          col_st(col + 4 * m, ld32(ws + so), csc1);
        }
        // ---- filter window: rows above from fbot (the MB body was written into it by the
        //      prediction sections, next to the workspace)
        if (y > 0) {
          st32(fw + kFwY + (m >> 2) * FWY + 4 + 4 * (m & 3), col_ld(col + 32 + 4 * m, csc1));
          const int p = m >> 3, rr = (m >> 1) & 3, dd = m & 1;
          st32(fw + (p ? kFwV : kFwU) + rr * FWC + 4 + 4 * dd, col_ld(col + 96 + 32 * p + 8 * rr + 4 * dd, csc1));
        }
      }
      lds_sync();

      K1_SECT(8);
      // ---- loop filter on the window
      {
        const uint32_t fi = rc.finfo;
        const int limit = fi & 0xff;
        const bool on = act && limit > 0;
#ifdef WG_ABL_FILTER
        if (false) {
#else
        if (ftype > 0 && __any(on)) {
#endif
          const int ilevel = (fi >> 8) & 0xff, inner = (fi >> 16) & 0xff, hev_t = (fi >> 24) & 0xff;
          if (ftype == 2) filter_mb<true>(fw, m, on, x > 0, y > 0, inner != 0, limit, ilevel, hev_t);
          else filter_mb<false>(fw, m, on, x > 0, y > 0, inner != 0, limit, ilevel, hev_t);
        }
      }

      K1_SECT(9);
      // ---- deposit final bottom rows of this MB column (and the left neighbour's cols 12..15
      //      / 4..7, final now) for the row below's top-edge filter: luma role m, chroma m+16
      if (act && !last_row) {
        {
          const int rr = m >> 2, d = m & 3;
          const uint8_t* src = fw + kFwY + (rr + 16) * FWY;
          if (d == 0) {
            if (x > 0) col_st(col - kColBytes + 32 + rr * 16 + 12, ld32(src), csc1);
            if (last_x) col_st(col + 32 + rr * 16 + 12, ld32(src + 16), csc1);
          } else {
            col_st(col + 32 + rr * 16 + 4 * (d - 1), ld32(src + 4 * d), csc1);
          }
        }
        {
          const int p = m >> 3, rr = (m >> 1) & 3, d = m & 1;
          const uint8_t* src = fw + (p ? kFwV : kFwU) + (rr + 8) * FWC;
          const ColPtr cb0 = col + 96 + 32 * p + 8 * rr;
          if (d == 0) {
            if (x > 0) col_st(cb0 - kColBytes + 4, ld32(src), csc1);
            if (last_x) col_st(cb0 + 4, ld32(src + 8), csc1);
          } else {
            col_st(cb0, ld32(src + 4), csc1);
          }
        }
      }
      K1_SECT(10);
      // ---- final pixels to HBM.  After this MB's filter, its rows 0..12 (chroma 0..4) are final
      //      in cols 0..11 (0..3), and so are the left neighbour's cols 12..15 (4..7) and the
      //      bottom rows 13..15 (5..7) of the MB above: one 16-byte (8-byte chroma) row segment
      //      per lane, two buffer stores per MB step, against one descriptor spanning the
      //      frame's Y|U|V planes.  At x = 0 the segment starts at col 0 instead of -4: its
      //      last 4 (chroma 4) bytes are not final yet and are rewritten, final, by the same
      //      lane at x = 1 (same-address stores of a lane stay in order) or by the last-column
      //      store below.  The bottom MB row and the last MB column add their rows 13..15
      //      (5..7) and cols 12..15 (4..7) under branches.
      {
        const bool tl = m >= 13, tc = (m & 7) >= 5;
        const int wcy = (tl || x == 0) ? 4 : 0, wcc = (tc || x == 0) ? 4 : 0;
        const uint8_t* sy = fw + kFwY + (tl ? m - 12 : m + 4) * FWY + wcy;
        const uint8_t* sc = fw + (m >= 8 ? kFwV : kFwU) + (tc ? (m & 7) - 4 : (m & 7) + 4) * FWC + wcc;
        const u32x4 vy = {ld32(sy), ld32(sy + 4), ld32(sy + 8), ld32(sy + 12)};
        const u32x2 vc = {ld32(sc), ld32(sc + 4)};
        const uint32_t ux = (uint32_t)x;
        // (measurement builds WG_ABL_PLANES_Y / _C drop the luma / chroma stores: DESIGN.md §4)
#if defined(WG_ABL_PLANES_Y64)  // measurement only: own luma rows as full 64-byte chunks (data wrong)
        const uint32_t oy = act && tl ? sb_y + (ux << 4) + wcy : kDrop;
        {
          const bool fl = act && (x & 3) == 0 && x >= 4;
          if (__any(fl)) {
#pragma unroll
            for (int A = 0; A < 4; ++A) {
              const int r = 4 * A + (m >> 2);
              const uint32_t o = fl && r < 13 ? (uint32_t)__mul24(16 * y + r, ys) + 16u * (ux - 4u) + 16u * (m & 3) : kDrop;
              __builtin_amdgcn_raw_buffer_store_b128(vy, planes, (int)o, 0, 0);
            }
          }
        }
#elif !defined(WG_ABL_PLANES_Y)
        const uint32_t oy = act ? sb_y + (ux << 4) + wcy : kDrop;
#else
        const uint32_t oy = kDrop;
#endif
#ifndef WG_ABL_PLANES_C
        const uint32_t oc = act ? sb_c + (ux << 3) + wcc : kDrop;
#else
        const uint32_t oc = kDrop;
#endif
        __builtin_amdgcn_raw_buffer_store_b128(vy, planes, (int)oy, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b64(vc, planes, (int)oc, 0, 0);
        const int w0 = x == 0 ? 4 : 0;  // the own-row segments' window column
        if (act && last_row && tl) {  // rows 13..15 of the bottom MB row (no MB below)
          const uint8_t* s2 = fw + kFwY + (m + 4) * FWY + w0;
          const u32x4 v2 = {ld32(s2), ld32(s2 + 4), ld32(s2 + 8), ld32(s2 + 12)};
          __builtin_amdgcn_raw_buffer_store_b128(v2, planes, __mul24(16 * y + m, ys) + 16 * x + w0 - 4, 0, 0);
        }
        if (act && last_row && tc) {  // chroma rows 5..7 of the bottom MB row
          const uint8_t* s2 = fw + (m >= 8 ? kFwV : kFwU) + ((m & 7) + 4) * FWC + w0;
          const u32x2 v2 = {ld32(s2), ld32(s2 + 4)};
          __builtin_amdgcn_raw_buffer_store_b64(
              v2, planes, (int)((m >= 8 ? voff : uoff) + __mul24(8 * y + (m & 7), uvs)) + 8 * x + w0 - 4, 0, 0);
        }
        if (act && last_x) {  // the last MB column's cols 12..15 (chroma 4..7) of its own rows
          if (m < 13 || last_row)
            __builtin_amdgcn_raw_buffer_store_b32(ld32(fw + kFwY + (m + 4) * FWY + 16), planes,
                                                  __mul24(16 * y + m, ys) + 16 * x + 12, 0, 0);
          if ((m & 7) < 5 || last_row)
            __builtin_amdgcn_raw_buffer_store_b32(
                ld32(fw + (m >= 8 ? kFwV : kFwU) + ((m & 7) + 4) * FWC + 8), planes,
                (int)((m >= 8 ? voff : uoff) + __mul24(8 * y + (m & 7), uvs)) + 8 * x + 4, 0, 0);
        }
      }
      lds_sync();

      K1_SECT(11);
      // ---- rotate for the next MB (frame_dec.c.go:106-114) + the filter window: cols 12..15
      //      (chroma 4..7) become cols -4..-1 for rows 0..15 (0..7); row -1 is not needed
      //      (its col -1 comes from the top-left carry).  Role m: luma row m; role m+16:
      //      chroma row m&7 (U for m < 8, else V).
      if (act) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int l = m + 16 * s;
          const bool ly = s == 0;
          const int cp = (l >> 3) & 1, cr = l & 7;
          uint8_t* src = ly ? ws + Y_OFF + l * BPS + 12 : ws + (cp ? V_OFF : U_OFF) + cr * BPS + 4;
          const uint32_t v = ld32(src);
          st32(src - (ly ? 16 : 8), v);
          left[l] = (uint8_t)(v >> 24);
          uint8_t* src2 = ly ? fw + kFwY + (l + 4) * FWY + 16 : fw + (cp ? kFwV : kFwU) + (cr + 4) * FWC + 8;
          st32(src2 - (ly ? 16 : 8), ld32(src2));
        }
      }
      lds_sync();
      if (g_pub) {
        // the next part's first quad: every 4th column of the last row, and its last (after this
        // wave's sc1 column-store stores have completed: vmcnt(0), then the sc1 flag store)
        const int xl = i - 2 * (kRows - 1);
        if (xl >= 0 && ((xl & 3) == 3 || xl + 1 == mb_w)) {
          // (also a compiler barrier: the flag store stays behind every sc1 column-store store;
          // tests/test_k1_isa.py checks the machine code at this marker)
          asm volatile("s_waitcnt vmcnt(0) ; wg-gprog-publish" ::: "memory");
          if (lane == 16 * (kRows - 1))
            __hip_atomic_store(gprog + 32 * part, ((epoch & 0xffffu) << 16) | (uint32_t)(xl + 1), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
      } else if (lane == 16 * (kRows - 1) && has_next && x >= 0) {
        __hip_atomic_store(progress + (k & (kWaves - 1)), ((uint32_t)k << 16) | (uint32_t)(x + 1), __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      K1_SECT(12);
      rc = rn;
      rn = rnn;
      blk = blk_next;
    }
    K1_QUAD_MARK(k, 1);
  }
  K1_SECT_FLUSH();
#ifdef WG_ABL_TAIL
  if (false) {
#else
  if (emit) {
#endif
    // Own plane stores complete before announcing the wave done: converters may read the
    // bottom rows right after the last wave's increment, with no row of margin left.
    // (Workgroup-scope release alone emits no vmcnt wait; this costs one wait per wave.)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    if (lane == 0) __hip_atomic_fetch_add(&recon_done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_s_setprio(0);
    if (F->flags & kFrameNoFancy) emit_tail<false>(*F, progress, &recon_done, &next_unit, lane, err);
    else emit_tail<true>(*F, progress, &recon_done, &next_unit, lane, err);
  }
  K1_TIMELINE_END();
}

#ifdef WG_K1_SECTION_TIMING
extern "C" int wg_debug_k1_sections(unsigned long long* out, int n, int reset) {
  if (n > kSections) n = kSections;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k1_sections), n * sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[kSections] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_k1_sections), z, sizeof(z)) != hipSuccess) return -1;
  }
  return n;
}

// per frame: start, each wave's exit from reconstruction, each wave's exit from the kernel
// (memrealtime ticks, 100 MHz)
extern "C" int wg_debug_k1_timeline(unsigned long long* out, int n_frames) {
  if (n_frames > kTimelineFrames) n_frames = kTimelineFrames;
  const size_t bytes = (size_t)n_frames * (1 + 2 * kWaves) * sizeof(unsigned long long);
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k1_timeline), bytes) != hipSuccess) return -1;
  return n_frames;
}

extern "C" int wg_debug_k1_quads(unsigned long long* out, int n_frames) {
  if (n_frames > kTimelineFrames) n_frames = kTimelineFrames;
  const size_t bytes = (size_t)n_frames * kTimelineQuads * 2 * sizeof(unsigned long long);
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k1_quads), bytes) != hipSuccess) return -1;
  return n_frames;
}
#endif

size_t vp8_recon_lds_bytes(int mb_w) {
  return (size_t)kHdrBytes + (size_t)kMaxRecon * kRows * kSlotBytes + (size_t)mb_w * kColBytes;
}

int vp8_recon_max_mb_w() { return (int)((163840 - kHdrBytes - kMaxRecon * kRows * kSlotBytes) / kColBytes); }

hipError_t launch_vp8_recon_filter(const FrameDesc* d_frames, int n_frames, int max_mb_w, bool lds_frames,
                                   bool wide_frames, int* d_err, hipStream_t stream, int split_parts, uint32_t epoch,
                                   int slab) {
  // WG_K1_LEAD overrides the inter-quad lead (tuning experiments only).
  static const int lead = [] {
    const char* e = getenv("WG_K1_LEAD");
    return e ? atoi(e) : 0;
  }();
  // WG_K1_RECON_WAVES: waves per frame that reconstruct (at most 12; with the RGBA tail the
  // rest convert finished bands from the start); 0 / unset = 12.
  static const int recon_waves = [] {
    const char* e = getenv("WG_K1_RECON_WAVES");
    return e ? atoi(e) : 0;
  }();
  if (split_parts >= 2) {  // every frame on split_parts workgroups, column stores in global memory
    if (split_parts > kMaxSplitParts) return hipErrorInvalidValue;
    const size_t lds = vp8_recon_lds_bytes(0);
    static bool configured = false;
    if (lds > 65536 && !configured) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&vp8_recon_filter_kernel<true, true>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
      configured = true;
    }
    const int grid = ((n_frames + 7) / 8) * 8 * split_parts;
    // (the slab: balanced over the parts by the caller -- fewer reconstructing waves per CU, each
    // issuing faster; WG_K1_RECON_WAVES still overrides it for measurements)
    hipLaunchKernelGGL((vp8_recon_filter_kernel<true, true>), dim3(grid), dim3(1024), lds, stream, d_frames, d_err,
                       lead, recon_waves > 0 ? recon_waves : slab, n_frames, split_parts, epoch);
    return hipGetLastError();
  }
  if (lds_frames) {
    const size_t lds = vp8_recon_lds_bytes(max_mb_w);
    static size_t configured = 0;
    if (lds > 65536 && lds > configured) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&vp8_recon_filter_kernel<false, false>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
      configured = lds;
    }
    hipLaunchKernelGGL((vp8_recon_filter_kernel<false, false>), dim3(n_frames), dim3(1024), lds, stream, d_frames,
                       d_err, lead, recon_waves, n_frames, 1, 0u);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (wide_frames) {
    const size_t lds = vp8_recon_lds_bytes(0);
    static bool configured = false;
    if (lds > 65536 && !configured) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&vp8_recon_filter_kernel<true, false>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
      configured = true;
    }
    hipLaunchKernelGGL((vp8_recon_filter_kernel<true, false>), dim3(n_frames), dim3(1024), lds, stream, d_frames,
                       d_err, lead, recon_waves, n_frames, 1, 0u);
    return hipGetLastError();
  }
  return hipSuccess;
}

}  // namespace wg
