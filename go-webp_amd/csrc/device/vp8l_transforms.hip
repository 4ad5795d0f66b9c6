// K3: VP8L (lossless) inverse transforms + BGRA->RGBA for a batch of frames.
//
// Replaces the reference's lossless DSP stage (pkg/libwebp/dsp/lossless.go):
//   PredictorInverseTransform + VP8LPredictor0..13      :91-148, 290-333
//   ColorSpaceInverseTransform / TransformColorInverse  :349-413
//   VP8LAddGreenToBlueAndRed                            :337-347
//   ColorIndexInverseTransform (+ ExpandColorMap)       :428-459 (vp8l_dec.c.go:1196-1219)
//   VP8LInverseTransform order, VP8LConvertBGRAToRGBA   :511-547, 561-573
// applied to the host entropy stage's output (host/vp8l_parse.cpp).
//
// One 1024-thread workgroup per frame.  Transforms are grouped into at most two passes
// (each type occurs once): [per-pixel ops] core [per-pixel ops], core = predictor or color
// indexing; the last pass writes RGBA, an earlier one the frame's scratch image.
//
// Predictor pass (the only dependent one): each pixel adds a prediction from its left,
// top-left, top and top-right OUTPUT neighbours -- a t = x + 2y wavefront.  Wave w owns
// 64-row bands b = w, w+16, ...; lane i (row 64b+i) handles column x = s - 2i at step s,
// so the row above is lane i-1 two steps earlier: T, TL, TR are lane i-1's last three
// outputs, moved one lane up with DPP wave_shr:1 (no LDS).  Lane 0 takes them from the
// previous band's last row through an LDS ring (kRing columns per band, flow-controlled
// by per-wave progress counters).  Pixels move in 8-step chunks through a per-row
// LDS column ring; HBM sees row-wise loads and whole aligned 64-byte row blocks.  Cross-color / add-green before the predictor are
// applied to its input, those after it to its output (the recurrence keeps the raw
// predictor output).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "../device_format.h"
#include "kernels.h"

namespace wg {
namespace {

constexpr int kWaves = 16;
constexpr int kBand = 64;
constexpr int kChunk = 8;
constexpr int kRing = 256;  // columns per inter-band ring slot (power of two; 512 measured the same)
constexpr int kRingBytes = kWaves * kRing * 4;
constexpr int kModeTabMax = 16384;  // predictor tiles staged in LDS (1 byte each)
constexpr int kCCTabMax = 4096;     // cross-color tiles staged in LDS (4 bytes each)
// Per-wave staging slot: the band's 64 rows x a 24-column ring (see pred_wavefront).
constexpr int kGroup = 2 * kChunk;
constexpr int kOutCols = 24;  // per-row column ring: column x at position x mod 24
constexpr int kSlotStride = 4 * kOutCols;
constexpr int kSlotBytes = kBand * kSlotStride;
constexpr int kLdsBytes = kRingBytes + kModeTabMax + kCCTabMax * 4 + kWaves * kSlotBytes;
static_assert(kLdsBytes + 4 * kWaves <= 160 * 1024, "K3 LDS (dynamic + the progress counters) exceeds gfx950's 160 KB");
static_assert(kOutCols >= 14 + kChunk && kOutCols % 4 == 0, "row ring: 14 open columns + a chunk; 16-byte pieces never wrap");
constexpr uint32_t kDrop = 0x80000000u;
#ifndef WG_K3_STORE_AUX
// Cache policy of the output block stores (buffer aux bits): sc1 (16) writes the lines
// through, so they do not hold L2 capacity the input rows' lines need until their next chunk:
// c5 reads 7.9 -> 5.7 GB per launch, K3 3.09 -> 3.04-3.06 ms (nt, 2: 5.9 GB, 3.06 ms; same call)
#define WG_K3_STORE_AUX 16
#endif
constexpr int T_PRED = 0, T_CC = 1, T_AG = 2;  // 3 = color indexing

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t uint32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t uint32x2_t __attribute__((ext_vector_type(2)));

// Opt-in per-section cycle accounting (make VARIANT=timing, read back by
// scripts/k3_sections.py): s_memtime deltas summed per chunk section in registers,
// flushed with one atomic per section per wave.  Measurement only.
[[maybe_unused]] constexpr int kK3Sections = 10;
#ifdef WG_K3_SECTION_TIMING
__device__ unsigned long long g_k3_sections[kK3Sections];
// per frame (workgroup) and band: start and end of the band's predictor loop (s_memrealtime)
constexpr int kK3TimelineFrames = 1024, kK3TimelineBands = 64;
__device__ unsigned long long g_k3_bands[kK3TimelineFrames][kK3TimelineBands + 1][2];
#define K3_BAND_MARK(b, which)                                                              \
  do {                                                                                      \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < kK3TimelineFrames && (b) < kK3TimelineBands) \
      g_k3_bands[blockIdx.x][1 + (b)][which] = __builtin_amdgcn_s_memrealtime();           \
  } while (0)
#define K3_START_MARK()                                                                     \
  do {                                                                                      \
    if (threadIdx.x == 0 && blockIdx.x < kK3TimelineFrames)                                 \
      g_k3_bands[blockIdx.x][0][0] = __builtin_amdgcn_s_memrealtime();                     \
  } while (0)
#define K3_SECT_DECL() uint64_t sect_acc[kK3Sections] = {}, sect_t = __builtin_amdgcn_s_memtime()
#define K3_SECT(id)                                       \
  do {                                                    \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();     \
    sect_acc[id] += t_ - sect_t;                          \
    sect_t = t_;                                          \
  } while (0)
#define K3_SECT_FLUSH()                                                                   \
  do {                                                                                    \
    if ((threadIdx.x & 63) == 0)                                                          \
      for (int s_ = 0; s_ < kK3Sections; ++s_) atomicAdd(&g_k3_sections[s_], sect_acc[s_]); \
  } while (0)
#else
#define K3_SECT_DECL() (void)0
#define K3_SECT(id) (void)0
#define K3_SECT_FLUSH() (void)0
#define K3_BAND_MARK(b, which) (void)0
#define K3_START_MARK() (void)0
#endif

// Per-byte a + b mod 256: add the low 7 bits of every byte (no carry can leave a byte),
// then set each top bit to the xor of the operands' top bits and the carry into it; the
// masked xor is one v_bitop3 (truth table 0x28 = (S0 ^ S1) & S2).
__device__ __forceinline__ uint32_t add_pixels(uint32_t a, uint32_t b) {
  return ((a & 0x7f7f7f7fu) + (b & 0x7f7f7f7fu)) ^ (uint32_t)__builtin_amdgcn_bitop3_b32(a, b, 0x80808080u, 0x28);
}
// Per-byte floor((a + b) / 2) (Average2, lossless.go): one v_lerp_u8 with a zero rounding
// operand (the SWAR form (a & b) + ((a ^ b) & 0xfe..) / 2 took four instructions); checked
// against it on the device over all byte pairs and 2^24 random dwords
// (scripts/probes/lerp_u8.hip).
__device__ __forceinline__ uint32_t avg2(uint32_t a, uint32_t b) { return __builtin_amdgcn_lerp(a, b, 0u); }
__device__ __forceinline__ int clamp255(int v) { return min(max(v, 0), 255); }
__device__ __forceinline__ int chan(uint32_t v, int s) { return (int)((v >> s) & 0xff); }

__device__ __forceinline__ uint32_t add_sub_full(uint32_t c0, uint32_t c1, uint32_t c2) {
  uint32_t r = 0;
#pragma unroll
  for (int s = 0; s < 32; s += 8) r |= (uint32_t)clamp255(chan(c0, s) + chan(c1, s) - chan(c2, s)) << s;
  return r;
}
__device__ __forceinline__ uint32_t add_sub_half(uint32_t c0, uint32_t c1, uint32_t c2) {
  const uint32_t ave = avg2(c0, c1);
  uint32_t r = 0;
#pragma unroll
  for (int s = 0; s < 32; s += 8) {
    const int a = chan(ave, s), d = a - chan(c2, s);
    r |= (uint32_t)clamp255(a + d / 2) << s;  // C division: toward zero
  }
  return r;
}
// Select (lossless.go): sum|L - TL| <= sum|T - TL| ? T : L, via v_sad_u8 on packed bytes
__device__ __forceinline__ uint32_t select_px(uint32_t T, uint32_t L, uint32_t TL) {
  const uint32_t dl = __builtin_amdgcn_sad_u8(L, TL, 0), dt = __builtin_amdgcn_sad_u8(T, TL, 0);
  return dl <= dt ? T : L;
}

__device__ __forceinline__ uint32_t predict(int mode, uint32_t L, uint32_t T, uint32_t TL, uint32_t TR) {
  switch (mode) {
    case 1: return L;
    case 2: return T;
    case 3: return TR;
    case 4: return TL;
    case 5: return avg2(avg2(L, TR), T);
    case 6: return avg2(L, TL);
    case 7: return avg2(L, T);
    case 8: return avg2(TL, T);
    case 9: return avg2(T, TR);
    case 10: return avg2(avg2(L, TL), avg2(T, TR));
    case 11: return select_px(T, L, TL);
    case 12: return add_sub_full(L, T, TL);
    case 13: return add_sub_half(L, T, TL);
    default: return 0xff000000u;  // 0 and the padding modes 14, 15
  }
}

// Predictor modes as staged for the steps (enc_mode): 0 = mode 10 (ClampedAverage of four, most
// tiles of a natural image); the copies 1..4 = 4 | sel with sel's bits choosing
// b1 ? (b0 ? TR : T) : (b0 ? L : TL); every other mode = 0x80 | mode << 3.
__device__ __forceinline__ int enc_mode(int m) {
  if (m == 10) return 0;
  if (m >= 1 && m <= 4) return 4 | (m & 3);
  return 0x80 | (m << 3);
}
// v_bfi_b32: bitwise mask ? a : b.  One-bit field of e sign-extended to a full mask: v_bfe_i32.
// (Inline asm: written as C, the compiler turns the masks back into compares + v_cndmask.)
__device__ __forceinline__ uint32_t bitsel(uint32_t mask, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(mask), "v"(a), "v"(b));
  return r;
}
template <int kBit>
__device__ __forceinline__ uint32_t bitmask(int e) {
  uint32_t r;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(r) : "v"(e), "i"(kBit));
  return r;
}

// Per-lane predictor with the common modes cheap: the ClampedAverage of four for every lane;
// when some lane is on another mode, the copies by three bitwise selects on masks taken
// straight from the encoded mode's bits (no compares: 7 instructions, the compare-and-select
// form took 14), and the per-lane switch only on lanes with the remaining modes, skipped when
// none is.
// kSel (chosen per chunk, see chunk_impl): 0 = every lane of the chunk on mode 10, 1 = mode 10 or
// copies only (selects without the per-step checks), 2 = anything (per-step checks).  kMS: bit
// position of the encoded mode in e (24 when it shares a word with the cross-color multipliers).
template <int kSel, int kMS>
__device__ __forceinline__ uint32_t predict_fast(int e, uint32_t L, uint32_t T, uint32_t TL, uint32_t TR) {
  uint32_t p = avg2(avg2(L, TL), avg2(T, TR));
  if (kSel == 1) {
    const uint32_t b0 = bitmask<kMS>(e);
    const uint32_t cp = bitsel(bitmask<kMS + 1>(e), bitsel(b0, TR, T), bitsel(b0, L, TL));
    return bitsel(bitmask<kMS + 2>(e), cp, p);
  }
#ifdef WG_ABL_K3_FAST  // measurement only: every pixel takes the mode-10 predictor (output wrong)
  if (false) {
#else
  if (kSel == 2 && __any((unsigned)e >= (1u << kMS))) {
#endif
    const uint32_t b0 = bitmask<kMS>(e);
    const uint32_t cp = bitsel(bitmask<kMS + 1>(e), bitsel(b0, TR, T), bitsel(b0, L, TL));
    p = bitsel(bitmask<kMS + 2>(e), cp, p);
    const bool rest = (unsigned)e >= (0x80u << kMS);
#ifdef WG_ABL_K3_NOREST  // measurement only: modes other than 1..4 and 10 not predicted (output wrong)
    if (false) {
#else
    if (__any(rest)) {
#endif
      if (rest) p = predict((int)(((unsigned)e >> (kMS + 3)) & 0xf), L, T, TL, TR);
    }
  }
  return p;
}

__device__ __forceinline__ int cdelta(int t, int c) {  // ColorTransformDelta on int8 values
  return ((int)(int8_t)t * (int)(int8_t)c) >> 5;
}
__device__ __forceinline__ uint32_t cross_color_inv(uint32_t argb, uint32_t m) {
  const int g = (int)((argb >> 8) & 0xff);
  int r = (int)((argb >> 16) & 0xff), b = (int)(argb & 0xff);
  r = r + cdelta((int)(m & 0xff), g);  // only the low byte is kept
  b = b + cdelta((int)((m >> 8) & 0xff), g) + cdelta((int)((m >> 16) & 0xff), r & 0xff);
  // the low bytes of r and b into bytes 2 and 0 of argb: two v_perm instead of masks + shifts
  const uint32_t t = __builtin_amdgcn_perm((uint32_t)r, argb, 0x03040100u);
  return __builtin_amdgcn_perm((uint32_t)b, t, 0x03020104u);
}
__device__ __forceinline__ uint32_t add_green(uint32_t argb) {
  const uint32_t g = (argb >> 8) & 0xff;
  return (argb & 0xff00ff00u) | (((argb & 0x00ff00ffu) + ((g << 16) | g)) & 0x00ff00ffu);
}
// VP8LAddGreenToBlueAndRed of one pixel with the output byte order folded into the final
// v_perm: bytes 0 and 2 of x are blue + green and red + green (the 0x00ff00ff mask keeps a
// byte-0 carry out of byte 2), bytes 1 and 3 (green, alpha) come from the input.  sel =
// 0x03060104 keeps ARGB (B,G,R,A in memory), 0x03040106 swaps to R,G,B,A.
__device__ __forceinline__ uint32_t add_green_emit(uint32_t argb, uint32_t sel) {
  const uint32_t gg = __builtin_amdgcn_perm(argb, argb, 0x0c010c01u);  // green in bytes 0 and 2
  const uint32_t x = (argb & 0x00ff00ffu) + gg;
  return __builtin_amdgcn_perm(x, argb, sel);
}
__device__ __forceinline__ uint32_t bgra_to_rgba(uint32_t c) {
  return __builtin_amdgcn_perm(c, c, 0x07040506u);  // bytes B,G,R,A -> R,G,B,A
}

__device__ __forceinline__ uint32_t shr1(uint32_t old, uint32_t v) {  // lane i <- lane i-1; lane 0 <- old
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

// Bounded spin on a progress counter (need is wave-uniform): the counter is read into an
// SGPR so the spin is a scalar branch.  After 2 s (s_memrealtime is 100 MHz) it flags the
// batch error word and sets `aborted`, which turns every later wait of the wave into a
// no-op: the wave runs to its end instead of leaving its loops early -- an exit path that
// skips a group's stores would make the waitcnt pass extend the loop's load waits over
// those stores.
__device__ __forceinline__ void wait_progress(uint32_t* pr, uint32_t need, int* err, bool& aborted) {
  auto cur = [&] {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(pr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
  };
  if (aborted || cur() >= need) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    __builtin_amdgcn_s_sleep(1);
    if (cur() >= need) return;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or(as_global(err), 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      aborted = true;
      return;
    }
  }
}

// Per-pass context, all wave-uniform.  Per-pixel ops: up to two (cross-color, add-green;
// each type occurs once per frame) before and after the core.  The cross-color table and
// the predictor modes live in LDS when they fit, else they are read from HBM.
struct Pass {
  int npre, pre0, pre1;    // op types, application order
  int npost, post0, post1;
  int cc_bits, cc_tpr, cc_in_lds;
  gptr<const uint32_t> cc_g;
  int m_bits, m_tpr, m_in_lds;
  gptr<const uint32_t> m_g;
  int joint;               // modes staged in byte 3 of the cross-color words (pred_wavefront kMS)
};

__device__ __forceinline__ uint32_t cc_word(const Pass& P, const uint32_t* cc_lds, int x, int y) {
  const int t = (y >> P.cc_bits) * P.cc_tpr + (x >> P.cc_bits);
  return P.cc_in_lds ? cc_lds[t] : P.cc_g[t];
}
__device__ __forceinline__ uint32_t op(int type, const Pass& P, const uint32_t* cc_lds, uint32_t v, int x, int y) {
  return type == T_AG ? add_green(v) : cross_color_inv(v, cc_word(P, cc_lds, x, y));
}
__device__ __forceinline__ uint32_t pre_ops(const Pass& P, const uint32_t* cc_lds, uint32_t v, int x, int y) {
  if (P.npre > 0) v = op(P.pre0, P, cc_lds, v, x, y);
  if (P.npre > 1) v = op(P.pre1, P, cc_lds, v, x, y);
  return v;
}
__device__ __forceinline__ uint32_t post_ops(const Pass& P, const uint32_t* cc_lds, uint32_t v, int x, int y) {
  if (P.npost > 0) v = op(P.post0, P, cc_lds, v, x, y);
  if (P.npost > 1) v = op(P.post1, P, cc_lds, v, x, y);
  return v;
}

// Compile-time per-pixel op sequences: 0 none, 1 cross-color, 2 add-green,
// 3 cross-color then add-green, 4 add-green then cross-color.  ccw: the pixel's
// cross-color tile word.
template <int OPS>
__device__ __forceinline__ uint32_t ops_ct(uint32_t v, uint32_t ccw) {
#ifdef WG_ABL_K3_NOCC  // measurement only: cross-color skipped (output wrong)
  if (OPS == 1) return v;
  if (OPS == 3) return add_green(v);
#endif
  if (OPS == 1) return cross_color_inv(v, ccw);
  if (OPS == 2) return add_green(v);
  if (OPS == 3) return add_green(cross_color_inv(v, ccw));
  if (OPS == 4) return cross_color_inv(add_green(v), ccw);
  return v;
}
constexpr bool ops_cc(int ops) { return ops == 1 || ops == 3 || ops == 4; }

// The predictor wavefront of one pass (see the file comment).  GENERIC: ops and tables
// at run time (tables may be in HBM); otherwise PRE/POST ops are compile-time and both
// tables are in LDS.  Returns false if a wave gave up waiting.
//
// Per 8-step chunk: the row above arrives as ONE DPP per step (lane i-1's previous output
// = this step's TR; T and TL are the TRs of the two steps before), lane 0's from nine ring
// columns read once per chunk.  Interior chunks (every lane's columns inside [1, W-2])
// carry no edge logic.  The chunk's LDS reads (inputs, modes, cross-color words, ring)
// issue together at its start and are waited on once.  Row 0 / column 0 use fixed modes
// (L / T, black at the origin), folded into the fetched modes.
//
// HBM traffic goes through the wave's staging slot, a 24-column ring per row: each chunk's
// inputs are loaded row-wise (two lanes per row) two chunks ahead and staged into the ring,
// the steps read and overwrite them transposed (lane = row), and every row's output leaves
// in whole aligned 64-byte blocks as soon as it completes one.  (Writing each group's
// 64 bytes per row where the skew puts them, 8 bytes off alignment, left HBM sectors half
// written between groups: 3.93 vs 3.47 ms on C5, see DESIGN.md.)
//
// kMS = 24: the pass's predictor modes share the cross-color table's words (equal tile
// sizes, both staged in LDS; encoded mode in byte 3, which cross-color does not read), so a
// step reads one table word instead of two and computes one address.
template <int PRE, int POST, bool GENERIC, int kMS = 0>
__device__ __forceinline__ bool pred_wavefront(const Pass& P, int W, int H, int w_in, bool last, __amdgpu_buffer_rsrc_t in_rs,
                               __amdgpu_buffer_rsrc_t out_rs, int dst_stride, uint32_t* ring, const uint8_t* mode_tab,
                               const uint32_t* cc_tab, uint8_t* slots, uint32_t* prog, int* err) {
  constexpr bool kCC = !GENERIC && (ops_cc(PRE) || ops_cc(POST));
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // wave in an SGPR
  bool aborted = false;
  const int nbands = (H + kBand - 1) / kBand;
  const int steps = W + 2 * (kBand - 1);
  const int ngroups = (steps + kGroup - 1) / kGroup;
  // interior chunks: 8c - 2*63 >= 1 and 8c + 7 <= W - 2
  const int c_lo = (2 * (kBand - 1) + kChunk) / kChunk, c_hi = (W - 1 - kChunk) / kChunk;
  uint8_t* slot = slots + wave * kSlotBytes;
  uint8_t* my_lds = slot + lane * kSlotStride;
  K3_SECT_DECL();
  for (int b = wave; b < nbands; b += kWaves) {
    K3_BAND_MARK(b, 0);
    const int y = b * kBand + lane;
    const bool row0 = y == 0;
    const int yc = min(y, H - 1);
    const uint32_t* ring_prev = ring + ((b - 1) & (kWaves - 1)) * kRing;  // band b-1's last row
    uint32_t* ring_mine = ring + (b & (kWaves - 1)) * kRing;
    // ring slot b&15 was last written by band b-16 and read by band b-15: that reader
    // must be done before this band overwrites it
    if (b >= kWaves)
      wait_progress(prog + ((b - kWaves + 1) & (kWaves - 1)), ((uint32_t)(b - kWaves + 1) << 16) | (uint32_t)steps, err,
                    aborted);
    K3_SECT(6);
    const int mrow = (yc >> P.m_bits) * P.m_tpr;
    const int crow = (yc >> P.cc_bits) * P.cc_tpr;
    // Rows past the frame get kDrop.  Columns left of the frame read the previous row
    // (ignored) or, in row 0, wrap to an out-of-range offset (reads 0).
    const int rows_left = H - b * kBand;
    // Row ring of 24 columns (column x at position x mod 24), inputs staged and outputs
    // emitted per chunk.  Loads: per chunk one aligned 32-byte block (8 columns) of each
    // row, the block holding the chunk's last column (c - r/4 for row r; the block before it
    // came with the previous chunk), by two lanes, rows lane/2 and lane/2 + 32, issued two
    // chunks ahead: every HBM sector of the input is requested once (an unaligned 32-byte
    // row piece touches two, and the L2 does not keep the shared one for the next chunk).
    // Staged blocks reach at most 6 columns past the chunk: with the <= 14 un-emitted output
    // columns the ring still holds <= 24.  Stores: whenever a row completes an
    // aligned 16-column block (64 B, every other chunk per row; 32 rows per chunk, 4 lanes
    // each) it goes out whole, so no HBM sector is left half written between groups.
    // Occupancy: at most 14 un-emitted columns + the chunk's 8 <= 24.
    auto ring_pos = [](int v) { return v >= kOutCols ? v - kOutCols : v; };
    const int cpos0 = (kOutCols - (2 * lane) % kOutCols) % kOutCols;  // column -2*lane
    const int l_row0 = lane >> 1, l_piece = lane & 1;
    const int spos0 = ((4 * l_piece - 8 * (l_row0 >> 2)) % kOutCols + kOutCols) % kOutCols;  // h = 0, c = 0
    const int spos1 = ((4 * l_piece - 8 * ((l_row0 + 32) >> 2)) % kOutCols + kOutCols) % kOutCols;
    const uint32_t l_off0 = (uint32_t)((b * kBand + l_row0) * w_in * 4) + 16u * l_piece - 32u * (uint32_t)(l_row0 >> 2);
    const uint32_t l_off1 = l_off0 + 32u * (uint32_t)w_in * 4u - 256u;  // +32 rows, -64 columns
    auto load_chunk = [&](int c, uint32x4_t* L) {
      L[0] = __builtin_amdgcn_raw_buffer_load_b128(in_rs, l_row0 < rows_left ? l_off0 + 32u * c : kDrop, 0, 0);
      L[1] = __builtin_amdgcn_raw_buffer_load_b128(in_rs, l_row0 + 32 < rows_left ? l_off1 + 32u * c : kDrop, 0, 0);
    };
    auto stage_chunk = [&](int c, const uint32x4_t* L) {
      const int c8 = 8 * (c % 3);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int pa = ring_pos((h ? spos1 : spos0) + c8);  // a multiple of 4 below 24: no wrap
        uint8_t* const row = slot + (l_row0 + 32 * h) * kSlotStride;
        *reinterpret_cast<uint32x4_t*>(row + 4 * pa) = L[h];
      }
    };
    // rows completing a block after chunk c (a multiple of 16 in (8c - 2r, 8c + 8 - 2r]):
    // r mod 8 in {1..4} (c even) or {5, 6, 7, 0} (c odd); lane -> (i = lane/4 + 16h,
    // quad = lane & 3), row = (8(i/4) + (i&3) + 1 + 4(c&1)) mod 64
    const int e_quad = lane & 3;
    auto emit_chunk = [&](int c) {
      const int K_hi = ((kChunk * c + kChunk) >> 4) - 1;  // row 0's block
      const bool inner = 8 * c >= 2 * (kBand - 1) + 16 && 16 * K_hi + 16 <= W;
      // both halves' LDS reads first, then both stores: one LDS round trip per chunk
      uint32x4_t d[2];
      uint32_t off[2];
      int x0[2];
      bool rok[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int i = (lane >> 2) + 16 * h;
        const int row = (8 * (i >> 2) + (i & 3) + 1 + 4 * (c & 1)) & (kBand - 1);
        const int K = ((kChunk * c + kChunk - 2 * row) >> 4) - 1;  // floor
        const int km3 = K >= 0 ? K % 3 : 0;
        const int pos = ring_pos(16 * km3 - (km3 == 2 ? 24 : 0) + 4 * e_quad);
        d[h] = *reinterpret_cast<const uint32x4_t*>(slot + row * kSlotStride + 4 * pos);
        x0[h] = 16 * K + 4 * e_quad;
        off[h] = (uint32_t)((b * kBand + row) * dst_stride) + 4u * (uint32_t)x0[h];
        rok[h] = row < rows_left && K >= 0;
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
        __builtin_amdgcn_raw_buffer_store_b128(d[h], out_rs, rok[h] && x0[h] + 3 < W ? off[h] : kDrop, 0, WG_K3_STORE_AUX);
      if (!inner) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bool ok = rok[h] && x0[h] + 3 >= W && x0[h] + j < W;
            __builtin_amdgcn_raw_buffer_store_b32(d[h][j], out_rs, ok ? off[h] + 4 * j : kDrop, 0, 0);
          }
        }
      }
    };
    // modes and cross-color words of chunk c: all reads issued back to back (column
    // clamped into the frame), the fixed modes of row 0 / column 0 applied afterwards
    // (interior chunks: every lane's columns lie inside the frame, no clamp)
    auto fetch_tables = [&](int c, int* md, uint32_t* cw, auto kInterior) {
#pragma unroll
      for (int k = 0; k < kChunk; ++k) {
        const int xr = c * kChunk + k - 2 * lane;
        const int x = decltype(kInterior)::value ? xr : min(max(xr, 0), W - 1);
        if constexpr (kMS != 0) {
          cw[k] = cc_tab[crow + (x >> P.cc_bits)];
          md[k] = (int)cw[k];
        } else {
          if (GENERIC && !P.m_in_lds)
            md[k] = enc_mode((int)((P.m_g[mrow + (x >> P.m_bits)] >> 8) & 0xf));
          else
            md[k] = mode_tab[mrow + (x >> P.m_bits)];
          if (kCC) cw[k] = cc_tab[crow + (x >> P.cc_bits)];
        }
      }
    };
    auto fix_modes = [&](int c, int* md) {
      if (!(c >= c_lo && c <= c_hi) || b == 0) {
#pragma unroll
        for (int k = 0; k < kChunk; ++k) {
          const int xr = c * kChunk + k - 2 * lane;
          const int fixed = row0 ? (xr == 0 ? enc_mode(0) : enc_mode(1)) : enc_mode(2);
          if (row0 || xr == 0) md[k] = kMS ? (int)(((uint32_t)md[k] & 0xffffffu) | ((uint32_t)fixed << kMS)) : fixed;
        }
      }
    };

    uint32_t o_prev = 0, t1 = 0, t2 = 0, first = 0;  // L; TR of the last two steps (= T, TL)
    // v_perm selectors of the chunk outputs: add-green's result bytes with RGBA (last pass)
    // or ARGB (scratch) order, and the plain RGBA / identity swizzle
    const uint32_t out_sel = last ? 0x03040106u : 0x03060104u;
    const uint32_t out_sel0 = last ? 0x07040506u : 0x07060504u;
    // one chunk (cl = 0/1 within its group): inputs from the slot, outputs back to it
    // kInterior (std::true_type / false_type): every lane's columns inside [1, W-2], so the
    // per-step frame-edge logic compiles out (two instantiations of the chunk)
    auto chunk_impl = [&](const int c, const int cl, auto kInterior) {
      constexpr bool interior = decltype(kInterior)::value;
      int cp[4];
      {
        const int p0 = ring_pos(cpos0 + 8 * (c % 3));
#pragma unroll
        for (int j = 0; j < 4; ++j) cp[j] = ring_pos(p0 + 2 * j);
      }
      const uint32x2_t i0 = *reinterpret_cast<const uint32x2_t*>(my_lds + 4 * cp[0]);
      const uint32x2_t i1 = *reinterpret_cast<const uint32x2_t*>(my_lds + 4 * cp[1]);
      const uint32x2_t i2 = *reinterpret_cast<const uint32x2_t*>(my_lds + 4 * cp[2]);
      const uint32x2_t i3 = *reinterpret_cast<const uint32x2_t*>(my_lds + 4 * cp[3]);
      const uint32x4_t in0 = uint32x4_t{i0[0], i0[1], i1[0], i1[1]};
      const uint32x4_t in1 = uint32x4_t{i2[0], i2[1], i3[0], i3[1]};
      uint32_t ccw[kChunk];
      int md[kChunk];
      fetch_tables(c, md, ccw, kInterior);
      K3_SECT(0);
      // band b-1 must be 135 steps ahead of this chunk's end (its last row, lane 63, then
      // covers column x+1 of lane 0); band b+1 must have consumed the ring columns this
      // chunk overwrites
      if (b > 0) {
        const uint32_t need = ((uint32_t)(b - 1) << 16) | (uint32_t)min(c * kChunk + kChunk + 127, steps);
        wait_progress(prog + ((b - 1) & (kWaves - 1)), need, err, aborted);
      }
      K3_SECT(1);
      if (b + 1 < nbands) {
        const int lag = c * kChunk + kChunk - 2 * (kBand - 1) - kRing + 16;  // oldest column still needed
        if (lag > 0) wait_progress(prog + ((b + 1) & (kWaves - 1)), ((uint32_t)(b + 1) << 16) | (uint32_t)lag, err, aborted);
      }
      K3_SECT(2);
      fix_modes(c, md);
      // lane 0's row above: columns 8c .. 8c+8 of band b-1's last row
      uint32_t r[kChunk + 1];
      {
        const int base = (c * kChunk) & (kRing - 1);
        const uint4 r0 = *reinterpret_cast<const uint4*>(ring_prev + base);
        const uint4 r1 = *reinterpret_cast<const uint4*>(ring_prev + base + 4);
        r[0] = r0.x; r[1] = r0.y; r[2] = r0.z; r[3] = r0.w;
        r[4] = r1.x; r[5] = r1.y; r[6] = r1.z; r[7] = r1.w;
        r[8] = ring_prev[(c * kChunk + kChunk) & (kRing - 1)];
      }
      if (c == 0) t1 = r[0];
      const uint32_t cin[kChunk] = {in0[0], in0[1], in0[2], in0[3], in1[0], in1[1], in1[2], in1[3]};
      K3_SECT(3);
      uint32_t ov[kChunk];
      auto run_steps = [&](auto kSelC) {
      constexpr int kSel = decltype(kSelC)::value;
#pragma unroll
      for (int k = 0; k < kChunk; ++k) {
        const int x = c * kChunk + k - 2 * lane;
        const uint32_t tr = shr1(r[k + 1], o_prev);
        const uint32_t TR = (!interior && x == W - 1) ? first : tr;  // rightmost: this row's first pixel
        // (generic: tables may be in HBM, so the column is clamped into the frame)
        const uint32_t v =
            GENERIC ? pre_ops(P, cc_tab, cin[k], min(max(x, 0), W - 1), yc) : ops_ct<PRE>(cin[k], ccw[k]);
        const uint32_t o = add_pixels(v, predict_fast<kSel, kMS>(md[k], o_prev, t1, t2, TR));
        if (!interior && x == 0) first = o;
        t2 = t1;
        t1 = tr;
        o_prev = o;
        ov[k] = o;
      }
      };
      // interior chunks pick the step code once for the chunk: the per-step checks of
      // predict_fast<2> (a compare and a branch each, two when some lane is off mode 10)
      // are only needed where some lane of the chunk is on a mode other than 10 and 1-4
      if constexpr (interior) {
        const int any_mode = (md[0] | md[1] | md[2] | md[3]) | (md[4] | md[5] | md[6] | md[7]);
#ifdef WG_ABL_K3_FAST
        run_steps(std::integral_constant<int, 0>{});
#else
        if (!__any((unsigned)any_mode >= (1u << kMS))) run_steps(std::integral_constant<int, 0>{});
        else if (!__any((unsigned)any_mode >= (0x80u << kMS))) run_steps(std::integral_constant<int, 1>{});
        else run_steps(std::integral_constant<int, 2>{});
#endif
      } else {
        run_steps(std::integral_constant<int, 2>{});
      }
      K3_SECT(4);
      // band b's last row into the ring (lane 63)
      if (lane == kBand - 1) {
        if (interior) {
#pragma unroll
          for (int k = 0; k < kChunk; k += 2)
            *reinterpret_cast<uint2*>(ring_mine + ((c * kChunk + k - 2 * lane) & (kRing - 1))) = make_uint2(ov[k], ov[k + 1]);
        } else {
#pragma unroll
          for (int k = 0; k < kChunk; ++k) {
            const int x = c * kChunk + k - 2 * lane;
            if (x >= 0 && x < W) ring_mine[x & (kRing - 1)] = ov[k];
          }
        }
      }
      // the chunk's outputs (post ops, RGBA on the last pass) over its inputs in the slot
      uint32_t f[kChunk];
#pragma unroll
      for (int k = 0; k < kChunk; ++k) {
        if constexpr (!GENERIC && POST == 2) {
          f[k] = add_green_emit(ov[k], out_sel);  // add-green and the output byte order in one
        } else if constexpr (!GENERIC && POST == 0) {
          f[k] = __builtin_amdgcn_perm(ov[k], ov[k], out_sel0);
        } else {
          f[k] = GENERIC ? post_ops(P, cc_tab, ov[k], min(max(c * kChunk + k - 2 * lane, 0), W - 1), yc)
                         : ops_ct<POST>(ov[k], ccw[k]);
          if (last) f[k] = bgra_to_rgba(f[k]);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) *reinterpret_cast<uint32x2_t*>(my_lds + 4 * cp[j]) = uint32x2_t{f[2 * j], f[2 * j + 1]};
      if (lane == 0)
        __hip_atomic_store(prog + (b & (kWaves - 1)), ((uint32_t)b << 16) | (uint32_t)min(c * kChunk + kChunk, steps),
                           __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      K3_SECT(5);
    };
    auto chunk = [&](const int c, const int cl) {
      if (c >= c_lo && c <= c_hi) chunk_impl(c, cl, std::true_type{});
      else chunk_impl(c, cl, std::false_type{});
    };
    uint32x4_t LA[2], LB[2];  // chunk inputs in flight: even chunks in LA, odd in LB
    load_chunk(0, LA);
    load_chunk(1, LB);
    const int nch = 2 * ngroups;
    for (int c = 0; c < nch; c += 2) {
      stage_chunk(c, LA);
      K3_SECT(8);
      load_chunk(c + 2, LA);
      K3_SECT(9);
      chunk(c, 0);
      emit_chunk(c);
      K3_SECT(7);
      stage_chunk(c + 1, LB);
      K3_SECT(8);
      load_chunk(c + 3, LB);
      K3_SECT(9);
      chunk(c + 1, 1);
      emit_chunk(c + 1);
      K3_SECT(7);
    }
    // blocks still open after the last chunk (row 63 completes one more, two chunks on)
    for (int c = nch; c < nch + 3; ++c) emit_chunk(c);
    K3_BAND_MARK(b, 1);
  }
  K3_SECT_FLUSH();
  return !aborted;
}

// VARIANT (chosen per frame on the host, vp8l_variant()): 1..4 = the predictor pass with
// compile-time ops (CC|PRED|AG, PRED|AG, CC|PRED, PRED) and LDS tables, 0 = generic.
template <int VARIANT>
__global__ void __launch_bounds__(1024) vp8l_transforms_kernel(const LLDesc* __restrict__ frames, int* err) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ uint32_t prog[kWaves];
  const LLDesc& F = frames[blockIdx.x];
  if (!F.valid) return;
  uint32_t* ring = reinterpret_cast<uint32_t*>(lds);
  uint8_t* mode_tab = lds + kRingBytes;
  uint32_t* cc_tab = reinterpret_cast<uint32_t*>(lds + kRingBytes + kModeTabMax);
  uint8_t* slots = lds + kRingBytes + kModeTabMax + kCCTabMax * 4;
  const int W = F.width, H = F.height, n = F.n_stages;
  K3_START_MARK();

  int i = 0, w_in = F.coded_width;
  const uint32_t* src = F.coded;
  int src_bytes = F.coded_bytes;
  bool first_pass = true;
  while (first_pass || i < n) {
    first_pass = false;
    // ---- plan one pass: [ops] core [ops]
    Pass P{};
    int cc_stage = -1;
    while (i < n && (F.stages[i].type == T_CC || F.stages[i].type == T_AG)) {
      if (F.stages[i].type == T_CC) cc_stage = i;
      if (P.npre == 0) P.pre0 = F.stages[i].type; else P.pre1 = F.stages[i].type;
      ++P.npre;
      ++i;
    }
    const int core = i < n ? i++ : -1;
    while (i < n && (F.stages[i].type == T_CC || F.stages[i].type == T_AG)) {
      if (F.stages[i].type == T_CC) cc_stage = i;
      if (P.npost == 0) P.post0 = F.stages[i].type; else P.post1 = F.stages[i].type;
      ++P.npost;
      ++i;
    }
    const bool last = i >= n;
    const int w_out = core >= 0 ? F.stages[core].xsize : W;
    const bool pred = core >= 0 && F.stages[core].type == T_PRED;
    // ---- stage the cross-color and predictor-mode tables
    __syncthreads();
    if (cc_stage >= 0) {
      const LLStage& st = F.stages[cc_stage];
      P.cc_bits = st.bits;
      P.cc_tpr = st.tiles_per_row;
      P.cc_g = as_global(st.data);
      const int nt = st.tiles_per_row * ((H + (1 << st.bits) - 1) >> st.bits);
      P.cc_in_lds = nt <= kCCTabMax;
      if (P.cc_in_lds)
        for (int t = threadIdx.x; t < nt; t += blockDim.x) cc_tab[t] = P.cc_g[t];
    }
    if (pred) {
      const LLStage& ps = F.stages[core];
      P.m_bits = ps.bits;
      P.m_tpr = ps.tiles_per_row;
      P.m_g = as_global(ps.data);
      const int nt = P.m_tpr * ((H + (1 << P.m_bits) - 1) >> P.m_bits);
      P.m_in_lds = nt <= kModeTabMax;
      P.joint = (VARIANT == 1 || VARIANT == 3) && cc_stage >= 0 && P.cc_in_lds && nt <= kModeTabMax &&
                P.cc_bits == P.m_bits && P.cc_tpr == P.m_tpr;
      if (P.joint)  // same thread, same t as the cross-color staging above
        for (int t = threadIdx.x; t < nt; t += blockDim.x)
          cc_tab[t] = (cc_tab[t] & 0xffffffu) | ((uint32_t)enc_mode((int)((P.m_g[t] >> 8) & 0xf)) << 24);
      else if (P.m_in_lds)
        for (int t = threadIdx.x; t < nt; t += blockDim.x) mode_tab[t] = (uint8_t)enc_mode((int)((P.m_g[t] >> 8) & 0xf));
    }
    if (threadIdx.x < kWaves) prog[threadIdx.x] = 0;
    __syncthreads();

    const __amdgpu_buffer_rsrc_t in_rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(src), 0, src_bytes, 0x00020000);
    uint8_t* dst_base = last ? F.rgba : reinterpret_cast<uint8_t*>(F.scratch);
    const int dst_stride = last ? F.rgba_stride : w_out * 4;
    const int dst_bytes = last ? F.rgba_stride * H : F.scratch_bytes;
    const __amdgpu_buffer_rsrc_t out_rs = __builtin_amdgcn_make_buffer_rsrc(dst_base, 0, dst_bytes, 0x00020000);

    if (pred) {
      // ---------------- predictor wavefront: compile-time op variants for the common
      // transform orders (all tables in LDS), the generic one otherwise
      bool ok;
#define WG_PRED(PRE, POST, GEN, MS) \
  pred_wavefront<PRE, POST, GEN, MS>(P, W, H, w_in, last, in_rs, out_rs, dst_stride, ring, mode_tab, cc_tab, slots, prog, err)
      // CC | PRED | AG (libwebp's usual order)
      if (VARIANT == 1) ok = P.joint ? WG_PRED(1, 2, false, 24) : WG_PRED(1, 2, false, 0);
      else if (VARIANT == 2) ok = WG_PRED(0, 2, false, 0);  // PRED | AG
      else if (VARIANT == 3) ok = P.joint ? WG_PRED(1, 0, false, 24) : WG_PRED(1, 0, false, 0);  // CC | PRED
      else if (VARIANT == 4) ok = WG_PRED(0, 0, false, 0);  // PRED
      else ok = WG_PRED(0, 0, true, 0);
#undef WG_PRED
      if (!ok) return;
    } else {
      // ---------------- per-pixel pass (color indexing or ops only)
      const bool ci = core >= 0;
      const int cbits = ci ? F.stages[core].bits : 0;
      const gptr<const uint32_t> pal = as_global(ci ? F.stages[core].data : F.coded);
      const gptr<const uint32_t> sg = as_global(src);
      const int bpp = 8 >> cbits;
      const int total = w_out * H;
      for (int p = threadIdx.x; p < total; p += blockDim.x) {
        const int y = p / w_out, x = p - y * w_out;
        uint32_t v;
        if (ci) {
          const int xs = x >> cbits;
          const uint32_t packed = pre_ops(P, cc_tab, sg[y * w_in + xs], xs, y);
          const int idx = cbits ? (int)(((packed >> 8) >> ((x & ((1 << cbits) - 1)) * bpp)) & ((1u << bpp) - 1))
                                : (int)((packed >> 8) & 0xff);
          v = pal[idx];
        } else {
          v = pre_ops(P, cc_tab, sg[y * w_in + x], x, y);
        }
        v = post_ops(P, cc_tab, v, x, y);
        __builtin_amdgcn_raw_buffer_store_b32(last ? bgra_to_rgba(v) : v, out_rs, y * dst_stride + 4 * x, 0, 0);
      }
    }
    __syncthreads();
    src = F.scratch;
    src_bytes = F.scratch_bytes;
    w_in = w_out;
  }
}

}  // namespace

size_t vp8l_lds_bytes() { return kLdsBytes; }

#ifdef WG_K3_SECTION_TIMING
extern "C" int wg_debug_k3_bands(unsigned long long* out, int n_frames) {
  if (n_frames > kK3TimelineFrames) n_frames = kK3TimelineFrames;
  const size_t bytes = (size_t)n_frames * (kK3TimelineBands + 1) * 2 * sizeof(unsigned long long);
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k3_bands), bytes) != hipSuccess) return -1;
  return n_frames;
}

extern "C" int wg_debug_k3_sections(unsigned long long* out, int n, int reset) {
  if (n > kK3Sections) n = kK3Sections;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k3_sections), n * sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[kK3Sections] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_k3_sections), z, sizeof(z)) != hipSuccess) return -1;
  }
  return n;
}
#endif

int vp8l_variant(const int* types, const int* bits, const int* tiles, int n_stages) {
  // mirror of the kernel's pass planning for the predictor pass: [ops] PRED [ops]
  int p = -1;
  for (int i = 0; i < n_stages; ++i)
    if (types[i] == T_PRED) p = i;
  if (p < 0) return 0;
  int pre = 0, post = 0, npre = 0, npost = 0;
  bool cc_fits = true;
  for (int i = p - 1; i >= 0 && (types[i] == T_CC || types[i] == T_AG); --i) {
    pre = pre * 4 + (types[i] == T_CC ? 1 : 2);  // innermost first
    ++npre;
    if (types[i] == T_CC) cc_fits = tiles[i] <= kCCTabMax;
  }
  for (int i = p + 1; i < n_stages && (types[i] == T_CC || types[i] == T_AG); ++i) {
    post = post * 4 + (types[i] == T_CC ? 1 : 2);
    ++npost;
    if (types[i] == T_CC) cc_fits = tiles[i] <= kCCTabMax;
  }
  if (tiles[p] > kModeTabMax || !cc_fits || npre > 1 || npost > 1) return 0;
  if (pre == 1 && post == 2) return 1;
  if (pre == 0 && post == 2) return 2;
  if (pre == 1 && post == 0) return 3;
  if (pre == 0 && post == 0) return 4;
  return 0;
}

hipError_t launch_vp8l_transforms(const LLDesc* d_frames, const int* group_count, int* d_err, hipStream_t stream) {
  static bool configured = false;
  auto kern = [](int v) -> const void* {
    switch (v) {
      case 1: return reinterpret_cast<const void*>(&vp8l_transforms_kernel<1>);
      case 2: return reinterpret_cast<const void*>(&vp8l_transforms_kernel<2>);
      case 3: return reinterpret_cast<const void*>(&vp8l_transforms_kernel<3>);
      case 4: return reinterpret_cast<const void*>(&vp8l_transforms_kernel<4>);
      default: return reinterpret_cast<const void*>(&vp8l_transforms_kernel<0>);
    }
  };
  if (!configured) {
    for (int v = 0; v < kVP8LVariants; ++v) {
      const hipError_t e = hipFuncSetAttribute(kern(v), hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
      if (e != hipSuccess) return e;
    }
    configured = true;
  }
  int start = 0;
  for (int v = 0; v < kVP8LVariants; ++v) {
    const int n = group_count[v];
    if (n <= 0) continue;
    const LLDesc* f = d_frames + start;
    switch (v) {
      case 1: hipLaunchKernelGGL(vp8l_transforms_kernel<1>, dim3(n), dim3(64 * kWaves), kLdsBytes, stream, f, d_err); break;
      case 2: hipLaunchKernelGGL(vp8l_transforms_kernel<2>, dim3(n), dim3(64 * kWaves), kLdsBytes, stream, f, d_err); break;
      case 3: hipLaunchKernelGGL(vp8l_transforms_kernel<3>, dim3(n), dim3(64 * kWaves), kLdsBytes, stream, f, d_err); break;
      case 4: hipLaunchKernelGGL(vp8l_transforms_kernel<4>, dim3(n), dim3(64 * kWaves), kLdsBytes, stream, f, d_err); break;
      default: hipLaunchKernelGGL(vp8l_transforms_kernel<0>, dim3(n), dim3(64 * kWaves), kLdsBytes, stream, f, d_err);
    }
    start += n;
  }
  return hipGetLastError();
}

}  // namespace wg
