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
// by per-wave progress counters).  Pixels move in 8-step chunks: at step 8c every lane
// loads/stores the 8 columns it will touch next (aligned to its own skew), so memory
// instructions are wave-uniform.  Cross-color / add-green before the predictor are
// applied to its input, those after it to its output (the recurrence keeps the raw
// predictor output).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device_format.h"
#include "kernels.h"

namespace wg {
namespace {

constexpr int kWaves = 16;
constexpr int kBand = 64;
constexpr int kChunk = 8;
constexpr int kRing = 512;  // columns per inter-band ring slot (power of two)
constexpr int kRingBytes = kWaves * kRing * 4;
constexpr int kModeTabMax = 16384;  // predictor tiles staged in LDS (1 byte each)
constexpr int kCCTabMax = 4096;     // cross-color tiles staged in LDS (4 bytes each)
constexpr int kLdsBytes = kRingBytes + kModeTabMax + kCCTabMax * 4;
constexpr uint32_t kDrop = 0x80000000u;
constexpr int T_PRED = 0, T_CC = 1, T_AG = 2;  // 3 = color indexing

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t add_pixels(uint32_t a, uint32_t b) {
  return (((a & 0xff00ff00u) + (b & 0xff00ff00u)) & 0xff00ff00u) |
         (((a & 0x00ff00ffu) + (b & 0x00ff00ffu)) & 0x00ff00ffu);
}
__device__ __forceinline__ uint32_t avg2(uint32_t a, uint32_t b) { return (((a ^ b) & 0xfefefefeu) >> 1) + (a & b); }
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

// Per-lane predictor with the common modes cheap: ClampedAverage of four (mode 10, most
// tiles of a natural image) for every lane; the copies 1..4 by a two-level select on the
// mode bits when some lane uses them; the per-lane switch only for lanes on the remaining
// modes, skipped when none is.
__device__ __forceinline__ uint32_t predict_fast(int m, uint32_t L, uint32_t T, uint32_t TL, uint32_t TR) {
  uint32_t p = avg2(avg2(L, TL), avg2(T, TR));
  if (__any(m != 10)) {
    const uint32_t cp = (m & 1) ? ((m & 2) ? TR : L) : ((m & 2) ? T : TL);  // 1 L, 2 T, 3 TR, 4 TL
    p = (unsigned)(m - 1) < 4u ? cp : p;
    const bool rest = ((unsigned)(m - 1) >= 4u) & (m != 10);
    if (__any(rest)) {
      if (rest) p = predict(m, L, T, TL, TR);
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
  r = (r + cdelta((int)(m & 0xff), g)) & 0xff;
  b = (b + cdelta((int)((m >> 8) & 0xff), g) + cdelta((int)((m >> 16) & 0xff), r)) & 0xff;
  return (argb & 0xff00ff00u) | ((uint32_t)r << 16) | (uint32_t)b;
}
__device__ __forceinline__ uint32_t add_green(uint32_t argb) {
  const uint32_t g = (argb >> 8) & 0xff;
  return (argb & 0xff00ff00u) | (((argb & 0x00ff00ffu) + ((g << 16) | g)) & 0x00ff00ffu);
}
__device__ __forceinline__ uint32_t bgra_to_rgba(uint32_t c) {
  return __builtin_amdgcn_perm(c, c, 0x07040506u);  // bytes B,G,R,A -> R,G,B,A
}

__device__ __forceinline__ uint32_t shr1(uint32_t old, uint32_t v) {  // lane i <- lane i-1; lane 0 <- old
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

// Bounded spin on a progress counter: gives up after 2 s (s_memrealtime is 100 MHz),
// flags the batch error word and makes the caller return.
__device__ __forceinline__ bool wait_progress(uint32_t* pr, uint32_t need, int* err) {
  if (__hip_atomic_load(pr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= need) return true;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(pr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
      atomicOr(err, 2);
      return false;
    }
  }
  return true;
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
// columns read once per chunk.  Interior chunks (every lane's columns inside
// [1, W-2]) carry no edge logic and move pixels with 8-byte loads/stores at immediate
// offsets; edge chunks predicate per pixel.  The chunk's LDS reads (modes, cross-color
// words, ring) issue together at its start and are waited on once.  Row 0 / column 0 use fixed modes (L / T,
// black at the origin), folded into the prefetched modes.
template <int PRE, int POST, bool GENERIC>
__device__ __forceinline__ bool pred_wavefront(const Pass& P, int W, int H, int w_in, bool last, __amdgpu_buffer_rsrc_t in_rs,
                               __amdgpu_buffer_rsrc_t out_rs, int dst_stride, uint32_t* ring, const uint8_t* mode_tab,
                               const uint32_t* cc_tab, uint32_t* prog, int* err) {
  constexpr bool kCC = !GENERIC && (ops_cc(PRE) || ops_cc(POST));
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nbands = (H + kBand - 1) / kBand;
  const int steps = W + 2 * (kBand - 1);
  const int nchunks = (steps + kChunk - 1) / kChunk;
  // interior chunks: 8c - 2*63 >= 1 and 8c + 7 <= W - 2
  const int c_lo = (2 * (kBand - 1) + kChunk) / kChunk, c_hi = (W - 1 - kChunk) / kChunk;
  for (int b = wave; b < nbands; b += kWaves) {
    const int y = b * kBand + lane;
    const bool row_ok = y < H;
    const bool row0 = y == 0;
    const int yc = min(y, H - 1);
    const uint32_t* ring_prev = ring + ((b - 1) & (kWaves - 1)) * kRing;  // band b-1's last row
    uint32_t* ring_mine = ring + (b & (kWaves - 1)) * kRing;
    // ring slot b&15 was last written by band b-16 and read by band b-15: that reader
    // must be done before this band overwrites it
    if (b >= kWaves && !wait_progress(prog + ((b - kWaves + 1) & (kWaves - 1)),
                                      ((uint32_t)(b - kWaves + 1) << 16) | (uint32_t)steps, err))
      return false;
    const int mrow = (yc >> P.m_bits) * P.m_tpr;
    const int crow = (yc >> P.cc_bits) * P.cc_tpr;
    const uint32_t in_row = row_ok ? (uint32_t)(y * w_in * 4) : kDrop;
    const uint32_t out_row = row_ok ? (uint32_t)(y * dst_stride) : kDrop;

    auto load_chunk = [&](int c, uint32_t* dstv) {
      const int x0 = c * kChunk - 2 * lane;
      if (c >= c_lo && c <= c_hi) {
#pragma unroll
        for (int k = 0; k < kChunk; k += 2) {
          const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(in_rs, in_row + 4 * x0, 4 * k, 0);
          dstv[k] = v.x;
          dstv[k + 1] = v.y;
        }
      } else {
#pragma unroll
        for (int k = 0; k < kChunk; k += 2) {
          const int x = x0 + k;
          const bool ok = x >= 0 && x < W;
          const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(in_rs, ok ? in_row + 4 * x : kDrop, 0, 0);
          dstv[k] = v.x;
          dstv[k + 1] = v.y;
        }
      }
    };
    // modes (fixed ones folded in) and cross-color words of chunk c
    auto fetch_tables = [&](int c, int* md, uint32_t* cw) {
      const bool edge = !(c >= c_lo && c <= c_hi);
#pragma unroll
      for (int k = 0; k < kChunk; ++k) {
        const int xr = c * kChunk + k - 2 * lane;
        const int x = edge ? min(max(xr, 0), W - 1) : xr;
        int m;
        if (GENERIC && !P.m_in_lds)
          m = (int)((P.m_g[mrow + (x >> P.m_bits)] >> 8) & 0xf);
        else
          m = mode_tab[mrow + (x >> P.m_bits)];
        if (edge) m = row0 ? (xr == 0 ? 0 : 1) : (xr == 0 ? 2 : m);
        else if (b == 0) m = row0 ? 1 : m;
        md[k] = m;
        if (kCC) cw[k] = cc_tab[crow + (x >> P.cc_bits)];
      }
    };

    uint32_t o_prev = 0, t1 = 0, t2 = 0, first = 0;  // L; TR of the last two steps (= T, TL)
    uint32_t cin[kChunk], cnext[kChunk];
    load_chunk(0, cin);
    for (int c = 0; c < nchunks; ++c) {
      const bool interior = c >= c_lo && c <= c_hi;
      if (c + 1 < nchunks) load_chunk(c + 1, cnext);
      uint32_t ccw[kChunk];
      int md[kChunk];
      fetch_tables(c, md, ccw);
      // band b-1 must be 135 steps ahead of this chunk's end (its last row, lane 63, then
      // covers column x+1 of lane 0); band b+1 must have consumed the ring columns this
      // chunk overwrites
      if (b > 0) {
        const uint32_t need = ((uint32_t)(b - 1) << 16) | (uint32_t)min(c * kChunk + kChunk + 127, steps);
        if (!wait_progress(prog + ((b - 1) & (kWaves - 1)), need, err)) return false;
      }
      if (b + 1 < nbands) {
        const int lag = c * kChunk + kChunk - 2 * (kBand - 1) - kRing + 16;  // oldest column still needed
        if (lag > 0 &&
            !wait_progress(prog + ((b + 1) & (kWaves - 1)), ((uint32_t)(b + 1) << 16) | (uint32_t)lag, err))
          return false;
      }
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
      uint32_t ov[kChunk];
#pragma unroll
      for (int k = 0; k < kChunk; ++k) {
        const int x = c * kChunk + k - 2 * lane;
        const uint32_t tr = shr1(r[k + 1], o_prev);
        const uint32_t TR = (!interior && x == W - 1) ? first : tr;  // rightmost: this row's first pixel
        // (generic: tables may be in HBM, so the column is clamped into the frame)
        const uint32_t v =
            GENERIC ? pre_ops(P, cc_tab, cin[k], min(max(x, 0), W - 1), yc) : ops_ct<PRE>(cin[k], ccw[k]);
        const uint32_t o = add_pixels(v, predict_fast(md[k], o_prev, t1, t2, TR));
        if (!interior && x == 0) first = o;
        t2 = t1;
        t1 = tr;
        o_prev = o;
        ov[k] = o;
      }
      // band b's last row into the ring (lane 63), then the chunk's outputs
      if (interior) {
        if (lane == kBand - 1) {
#pragma unroll
          for (int k = 0; k < kChunk; k += 2)
            *reinterpret_cast<uint2*>(ring_mine + ((c * kChunk + k - 2 * lane) & (kRing - 1))) = make_uint2(ov[k], ov[k + 1]);
        }
        const uint32_t off = out_row + 4 * (c * kChunk - 2 * lane);
#pragma unroll
        for (int k = 0; k < kChunk; k += 2) {
          uint32_t f0, f1;
          if (GENERIC) {
            f0 = post_ops(P, cc_tab, ov[k], c * kChunk + k - 2 * lane, yc);
            f1 = post_ops(P, cc_tab, ov[k + 1], c * kChunk + k + 1 - 2 * lane, yc);
          } else {
            f0 = ops_ct<POST>(ov[k], ccw[k]);
            f1 = ops_ct<POST>(ov[k + 1], ccw[k + 1]);
          }
          if (last) {
            f0 = bgra_to_rgba(f0);
            f1 = bgra_to_rgba(f1);
          }
          u32x2 pair;
          pair.x = f0;
          pair.y = f1;
          __builtin_amdgcn_raw_buffer_store_b64(pair, out_rs, off, 4 * k, 0);
        }
      } else {
#pragma unroll
        for (int k = 0; k < kChunk; ++k) {
          const int x = c * kChunk + k - 2 * lane;
          const bool ok = row_ok && x >= 0 && x < W;
          if (lane == kBand - 1 && ok) ring_mine[x & (kRing - 1)] = ov[k];
          uint32_t f = GENERIC ? post_ops(P, cc_tab, ov[k], min(max(x, 0), W - 1), yc) : ops_ct<POST>(ov[k], ccw[k]);
          if (last) f = bgra_to_rgba(f);
          __builtin_amdgcn_raw_buffer_store_b32(f, out_rs, ok ? out_row + 4 * x : kDrop, 0, 0);
        }
      }
      if (lane == 0)
        __hip_atomic_store(prog + (b & (kWaves - 1)), ((uint32_t)b << 16) | (uint32_t)min(c * kChunk + kChunk, steps),
                           __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
      for (int k = 0; k < kChunk; ++k) cin[k] = cnext[k];
    }
  }
  return true;
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
  const int W = F.width, H = F.height, n = F.n_stages;

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
        for (int t = threadIdx.x; t < nt; t += blockDim.x) cc_tab[t] = st.data[t];
    }
    if (pred) {
      const LLStage& ps = F.stages[core];
      P.m_bits = ps.bits;
      P.m_tpr = ps.tiles_per_row;
      P.m_g = as_global(ps.data);
      const int nt = P.m_tpr * ((H + (1 << P.m_bits) - 1) >> P.m_bits);
      P.m_in_lds = nt <= kModeTabMax;
      if (P.m_in_lds)
        for (int t = threadIdx.x; t < nt; t += blockDim.x) mode_tab[t] = (uint8_t)((ps.data[t] >> 8) & 0xf);
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
#define WG_PRED(PRE, POST, GEN) \
  pred_wavefront<PRE, POST, GEN>(P, W, H, w_in, last, in_rs, out_rs, dst_stride, ring, mode_tab, cc_tab, prog, err)
      if (VARIANT == 1) ok = WG_PRED(1, 2, false);       // CC | PRED | AG (libwebp's usual order)
      else if (VARIANT == 2) ok = WG_PRED(0, 2, false);  // PRED | AG
      else if (VARIANT == 3) ok = WG_PRED(1, 0, false);  // CC | PRED
      else if (VARIANT == 4) ok = WG_PRED(0, 0, false);  // PRED
      else ok = WG_PRED(0, 0, true);
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
