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

// A per-pixel op (cross-color or add-green) with its tile table.
struct PixOp {
  int type, bits, tpr, idx;  // idx: stage index in the frame's list
  const uint32_t* cc;        // LDS or global multipliers (cross-color)
};

__device__ __forceinline__ uint32_t apply_ops(const PixOp* ops, int n, uint32_t v, int x, int y) {
  for (int k = 0; k < n; ++k) {
    if (ops[k].type == T_AG) {
      v = add_green(v);
    } else {
      v = cross_color_inv(v, ops[k].cc[(y >> ops[k].bits) * ops[k].tpr + (x >> ops[k].bits)]);
    }
  }
  return v;
}

__device__ __forceinline__ uint32_t shr1(uint32_t old, uint32_t v) {  // lane i <- lane i-1; lane 0 <- old
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

// Stage a cross-color table into LDS when it fits; returns the table to use.
__device__ const uint32_t* stage_cc(const LLStage& st, uint32_t* lds_cc, int ysize) {
  const int n = st.tiles_per_row * ((ysize + (1 << st.bits) - 1) >> st.bits);
  if (n > kCCTabMax) return st.data;
  for (int t = threadIdx.x; t < n; t += blockDim.x) lds_cc[t] = st.data[t];
  return lds_cc;
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

__global__ void __launch_bounds__(1024) vp8l_transforms_kernel(const LLDesc* __restrict__ frames, int* err) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ uint32_t prog[kWaves];
  const LLDesc& F = frames[blockIdx.x];
  if (!F.valid) return;
  uint32_t* ring = reinterpret_cast<uint32_t*>(lds);
  uint8_t* mode_tab = lds + kRingBytes;
  uint32_t* cc_tab = reinterpret_cast<uint32_t*>(lds + kRingBytes + kModeTabMax);
  const int W = F.width, H = F.height, n = F.n_stages;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;

  int i = 0, w_in = F.coded_width;
  const uint32_t* src = F.coded;
  int src_bytes = F.coded_bytes;
  bool first_pass = true;
  while (first_pass || i < n) {
    first_pass = false;
    // ---- plan one pass: [ops] core [ops]
    PixOp pre[2], post[2];
    int npre = 0, npost = 0, core = -1;
    while (i < n && (F.stages[i].type == T_CC || F.stages[i].type == T_AG)) {
      pre[npre] = PixOp{F.stages[i].type, F.stages[i].bits, F.stages[i].tiles_per_row, i, F.stages[i].data};
      ++npre;
      ++i;
    }
    if (i < n) core = i++;
    while (i < n && (F.stages[i].type == T_CC || F.stages[i].type == T_AG)) {
      post[npost] = PixOp{F.stages[i].type, F.stages[i].bits, F.stages[i].tiles_per_row, i, F.stages[i].data};
      ++npost;
      ++i;
    }
    const bool last = i >= n;
    const int w_out = core >= 0 ? F.stages[core].xsize : W;
    // ---- stage tables (one cross-color table at most: the type occurs once)
    __syncthreads();
    for (int k = 0; k < npre; ++k)
      if (pre[k].type == T_CC) pre[k].cc = stage_cc(F.stages[pre[k].idx], cc_tab, H);
    for (int k = 0; k < npost; ++k)
      if (post[k].type == T_CC) post[k].cc = stage_cc(F.stages[post[k].idx], cc_tab, H);
    const bool pred = core >= 0 && F.stages[core].type == T_PRED;
    const uint8_t* modes = nullptr;
    int mbits = 0, mtpr = 0;
    const uint32_t* gmodes = nullptr;
    if (pred) {
      const LLStage& ps = F.stages[core];
      mbits = ps.bits;
      mtpr = ps.tiles_per_row;
      const int nt = mtpr * ((H + (1 << mbits) - 1) >> mbits);
      if (nt <= kModeTabMax) {
        for (int t = threadIdx.x; t < nt; t += blockDim.x) mode_tab[t] = (uint8_t)((ps.data[t] >> 8) & 0xf);
        modes = mode_tab;
      } else {
        gmodes = ps.data;
      }
    }
    if (threadIdx.x < kWaves) prog[threadIdx.x] = 0;
    __syncthreads();

    const __amdgpu_buffer_rsrc_t in_rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(src), 0, src_bytes,
                                                                           0x00020000);
    uint8_t* dst_base = last ? F.rgba : reinterpret_cast<uint8_t*>(F.scratch);
    const int dst_stride = last ? F.rgba_stride : w_out * 4;
    const int dst_bytes = last ? F.rgba_stride * H : F.scratch_bytes;
    const __amdgpu_buffer_rsrc_t out_rs = __builtin_amdgcn_make_buffer_rsrc(dst_base, 0, dst_bytes, 0x00020000);

    if (pred) {
      // ---------------- predictor wavefront
      const int nbands = (H + kBand - 1) / kBand;
      const int steps = W + 2 * (kBand - 1);
      const int nchunks = (steps + kChunk - 1) / kChunk;
      for (int b = wave; b < nbands; b += kWaves) {
        const int y = b * kBand + lane;
        const bool row_ok = y < H;
        uint32_t* ring_prev = ring + ((b - 1) & (kWaves - 1)) * kRing;  // band b-1's last row
        uint32_t* ring_mine = ring + (b & (kWaves - 1)) * kRing;
        // ring slot b&15 was last written by band b-16 and read by band b-15: that reader
        // must be done before this band overwrites it
        if (b >= kWaves && !wait_progress(prog + ((b - kWaves + 1) & (kWaves - 1)),
                                          ((uint32_t)(b - kWaves + 1) << 16) | (uint32_t)steps, err))
          return;
        uint32_t h1 = 0, h2 = 0, h3 = 0, first = 0;
        uint32_t cin[kChunk], cnext[kChunk];
        auto load_chunk = [&](int c, uint32_t* dstv) {
#pragma unroll
          for (int k = 0; k < kChunk; k += 2) {
            const int x = c * kChunk + k - 2 * lane;
            const bool ok = row_ok && x >= 0 && x < W;
            const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(in_rs, ok ? (y * w_in + x) * 4 : (int)kDrop, 0, 0);
            dstv[k] = v.x;
            dstv[k + 1] = v.y;
          }
        };
        load_chunk(0, cin);
        for (int c = 0; c < nchunks; ++c) {
          if (c + 1 < nchunks) load_chunk(c + 1, cnext);
          // wait for band b-1 to be 135 steps ahead of this chunk's end; the ring is
          // not overwritten before band b+1 has consumed it
          if (b > 0) {
            const uint32_t need = ((uint32_t)(b - 1) << 16) | (uint32_t)min(c * kChunk + kChunk + 127, steps);
            if (!wait_progress(prog + ((b - 1) & (kWaves - 1)), need, err)) return;
          }
          if (b + 1 < nbands) {
            const int lag = c * kChunk + kChunk - 2 * (kBand - 1) - kRing + 16;  // oldest column still needed
            if (lag > 0 &&
                !wait_progress(prog + ((b + 1) & (kWaves - 1)), ((uint32_t)(b + 1) << 16) | (uint32_t)lag, err))
              return;
          }
          uint32_t cout[kChunk];
#pragma unroll
          for (int k = 0; k < kChunk; ++k) {
            const int s = c * kChunk + k;
            const int x = s - 2 * lane;
            const bool ok = row_ok && x >= 0 && x < W;
            // row above: lane i-1's outputs at steps s-1 (x+1), s-2 (x), s-3 (x-1);
            // lane 0 reads the previous band's last row from the ring
            const uint32_t rTR = ring_prev[(x + 1) & (kRing - 1)];
            const uint32_t rT = ring_prev[x & (kRing - 1)];
            const uint32_t rTL = ring_prev[(x - 1) & (kRing - 1)];
            uint32_t TR = shr1(rTR, h1), T = shr1(rT, h2), TL = shr1(rTL, h3);
            uint32_t v = apply_ops(pre, npre, cin[k], x, y);
            uint32_t p;
            if (y == 0) {
              p = x == 0 ? 0xff000000u : h1;
            } else if (x == 0) {
              p = T;
            } else {
              if (x == W - 1) TR = first;
              const int tile = (y >> mbits) * mtpr + (x >> mbits);
              const int mode = modes ? (int)modes[tile] : (int)((gmodes[tile] >> 8) & 0xf);
              p = predict(mode, h1, T, TL, TR);
            }
            const uint32_t o = add_pixels(v, p);
            if (x == 0) first = o;
            if (lane == kBand - 1 && ok) ring_mine[x & (kRing - 1)] = o;
            h3 = h2;
            h2 = h1;
            h1 = o;
            const uint32_t f = apply_ops(post, npost, o, x, y);
            cout[k] = last ? bgra_to_rgba(f) : f;
          }
#pragma unroll
          for (int k = 0; k < kChunk; ++k) {
            const int x = c * kChunk + k - 2 * lane;
            const bool ok = row_ok && x >= 0 && x < W;
            __builtin_amdgcn_raw_buffer_store_b32(cout[k], out_rs, ok ? y * dst_stride + 4 * x : (int)kDrop, 0, 0);
          }
          if (lane == 0)
            __hip_atomic_store(prog + (b & (kWaves - 1)), ((uint32_t)b << 16) | (uint32_t)min(c * kChunk + kChunk, steps),
                               __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
          for (int k = 0; k < kChunk; ++k) cin[k] = cnext[k];
        }
      }
    } else {
      // ---------------- per-pixel pass (color indexing or ops only)
      const bool ci = core >= 0;
      const int cbits = ci ? F.stages[core].bits : 0;
      const uint32_t* pal = ci ? F.stages[core].data : nullptr;
      const int bpp = 8 >> cbits;
      const int total = w_out * H;
      for (int p = threadIdx.x; p < total; p += blockDim.x) {
        const int y = p / w_out, x = p - y * w_out;
        uint32_t v;
        if (ci) {
          const int xs = x >> cbits;
          uint32_t packed = apply_ops(pre, npre, src[y * w_in + xs], xs, y);
          const int idx = cbits ? (int)(((packed >> 8) >> ((x & ((1 << cbits) - 1)) * bpp)) & ((1u << bpp) - 1))
                                : (int)((packed >> 8) & 0xff);
          v = pal[idx];
        } else {
          v = apply_ops(pre, npre, src[y * w_in + x], x, y);
        }
        v = apply_ops(post, npost, v, x, y);
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

hipError_t launch_vp8l_transforms(const LLDesc* d_frames, int n_frames, int* d_err, hipStream_t stream) {
  static bool configured = false;
  if (!configured) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&vp8l_transforms_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    if (e != hipSuccess) return e;
    configured = true;
  }
  hipLaunchKernelGGL(vp8l_transforms_kernel, dim3(n_frames), dim3(64 * kWaves), kLdsBytes, stream, d_frames, d_err);
  return hipGetLastError();
}

}  // namespace wg
