// Probe: achievable HBM bandwidth for K2's read/write mix (YUV420 -> RGBA: 1.5 B read per
// 4 B written).  Streams with ideal access shapes -- every wave instruction touches one
// contiguous run (384 B read by 24 lanes, 1 KB written by 64 lanes, like K2's luma/chroma
// loads and RGBA stores) -- over buffers the size of the c3 batch (3.19 GB in, 8.49 GB out),
// and for comparison write-only, read-only and 1:1 copy streams.  Prints GB/s of
// (bytes read + bytes written) per kernel, best of 5.
// Build: hipcc -w --offload-arch=gfx950 -O3 rw_mix.hip -o rw_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// rd_lanes of 64 lanes read 16 B each, wr_lanes write 16 B each, per unit.
template <int RD, int WR, bool NT>
__global__ void __launch_bounds__(256) stream(const u32x4* __restrict__ src, u32x4* __restrict__ dst, long units) {
  const int lane = threadIdx.x & 63;
  const long wave = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  uint32_t acc = 0;
  for (long u = wave; u < units; u += nwaves) {
    u32x4 r = {0, 0, 0, 0};
    if (RD > 0 && lane < RD) r = NT ? __builtin_nontemporal_load(src + u * RD + lane) : src[u * RD + lane];
    if (WR > 0) {
      const int s = RD > 0 ? lane % RD : 0;
      u32x4 w;
      w.x = __shfl(r.x, s) ^ lane;
      w.y = __shfl(r.y, s);
      w.z = __shfl(r.z, s);
      w.w = __shfl(r.w, s) + (uint32_t)u;
      if (lane < WR) {
        if (NT) __builtin_nontemporal_store(w, dst + u * WR + lane);
        else dst[u * WR + lane] = w;
      }
    } else {
      acc += r.x ^ r.y ^ r.z ^ r.w;
    }
  }
  if (WR == 0 && acc == 0x12345678u) dst[0] = u32x4{acc, 0, 0, 0};  // keep the reads
}

template <int RD, int WR, bool NT>
static void run(const char* name, const u32x4* src, u32x4* dst, long units) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int grid = 256 * 8;
  float best = 1e30f;
  for (int it = 0; it < 6; ++it) {
    (void)hipEventRecord(a);
    stream<RD, WR, NT><<<grid, 256>>>(src, dst, units);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    if (it > 0 && ms < best) best = ms;
  }
  const double bytes = (double)units * 16.0 * (RD + WR);
  printf("%-34s %8.3f ms  %7.1f GB moved  %7.1f GB/s  (%.1f%% of 8 TB/s)\n", name, best, bytes / 1e9,
         bytes / best / 1e6, bytes / best / 1e6 / 80.0);
}

int main() {
  const long out_bytes = 8493465600L;  // 256 x 3840 x 2160 x 4
  const long units = out_bytes / 1024;  // 1 KB written per unit
  u32x4 *src, *dst;
  if (hipMalloc(&src, units * 24 * 16 + 4096) != hipSuccess || hipMalloc(&dst, out_bytes + 4096) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  (void)hipMemset(src, 1, units * 24 * 16);
  (void)hipMemset(dst, 0, out_bytes);
  run<24, 64, true>("mix 0.375:1 (K2 shape), nt", src, dst, units);
  run<24, 64, false>("mix 0.375:1 (K2 shape), plain", src, dst, units);
  run<0, 64, true>("write only, nt", src, dst, units);
  run<0, 64, false>("write only, plain", src, dst, units);
  run<64, 0, true>("read only, nt", dst, src, units);
  run<64, 0, false>("read only, plain", dst, src, units);
  run<24, 24, true>("copy 1:1, nt", src, dst, units);
  return 0;
}
