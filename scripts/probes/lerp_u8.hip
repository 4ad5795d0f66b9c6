// Probe: v_lerp_u8 (__builtin_amdgcn_lerp) with a zero round operand is VP8L's Average2
// (per-byte floor((a + b) / 2), lossless.go Average2) on all byte pairs: checks the
// device result against the SWAR formula K3 used before for 2^24 random dword pairs and the
// full 256 x 256 byte grid.  Build: hipcc -w --offload-arch=gfx950 -O3 lerp_u8.hip -o lerp_u8
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t avg2_swar(uint32_t a, uint32_t b) {
  return (((a ^ b) & 0xfefefefeu) >> 1) + (a & b);
}
__device__ __forceinline__ uint32_t hash(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
__global__ void k(unsigned* bad, int n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint32_t)n) return;
  uint32_t a, b;
  if (i < 65536u) { a = (i & 255u) * 0x01010101u; b = (i >> 8) * 0x01010101u; }
  else { a = hash(2 * i); b = hash(2 * i + 1); }
  if (__builtin_amdgcn_lerp(a, b, 0u) != avg2_swar(a, b)) atomicAdd(bad, 1u);
}
int main() {
  unsigned* d;
  (void)hipMalloc(&d, 4);
  (void)hipMemset(d, 0, 4);
  const int n = 1 << 24;
  k<<<n / 256, 256>>>(d, n);
  unsigned h = 0;
  (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  printf("lerp_u8 vs Average2 mismatches: %u of %d\n", h, n);
  return h != 0;
}
