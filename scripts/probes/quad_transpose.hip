#include <hip/hip_runtime.h>
// 4x4 transpose across a lane quad: lane q holds t[0..3] = row q; returns column q.
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
  t[0] = m0; t[1] = m1; t[2] = m2; t[3] = m3;
}
__global__ void k(int* p) {
  int t[4] = {p[4 * threadIdx.x], p[4 * threadIdx.x + 1], p[4 * threadIdx.x + 2], p[4 * threadIdx.x + 3]};
  quad_transpose(t);
  for (int i = 0; i < 4; ++i) p[1024 + 4 * threadIdx.x + i] = t[i];
}
int main() {
  int h[2048], *d;
  for (int i = 0; i < 1024; ++i) h[i] = i;
  (void)hipMalloc(&d, sizeof(h));
  (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  k<<<1, 256>>>(d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 256; ++l)
    for (int i = 0; i < 4; ++i) {
      const int q = l & 3, base = l & ~3;
      const int want = 4 * (base + i) + q;  // lane q of the quad gets element q of lane i
      if (h[1024 + 4 * l + i] != want) ++bad;
    }
  printf("quad_transpose mismatches: %d\n", bad);
  return bad != 0;
}
