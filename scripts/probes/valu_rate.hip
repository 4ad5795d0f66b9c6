// Probe: issue rate of a SIMD for one instruction kind with 1..4 co-resident waves (gfx950).
// One 1024-thread workgroup per CU (256 workgroups); waves with index < A run a loop of
// 16 independent instructions of one kind per iteration, the others exit at once.  Prints
// ns per wave-instruction per SIMD.  Used to price K1's instruction mix.
// Build: hipcc -w --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define KINDS(X) \
  X(0, "v_add_u32", "v_add_u32 %0, %0, %1") \
  X(1, "v_sub_u32", "v_sub_u32 %0, %0, %1") \
  X(2, "v_or_b32", "v_or_b32 %0, %0, %1") \
  X(3, "v_lshrrev_b32", "v_lshrrev_b32 %0, 3, %0") \
  X(4, "v_max_i32", "v_max_i32 %0, %0, %1") \
  X(5, "v_min_u32", "v_min_u32 %0, %0, %1") \
  X(6, "v_mov_b32", "v_mov_b32 %0, %1") \
  X(7, "v_add_u32_e64", "v_add_u32_e64 %0, %0, %1") \
  X(8, "v_sub_u32 clamp", "v_sub_u32_e64 %0, %0, %1 clamp") \
  X(9, "v_mul_u32_u24", "v_mul_u32_u24 %0, %0, %1") \
  X(10, "v_mad_u32_u24", "v_mad_u32_u24 %0, %0, %1, %2") \
  X(11, "v_sad_u8", "v_sad_u8 %0, %0, %1, %0") \
  X(12, "v_med3_i32", "v_med3_i32 %0, %0, %1, %2") \
  X(13, "v_max3_i32", "v_max3_i32 %0, %0, %1, %2") \
  X(14, "v_add3_u32", "v_add3_u32 %0, %0, %1, %2") \
  X(15, "v_lshl_add_u32", "v_lshl_add_u32 %0, %0, 2, %1") \
  X(16, "v_lshl_or_b32", "v_lshl_or_b32 %0, %0, 2, %1") \
  X(17, "v_and_or_b32", "v_and_or_b32 %0, %0, %1, %2") \
  X(18, "v_bfi_b32", "v_bfi_b32 %0, %0, %1, %2") \
  X(19, "v_bitop3_b32", "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca") \
  X(20, "v_bfe_u32", "v_bfe_u32 %0, %0, %1, 8") \
  X(21, "v_perm_b32", "v_perm_b32 %0, %0, %1, %2") \
  X(22, "v_alignbit_b32", "v_alignbit_b32 %0, %0, %1, 8") \
  X(23, "v_cndmask_e64", "v_cndmask_b32_e64 %0, %0, %1, s[20:21]") \
  X(24, "v_cmp_lt(vcc)", "v_cmp_lt_u32 vcc, %0, %1") \
  X(25, "v_cmp_lt_e64", "v_cmp_lt_u32_e64 s[20:21], %0, %1") \
  X(26, "dpp_mov", "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf") \
  X(27, "dpp_add", "v_add_u32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf") \
  X(28, "v_add_sdwa", "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1") \
  X(29, "v_pk_add_u16", "v_pk_add_u16 %0, %0, %1") \
  X(30, "v_pk_max_i16", "v_pk_max_i16 %0, %0, %1") \
  X(31, "v_pk_mad_u16", "v_pk_mad_u16 %0, %0, %1, %2") \
  X(32, "v_add_u16", "v_add_u16 %0, %0, %1") \
  X(33, "v_mul_lo_u16", "v_mul_lo_u16 %0, %0, %1") \
  X(34, "v_ashr_pk_u8", "v_ashr_pk_u8_i32 %0, %0, %1, 0") \
  X(35, "v_readfirstlane", "v_readfirstlane_b32 s20, %0") \
  X(36, "v_mul_lo_u32", "v_mul_lo_u32 %0, %0, %1") \
  X(37, "add+ds_read(1:4)", "v_add_u32 %0, %0, %1")

template <int KIND>
__device__ __forceinline__ void op(unsigned& x, unsigned a0, unsigned a7) {
#define X(k, name, txt) \
  if (KIND == k) asm volatile(txt : "+v"(x) : "v"(a0), "v"(a7) : "vcc", "scc", "s20", "s21", "s22");
  KINDS(X)
#undef X
}

template <int KIND>
__global__ void __launch_bounds__(1024) probe(int active, int iters, unsigned* out) {
  extern __shared__ unsigned lds[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave >= active) return;
  unsigned a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 11, a5 = a0 + 13, a6 = a0 ^ 17,
           a7 = a0 ^ 19, a8 = a0 | 23;
  lds[threadIdx.x] = a0;
  unsigned r = 0;
  for (int i = 0; i < iters; ++i) {
#define OP(x) op<KIND>(x, a0, a7);
#define EIGHT OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7) OP(a8)
    EIGHT EIGHT
    if (KIND == 37) {  // one LDS read per four VALU
      unsigned t0, t1, t2, t3;
      asm volatile("ds_read_b32 %0, %4\n\tds_read_b32 %1, %4 offset:256\n\tds_read_b32 %2, %4 offset:512\n\t"
                   "ds_read_b32 %3, %4 offset:768\n\ts_waitcnt lgkmcnt(0)"
                   : "=v"(t0), "=v"(t1), "=v"(t2), "=v"(t3)
                   : "v"(threadIdx.x * 4));
      r += t0 ^ t1 ^ t2 ^ t3;
    }
  }
  out[blockIdx.x * 1024 + threadIdx.x] = a1 + a2 + a3 + a4 + a5 + a6 + a7 + a8 + r;
}

template <int KIND>
void run(const char* name, unsigned* d) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 32768;
  float t[4];
  for (int a = 1; a <= 4; ++a) {
    for (int w = 0; w < 3; ++w) probe<KIND><<<256, 1024, 4096>>>(4 * a, iters, d);
    (void)hipEventRecord(e0);
    probe<KIND><<<256, 1024, 4096>>>(4 * a, iters, d);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    t[a - 1] = ms * 1e6f / (a * iters * 16.0f);  // ns per (16-op group member) per SIMD
  }
  printf("%-18s ns/instr/SIMD at 1,2,3,4 waves per SIMD: %.2f %.2f %.2f %.2f\n", name, t[0], t[1], t[2], t[3]);
}

int main() {
  unsigned* d;
  setvbuf(stdout, nullptr, _IONBF, 0);
  (void)hipMalloc(&d, 256 * 1024 * 4);
#define R(k, name, txt) run<k>(name, d);
  KINDS(R)
  return 0;
}
