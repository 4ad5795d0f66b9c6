// Probe: cost of a workgroup barrier and of an LDS round trip between barriers (gfx950), the
// two things K7 (vp8l_resolve.hip) pays per 4096-pixel block.  One 1024-thread workgroup per CU
// (256 workgroups), each runs N iterations of: [optional LDS write + read of a neighbour's
// word] + __syncthreads().  Prints ns per iteration.
// Build: hipcc -w --offload-arch=gfx950 -O3 barrier_rate.hip -o barrier_rate
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(1024) probe(int iters, unsigned* out) {
  __shared__ unsigned buf[1024];
  unsigned x = threadIdx.x;
  buf[threadIdx.x] = x;
  __syncthreads();
  for (int i = 0; i < iters; ++i) {
    if (MODE >= 1) {  // one dependent LDS round trip through another wave's word
      buf[threadIdx.x] = x;
      __syncthreads();
      x += buf[(threadIdx.x + 64 * (i & 15) + 1) & 1023];
    }
    if (MODE == 2) {  // plus 100 dependent VALU ops
#pragma unroll
      for (int k = 0; k < 100; ++k) asm volatile("v_add_u32 %0, %0, 1" : "+v"(x));
    }
    __syncthreads();
  }
  if (x == 0xdeadbeef) out[0] = x;
}

int main() {
  unsigned* d;
  hipMalloc(&d, 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 20000;
  const char* names[3] = {"barrier only", "LDS round trip + 2 barriers", "LDS round trip + 100 VALU + 2 barriers"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(256), dim3(1024), 0, 0, iters, d);
      if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(256), dim3(1024), 0, 0, iters, d);
      if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(256), dim3(1024), 0, 0, iters, d);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep) printf("%-44s %8.1f ns per iteration\n", names[mode], ms * 1e6 / iters);
    }
  }
  return 0;
}
