// Probe: semantics of gfx950 v_ashr_pk_u8_i32 (operand order, saturation, upper bits).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out, int a, int b, int sh) {
  unsigned d = 0xDEADBEEFu;
  asm volatile("v_ashr_pk_u8_i32 %0, %1, %2, %3" : "+v"(d) : "v"(a), "v"(b), "v"(sh));
  out[threadIdx.x] = d;
}
int main() {
  unsigned* o;
  hipMalloc(&o, 64 * 4);
  const int cases[][3] = {{10, 20, 0}, {-5, 300, 0}, {256, 255, 0}, {1000, -1000, 2}, {0x12, 0x34, 0}};
  for (auto& c : cases) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, c[0], c[1], c[2]);
    unsigned h;
    hipMemcpy(&h, o, 4, hipMemcpyDeviceToHost);
    std::printf("a=%d b=%d sh=%d -> 0x%08x\n", c[0], c[1], c[2], h);
  }
  return 0;
}
