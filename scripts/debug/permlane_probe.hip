// Probe of v_permlane32_swap semantics (which halves move, which builtin result is which).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  const unsigned l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane32_swap(1000u + l, 2000u + l, false, false);
  o[l] = r[0];
  o[64 + l] = r[1];
}
int main() {
  unsigned* d;
  unsigned h[128];
  hipMalloc(&d, 512);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  printf("r0: lane0 %u lane31 %u lane32 %u lane63 %u\n", h[0], h[31], h[32], h[63]);
  printf("r1: lane0 %u lane31 %u lane32 %u lane63 %u\n", h[64], h[95], h[96], h[127]);
  return 0;
}
