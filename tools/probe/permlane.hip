// prints what v_permlane16_swap returns for (old = lane, src = 100 + lane)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  const unsigned l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap(l, 100 + l, false, false);
  o[l] = r[0];
  o[64 + l] = r[1];
}
int main() {
  unsigned* d;
  unsigned h[128];
  hipMalloc(&d, 512);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l += 4) printf("lane %2d: r0=%3u r1=%3u\n", l, h[l], h[64 + l]);
  return 0;
}
