// v_permlane32_swap semantics check (diagnostic, GPU box): prints lanes 0, 31, 32, 63 of both results
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  const unsigned a = threadIdx.x, b = 100 + threadIdx.x;
  const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  out[threadIdx.x] = r[0];
  out[64 + threadIdx.x] = r[1];
}
int main() {
  unsigned* d;
  unsigned h[128];
  if (hipMalloc(&d, 512) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int l : {0, 31, 32, 63}) printf("lane %d: r0 %u r1 %u\n", l, h[l], h[64 + l]);
  return hipFree(d) == hipSuccess ? 0 : 1;
}
