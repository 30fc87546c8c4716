// probe: which XCD (s_getreg HW_REG_XCC_ID) each block of a 256-block launch runs on
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (threadIdx.x == 0) out[blockIdx.x] = (int)x;
}
int main() {
  int* d; int h[256];
  hipMalloc(&d, 256 * sizeof(int));
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k, dim3(256), dim3(256), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int cnt[16] = {0};
    for (int b = 0; b < 256; ++b) cnt[h[b] & 15]++;
    printf("rep %d: first 16:", rep);
    for (int b = 0; b < 16; ++b) printf(" %d", h[b]);
    printf(" | raw[0]=0x%x counts:", h[0]);
    for (int i = 0; i < 16; ++i) printf(" %d", cnt[i]);
    printf("\n");
  }
  return 0;
}
