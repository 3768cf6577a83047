#include <hip/hip_runtime.h>
__global__ void k(unsigned *o, const unsigned *a, const unsigned *b) {
  const int l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane32_swap(a[l], b[l], false, false);
  o[l] = r[0]; o[64 + l] = r[1];
}
int main() {
  unsigned *a, *b, *o; hipMalloc(&a, 256); hipMalloc(&b, 256); hipMalloc(&o, 512);
  unsigned ha[64], hb[64], ho[128];
  for (int i = 0; i < 64; i++) { ha[i] = i; hb[i] = 100 + i; }
  hipMemcpy(a, ha, 256, hipMemcpyHostToDevice); hipMemcpy(b, hb, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, a, b);
  hipMemcpy(ho, o, 512, hipMemcpyDeviceToHost);
  printf("r0:"); for (int i = 0; i < 64; i += 8) printf(" [%d]=%u", i, ho[i]);
  printf("\nr1:"); for (int i = 0; i < 64; i += 8) printf(" [%d]=%u", i, ho[64 + i]);
  printf("\n");
}
