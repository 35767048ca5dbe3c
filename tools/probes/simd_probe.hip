/*
 * simd_probe.hip -- which SIMD does wave w of a 512-thread workgroup run on?
 * (HW_REG_HW_ID: WAVE_ID [3:0], SIMD_ID [5:4], CU_ID [11:8]).  One
 * workgroup per CU (the mf_kernel shape: 8 waves at 2 waves per SIMD),
 * a few workgroups reported.
 * Build: hipcc --offload-arch=gfx950 -O2 simd_probe.hip -o simd_probe
 */
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(512) void k(int *out)
{
  extern __shared__ int pad[];
  const int hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | ((32 - 1) << 11));
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + threadIdx.x / 64] = hw;
  if (threadIdx.x == 0) pad[0] = hw;
}

int main()
{
  const int G = 256;
  int *d;
  (void)hipMalloc(&d, G * 8 * sizeof(int));
  (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  hipLaunchKernelGGL(k, dim3(G), dim3(512), 96 * 1024, 0, d);
  int h[G * 8];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int hist[8][4] = {};
  for (int b = 0; b < G; b++)
    for (int w = 0; w < 8; w++) hist[w][(h[b * 8 + w] >> 4) & 3]++;
  for (int b = 0; b < 3; b++) {
    printf("wg %d:", b);
    for (int w = 0; w < 8; w++) printf(" w%d->simd%d", w, (h[b * 8 + w] >> 4) & 3);
    printf("\n");
  }
  printf("histogram over %d workgroups (wave: simd0..3):\n", G);
  for (int w = 0; w < 8; w++) printf("  w%d: %d %d %d %d\n", w, hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
  (void)hipFree(d);
  return 0;
}
