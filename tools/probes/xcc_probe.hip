/*
 * xcc_probe.hip -- which XCD does a one-workgroup launch land on, launch
 * after launch?  Two one-workgroup kernels alternate on one stream (the
 * batch-1 frame/sample pattern); each records HW_REG_XCC_ID.  Also a
 * grid-8 launch, to see whether 8 workgroups cover the 8 XCDs.
 * Build: hipcc --offload-arch=gfx950 -O2 xcc_probe.hip -o xcc_probe
 */
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ int xcc_id()
{
  /* s_getreg_b32 HW_REG_XCC_ID (id 20), bits [3:0] */
  return __builtin_amdgcn_s_getreg(20 | (0 << 6) | ((4 - 1) << 11));
}

__global__ void k_a(int *out, int slot)
{
  if (threadIdx.x == 0) out[slot * 8 + blockIdx.x] = xcc_id();
}

__global__ void k_b(int *out, int slot)
{
  if (threadIdx.x == 0) out[slot * 8 + blockIdx.x] = 100 + xcc_id();
}

int main()
{
  const int n = 32;
  int *d;
  hipMalloc(&d, (2 * n + 8) * 8 * sizeof(int));
  hipMemset(d, 0xff, (2 * n + 8) * 8 * sizeof(int));
  for (int i = 0; i < n; i++) {
    hipLaunchKernelGGL(k_b, dim3(1), dim3(256), 0, 0, d, 2 * i);
    hipLaunchKernelGGL(k_a, dim3(1), dim3(512), 0, 0, d, 2 * i + 1);
  }
  for (int i = 0; i < 4; i++) hipLaunchKernelGGL(k_a, dim3(8), dim3(512), 0, 0, d, 2 * n + i);
  int h[(2 * n + 8) * 8];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("alternating 1-WG launches (frame=1xx, sample=x):");
  for (int i = 0; i < 2 * n; i++) printf(" %d", h[i * 8]);
  printf("\ngrid-8 launches:");
  for (int i = 0; i < 4; i++) {
    printf(" [");
    for (int b = 0; b < 8; b++) printf("%d", h[(2 * n + i) * 8 + b]);
    printf("]");
  }
  printf("\n");
  hipFree(d);
  return 0;
}
