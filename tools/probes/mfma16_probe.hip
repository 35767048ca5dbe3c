// Probe: v_mfma_i32_16x16x64_i8 operand/result layout on gfx950 (random
// int8 operands; the host checks lane-layout hypotheses).  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k16(const v4i *a, const v4i *b, v4i *c) {
  int l = threadIdx.x;
  v4i acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[l], b[l], acc, 0, 0, 0);
  c[l] = acc;
}
int main() {
  signed char A[64][16], B[64][16];
  srand(7);
  for (int l = 0; l < 64; l++)
    for (int j = 0; j < 16; j++) { A[l][j] = (signed char)(rand() % 255 - 127); B[l][j] = (signed char)(rand() % 255 - 127); }
  v4i *da, *db, *dc;
  (void)hipMalloc(&da, 1024); (void)hipMalloc(&db, 1024); (void)hipMalloc(&dc, 1024);
  (void)hipMemcpy(da, A, 1024, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, B, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, da, db, dc);
  int C[64][4];
  (void)hipMemcpy(C, dc, 1024, hipMemcpyDeviceToHost);
  FILE *f = fopen("gpurun_out/mfma16.bin", "wb");
  fwrite(A, 1, 1024, f); fwrite(B, 1, 1024, f); fwrite(C, 4, 256, f);
  fclose(f);
  printf("C[0] = %d %d %d %d\n", C[0][0], C[0][1], C[0][2], C[0][3]);
  return 0;
}
