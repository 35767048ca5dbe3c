// Probe: operand/result lane layout and issue/latency cycles of the i8 MFMAs
// the GRU matvecs could use on gfx950 (v_mfma_i32_4x4x4_16b_i8,
// v_mfma_i32_16x16x64_i8).  Diagnostic only; not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void layout4(const int *a, const int *b, v4i *c) {
  int l = threadIdx.x;
  v4i acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_4x4x4i8(a[l], b[l], acc, 0, 0, 0);
  c[l] = acc;
}

template <int DEP>
__global__ void time4(const int *a, const int *b, v4i *c, unsigned long long *t) {
  int l = threadIdx.x;
  int x = a[l], y = b[l];
  v4i acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 64; i++) {
    if (DEP) {
      acc0 = __builtin_amdgcn_mfma_i32_4x4x4i8(x, y, acc0, 0, 0, 0);
    } else {
      acc0 = __builtin_amdgcn_mfma_i32_4x4x4i8(x, y, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_i32_4x4x4i8(x, y, acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_i32_4x4x4i8(x, y, acc2, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_i32_4x4x4i8(x, y, acc3, 0, 0, 0);
    }
  }
  v4i s = acc0 + acc1 + acc2 + acc3;
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  c[l] = s;
  if (l == 0) t[0] = t1 - t0;
}

typedef int v4 __attribute__((ext_vector_type(4)));
__global__ void time16(const v4 *a, const v4 *b, v4i *c, unsigned long long *t) {
  int l = threadIdx.x;
  v4 x = a[l], y = b[l];
  v4i acc0 = {0, 0, 0, 0};
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 64; i++) acc0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, y, acc0, 0, 0, 0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  c[l] = acc0;
  if (l == 0) t[0] = t1 - t0;
}

int main() {
  int *da, *db; v4i *dc; unsigned long long *dt;
  hipMalloc(&da, 64 * 16); hipMalloc(&db, 64 * 16); hipMalloc(&dc, 64 * 16); hipMalloc(&dt, 8);
  std::vector<int> A(64), B(64); std::vector<v4i> C(64);
  // test 1: A = 1 everywhere, B byte k of lane l = (l+1) if k==0 -> C shows which B lane feeds (lane, reg)
  // test 2: B = 1 everywhere, A byte 0 of lane l = l+1 -> C shows which A lane feeds
  // test 3: A lane l = byte k set to 1 only for k == kk, B lane l byte kk = l+1 (probe K pairing)
  for (int test = 0; test < 3; test++) {
    for (int l = 0; l < 64; l++) {
      if (test == 0) { A[l] = 0x01010101; B[l] = l + 1; }
      else if (test == 1) { B[l] = 0x01010101; A[l] = l + 1; }
      else { A[l] = 0x01000000; B[l] = (l + 1) << 24; }
    }
    hipMemcpy(da, A.data(), 256, hipMemcpyHostToDevice);
    hipMemcpy(db, B.data(), 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(layout4, dim3(1), dim3(64), 0, 0, da, db, dc);
    hipMemcpy(C.data(), dc, 64 * 16, hipMemcpyDeviceToHost);
    printf("test %d:", test);
    for (int l = 0; l < 64; l++) printf(" [%d:%d,%d,%d,%d]", l, C[l][0], C[l][1], C[l][2], C[l][3]);
    printf("\n");
  }
  unsigned long long t;
  for (int r = 0; r < 3; r++) {
    hipLaunchKernelGGL(time4<1>, dim3(1), dim3(64), 0, 0, da, db, dc, dt);
    hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
    printf("4x4x4_16b_i8 dependent chain: %.1f cyc/mfma\n", t / 64.0);
    hipLaunchKernelGGL(time4<0>, dim3(1), dim3(64), 0, 0, da, db, dc, dt);
    hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
    printf("4x4x4_16b_i8 4 independent accs: %.1f cyc/mfma\n", t / 256.0);
    hipLaunchKernelGGL(time16, dim3(1), dim3(64), 0, 0, (const v4 *)da, (const v4 *)db, dc, dt);
    hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
    printf("16x16x64_i8 dependent chain: %.1f cyc/mfma\n", t / 64.0);
  }
  return 0;
}
