// Probe: issue and dependent-chain cycles of the i8 MFMAs used by mf_kernel
// (one wave per SIMD, operands in registers, s_memtime around 64 MFMAs).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void bench(const v4i *in, v4i *out, unsigned long long *t) {
  const int l = threadIdx.x;
  v4i a = in[l], b = in[64 + l];
  int a1 = a.x, b1 = b.x;
  v4i c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 16; i++) {
    if (MODE == 0) {  // 16x16x64 dependent chain
      asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
      asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
      asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
      asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
    } else if (MODE == 1) {  // 16x16x64, 4 independent accumulators
      asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
      asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(c1) : "v"(a), "v"(b));
      asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(c2) : "v"(a), "v"(b));
      asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(c3) : "v"(a), "v"(b));
    } else if (MODE == 2) {  // 4x4x4_16b dependent chain
      asm volatile("v_mfma_i32_4x4x4_16b_i8 %0, %1, %2, %0" : "+v"(c0) : "v"(a1), "v"(b1));
      asm volatile("v_mfma_i32_4x4x4_16b_i8 %0, %1, %2, %0" : "+v"(c0) : "v"(a1), "v"(b1));
      asm volatile("v_mfma_i32_4x4x4_16b_i8 %0, %1, %2, %0" : "+v"(c0) : "v"(a1), "v"(b1));
      asm volatile("v_mfma_i32_4x4x4_16b_i8 %0, %1, %2, %0" : "+v"(c0) : "v"(a1), "v"(b1));
    } else {  // 4x4x4_16b, 4 independent accumulators
      asm volatile("v_mfma_i32_4x4x4_16b_i8 %0, %1, %2, %0" : "+v"(c0) : "v"(a1), "v"(b1));
      asm volatile("v_mfma_i32_4x4x4_16b_i8 %0, %1, %2, %0" : "+v"(c1) : "v"(a1), "v"(b1));
      asm volatile("v_mfma_i32_4x4x4_16b_i8 %0, %1, %2, %0" : "+v"(c2) : "v"(a1), "v"(b1));
      asm volatile("v_mfma_i32_4x4x4_16b_i8 %0, %1, %2, %0" : "+v"(c3) : "v"(a1), "v"(b1));
    }
  }
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
  v4i s = c0 + c1 + c2 + c3;
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = s;
  if (l == 0) t[0] = t1 - t0;
}

int main() {
  v4i *in, *out; unsigned long long *t;
  (void)hipMalloc(&in, 128 * 16); (void)hipMalloc(&out, 64 * 16); (void)hipMalloc(&t, 8);
  (void)hipMemset(in, 1, 128 * 16);
  const char *names[4] = {"16x16x64_i8 dependent", "16x16x64_i8 4 accs", "4x4x4_16b_i8 dependent", "4x4x4_16b_i8 4 accs"};
  for (int rep = 0; rep < 2; rep++)
    for (int m = 0; m < 4; m++) {
      if (m == 0) hipLaunchKernelGGL(bench<0>, dim3(1), dim3(64), 0, 0, in, out, t);
      if (m == 1) hipLaunchKernelGGL(bench<1>, dim3(1), dim3(64), 0, 0, in, out, t);
      if (m == 2) hipLaunchKernelGGL(bench<2>, dim3(1), dim3(64), 0, 0, in, out, t);
      if (m == 3) hipLaunchKernelGGL(bench<3>, dim3(1), dim3(64), 0, 0, in, out, t);
      unsigned long long h;
      (void)hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
      printf("%-26s %.1f cycles/MFMA\n", names[m], h / 64.0);
    }
  return 0;
}
