// Probe: issue cost (cycles per instruction, one wave alone on its SIMD, 8
// independent chains) of the VALU ops the GRU_A elementwise step uses.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ void bench(const float *in, float *out, unsigned long long *t)
{
  const int l = threadIdx.x;
  float v[8];
  int iv[8];
  for (int k = 0; k < 8; k++) { v[k] = in[l] + k; iv[k] = (int)in[l] + k; }
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 32; i++) {
#define STEP(k)                                                                                     \
    if (OP == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[k]) : "v"(v[(k + 1) & 7]));            \
    if (OP == 1) asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(iv[k]) : "v"(v[k]));                    \
    if (OP == 2) asm volatile("v_rndne_f32 %0, %0" : "+v"(v[k]));                                   \
    if (OP == 3) asm volatile("v_cvt_f32_i32 %0, %1" : "=v"(v[k]) : "v"(iv[k]));                    \
    if (OP == 4) asm volatile("v_cvt_pk_u8_f32 %0, %1, 0, %0" : "+v"(iv[k]) : "v"(v[k]));          \
    if (OP == 5) asm volatile("v_med3_f32 %0, %0, 0, 1.0" : "+v"(v[k]));                            \
    if (OP == 6) asm volatile("v_rcp_f32 %0, %0" : "+v"(v[k]));                                     \
    if (OP == 7) asm volatile("v_fma_f32 %0, %0, %1, 1.0" : "+v"(v[k]) : "v"(v[(k + 3) & 7]));      \
    if (OP == 8) asm volatile("v_bfe_u32 %0, %0, 12, 11" : "+v"(iv[k]));                            \
    if (OP == 9) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(*(unsigned long long *)&iv[k & 6]) : "s"(0ull));
    REP8(STEP)
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int k = 0; k < 8; k++) s += v[k] + (float)iv[k];
  out[l] = s;
  if (l == 0) t[0] = t1 - t0;
}

int main()
{
  float *in, *out; unsigned long long *t;
  (void)hipMalloc(&in, 256 * 4); (void)hipMalloc(&out, 256 * 4); (void)hipMalloc(&t, 8);
  (void)hipMemset(in, 0, 256 * 4);
  const char *names[10] = {"v_add_f32", "v_cvt_i32_f32", "v_rndne_f32", "v_cvt_f32_i32", "v_cvt_pk_u8_f32",
                           "v_med3_f32", "v_rcp_f32", "v_fma_f32", "v_bfe_u32", "v_lshl_add_u64"};
  for (int rep = 0; rep < 2; rep++)
    for (int op = 0; op < 10; op++) {
      switch (op) {
        case 0: hipLaunchKernelGGL(bench<0>, dim3(1), dim3(64), 0, 0, in, out, t); break;
        case 1: hipLaunchKernelGGL(bench<1>, dim3(1), dim3(64), 0, 0, in, out, t); break;
        case 2: hipLaunchKernelGGL(bench<2>, dim3(1), dim3(64), 0, 0, in, out, t); break;
        case 3: hipLaunchKernelGGL(bench<3>, dim3(1), dim3(64), 0, 0, in, out, t); break;
        case 4: hipLaunchKernelGGL(bench<4>, dim3(1), dim3(64), 0, 0, in, out, t); break;
        case 5: hipLaunchKernelGGL(bench<5>, dim3(1), dim3(64), 0, 0, in, out, t); break;
        case 6: hipLaunchKernelGGL(bench<6>, dim3(1), dim3(64), 0, 0, in, out, t); break;
        case 7: hipLaunchKernelGGL(bench<7>, dim3(1), dim3(64), 0, 0, in, out, t); break;
        case 8: hipLaunchKernelGGL(bench<8>, dim3(1), dim3(64), 0, 0, in, out, t); break;
        case 9: hipLaunchKernelGGL(bench<9>, dim3(1), dim3(64), 0, 0, in, out, t); break;
      }
      unsigned long long h;
      (void)hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%-16s %.2f cycles per instruction (8 independent chains, one wave)\n", names[op], h / 256.0);
    }
  return 0;
}
