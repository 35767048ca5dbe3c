// Probe: issue cost (cycles per instruction, 8 independent chains per wave)
// of the VALU ops the GRU_A elementwise step uses, with one wave alone on its
// SIMD (64 threads) and with two waves per SIMD (512 threads: waves w, w+4
// share a SIMD): if the two-wave figure doubles, one wave already saturates
// the SIMD's VALU; packed f32 ops included.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
typedef float v2f __attribute__((ext_vector_type(2)));

template <int OP>
__global__ void bench(const float *in, float *out, unsigned long long *t)
{
  const int l = threadIdx.x;
  float v[8];
  int iv[8];
  v2f p[8];
  for (int k = 0; k < 8; k++) { v[k] = in[l] + k; iv[k] = (int)in[l] + k; p[k] = v2f{v[k], v[k] + 1.f}; }
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
    if (OP == 9) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v[k]) : "v"(v[(k + 3) & 7]));           \
    if (OP == 10) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p[k]) : "v"(p[(k + 3) & 7]));  \
    if (OP == 11) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[k]) : "v"(p[(k + 3) & 7]));      \
    if (OP == 12) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[k]) : "v"(p[(k + 3) & 7]));      \
    if (OP == 13) asm volatile("v_and_b32 %0, 0x7f800000, %0" : "+v"(iv[k]));                       \
    if (OP == 14) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(iv[k]) : "v"(iv[(k + 1) & 7]));
    REP8(STEP)
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int k = 0; k < 8; k++) s += v[k] + (float)iv[k] + p[k].x + p[k].y;
  out[l] = s;
  if ((l & 63) == 0) t[l >> 6] = t1 - t0;
}

template <int OP>
static void run(int threads, const float *in, float *out, unsigned long long *t)
{
  hipLaunchKernelGGL(bench<OP>, dim3(1), dim3(threads), 0, 0, in, out, t);
}

int main()
{
  float *in, *out; unsigned long long *t;
  (void)hipMalloc(&in, 512 * 4); (void)hipMalloc(&out, 512 * 4); (void)hipMalloc(&t, 8 * 8);
  (void)hipMemset(in, 0, 512 * 4);
  const char *names[15] = {"v_add_f32", "v_cvt_i32_f32", "v_rndne_f32", "v_cvt_f32_i32", "v_cvt_pk_u8_f32",
                           "v_med3_f32", "v_rcp_f32", "v_fma_f32", "v_bfe_u32", "v_mul_f32",
                           "v_pk_fma_f32", "v_pk_mul_f32", "v_pk_add_f32", "v_and_b32", "v_sub_u32"};
  void (*fns[15])(int, const float *, float *, unsigned long long *) = {
      run<0>, run<1>, run<2>, run<3>, run<4>, run<5>, run<6>, run<7>, run<8>, run<9>, run<10>, run<11>, run<12>, run<13>, run<14>};
  for (int op = 0; op < 15; op++) {
    double c[2];
    for (int m = 0; m < 2; m++) {
      const int threads = m ? 512 : 64;
      for (int rep = 0; rep < 2; rep++) fns[op](threads, in, out, t);
      unsigned long long h[8];
      (void)hipMemcpy(h, t, 8 * 8, hipMemcpyDeviceToHost);
      unsigned long long mx = 0;
      for (int w = 0; w < threads / 64; w++) mx = h[w] > mx ? h[w] : mx;
      c[m] = mx / 256.0;
    }
    printf("%-16s %.2f cycles/instr one wave per SIMD, %.2f with two waves per SIMD\n", names[op], c[0], c[1]);
  }
  return 0;
}
