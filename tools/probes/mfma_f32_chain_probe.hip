// Probe: dependent-chain cycles of an fp32 fused multiply-add chain as
// v_fma_f32, v_mfma_f32_4x4x1_16b_f32 (one k step per instruction) and
// v_mfma_f32_16x16x4_f32 (four k steps), one wave alone; and whether the
// 4x4x1 MFMA chain equals the fmaf chain bit for bit under the layout
// D[block b][row r][col c] += A[lane 4b + r] * B[lane 4b + c], D in lane
// 4b + c, register r.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstring>
typedef float v4f __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void bench(const float *in, float *out, unsigned long long *t)
{
  const int l = threadIdx.x;
  float a = in[l], b = in[64 + l];
  float y = 0.f;
  v4f c = {0.f, 0.f, 0.f, 0.f}, c1 = c, c2 = c;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 16; i++) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (MODE == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(y) : "v"(a), "v"(b));
      if (MODE == 1) asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
      if (MODE == 2) asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
      if (MODE == 3) {
        asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
        asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(c1) : "v"(a), "v"(b));
        asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(c2) : "v"(a), "v"(b));
      }
    }
  }
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
  const float s = y + c.x + c.y + c.z + c.w + c1.x + c2.x;
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = s;
  if (l == 0) t[0] = t1 - t0;
}

/* the same chains through the compiler intrinsics (the compiler inserts
 * whatever wait states the dependent MFMAs need): time per k step */
template <int MODE>
__global__ void chain_timed(const float *A, const float *B, float *out, unsigned long long *t, int K)
{
  const int l = threadIdx.x;
  constexpr int R = 32; /* operands in registers, the chain repeated K / R times */
  float a[R], b[R];
#pragma unroll
  for (int k = 0; k < R; k++) { a[k] = A[k * 64 + l]; b[k] = B[k * 64 + l]; }
  v4f c = {0.f, 0.f, 0.f, 0.f};
  float y = 0.f;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < K / R; i++) {
    if (MODE == 0) {
#pragma unroll
      for (int k = 0; k < R; k++) y = __builtin_fmaf(a[k], b[k], y);
    }
    if (MODE == 1) {
#pragma unroll
      for (int k = 0; k < R; k++) c = __builtin_amdgcn_mfma_f32_4x4x1f32(a[k], b[k], c, 0, 0, 0);
    }
    if (MODE == 2) {
#pragma unroll
      for (int k = 0; k < R; k += 4) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[k], b[k], c, 0, 0, 0);
    }
    asm volatile("" : "+v"(y), "+v"(c));
  }
  const float s = y + c.x + c.y + c.z + c.w;
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = s;
  if (l == 0) t[0] = t1 - t0;
}

/* 4x4x1 chain over K steps with per-step operands; out[l*4+r] = D */
__global__ void chain(const float *A, const float *B, float *out, int K)
{
  const int l = threadIdx.x;
  v4f c = {0.25f, -0.5f, 1.f / 3.f, 7.f};
  for (int k = 0; k < K; k++)
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(A[k * 64 + l], B[k * 64 + l], c, 0, 0, 0);
  for (int r = 0; r < 4; r++) out[l * 4 + r] = c[r];
}

int main()
{
  float *in, *out; unsigned long long *t;
  (void)hipMalloc(&in, 128 * 4); (void)hipMalloc(&out, 64 * 4); (void)hipMalloc(&t, 8);
  (void)hipMemset(in, 0, 128 * 4);
  const char *names[4] = {"v_fma_f32 dependent", "4x4x1_16b_f32 dependent", "16x16x4_f32 dependent", "4x4x1_16b_f32 3 accs"};
  const double steps[4] = {1, 1, 4, 3};
  for (int rep = 0; rep < 2; rep++)
    for (int m = 0; m < 4; m++) {
      if (m == 0) hipLaunchKernelGGL(bench<0>, dim3(1), dim3(64), 0, 0, in, out, t);
      if (m == 1) hipLaunchKernelGGL(bench<1>, dim3(1), dim3(64), 0, 0, in, out, t);
      if (m == 2) hipLaunchKernelGGL(bench<2>, dim3(1), dim3(64), 0, 0, in, out, t);
      if (m == 3) hipLaunchKernelGGL(bench<3>, dim3(1), dim3(64), 0, 0, in, out, t);
      unsigned long long h;
      (void)hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%-26s %.1f cycles/instr, %.2f cycles per k step\n", names[m], h / 64.0, h / 64.0 / steps[m]);
    }
  /* exactness of the 4x4x1 chain vs fmaf, incl. denormal and signed-zero cases */
  const int K = 384;
  float *hA = new float[K * 64], *hB = new float[K * 64], hO[256];
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) / 16777216.f - 0.5f) * 2.f; };
  for (int i = 0; i < K * 64; i++) {
    hA[i] = rnd();
    hB[i] = rnd();
    if (i % 97 == 0) hA[i] = 1e-39f;   /* denormal operand */
    if (i % 89 == 0) hB[i] = -0.f;
  }
  float *dA, *dB, *dO;
  (void)hipMalloc(&dA, K * 64 * 4); (void)hipMalloc(&dB, K * 64 * 4); (void)hipMalloc(&dO, 256 * 4);
  (void)hipMemcpy(dA, hA, K * 64 * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB, K * 64 * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, dA, dB, dO, K);
  (void)hipMemcpy(hO, dO, 256 * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; l++)
    for (int r = 0; r < 4; r++) {
      const int b = l / 4, col = l % 4;
      const float init[4] = {0.25f, -0.5f, 1.f / 3.f, 7.f};
      float y = init[r];
      for (int k = 0; k < K; k++) y = fmaf(hA[k * 64 + 4 * b + r], hB[k * 64 + 4 * b + col], y);
      if (memcmp(&y, &hO[l * 4 + r], 4)) {
        if (bad < 4) printf("mismatch lane %d reg %d: mfma %a fmaf %a\n", l, r, hO[l * 4 + r], y);
        bad++;
      }
    }
  printf("4x4x1_16b_f32 chain of %d steps vs fmaf: %d of 256 outputs differ\n", K, bad);
  /* operands from global memory (L1/L2-resident after the first pass) */
  const char *tn[3] = {"fmaf chain (intrinsic)", "4x4x1_16b_f32 chain (intrinsic)", "16x16x4_f32 chain (intrinsic)"};
  for (int m = 0; m < 3; m++)
    for (int rep = 0; rep < 3; rep++) {
      if (m == 0) hipLaunchKernelGGL(chain_timed<0>, dim3(1), dim3(64), 0, 0, dA, dB, out, t, K);
      if (m == 1) hipLaunchKernelGGL(chain_timed<1>, dim3(1), dim3(64), 0, 0, dA, dB, out, t, K);
      if (m == 2) hipLaunchKernelGGL(chain_timed<2>, dim3(1), dim3(64), 0, 0, dA, dB, out, t, K);
      unsigned long long h;
      (void)hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
      if (rep == 2) printf("%-34s %.2f per k step (%d steps, operands in registers)\n", tn[m], h / (double)K, K);
    }
  return 0;
}
