// Probe: dependent v_fma_f32 chain cycles (1..4 interleaved chains, one wave),
// ds_read_b128 / global_load pointer-chase latency, s_memtime around the loop.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void bench(const float *in, float *out, unsigned long long *t, const int *chase)
{
  extern __shared__ int lds[];
  const int l = threadIdx.x;
  float a = in[l], b = in[64 + l];
  float c0 = in[128 + l], c1 = c0 + 1.f, c2 = c0 + 2.f, c3 = c0 + 3.f;
  for (int k = l; k < 4096; k += 64) lds[k] = chase[k];
  int p = l & 0;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 16; i++) {
    if (MODE == 0) {
#pragma unroll
      for (int k = 0; k < 16; k++) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
    } else if (MODE == 1) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c1) : "v"(a), "v"(b));
      }
    } else if (MODE == 2) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c1) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c2) : "v"(a), "v"(b));
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c3) : "v"(a), "v"(b));
      }
    } else if (MODE == 5) { /* dependent chain, lanes 0..31 active */
      if (l < 32) {
#pragma unroll
        for (int k = 0; k < 16; k++) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
      }
    } else if (MODE == 6) { /* dependent chain, lanes 0..15 active */
      if (l < 16) {
#pragma unroll
        for (int k = 0; k < 16; k++) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
      }
    } else if (MODE == 7) { /* dependent packed chain */
      typedef float v2f __attribute__((ext_vector_type(2)));
      v2f p = {c0, c1}, q = {a, b};
#pragma unroll
      for (int k = 0; k < 16; k++) asm volatile("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(p) : "v"(q));
      c0 = p.x; c1 = p.y;
    } else if (MODE == 8) { /* dependent v_fmac_f32 */
#pragma unroll
      for (int k = 0; k < 16; k++) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(c0) : "v"(a), "v"(b));
    } else if (MODE == 3) { /* LDS pointer chase, 16 hops */
#pragma unroll
      for (int k = 0; k < 16; k++) p = lds[p];
    } else { /* global (L2) pointer chase, 16 hops */
#pragma unroll
      for (int k = 0; k < 16; k++) p = __builtin_nontemporal_load(chase + p);
    }
  }
  asm volatile("s_nop 7\n s_nop 7" ::: "memory");
  float s = c0 + c1 + c2 + c3 + (float)p;
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = s;
  if (l == 0) t[0] = t1 - t0;
}

int main()
{
  float *in, *out;
  unsigned long long *t;
  int *chase;
  (void)hipMalloc(&in, 192 * 4);
  (void)hipMalloc(&out, 64 * 4);
  (void)hipMalloc(&t, 8);
  (void)hipMalloc(&chase, 4096 * 4 * 64);
  (void)hipMemset(in, 0, 192 * 4);
  int h[4096];
  for (int k = 0; k < 4096; k++) h[k] = (k * 64 + 64 * 37) % 4096; /* stride-64 cycle */
  (void)hipMemcpy(chase, h, sizeof(h), hipMemcpyHostToDevice);
  const char *names[9] = {"fma dependent", "fma 2 chains", "fma 4 chains", "lds chase", "global chase",
                          "fma dep 32 lanes", "fma dep 16 lanes", "pk_fma dependent", "fmac dependent"};
  for (int rep = 0; rep < 2; rep++)
    for (int m = 0; m < 9; m++) {
      if (m == 0) hipLaunchKernelGGL(bench<0>, dim3(1), dim3(64), 16384, 0, in, out, t, chase);
      if (m == 1) hipLaunchKernelGGL(bench<1>, dim3(1), dim3(64), 16384, 0, in, out, t, chase);
      if (m == 2) hipLaunchKernelGGL(bench<2>, dim3(1), dim3(64), 16384, 0, in, out, t, chase);
      if (m == 3) hipLaunchKernelGGL(bench<3>, dim3(1), dim3(64), 16384, 0, in, out, t, chase);
      if (m == 4) hipLaunchKernelGGL(bench<4>, dim3(1), dim3(64), 16384, 0, in, out, t, chase);
      if (m == 5) hipLaunchKernelGGL(bench<5>, dim3(1), dim3(64), 16384, 0, in, out, t, chase);
      if (m == 6) hipLaunchKernelGGL(bench<6>, dim3(1), dim3(64), 16384, 0, in, out, t, chase);
      if (m == 7) hipLaunchKernelGGL(bench<7>, dim3(1), dim3(64), 16384, 0, in, out, t, chase);
      if (m == 8) hipLaunchKernelGGL(bench<8>, dim3(1), dim3(64), 16384, 0, in, out, t, chase);
      unsigned long long v;
      (void)hipMemcpy(&v, t, 8, hipMemcpyDeviceToHost);
      printf("%-16s %.1f cycles per instruction / hop\n", names[m], v / 256.0);
    }
  return 0;
}
