// Probe: does v_cvt_pk_u8_f32 round to nearest even, saturate to [0,255] and
// map NaN to 0 on gfx950?  Compares against sat_u8(rne(x)) for a sweep of
// inputs (every float in [-2, 258] at 1/64 steps, halves, specials).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <vector>

__global__ void k(const float *x, unsigned *o, int n)
{
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = __builtin_amdgcn_cvt_pk_u8_f32(x[i], 0, 0u) & 0xffu;
}

int main()
{
  std::vector<float> x;
  for (int i = -256; i <= 258 * 64; i++) x.push_back(i / 64.f);
  for (int i = -2; i < 260; i++) x.push_back(i + 0.5f);
  const float sp[] = {NAN, -NAN, INFINITY, -INFINITY, 2147483648.f, 4e9f, -4e9f, 1e-40f, -0.f, 255.49f, 255.5f, 254.5f, 0.5f, 1.5f, 2.5f};
  for (float f : sp) x.push_back(f);
  int n = (int)x.size();
  float *dx; unsigned *dout;
  hipMalloc(&dx, n * 4); hipMalloc(&dout, n * 4);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dout, n);
  std::vector<unsigned> o(n);
  hipMemcpy(o.data(), dout, n * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; i++) {
    float r = rintf(x[i]);
    unsigned e = (x[i] != x[i]) ? 0u : (r <= 0 ? 0u : (r >= 255 ? 255u : (unsigned)r));
    if (o[i] != e) { if (bad++ < 20) printf("x=%a got %u expected(sat rne) %u\n", x[i], o[i], e); }
  }
  printf("%d inputs, %d differ from sat_u8(rne(x)) with NaN->0\n", n, bad);
  return 0;
}
