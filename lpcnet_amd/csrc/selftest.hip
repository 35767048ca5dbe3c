/*
 * selftest.hip -- the device numerics of device_math.h evaluated elementwise
 * on the GPU, so tests can pin each routine the sample kernels use against
 * the reference's own compiled kernels (tests/golden/kernels.npz: NaN, inf
 * and denormal inputs included) independently of the end-to-end PCM tests.
 * Diagnostic C-ABI, not part of the synthesis path.
 */
#include <hip/hip_runtime.h>

#include <vector>

#include "device_math.h"
#include "lpcnet.h"
#include "lpcnet_engine.h"
#include "lpcnet_mi355x.h"
#include "pow10_dd.h"

namespace lpcnet_mi355x {

/* op codes: see lpcnet_mi355x_device_numerics in include/lpcnet_mi355x.h */
__global__ void numerics_kernel(int op, const uint32_t *__restrict__ in, uint32_t *__restrict__ out, int n,
                                const uint32_t *__restrict__ rcp_g)
{
  __shared__ uint32_t rcp[RCP_ENTRIES];
  for (int k = threadIdx.x; k < RCP_ENTRIES; k += blockDim.x) rcp[k] = rcp_g[k];
  __syncthreads();
  if (op == 8) {
    /* kiss99 (kiss99.c:59-81): n draws from the state in[0..3], one lane */
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      uint32_t z = in[0], w = in[1], j = in[2], c = in[3];
      for (int k = 0; k < n; k++) out[k] = kiss99_next(z, w, j, c);
    }
    return;
  }
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const float x = __uint_as_float(in[e]);
  switch (op) {
    case 0: out[e] = __float_as_uint(tanh_x86(x, rcp)); break;
    case 1: out[e] = __float_as_uint(sigmoid_x86(x, rcp)); break;
    case 2: {
      float v[1] = {x};
      tanh_x86_n<1, true>(v, rcp);
      out[e] = __float_as_uint(v[0]);
      break;
    }
    case 3: {
      float v[1] = {x};
      sigmoid_x86_n<1, true>(v, rcp);
      out[e] = __float_as_uint(v[0]);
      break;
    }
    case 4: out[e] = quant_s8(x) ^ 0x80u; break; /* vector_ps_to_epi8 byte */
    case 5: out[e] = (uint32_t)lin2ulaw_x86(x); break;
    case 6: out[e] = (uint32_t)round_half_up(x); break;
    case 7: out[e] = (uint32_t)cvt_rne(x); break;
    case 9: {
      /* band power of lpc_from_cepstrum (freq.c:318) with compensation[e % 18] */
      const float comp[18] = {0.8f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 0.666667f, 0.5f, 0.5f, 0.5f,
                              0.333333f, 0.25f, 0.25f, 0.2f, 0.166667f, 0.173913f};
      out[e] = __float_as_uint((float)(pow10_dd((double)x) * (double)comp[e % 18]));
      break;
    }
    case 10: out[e] = __float_as_uint(rcp_x86<true>(x, rcp)); break; /* rcpps of a Pade denominator, hardware form */
    case 11: {
      /* sigmoid of the int8 products' gates: inputs |x| < 2^18 only */
      float v[1] = {x};
      sigmoid_x86_fin_n<1, true>(v, rcp);
      out[e] = __float_as_uint(v[0]);
      break;
    }
    case 12: {
      float v[1] = {x};
      sigmoid_x86_fin_n<1, false>(v, rcp); /* the table form */
      out[e] = __float_as_uint(v[0]);
      break;
    }
    default: out[e] = 0; break;
  }
}

}  // namespace lpcnet_mi355x

using namespace lpcnet_mi355x;

extern "C" LPCNET_EXPORT int lpcnet_mi355x_device_numerics(int device, int op, const void *in, void *out, int n)
{
  if (op < 0 || op > 12 || n < 0 || (n > 0 && (!in || !out))) return -1;
  if (n == 0) return 0;
  if (hipSetDevice(device) != hipSuccess) return -1;
  const size_t nin = op == 8 ? 4 : (size_t)n;
  uint32_t *d_in = nullptr, *d_out = nullptr, *d_rcp = nullptr;
  const uint32_t *tab = lpcnet_mi355x_rcp_table();
  std::vector<uint32_t> rcp_dev(RCP_ENTRIES);
  for (int i = 0; i < RCP_ENTRIES; i++) rcp_dev[i] = tab[i >> (RCP_TABLE_BITS - 11)] + kRcpBias; /* 11-bit x86 table */
  int rc = -1;
  if (hipMalloc(&d_in, nin * 4) == hipSuccess && hipMalloc(&d_out, (size_t)n * 4) == hipSuccess &&
      hipMalloc(&d_rcp, RCP_ENTRIES * 4) == hipSuccess && hipMemcpy(d_in, in, nin * 4, hipMemcpyHostToDevice) == hipSuccess &&
      hipMemcpy(d_rcp, rcp_dev.data(), RCP_ENTRIES * 4, hipMemcpyHostToDevice) == hipSuccess) {
    const int grid = op == 8 ? 1 : (n + 255) / 256;
    hipLaunchKernelGGL(numerics_kernel, dim3(grid), dim3(256), 0, 0, op, d_in, d_out, n, d_rcp);
    if (hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
        hipMemcpy(out, d_out, (size_t)n * 4, hipMemcpyDeviceToHost) == hipSuccess)
      rc = 0;
  }
  (void)hipFree(d_in);
  (void)hipFree(d_out);
  (void)hipFree(d_rcp);
  return rc;
}
