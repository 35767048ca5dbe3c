/*
 * lpc_kernel.hip -- lpc_from_cepstrum (freq.c:310-320) for every stream of a
 * batch on the GPU: one wavefront per stream, eight streams per workgroup.
 *
 * Restates, term for term and in the reference's operation order:
 *   idct                 freq.c:230-240   lanes 0..17, one band each
 *   pow(10, Ex)*comp     freq.c:318       pow10_dd.h (double-double, exact
 *                                         against glibc: pow10_exhaustive.c)
 *   interp_band_gain     freq.c:202-216   lane per spectrum bin
 *   inverse_transform    freq.c:256-273   Opus kiss FFT, 320 points, factors
 *                                         4,4,4,5 (kiss_fft.c:101-305, 518-586):
 *                                         one lane per butterfly, LDS between
 *                                         stages, digit-reversed scaled input
 *   lpc_from_bands       freq.c:275-297   noise floor + lag window (double)
 *   lpcn_lpc             freq.c:86-127    Levinson-Durbin, float build, lane 0
 * Must be compiled with -ffp-contract=off.  The output feeds the frame
 * kernel's two-frame LPC ring (lpcnet.c:110-112), so this kernel is two
 * frames ahead of its first use.
 */
#include <hip/hip_runtime.h>

#include "lpcnet_engine.h"
#include "pow10_dd.h"

namespace lpcnet_mi355x {

namespace {

constexpr int WIN = LPC_WIN; /* NBANDS (lpcnet_engine.h) == LPC_NBANDS */
#ifndef LPC_WG_STREAMS
#define LPC_WG_STREAMS 8
#endif
constexpr int LPC_STREAMS = LPC_WG_STREAMS; /* streams (waves) per workgroup */

struct alignas(8) C2 {
  float r, i;
};

__device__ __forceinline__ C2 cmul(C2 a, C2 b) { return C2{a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
__device__ __forceinline__ C2 cadd(C2 a, C2 b) { return C2{a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ C2 csub(C2 a, C2 b) { return C2{a.r - b.r, a.i - b.i}; }

/* radix-4 butterfly j of a group at p (kiss_fft_bfly4, kiss_fft.c:164-214,
 * m > 1 form; m == 1 has no twiddles) */
__device__ __forceinline__ void bfly4(C2 *p, int j, int m, int tstride, const C2 *tw)
{
  if (m == 1) {
    C2 f0 = p[0], f1 = p[1], f2 = p[2], f3 = p[3];
    const C2 s0 = csub(f0, f2);
    f0 = cadd(f0, f2);
    C2 s1 = cadd(f1, f3);
    f2 = csub(f0, s1);
    f0 = cadd(f0, s1);
    s1 = csub(f1, f3);
    p[0] = f0;
    p[2] = f2;
    p[1] = C2{s0.r + s1.i, s0.i - s1.r};
    p[3] = C2{s0.r - s1.i, s0.i + s1.r};
    return;
  }
  C2 *q = p + j;
  const C2 a = cmul(q[m], tw[j * tstride]);
  const C2 b = cmul(q[2 * m], tw[2 * j * tstride]);
  const C2 c = cmul(q[3 * m], tw[3 * j * tstride]);
  C2 q0 = q[0];
  const C2 d = csub(q0, b);
  q0 = cadd(q0, b);
  const C2 e = cadd(a, c), h = csub(a, c);
  q[2 * m] = csub(q0, e);
  q[0] = cadd(q0, e);
  q[m] = C2{d.r + h.i, d.i - h.r};
  q[3 * m] = C2{d.r - h.i, d.i + h.r};
}

/* radix-5 butterfly u of the last stage, m = 64 (kiss_fft_bfly5, kiss_fft.c:255-305) */
__device__ __forceinline__ void bfly5(C2 *f, int u, const C2 *tw)
{
  const int m = 64;
  const C2 ya = tw[m], yb = tw[2 * m];
  C2 *q0 = f + u, *q1 = q0 + m, *q2 = q0 + 2 * m, *q3 = q0 + 3 * m, *q4 = q0 + 4 * m;
  const C2 s0 = *q0;
  const C2 s1 = cmul(*q1, tw[u]), s2 = cmul(*q2, tw[2 * u]), s3 = cmul(*q3, tw[3 * u]), s4 = cmul(*q4, tw[4 * u]);
  const C2 s7 = cadd(s1, s4), s10 = csub(s1, s4), s8 = cadd(s2, s3), s9 = csub(s2, s3);
  C2 r0;
  r0.r = s0.r + (s7.r + s8.r);
  r0.i = s0.i + (s7.i + s8.i);
  const C2 s5{s0.r + ((s7.r * ya.r) + (s8.r * yb.r)), s0.i + ((s7.i * ya.r) + (s8.i * yb.r))};
  const C2 s6{(s10.i * ya.i) + (s9.i * yb.i), -((s10.r * ya.i) + (s9.r * yb.i))};
  const C2 s11{s0.r + ((s7.r * yb.r) + (s8.r * ya.r)), s0.i + ((s7.i * yb.r) + (s8.i * ya.r))};
  const C2 s12{(s9.i * ya.i) - (s10.i * yb.i), (s10.r * yb.i) - (s9.r * ya.i)};
  *q0 = r0;
  *q1 = csub(s5, s6);
  *q4 = cadd(s5, s6);
  *q2 = cadd(s11, s12);
  *q3 = csub(s11, s12);
}

}  // namespace

/* the warm-up of the next tick's chunk kernel weights (deferred form): the
 * workgroups of an XCD (workgroup b runs on XCD b % 8) split every line of
 * the matrices and touch it once; the XOR only keeps the loads alive */
__device__ __forceinline__ void l2_warm_lines(const L2Warm &W)
{
  const int x = blockIdx.x % 8, nx = ((int)gridDim.x - 1 - x) / 8 + 1, k = blockIdx.x / 8;
  uint32_t acc = 0;
#pragma unroll
  for (int t = 0; t < 5; t++)
    for (int o = k * (int)blockDim.x + (int)threadIdx.x; o < W.lines[t]; o += nx * (int)blockDim.x)
      acc ^= W.m[t][(size_t)o * 32];
  asm volatile("" ::"v"(acc));
}

__global__ __launch_bounds__(64 * LPC_STREAMS) void lpc_kernel(const float *features, float *lpc_out, int nstreams,
                                                               const LpcTables *T, StreamState *ring, int ring_depth,
                                                               L2Warm warm)
{
  if (warm.m[0]) l2_warm_lines(warm); /* issued first, in flight under the LPC work */
  __shared__ C2 ybuf[LPC_STREAMS][WIN];
  __shared__ C2 tw[WIN];
  __shared__ float dct[NBANDS * NBANDS];
  __shared__ LpcSlot slot[WIN];
  __shared__ float Eb[LPC_STREAMS][NBANDS + 2];
  __shared__ float acb[LPC_STREAMS][LPC_ORDER1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sid = blockIdx.x * LPC_STREAMS + w;
  const bool live = sid < nstreams; /* wave-uniform */
  /* every global read up front (one round of latency): this stream's
   * cepstrum, then the tables into LDS */
  float ceps[NBANDS];
  if (live && lane < NBANDS) {
    const float *c = features + (size_t)sid * NF;
#pragma unroll
    for (int j = 0; j < NBANDS; j++) ceps[j] = c[j];
  }
  for (int k = threadIdx.x; k < WIN; k += blockDim.x) {
    tw[k] = C2{T->twr[k], T->twi[k]};
    slot[k] = T->slot[k];
  }
  for (int k = threadIdx.x; k < NBANDS * NBANDS; k += blockDim.x) dct[k] = T->dct[k];
  const double sq = T->sqrt_2_18;
  const float cmp = lane < NBANDS ? T->comp[lane] : 0.f, scale = T->scale;
  C2 *y = ybuf[w];
  float *E = Eb[w];
  __syncthreads();

  /* idct + band powers (freq.c:230-240, 316-318) */
  if (live && lane < NBANDS) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < NBANDS; j++) {
      const float t = j == 0 ? ceps[0] + 4 : ceps[j];
      acc += t * dct[lane * NBANDS + j];
    }
    const float ex = (float)((double)acc * sq);
    E[lane] = (float)(pow10_dd((double)ex) * (double)cmp);
  }
  __syncthreads();

  /* scaled Hermitian spectrum in digit-reversed order (freq.c:202-216, 256-268;
   * kiss_fft_stride's input permutation and 1/nfft scaling): FFT slot i holds
   * bin perm[i]; bins above 160 are the conjugates (imaginary -0.f) */
  if (live)
    for (int i = lane; i < WIN; i += 64) {
      const LpcSlot sl = slot[i];
      float g = 0.f;
      if (sl.band < NBANDS - 1) g = (1 - sl.frac) * E[sl.band] + sl.frac * E[sl.band + 1];
      y[i] = C2{scale * g, scale * (sl.conj ? -0.f : 0.f)};
    }
  __syncthreads();
  /* radix-4 stages: (m, groups, span, twiddle stride) = (1, 80, 4, 80), (4, 20, 16, 20), (16, 5, 64, 5) */
  if (live)
    for (int t = lane; t < 80; t += 64) bfly4(y + 4 * t, 0, 1, 80, tw);
  __syncthreads();
  if (live)
    for (int t = lane; t < 80; t += 64) bfly4(y + 16 * (t >> 2), t & 3, 4, 20, tw);
  __syncthreads();
  if (live)
    for (int t = lane; t < 80; t += 64) bfly4(y + 64 * (t >> 4), t & 15, 16, 5, tw);
  __syncthreads();
  if (live) bfly5(y, lane, tw);
  __syncthreads();

  /* autocorrelation, noise floor and lag window (freq.c:268-296) */
  if (live && lane < LPC_ORDER1) {
    float a = WIN * y[lane == 0 ? 0 : WIN - lane].r;
    if (lane == 0) a += a * 1e-4 + 320 / 12 / 38.;
    else a *= (1 - 6e-5 * lane * lane);
    acb[w][lane] = a;
  }
  __syncthreads();

  /* Levinson-Durbin, float build of lpcn_lpc (freq.c:86-127): one lane
   * per stream of the workgroup, all in wave 0 (the recursion is serial: one
   * lane of each wave would issue it four times); fully unrolled, so lpc[]
   * and ac[] stay in registers (a dynamic index into a register array costs
   * a select chain per access) */
  const int lsid = blockIdx.x * LPC_STREAMS + lane;
  if (w == 0 && lane < LPC_STREAMS && lsid < nstreams) {
    float ac[LPC_ORDER1];
#pragma unroll
    for (int i = 0; i < LPC_ORDER1; i++) ac[i] = acb[lane][i];
    float lpc[LPC_ORDER1 - 1];
    float err = ac[0];
#pragma unroll
    for (int i = 0; i < LPC_ORDER1 - 1; i++) lpc[i] = 0;
    if (ac[0] != 0) {
#pragma unroll
      for (int i = 0; i < LPC_ORDER1 - 1; i++) {
        float rr = 0;
#pragma unroll
        for (int j = 0; j < i; j++) rr += lpc[j] * ac[i - j];
        rr += ac[i + 1];
        const float r = -rr / err;
        lpc[i] = r;
#pragma unroll
        for (int j = 0; j < (i + 1) >> 1; j++) {
          const float a = lpc[j], b = lpc[i - 1 - j];
          lpc[j] = a + r * b;
          lpc[i - 1 - j] = b + r * a;
        }
        err = err - (r * r) * err;
        if (err < .001f * ac[0]) break;
      }
    }
    if (ring) {
      /* deferred form (one-frame ticks, FEATURES_DELAY >= 1): push this
       * frame's LPC into the stream's ring (lpcnet.c:110-114: the oldest slot
       * was read by the frame's chunk_kernel already) */
      float4 *q = (float4 *)ring[lsid].old_lpc[0];
      for (int j = ring_depth - 1; j > 0; j--)
#pragma unroll
        for (int i = 0; i < NLPC / 4; i++) q[j * (NLPC / 4) + i] = q[(j - 1) * (NLPC / 4) + i];
#pragma unroll
      for (int i = 0; i < NLPC / 4; i++) q[i] = make_float4(lpc[4 * i], lpc[4 * i + 1], lpc[4 * i + 2], lpc[4 * i + 3]);
      return;
    }
    float4 *o = (float4 *)(lpc_out + (size_t)lsid * NLPC);
#pragma unroll
    for (int i = 0; i < NLPC / 4; i++) o[i] = make_float4(lpc[4 * i], lpc[4 * i + 1], lpc[4 * i + 2], lpc[4 * i + 3]);
  }
}

int launch_lpc(const float *features, float *lpc_out, int nstreams, const LpcTables *tables, void *stream,
               StreamState *ring, int ring_depth, const L2Warm *warm)
{
  if (ring && (ring_depth < 1 || ring_depth > MAX_FEATURES_DELAY)) return -1;
  const int grid = (nstreams + LPC_STREAMS - 1) / LPC_STREAMS;
  L2Warm w{};
  if (warm) w = *warm;
  hipLaunchKernelGGL(lpc_kernel, dim3(grid), dim3(64 * LPC_STREAMS), 0, (hipStream_t)stream, features, lpc_out, nstreams,
                     tables, ring, ring_depth, w);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lpcnet_mi355x
