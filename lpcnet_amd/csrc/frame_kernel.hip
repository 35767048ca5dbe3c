/*
 * frame_kernel.hip -- run_frame_network (lpcnet.c:82-120) for FRAME_STREAMS
 * streams per 512-thread workgroup: pitch embedding, conv1d x2
 * (compute_conv1d, nnet.c:452-470), dense x2 (_lpcnet_compute_dense,
 * nnet.c:122-135), the GRU_A / GRU_B conditioning projections, the
 * conv memories and the LPC ring.
 *
 * Numerics: every output row is a sequential FMA chain over its inputs in
 * index order, started from the bias -- sgemv_accum16 (vec_avx.h:618-643)
 * bit for bit; tanh is the Pade form with emulated rcpps (device_math.h).
 *
 * Layout and schedule.  A chain's steps are dependent, so the kernel is
 * built to never wait on memory inside one (chain_deep):
 *  - weights keep the blob's [in][out] layout, so a wave's load of one input
 *    for 64 consecutive rows is 256 contiguous bytes; the next 64 inputs'
 *    weights are always in flight (L2 latency under load ~1.3k cycles);
 *  - activations live in LDS as [stream][input] (16-byte aligned rows): the
 *    lanes of a wave share one stream, so a ds_read_b128 is a broadcast
 *    feeding 4 steps, read one block ahead;
 *  - 8 waves (2 per SIMD) so two chains' latencies interleave on every SIMD.
 * Every weight is fetched once per workgroup and used for all 4 streams
 * (the frame network's L2 traffic is 1.07 MB per workgroup), and one load
 * instruction feeds 4 FMAs per lane (the address unit, 4 cycles per
 * wave-load, bounds a 1-FMA-per-load mapping).  Thread mapping:
 * conv/dense layers: thread = row (128) x 4 streams; projections (1152 + 48
 * rows, gadf | gbdf as one [128][1200] matrix): thread = row tid + 512p
 * (3 passes) x 4 streams.
 */
#include <hip/hip_runtime.h>

#include "device_math.h"
#include "lpcnet_engine.h"

namespace lpcnet_mi355x {

constexpr int FK_THREADS = 512;
constexpr int FK_PROJ = GA_ROWS + GB_ROWS; /* gru_a | gru_b dense-feature rows */
static_assert(FRAME_STREAMS == 4, "thread mapping assumes 4 streams per workgroup");

/* plain v_fma_f32: keeps the compiler from forming broadcast v_pk_fma_f32
 * (which would read a weight's whole register pair and so wait on loads
 * landing in its other half) */
__device__ __forceinline__ float fma_step(float w, float x, float acc)
{
  float r;
  asm("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(w), "v"(x), "v"(acc));
  return r;
}

/* acc[s] = sequential FMA chain over NIN inputs of output `row` of W
 * ([NIN][nout], the blob's layout: lanes = consecutive rows, so a weight
 * load is 256 contiguous bytes per wave) against NS activation rows xs[s]
 * (LDS, [NIN], 16-byte aligned).  L2 latency under load is ~1.3k cycles, so
 * the weights of the next FD x FB inputs are always in flight: a ring of FD
 * register blocks of FB weights, the loop unrolled over the ring (no
 * register copies); activations are read one block ahead. */
constexpr int FB = 8;  /* inputs per block */
constexpr int FD = 8;  /* blocks in flight */

template <int NIN, int NOUT, int NS>
__device__ __forceinline__ void chain_deep(const float *__restrict__ W, int row, const float *const (&xs)[NS],
                                           float (&acc)[NS])
{
  static_assert(NIN % 4 == 0, "activation quads");
  constexpr int NB = (NIN + FB - 1) / FB;
  /* compile-time row stride, no clamp (the device copies carry
   * FRAME_PREFETCH zero rows past NIN): the loads of a block share one
   * address register and use immediate offsets */
  static_assert(FD * FB <= FRAME_PREFETCH, "prefetch beyond the padding");
  const float *wp = W + row;
  auto wld = [&](int j) -> float { return wp[(size_t)j * NOUT]; };
  float w[FD][FB];
  float4 x[NS][2], xn[NS][2];
#pragma unroll
  for (int d = 0; d < FD; d++)
#pragma unroll
    for (int k = 0; k < FB; k++) w[d][k] = wld(d * FB + k);
  auto load_x = [&](int blk, float4 (&dst)[NS][2]) {
#pragma unroll
    for (int s = 0; s < NS; s++)
#pragma unroll
      for (int h = 0; h < 2; h++) dst[s][h] = ((const float4 *)xs[s])[min(blk * 2 + h, NIN / 4 - 1)];
  };
  load_x(0, x);
#pragma unroll 1
  for (int base = 0; base < NB; base += FD) {
#pragma unroll
    for (int d = 0; d < FD; d++) {
      const int blk = base + d;
      load_x(blk + 1, xn);
      if (blk < NB) {
#pragma unroll
        for (int k = 0; k < FB; k++) {
          if (blk * FB + k < NIN) {
#pragma unroll
            for (int s = 0; s < NS; s++) {
              const float4 &q = x[s][k >> 2];
              const float xv = (k & 3) == 0 ? q.x : ((k & 3) == 1 ? q.y : ((k & 3) == 2 ? q.z : q.w));
              acc[s] = fma_step(w[d][k], xv, acc[s]);
            }
          }
        }
      }
      /* refill this slot with block blk + FD */
#pragma unroll
      for (int k = 0; k < FB; k++) w[d][k] = wld((blk + FD) * FB + k);
#pragma unroll
      for (int s = 0; s < NS; s++) {
        x[s][0] = xn[s][0];
        x[s][1] = xn[s][1];
      }
    }
  }
}

/* NS streams per workgroup: 4 (FRAME_STREAMS) for batches, 1 for a single
 * stream, where the three idle chains per thread would only cost issue slots
 * on the latency-bound chains. */
template <int NS>
__global__ __launch_bounds__(FK_THREADS) void frame_kernel(FrameArgs A)
{
  /* activations [stream][input], rows 16-byte aligned */
  __shared__ float4 x1_[NS][3 * FIN / 4]; /* conv1 window: 2 memory frames + current */
  __shared__ float4 x2_[NS][3 * COND / 4]; /* conv2 window */
  __shared__ float4 ya_[NS][COND / 4], yb_[NS][COND / 4];
  __shared__ int fc[NS];
  float(*x1)[3 * FIN] = (float(*)[3 * FIN])x1_;
  float(*x2)[3 * COND] = (float(*)[3 * COND])x2_;
  float(*ya)[COND] = (float(*)[COND])ya_;
  float(*yb)[COND] = (float(*)[COND])yb_;
  /* the single-stream launch has FK_B1_GRID workgroups of which only the
   * last works: one-workgroup launches all land on XCD 0, and moving this
   * kernel's 1 MB weight stream to another XCD's L2 leaves XCD 0's L2 to
   * the sample kernel's embedding tables (placement affects speed only) */
  if (NS == 1 && A.nstreams == 1 && blockIdx.x != gridDim.x - 1) return;
  const int grp = NS == 1 && A.nstreams == 1 ? 0 : blockIdx.x;
  const int tid = threadIdx.x;
  const int s0 = grp * NS;
  const uint32_t *rcp = A.rcp;
  unsigned long long t_prev = A.stamps ? __builtin_amdgcn_s_memtime() : 0, t_first = t_prev;
  unsigned long long stp[8] = {};
  auto stamp = [&](int q) {
    if (A.stamps) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      stp[q] += t - t_prev;
      t_prev = t;
    }
  };

  if (tid < NS) {
    const int sid = s0 + tid;
    fc[tid] = sid < A.nstreams ? A.st[sid].frame_count : 1000;
  }
  /* this frame's new LPC (host-computed; possibly pinned host memory read
   * over PCIe): fetched first, used in the epilogue */
  float lpc_in = 0.f;
  if (!A.mc.end2end && tid < NS * NLPC && s0 + tid / NLPC < A.nstreams)
    lpc_in = A.lpc_new[(s0 + tid / NLPC) * NLPC + tid % NLPC];
  /* inputs (lpcnet.c:91-99): conv1 window = conv1 memory | features | pitch
   * embedding; conv2 memory.  All loads of a thread in flight, then stores. */
  {
    constexpr int N1 = (NS * 3 * FIN + FK_THREADS - 1) / FK_THREADS;
    constexpr int N2 = (NS * 2 * COND + FK_THREADS - 1) / FK_THREADS;
    float v1[N1], v2[N2];
#pragma unroll
    for (int q = 0; q < N1; q++) {
      const int e = min(tid + q * FK_THREADS, NS * 3 * FIN - 1);
      const int s = e / (3 * FIN), j = e % (3 * FIN);
      const int sid = min(s0 + s, A.nstreams - 1);
      if (j < 2 * FIN) {
        v1[q] = A.st[sid].conv1_mem[j];
      } else if (j < 2 * FIN + NF) {
        v1[q] = A.features[sid * NF + (j - 2 * FIN)];
      } else {
        /* lpcnet.c:93-94: the 0.1 avoids rounding issues */
        const float f18 = A.features[sid * NF + 18];
        int pitch = (int)floor(.1 + (double)(50.f * f18) + 100);
        pitch = min(255, max(33, pitch));
        v1[q] = A.embed_pitch[pitch * EP + (j - 2 * FIN - NF)];
      }
    }
#pragma unroll
    for (int q = 0; q < N2; q++) {
      const int e = min(tid + q * FK_THREADS, NS * 2 * COND - 1);
      v2[q] = A.st[min(s0 + e / (2 * COND), A.nstreams - 1)].conv2_mem[e % (2 * COND)];
    }
#pragma unroll
    for (int q = 0; q < N1; q++) {
      const int e = tid + q * FK_THREADS;
      if (e < NS * 3 * FIN) x1[e / (3 * FIN)][e % (3 * FIN)] = v1[q];
    }
#pragma unroll
    for (int q = 0; q < N2; q++) {
      const int e = tid + q * FK_THREADS;
      if (e < NS * 2 * COND) x2[e / (2 * COND)][e % (2 * COND)] = v2[q];
    }
  }
  __syncthreads();
  stamp(0);

  /* conv/dense layers (128 rows): lane = row, all 4 streams (waves 0-1; the
   * others wait at the barrier) -- one weight load feeds 4 FMAs, each
   * weight fetched once per workgroup */
  const int i = tid;
  const float *xs1[NS], *xs2[NS], *xsa[NS], *xsb[NS];
#pragma unroll
  for (int q = 0; q < NS; q++) {
    xs1[q] = x1[q];
    xs2[q] = x2[q];
    xsa[q] = ya[q];
    xsb[q] = yb[q];
  }
  /* conv1 (nnet.c:452-470): 252 inputs -> 128, tanh; cleared while frame_count < 1 (lpcnet.c:99) */
  if (tid < COND) {
    float a[NS];
#pragma unroll
    for (int q = 0; q < NS; q++) a[q] = A.conv1_b[i];
    chain_deep<3 * FIN, COND, NS>(A.conv1_w, i, xs1, a);
#pragma unroll
    for (int q = 0; q < NS; q++) {
      const float t = tanh_x86(a[q], rcp);
      x2[q][2 * COND + i] = fc[q] < 1 ? 0.f : t;
    }
  }
  __syncthreads();
  stamp(1);
  /* conv2: 384 inputs -> 128, tanh; cleared while frame_count < FEATURES_DELAY (lpcnet.c:101) */
  if (tid < COND) {
    float a[NS];
#pragma unroll
    for (int q = 0; q < NS; q++) a[q] = A.conv2_b[i];
    chain_deep<3 * COND, COND, NS>(A.conv2_w, i, xs2, a);
#pragma unroll
    for (int q = 0; q < NS; q++) {
      const float t = tanh_x86(a[q], rcp);
      ya[q][i] = fc[q] < A.mc.delay ? 0.f : t;
    }
  }
  __syncthreads();
  stamp(2);
  if (tid < COND) {
    float a[NS];
#pragma unroll
    for (int q = 0; q < NS; q++) a[q] = A.dense1_b[i];
    chain_deep<COND, COND, NS>(A.dense1_w, i, xsa, a);
#pragma unroll
    for (int q = 0; q < NS; q++) yb[q][i] = tanh_x86(a[q], rcp); /* lpcnet.c:104 */
  }
  __syncthreads();
  stamp(3);
  if (tid < COND) {
    float a[NS];
#pragma unroll
    for (int q = 0; q < NS; q++) a[q] = A.dense2_b[i];
    chain_deep<COND, COND, NS>(A.dense2_w, i, xsb, a);
#pragma unroll
    for (int q = 0; q < NS; q++) ya[q][i] = tanh_x86(a[q], rcp); /* lpcnet.c:105 */
  }
  __syncthreads();
  stamp(4);
  /* conditioning projections (lpcnet.c:106-107), linear: gru_a_dense_feature |
   * gru_b_dense_feature as one [128][1200] matrix; thread = row tid + 512p
   * (3 passes), all 4 streams: every weight fetched once per workgroup */
  {
    const float *const(&xs)[NS] = xsa;
#pragma unroll 1
    for (int p = 0; p < (FK_PROJ + FK_THREADS - 1) / FK_THREADS; p++) {
      if (p * FK_THREADS + (tid & ~63) >= FK_PROJ) break; /* whole wave past the end */
      const int row = min(tid + p * FK_THREADS, FK_PROJ - 1);
      float acc[NS];
#pragma unroll
      for (int k = 0; k < NS; k++) acc[k] = A.proj_b[row];
      chain_deep<COND, FK_PROJ, NS>(A.proj_w, row, xs, acc);
      if (tid + p * FK_THREADS >= FK_PROJ || A.keep_cond) continue;
#pragma unroll
      for (int k = 0; k < NS; k++) {
        const int sid = s0 + k;
        if (sid >= A.nstreams) continue;
        if (row < GA_ROWS) A.st[sid].gru_a_cond[row] = acc[k];
        else A.st[sid].gru_b_cond[row - GA_ROWS] = acc[k];
      }
    }
  }
  stamp(5);
  /* conv memories (nnet.c:469) */
  for (int e = tid; e < NS * 2 * FIN; e += FK_THREADS) {
    const int q = e / (2 * FIN), j = e % (2 * FIN);
    if (s0 + q < A.nstreams) A.st[s0 + q].conv1_mem[j] = x1[q][FIN + j];
  }
  for (int e = tid; e < NS * 2 * COND; e += FK_THREADS) {
    const int q = e / (2 * COND), j = e % (2 * COND);
    if (s0 + q < A.nstreams) A.st[s0 + q].conv2_mem[j] = x2[q][COND + j];
  }
  /* the frame's LPC (lpcnet.c:107-118): END2END -> rc2lpc of the first
   * LPC_ORDER conditioning values (dense2's outputs, still in ya); else the
   * lpc_from_cepstrum ring of FEATURES_DELAY frames (none at delay 0); then
   * lpc_weighting by LPC_GAMMA */
  if (A.mc.end2end) {
    if (tid < NS && s0 + tid < A.nstreams && !A.keep_cond) {
      float rc[NLPC], l[NLPC];
#pragma unroll
      for (int k = 0; k < NLPC; k++) rc[k] = ya[tid][k];
      rc2lpc_dev(l, rc);
      StreamState *p = &A.st[s0 + tid];
      float gi = A.mc.lpc_gamma;
#pragma unroll
      for (int k = 0; k < NLPC; k++) {
        p->lpc[k] = l[k] * gi;
        gi *= A.mc.lpc_gamma;
      }
    }
  } else if (tid < NS * NLPC) {
    const int q = tid / NLPC, k = tid % NLPC, sid = s0 + q;
    if (sid < A.nstreams) {
      StreamState *p = &A.st[sid];
      const int D = A.mc.delay;
      const float cur = D > 0 ? p->old_lpc[D - 1][k] : lpc_in;
      for (int j = D - 1; j > 0; j--) p->old_lpc[j][k] = p->old_lpc[j - 1][k];
      if (D > 0) p->old_lpc[0][k] = lpc_in;
      if (!A.keep_cond) p->lpc[k] = lpc_weight(cur, k, A.mc.lpc_gamma);
    }
  }
  __syncthreads();
  if (tid < NS) {
    const int sid = s0 + tid;
    if (sid < A.nstreams && fc[tid] < 1000) A.st[sid].frame_count = fc[tid] + 1;
  }
  stamp(6);
  if (A.stamps && tid == 0) {
    stp[7] = t_prev - t_first;
    for (int q = 0; q < 8; q++) A.stamps[(size_t)grp * 16 + q] = stp[q];
  }
}

/* FrameCond copy of the frame step's outputs (overlapped multi-frame path,
 * engine.cpp launch_frame_step): a separate launch after the frame kernel,
 * which stays untouched (a store of the copy inside its projection loop
 * made it 2.4x slower at 1024 streams).  One workgroup for all (<= 128)
 * streams. */
__global__ __launch_bounds__(1024) void cond_copy_kernel(const StreamState *st, FrameCond *cond, int nstreams)
{
  constexpr int W = GA_ROWS + GB_ROWS + NLPC + 1;
  for (int e = threadIdx.x; e < nstreams * W; e += blockDim.x) {
    const int sid = e / W, j = e % W;
    const StreamState *p = &st[sid];
    FrameCond *q = &cond[sid];
    if (j < GA_ROWS) q->gru_a_cond[j] = p->gru_a_cond[j];
    else if (j < GA_ROWS + GB_ROWS) q->gru_b_cond[j - GA_ROWS] = p->gru_b_cond[j - GA_ROWS];
    else if (j < GA_ROWS + GB_ROWS + NLPC) q->lpc[j - GA_ROWS - GB_ROWS] = p->lpc[j - GA_ROWS - GB_ROWS];
    else q->frame_count = p->frame_count;
  }
}

int launch_cond_copy(const StreamState *st, FrameCond *cond, int nstreams, void *stream)
{
  hipLaunchKernelGGL(cond_copy_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, st, cond, nstreams);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* Stream-state moves of the shared drop-in pool (engine.cpp StatePool):
 * dst[dmap ? dmap[k] : k] = src[smap ? smap[k] : k] for k < n, one
 * workgroup per state, 16 bytes per thread. */
__global__ __launch_bounds__(256) void state_copy_kernel(StreamState *dst, const StreamState *src, const int *dmap,
                                                       const int *smap, int n)
{
  const int k = blockIdx.x;
  if (k >= n) return;
  uint4 *d = (uint4 *)&dst[dmap ? dmap[k] : k];
  const uint4 *s = (const uint4 *)&src[smap ? smap[k] : k];
  for (int e = threadIdx.x; e < (int)(sizeof(StreamState) / 16); e += blockDim.x) d[e] = s[e];
}

int launch_state_copy(StreamState *dst, const StreamState *src, const int *dmap, const int *smap, int n, void *stream)
{
  if (n <= 0) return 0;
  hipLaunchKernelGGL(state_copy_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, dst, src, dmap, smap, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

constexpr int FK_B1_GRID = 2;

/* Up to one stream per CU the single-stream kernel runs every stream in its
 * own workgroup at once (a workgroup's time is set by its weight ingest,
 * not by its stream count: 20 us for 1 stream, 44 us for 4). */
int frame_groups(int nstreams)
{
  return nstreams <= FK_ONE_STREAM_MAX ? nstreams : (nstreams + FRAME_STREAMS - 1) / FRAME_STREAMS;
}

int launch_frame(const FrameArgs &a, void *stream)
{
  if (a.nstreams == 1) {
    hipLaunchKernelGGL(frame_kernel<1>, dim3(FK_B1_GRID), dim3(FK_THREADS), 0, (hipStream_t)stream, a);
  } else if (a.nstreams <= FK_ONE_STREAM_MAX) {
    hipLaunchKernelGGL(frame_kernel<1>, dim3(a.nstreams), dim3(FK_THREADS), 0, (hipStream_t)stream, a);
  } else {
    const int grid = (a.nstreams + FRAME_STREAMS - 1) / FRAME_STREAMS;
    hipLaunchKernelGGL(frame_kernel<FRAME_STREAMS>, dim3(grid), dim3(FK_THREADS), 0, (hipStream_t)stream, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lpcnet_mi355x
