/*
 * fp_kernel.hip -- the fp32 latency kernel: lpcnet_synthesize_tail_impl
 * (lpcnet.c:235-271) of the reference's fp32 build (no DOT_PROD: GRU_A
 * recurrent product = the fp32 sparse_sgemv_accum8x4, vec_avx.h:865-902;
 * GRU_B = sgemv_accum16), one stream per 448-thread workgroup, persistent
 * over the N samples of a frame.  Default for fp32 models (BASELINE
 * configs[1], batch = 1).
 *
 * Every output row of the reference's fp32 products is one sequential FMA
 * chain (a block's 4 columns in order, blocks in index order), and a chain
 * cannot be reassociated without changing the result.  The kernel is built
 * around those chains' latency rather than bandwidth:
 *  - GRU_A waves g = 0..5 (hardware waves 1-6), thread = unit i: the z and r rows of unit i run as two
 *    interleaved chains from register-resident weights (they start from the
 *    sample-dependent input, nnet.c:434, so they are on the per-sample
 *    critical path); the h row starts from bias + diag*state only
 *    (nnet.c:439), so its chain for sample n+1 runs while the sampler works
 *    on sample n, with its weights streamed from L2.
 *  - sampler (hardware wave 0): GRU_B (48 rows = lanes, 384-step chains, weights in
 *    LDS as [column quad][row] float4), the GRU_B elementwise step and the
 *    dual-FC tree walk (sampler.h).
 *  - no workgroup barriers in the sample loop: LDS flags.  GRU_A wave w
 *    publishes done[w] = n+1 when its 64 units of h_A(n) are in LDS; the
 *    sampler's GRU_B chain consumes h_A(n) in column order, so it starts on
 *    wave 0's units while waves 1..5 are still finishing theirs.  ixseq =
 *    n+1 publishes the indices of sample n.
 * h_A(n) lives in LDS buffer (n+1)&1 (h_A(-1) = the stream's state in buffer
 * 0): a buffer is rewritten only after every reader of its previous contents
 * has passed a flag that depends on it (see the loop comments).
 * Numerics are term for term the reference's fp32 path (device_math.h).
 */
#include <hip/hip_runtime.h>

#include "device_math.h"
#include "l2_warm.h"
#include "lds_flags.h"
#include "lpcnet_engine.h"
#include "sampler.h"

namespace lpcnet_mi355x {

constexpr int FP_SLOTS = NA / 4 + 1; /* column quads of the GRU_A state + one +0 quad (padding) */
constexpr int FP_HD = 8;             /* h-gate weight blocks in flight per lane */
#ifndef FP_XD_N
#define FP_XD_N 8
#endif
/* GRU_A state quads in flight per chain (LDS): the z/r chains' x reads at
 * 8 slots ahead instead of 3, batch-1 fp32 sample kernel -2.2 % (5, 12, 16:
 * -1.2 %, +2.6 %, +29 %; same box, three alternating rounds, r05) */
constexpr int FP_XD = FP_XD_N;
#ifndef FP_SAMPLER_HW
#define FP_SAMPLER_HW 3
#endif
/* Hardware wave w runs on SIMD w % 4 (waves w and w+4 share one; wave 3 is
 * alone).  The z/r phase is VALU-issue bound where two GRU_A waves share a
 * SIMD, and GRU_B consumes the GRU_A waves' units in order g = 0..5, each
 * 64 columns (~700 cycles) after the previous: g = 0 gets SIMD 3 to itself,
 * g = 1, 2 share theirs with the least urgent g = 4, 3, and the sampler
 * (busy while the GRU_A waves wait, and vice versa) shares with g = 5. */
constexpr int FP_SAMPLER_WAVE = FP_SAMPLER_HW;
__device__ __forceinline__ int fp_gru_a_wave(int hw)
{
  if (FP_SAMPLER_HW == 3) return hw < 3 ? hw : 9 - hw;
  return hw == 3 ? 0 : (hw < 3 ? hw : 9 - hw);
}
#ifndef FP_GB_RING
#define FP_GB_RING 8
#endif
constexpr int GB_RING = FP_GB_RING;  /* GRU_B column quads in flight (LDS) */

struct FpLds {
  static constexpr int xs = 2 * FP_SLOTS * 16;        /* fp32 GRU_A state, [2][FP_SLOTS] float4 */
  static constexpr int gbw = (NA / 4) * GB_ROWS * 16; /* GRU_B input weights [96][48] float4 */
  static constexpr int sb = NB * 4;                   /* GRU_B state exchange */
  static constexpr int sync = 16 * 4;                 /* ix int4 | ixseq | abort | - | done[6] (+pad) */
  static constexpr int pcm = ((FRAME * 2 + 15) / 16) * 16;
  static constexpr int total = xs + gbw + sb + sync + pcm;
};

int fp_lds_bytes() { return IMG_VAR + FpLds::total; }

/* Keep packed offsets packed: without this the compiler hoists every
 * unpacked offset out of the sample loop (one register per slot). */
template <int N>
__device__ __forceinline__ void keep_packed(uint32_t (&o)[N])
{
#pragma unroll
  for (int k = 0; k < N; k++) asm volatile("" : "+v"(o[k]));
}

/* column quad t of packed byte offsets o (4 per word) -> the state float4 */
template <int NO>
__device__ __forceinline__ float4 fp_x(const float4 *xb, const uint32_t (&o)[NO], int t)
{
  return xb[(o[t >> 2] >> (8 * (t & 3))) & 0xFF];
}

__device__ __forceinline__ float fma4(const float4 &w, const float4 &x, float y)
{
  y = __builtin_fmaf(w.x, x.x, y);
  y = __builtin_fmaf(w.y, x.y, y);
  y = __builtin_fmaf(w.z, x.z, y);
  return __builtin_fmaf(w.w, x.w, y);
}

typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

/* fp_x as a native 4-vector (clean lane shuffles for the packed chain) */
template <int NO>
__device__ __forceinline__ v4f fp_xv(const float4 *xb, const uint32_t (&o)[NO], int t)
{
  return *(const v4f *)(xb + ((o[t >> 2] >> (8 * (t & 3))) & 0xFF));
}

/* The z and r chains of one unit over exactly NBK slots as one packed (z, r)
 * chain, from register weights (wz[t] = z.x r.x z.y r.y, wr[t] = z.z r.z
 * z.w r.w of slot t); xz / xr arrive holding slots 0..FP_XD-1.  Straight-line
 * code on purpose: a uniform branch around a ring step makes the compiler
 * copy the ring registers at the join and wait for their loads there. */
template <int NBK>
__device__ __forceinline__ void zr_chain(const float4 *xp, const v4f (&wz)[FP_ZF], const v4f (&wr)[FP_ZF],
                                         const uint32_t (&oz)[FP_ZF / 4], const uint32_t (&orr)[FP_ZF / 4],
                                         v4f (&xz)[FP_XD], v4f (&xr)[FP_XD], v2f &acc)
{
#pragma unroll
  for (int t = 0; t < NBK; t++) {
    /* two interleaved scalar chains (v_pk_fma_f32 needs (x_z, x_r) register
     * pairs, and the moves building them cost more than they save) */
    const v4f a = wz[t], b = wr[t], p = xz[t % FP_XD], q = xr[t % FP_XD];
    if (t + FP_XD < NBK) {
      xz[t % FP_XD] = fp_xv(xp, oz, t + FP_XD);
      xr[t % FP_XD] = fp_xv(xp, orr, t + FP_XD);
    }
    float gz = acc.x, gr = acc.y;
    gz = __builtin_fmaf(a.x, p.x, gz);
    gr = __builtin_fmaf(a.y, q.x, gr);
    gz = __builtin_fmaf(a.z, p.y, gz);
    gr = __builtin_fmaf(a.w, q.y, gr);
    gz = __builtin_fmaf(b.x, p.z, gz);
    gr = __builtin_fmaf(b.y, q.z, gr);
    gz = __builtin_fmaf(b.z, p.w, gz);
    gr = __builtin_fmaf(b.w, q.w, gr);
    asm volatile("" : "+v"(gz), "+v"(gr));
    acc = v2f{gz, gr};
    __builtin_amdgcn_sched_barrier(0);
  }
}

/* The h chain of one unit over exactly NBK slots: weights streamed from L2
 * (FP_HD slots in flight), state quads from LDS (FP_XD in flight). */
template <int NBK>
__device__ __forceinline__ float h_chain(const float4 *hw, const float4 *xb, const uint32_t (&oh)[FP_HF / 4], float y)
{
  float4 w[FP_HD], x[FP_XD];
#pragma unroll
  for (int d = 0; d < FP_HD && d < NBK; d++) w[d] = hw[d * 64];
#pragma unroll
  for (int d = 0; d < FP_XD && d < NBK; d++) x[d] = fp_x(xb, oh, d);
#pragma unroll
  for (int t = 0; t < NBK; t++) {
    const float4 wt = w[t % FP_HD], xt = x[t % FP_XD];
    if (t + FP_HD < NBK) w[t % FP_HD] = hw[(t + FP_HD) * 64];
    if (t + FP_XD < NBK) x[t % FP_XD] = fp_x(xb, oh, t + FP_XD);
    y = fma4(wt, xt, y);
    asm volatile("" : "+v"(y));
    __builtin_amdgcn_sched_barrier(0);
  }
  return y;
}

/* Long form (trained masks with block rows beyond the register tables):
 * the z/r chains over n slots streamed from the global tables, FPL_D slots
 * of weights and column quads in flight, the state quads read one slot
 * ahead.  Same FMA order as zr_chain (slot order = the reference's block
 * order; padding slots are -0 weights on the +0 quad). */
constexpr int FPL_D = 8;
__device__ __forceinline__ v2f zr_chain_stream(const float4 *xp, const float4 *w2 /* lane's slot 0 (lo, hi) */,
                                               const uint32_t *of /* lane's slot 0 */, int n, v2f acc)
{
  float4 lo[FPL_D], hi[FPL_D];
  uint32_t oo[FPL_D];
#pragma unroll
  for (int d = 0; d < FPL_D; d++)
    if (d < n) {
      lo[d] = w2[(size_t)d * 128];
      hi[d] = w2[(size_t)d * 128 + 1];
      oo[d] = of[(size_t)d * 64];
    }
  float gz = acc.x, gr = acc.y;
  float4 p = xp[oo[0] & 0xFF], q = xp[(oo[0] >> 8) & 0xFF];
#pragma unroll 1
  for (int base = 0; base < n; base += FPL_D) {
#pragma unroll
    for (int d = 0; d < FPL_D; d++) {
      const int t = base + d;
      if (t < n) {
        const float4 a = lo[d], b = hi[d];
        const float4 pc = p, qc = q;
        /* next slot's state quads (its offsets arrived FPL_D slots ago) */
        if (t + 1 < n) {
          const uint32_t on = oo[(d + 1) % FPL_D];
          p = xp[on & 0xFF];
          q = xp[(on >> 8) & 0xFF];
        }
        if (t + FPL_D < n) {
          lo[d] = w2[(size_t)(t + FPL_D) * 128];
          hi[d] = w2[(size_t)(t + FPL_D) * 128 + 1];
          oo[d] = of[(size_t)(t + FPL_D) * 64];
        }
        gz = __builtin_fmaf(a.x, pc.x, gz);
        gr = __builtin_fmaf(a.y, qc.x, gr);
        gz = __builtin_fmaf(a.z, pc.y, gz);
        gr = __builtin_fmaf(a.w, qc.y, gr);
        gz = __builtin_fmaf(b.x, pc.z, gz);
        gr = __builtin_fmaf(b.y, qc.z, gr);
        gz = __builtin_fmaf(b.z, pc.w, gz);
        gr = __builtin_fmaf(b.w, qc.w, gr);
        asm volatile("" : "+v"(gz), "+v"(gr));
      }
    }
  }
  return v2f{gz, gr};
}

/* the h chain of the long form: every slot streamed */
__device__ __forceinline__ float h_chain_stream(const float4 *hw /* lane's slot 0 */, const uint32_t *of, const float4 *xb, int n,
                                                float y)
{
  float4 w[FPL_D];
  uint32_t oo[FPL_D];
#pragma unroll
  for (int d = 0; d < FPL_D; d++)
    if (d < n) {
      w[d] = hw[(size_t)d * 64];
      oo[d] = of[(size_t)d * 64];
    }
  float4 x = xb[oo[0] & 0xFF];
#pragma unroll 1
  for (int base = 0; base < n; base += FPL_D) {
#pragma unroll
    for (int d = 0; d < FPL_D; d++) {
      const int t = base + d;
      if (t < n) {
        const float4 wt = w[d], xt = x;
        if (t + 1 < n) x = xb[oo[(d + 1) % FPL_D] & 0xFF];
        if (t + FPL_D < n) {
          w[d] = hw[(size_t)(t + FPL_D) * 64];
          oo[d] = of[(size_t)(t + FPL_D) * 64];
        }
        y = fma4(wt, xt, y);
        asm volatile("" : "+v"(y));
      }
    }
  }
  return y;
}

/* DIAG: 0 the production kernel, 1 with the logit / excitation trace, 2
 * with the s_memtime phase stamps (mf_kernel.hip) */
template <int DIAG, bool LONG, bool HWR>
__global__ __launch_bounds__(FP_THREADS) void fp_kernel(SampleArgs A)
{
  constexpr bool TRACE = DIAG == 1;
  extern __shared__ uint4 lds4[];
  unsigned char *lds = (unsigned char *)lds4;
  using L = FpLds;
  float4 *xs = (float4 *)lds;
  float4 *gbw = (float4 *)(lds + L::xs);
  float *sbuf = (float *)(lds + L::xs + L::gbw);
  int *sync = (int *)((unsigned char *)sbuf + L::sb);
  int *ix = sync, *ixseq = sync + 4, *abort_w = sync + 5, *done = sync + 8;
  short *pcmbuf = (short *)((unsigned char *)sync + L::sync);
  /* fixed image in static LDS: no dynamic-base add per table / dual-FC address */
  __shared__ uint4 img_s[IMG_VAR / 16];
  unsigned char *img = (unsigned char *)img_s;

  {
    const float *const fp_tabs[3] = {A.emb_sig, A.emb_pred, A.emb_exc};
    if (l2_warm_role(fp_tabs, A.nstreams)) return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sid = blockIdx.x;
  const uint32_t *rcp = (const uint32_t *)(img + IMG_RCP);
  const bool active = frame_count_of(A, sid) > A.delay;
  if (!active) {
    for (int n = tid; n < A.N; n += FP_THREADS) A.pcm[(size_t)sid * A.N + n] = 0;
    return;
  }
  const StreamState *ps = &A.st[sid];
  {
    for (int o = tid; o < IMG_VAR / 16; o += FP_THREADS) img_s[o] = A.image[o];
    for (int o = tid; o < (NA / 4) * GB_ROWS; o += FP_THREADS) gbw[o] = A.fp_gb[o];
  }
  for (int n = tid; n < A.preload; n += FP_THREADS) pcmbuf[n] = A.pcm[(size_t)sid * A.N + n];
  if (tid < 8) ((float *)xs)[(tid >> 2) * FP_SLOTS * 4 + NA + (tid & 3)] = 0.f;
  if (tid < 8) done[tid] = 0;
  if (tid == 0) *abort_w = 0;

  constexpr bool stamping = DIAG == 2;
  unsigned long long stp[10] = {};
  unsigned long long t_prev = 0, t_loop0 = 0;
  auto stamp = [&](int k) {
    if (stamping) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      stp[k] += t - t_prev;
      t_prev = t;
    }
  };
  auto stamp_start = [&]() {
    if (stamping) t_prev = t_loop0 = __builtin_amdgcn_s_memtime();
  };

  if (wv != FP_SAMPLER_WAVE) {
    /* ======================= GRU_A role ================================== */
    const int g = fp_gru_a_wave(wv); /* GRU_A wave: units 64g .. 64g+63 */
    const int i = 64 * g + lane;
    const float bz = A.ga_par[i], br = A.ga_par[NA + i], bh = A.ga_par[2 * NA + i];
    const float dz = A.ga_par[3 * NA + i], dr = A.ga_par[4 * NA + i], dh = A.ga_par[5 * NA + i];
    const float *ca = gru_a_cond_of(A, sid);
    const float cz = ca[i], cr = ca[NA + i], ch = ca[2 * NA + i];
    float st = ps->gru_a_state[i];
    v4f wz[FP_ZF], wr[FP_ZF];
    uint32_t oz[FP_ZF / 4], orr[FP_ZF / 4], oh[FP_HF / 4];
    if (!LONG) {
      const v4f *t = (const v4f *)A.fp_zr + (size_t)g * 2 * FP_ZF * 64 + lane;
#pragma unroll
      for (int k = 0; k < FP_ZF; k++) {
        wz[k] = t[k * 64];
        wr[k] = t[(FP_ZF + k) * 64];
      }
      const uint32_t *o = A.fp_off + (size_t)g * FP_OFF_WORDS * 64 + lane;
#pragma unroll
      for (int k = 0; k < FP_ZF / 4; k++) {
        oz[k] = o[k * 64];
        orr[k] = o[(FP_ZF / 4 + k) * 64];
      }
#pragma unroll
      for (int k = 0; k < FP_HF / 4; k++) oh[k] = o[(FP_ZF / 2 + k) * 64];
    }
    const int nzr = A.fp_nzr[g], nh = A.fp_nh[g]; /* chain blocks of this wave */
    ((float *)xs)[i] = st; /* h_A(-1) -> buffer 0 */
    __syncthreads();       /* image, GRU_B weights, initial state, ix(0) */
    /* the first units GRU_B consumes */
    if (g == 0) __builtin_amdgcn_s_setprio(2);
    else if (g < 3) __builtin_amdgcn_s_setprio(1);
    stamp_start();

    /* h row (nnet.c:439 + the h rows of the sparse product): bias + diag*state
     * then the chain over the column blocks of h_A(n) in buffer xb */
    auto hchain = [&](const float4 *xb) -> float {
      if constexpr (LONG) {
        size_t ho = (size_t)g * A.fpl_kh * 64 + lane;
        asm volatile("" : "+v"(ho));
        return h_chain_stream(A.fpl_h + ho, A.fpl_off + (size_t)SAMPLE_WAVES * A.fpl_kz * 64 + ho, xb, nh, bh + dh * st);
      }
      size_t ho = (size_t)(g * FP_HF * 64 + lane);
      asm volatile("" : "+v"(ho)); /* same weights every sample: do not hoist their loads */
      const float4 *hw = A.fp_h + ho;
      keep_packed(oh);
      float y = bh + dh * st;
      /* slot classes: the padding slots (-0 weights, +0 quad) are exact no-ops */
      switch ((nh + 3) / 4) {
        case 0: case 1: case 2: return h_chain<8>(hw, xb, oh, y);
        case 3: case 4: return h_chain<16>(hw, xb, oh, y);
        case 5: return h_chain<20>(hw, xb, oh, y);
        case 6: return h_chain<24>(hw, xb, oh, y);
        case 7: return h_chain<28>(hw, xb, oh, y);
        default: return h_chain<32>(hw, xb, oh, y);
      }
    };
    float hpre = hchain(xs);
    float tz = bz + dz * st, tr = br + dr * st;

    for (int n = 0; n < A.N; n++) {
      const float4 *xp = xs + (n & 1) * FP_SLOTS;   /* h_A(n-1) */
      float4 *xn = xs + ((n + 1) & 1) * FP_SLOTS;   /* h_A(n) */
      v4f xz[FP_XD], xr[FP_XD];
      if (!LONG) {
        keep_packed(oz);
        keep_packed(orr);
        /* first column quads of the z and r chains, before the indices land */
#pragma unroll
        for (int d = 0; d < FP_XD; d++) {
          xz[d] = fp_xv(xp, oz, d);
          xr[d] = fp_xv(xp, orr, d);
        }
      }
      stamp(5);
      flag_wait<1>(ixseq, n + 1, abort_w, A.spin_limit);
      stamp(0);
      /* GRU_A input (nnet.c:484-491): the 9 embedding gathers of this unit */
      float e[9];
      {
        const int4 v = *(const int4 *)ix;
        const float *e1 = A.emb_sig + (__builtin_amdgcn_readfirstlane(v.x) & 0xFF) * GA_ROWS;
        const float *e2 = A.emb_pred + (__builtin_amdgcn_readfirstlane(v.y) & 0xFF) * GA_ROWS;
        const float *e3 = A.emb_exc + (__builtin_amdgcn_readfirstlane(v.z) & 0xFF) * GA_ROWS;
#pragma unroll
        for (int g = 0; g < 3; g++) {
          e[g] = e1[g * NA + i];
          e[3 + g] = e2[g * NA + i];
          e[6 + g] = e3[g * NA + i];
        }
      }
      const float inz = ((cz + e[0]) + e[3]) + e[6];
      const float inr = ((cr + e[1]) + e[4]) + e[7];
      const float inh = ((ch + e[2]) + e[5]) + e[8];
      if (stamping) {
        /* diagnostic only: wait for the gathers before the stamp */
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("" ::"v"(inz), "v"(inr), "v"(inh));
      }
      stamp(1);
      /* z and r rows (nnet.c:434 + sparse product): two interleaved chains */
      v2f acc = {tz + inz, tr + inr};
      if constexpr (LONG) {
        size_t zo = (size_t)g * A.fpl_kz * 64 + lane;
        asm volatile("" : "+v"(zo));
        acc = zr_chain_stream(xp, A.fpl_zr + 2 * zo, A.fpl_off + zo, nzr, acc);
      } else
      switch ((nzr + 1) / 2) {
        case 0: case 1: zr_chain<2>(xp, wz, wr, oz, orr, xz, xr, acc); break;
        case 2: zr_chain<4>(xp, wz, wr, oz, orr, xz, xr, acc); break;
        case 3: zr_chain<6>(xp, wz, wr, oz, orr, xz, xr, acc); break;
        case 4: zr_chain<8>(xp, wz, wr, oz, orr, xz, xr, acc); break;
        case 5: zr_chain<10>(xp, wz, wr, oz, orr, xz, xr, acc); break;
        case 6: zr_chain<12>(xp, wz, wr, oz, orr, xz, xr, acc); break;
        case 7: zr_chain<14>(xp, wz, wr, oz, orr, xz, xr, acc); break;
        default: zr_chain<16>(xp, wz, wr, oz, orr, xz, xr, acc); break;
      }
      stamp(2);
      /* compute_sparse_gru elementwise (nnet.c:442-447) */
      float zr2[2] = {acc.x, acc.y};
      sigmoid_x86_n<2, HWR>(zr2, rcp);
      float hv[1] = {hpre * zr2[1] + inh};
      tanh_x86_n<1, HWR>(hv, rcp);
      st = zr2[0] * st + (1.f - zr2[0]) * hv[0];
      ((float *)xn)[i] = st;
      if (lane == 0) flag_publish(done + g, n + 1);
      stamp(3);
      if (n + 1 < A.N) {
        tz = bz + dz * st;
        tr = br + dr * st;
        /* the h chain of n+1 reads all of h_A(n) */
        {
          int m = flag_load(done);
#pragma unroll
          for (int w = 1; w < SAMPLE_WAVES; w++) m = min(m, flag_load(done + w));
          if (m < n + 1)
            for (int w = 0; w < SAMPLE_WAVES; w++) flag_wait(done + w, n + 1, abort_w, A.spin_limit);
          asm volatile("" ::: "memory");
        }
        stamp(4);
        hpre = hchain(xn);
      }
      stamp(8);
    }
    stamp(5);
    __syncthreads(); /* final */
    A.st[sid].gru_a_state[i] = st;
  } else {
    /* ======================= sampler role ================================ */
    const float *logit_tab = (const float *)(img + IMG_LOGIT);
    const int row = min(lane, GB_ROWS - 1), u = lane & (NB - 1);
    float lsr[NLPC], lpr[NLPC];
#pragma unroll
    for (int j = 0; j < NLPC; j++) {
      lsr[j] = ps->last_sig[j];
      lpr[j] = lpc_of(A, sid)[j];
    }
    float deemph = ps->deemph_mem, pred = 0.f;
    int last_exc = ps->last_exc & 0xFF;
    uint32_t rz = ps->rng[0], rw = ps->rng[1], rj = ps->rng[2], rc = ps->rng[3];
    float xv[NB]; /* GRU_B state, every lane */
#pragma unroll
    for (int j = 0; j < NB; j++) xv[j] = ps->gru_b_state[j];
    float sbv = xv[0];
#pragma unroll
    for (int j = 1; j < NB; j++) sbv = u == j ? xv[j] : sbv;
    /* GRU_B row seeds (nnet.c:347-356): bias + condition, recurrent bias, weights */
    const float gseed = A.gb_par[row] + gru_b_cond_of(A, sid)[row];
    const float rseed = A.gb_par[GB_ROWS + row];
    float rw16[NB];
#pragma unroll
    for (int j = 0; j < NB; j++) rw16[j] = A.gb_recf[j * GB_ROWS + row];
    {
      /* pred and the u-law indices of the first sample (lpcnet.c:252-254) */
      float p2 = 0.f;
#pragma unroll
      for (int j = 0; j < NLPC; j++) p2 = p2 - lsr[j] * lpr[j];
      pred = p2;
      if (lane == 0) {
        *(int4 *)ix = make_int4(lin2ulaw_x86(lsr[0]), lin2ulaw_x86(pred), last_exc, 0);
        *ixseq = 1;
      }
    }
    __syncthreads(); /* image, GRU_B weights, initial state, ix(0) */
    FcLane F;
    F.init(img, lane);
    stamp_start();
    /* the sampler chain is the per-sample critical path */
    __builtin_amdgcn_s_setprio(3);
    float t03 = 0.f, t47 = 0.f;
    float pend_pcm = 0.f, pend_pred = 0.f;
    int pend_exc = 0, pend_n = -1;
    auto finish = [&]() {
      if (pend_n < 0) return;
#pragma unroll
      for (int j = NLPC - 1; j > 0; j--) lsr[j] = lsr[j - 1];
      lsr[0] = pend_pcm;
        last_exc = pend_exc;
      pred = pend_pred;
      float o = pend_pcm + kPreemph * deemph;
      deemph = o;
      if (o < -32767) o = -32767;
      if (o > 32767) o = 32767;
      if (lane == 0 && pend_n >= A.preload) pcmbuf[pend_n] = (short)round_half_up(o);
      pend_n = -1;
    };
    for (int n = 0; n < A.N; n++) {
      finish();
      /* pred(n+1)'s candidate-independent products, off the walk */
      float lpd[NLPC];
      lpd[0] = 0.f;
#pragma unroll
      for (int j = 1; j < NLPC; j++) lpd[j] = lsr[j - 1] * lpr[j];
      /* the two kiss99 draws of this sample and their thresholds (nnet.c:178-184) */
      const uint32_t r0 = kiss99_next(rz, rw, rj, rc);
      const uint32_t r1 = kiss99_next(rz, rw, rj, rc);
      lane_thresholds(F, logit_tab, r0, r1, t03, t47);
      /* GRU_B recurrent rows (nnet.c:355-361) over h_B(n-1) */
      float y2 = rseed;
#pragma unroll
      for (int j = 0; j < NB; j++) y2 = __builtin_fmaf(rw16[j], xv[j], y2);
      stamp(0);
      /* GRU_B input rows (nnet.c:345-353): 384-step chains over h_A(n), in
       * column order, one GRU_A wave's 64 units at a time */
      const float4 *xb = xs + ((n + 1) & 1) * FP_SLOTS;
      uint32_t wrow = (uint32_t)row;
      asm volatile("" : "+v"(wrow)); /* same weights every sample: do not hoist their loads */
      const float4 *wp = gbw + wrow;
      float y = gseed;
      flag_wait(done, n + 1, abort_w, A.spin_limit);
      stamp(1);
      {
        /* ring of GB_RING blocks in flight; wave w+1's flag is read 8 blocks
         * before its first quad is needed and checked 4 blocks before */
        constexpr int NQ = NA / 4;
        float4 wq[GB_RING], xq[GB_RING];
#pragma unroll
        for (int d = 0; d < GB_RING; d++) {
          wq[d] = wp[d * GB_ROWS];
          xq[d] = xb[d];
        }
        int fnext = 0;
#pragma unroll
        for (int k = 0; k < NQ; k++) {
          const int d = k % GB_RING, seg = k / 16;
          if ((k & 15) == 16 - 2 * GB_RING && seg + 1 < SAMPLE_WAVES) fnext = flag_load(done + seg + 1);
          if ((k & 15) == 16 - GB_RING && seg + 1 < SAMPLE_WAVES && fnext < n + 1) flag_wait(done + seg + 1, n + 1, abort_w, A.spin_limit);
          const float4 a = wq[d], b = xq[d];
          if (k + GB_RING < NQ) {
            wq[d] = wp[(k + GB_RING) * GB_ROWS];
            xq[d] = xb[k + GB_RING];
          }
          y = fma4(a, b, y);
          asm volatile("" : "+v"(y)); /* keep the chain here, not sunk past the flag waits */
        }
      }
      stamp(2);
      /* GRU_B elementwise (nnet.c:362-371), unit u = lane % 16 (rows u,
       * 16+u, 32+u of the chains live in lanes u, 16+u, 32+u) */
      {
        /* lanes u < 16: rows u (own lane), 16+u (permlane16 swap), 32+u
         * (permlane32 swap); the other lanes compute values nobody reads */
        const float tsum = y + y2;
        const float zin = tsum;
        const float rin = __uint_as_float(__builtin_amdgcn_permlane16_swap(__float_as_uint(tsum), __float_as_uint(tsum), false, false)[1]);
        const float hin = __uint_as_float(__builtin_amdgcn_permlane32_swap(__float_as_uint(y), __float_as_uint(y), false, false)[1]);
        const float hrec = __uint_as_float(__builtin_amdgcn_permlane32_swap(__float_as_uint(y2), __float_as_uint(y2), false, false)[1]);
        float zr2[2] = {zin, rin};
        sigmoid_x86_n<2, HWR>(zr2, rcp);
        float hh[1] = {hin + hrec * zr2[1]};
        tanh_x86_n<1, HWR>(hh, rcp);
        sbv = zr2[0] * sbv + (1.f - zr2[0]) * hh[0];
        if (lane < NB) sbuf[lane] = sbv;
      }
      __builtin_amdgcn_wave_barrier();
      {
        const float4 *b4 = (const float4 *)sbuf;
#pragma unroll
        for (int j = 0; j < NB / 4; j++) {
          const float4 v = b4[j];
          xv[4 * j] = v.x; xv[4 * j + 1] = v.y; xv[4 * j + 2] = v.z; xv[4 * j + 3] = v.w;
        }
      }
      stamp(3);
      const WalkOut R = dual_fc_walk_p<TRACE, false, HWR>(F, t03, t47, xv, pred, lpd, lpr, n < A.preload ? pcmbuf + n : nullptr, deemph);
      if (n + 1 < A.N && lane == 0) {
        *(int4 *)ix = make_int4(R.su, R.pu, R.exc, 0);
        flag_publish(ixseq, n + 2);
      }
      stamp(4);
      if (TRACE && lane < 8) {
        float v = R.lg[0];
#pragma unroll
        for (int b = 1; b < 8; b++) v = lane == b ? R.lg[b] : v;
        A.trace_logits[((size_t)sid * A.N + n) * 8 + lane] = v;
      }
      if (TRACE && A.trace_exc && lane == 0) A.trace_exc[(size_t)sid * A.N + n] = R.exc;
      pend_pcm = R.pcm;
      pend_pred = R.pn;
      pend_exc = R.exc;
      pend_n = n;
      stamp(8);
    }
    finish();
    stamp(5);
    __syncthreads(); /* final */
    if (lane == 0) {
      StreamState *p = &A.st[sid];
#pragma unroll
      for (int j = 0; j < NLPC; j++) p->last_sig[j] = lsr[j];
      p->deemph_mem = deemph;
      p->last_exc = last_exc;
      p->rng[0] = rz; p->rng[1] = rw; p->rng[2] = rj; p->rng[3] = rc;
    }
    if (lane < NB) A.st[sid].gru_b_state[lane] = sbv;
  }
  if (stamping && lane == 0) {
    stp[6] = __builtin_amdgcn_s_memtime() - t_loop0;
    stp[7] = (unsigned long long)A.N;
    for (int k = 0; k < 16; k++) A.stamps[((size_t)blockIdx.x * STAMP_WAVES + wv) * 16 + k] = k < 10 ? stp[k] : 0;
  }
  for (int n = tid; n < A.N; n += FP_THREADS) A.pcm[(size_t)sid * A.N + n] = pcmbuf[n];
  /* every wave passed the final barrier: the abort word is settled */
  if (tid == 0 && flag_load(abort_w) && A.status) {
    A.status[0] = STATUS_FLAG_TIMEOUT; /* plain vector store to the pinned host word */
    __threadfence_system();
  }
}

template <int DIAG, bool LONG, bool HWR = true>
static int launch_fp_t(const SampleArgs &a, hipStream_t stream)
{
  if (ensure_dyn_lds((const void *)fp_kernel<DIAG, LONG, HWR>, 160 * 1024 - IMG_VAR)) return -1;
  hipLaunchKernelGGL((fp_kernel<DIAG, LONG, HWR>), dim3(warm_grid(a.nstreams, a.nstreams)), dim3(FP_THREADS), fp_lds_bytes() - IMG_VAR, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_fp(const SampleArgs &a, void *stream)
{
  hipStream_t st = (hipStream_t)stream;
  if (!a.rcp_hw) {
    /* another host's rcpps table: every activation through it (production
     * and trace forms; no stamped build) */
    if (a.stamps) return -1;
    if (a.fp_long) return a.trace_logits ? launch_fp_t<1, true, false>(a, st) : launch_fp_t<0, true, false>(a, st);
    return a.trace_logits ? launch_fp_t<1, false, false>(a, st) : launch_fp_t<0, false, false>(a, st);
  }
  if (a.fp_long)
    return a.trace_logits ? launch_fp_t<1, true>(a, st) : a.stamps ? launch_fp_t<2, true>(a, st) : launch_fp_t<0, true>(a, st);
  return a.trace_logits ? launch_fp_t<1, false>(a, st) : a.stamps ? launch_fp_t<2, false>(a, st) : launch_fp_t<0, false>(a, st);
}

}  // namespace lpcnet_mi355x
