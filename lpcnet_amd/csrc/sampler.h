/*
 * sampler.h -- dual-FC tree sampling of one output sample (sample_mdense,
 * nnet.c:163-214) and the next sample's indices (lpcnet.c:252-261), for one
 * stream per 32-lane half-wave.  Shared by the pipelined sample kernels.
 *
 * Lane hl of a half evaluates (node qq+1, channel ch2) of tree levels 0..3
 * (qq = hl/2 < 15), then the node of levels 4..7 under the chosen 4-bit
 * prefix.  While levels 4..7 are walked, lane c = hl & 15 speculatively
 * evaluates candidate exc = 16*prefix + c: its output sample, pred(n+1) and
 * both u-law indices -- the same operations in the same order as the
 * reference, so the walk then only selects a lane.
 */
#ifndef LPCNET_SAMPLER_H
#define LPCNET_SAMPLER_H

#include "device_math.h"

namespace lpcnet_mi355x {

struct FcLane {
  const uint32_t *rcp;
  const float *ulaw, *fcw, *fcb, *fcf;
  float w03[NB];   /* weights of this lane's level 0..3 node and channel (registers) */
  float b03, f03;
  int qq, lvl_in, ch2, hb, half, hl;

  __device__ __forceinline__ void init(const unsigned char *img, int lane)
  {
    init_sections((const uint32_t *)(img + IMG_RCP), (const float *)(img + IMG_ULAW), (const float *)(img + IMG_FCW),
                  (const float *)(img + IMG_FCB), (const float *)(img + IMG_FCF), lane);
  }

  /* the same from the image's sections placed anywhere in LDS (mfw_kernel
   * keeps no rcpps table: hardware reciprocal only, rcp_ = nullptr) */
  __device__ __forceinline__ void init_sections(const uint32_t *rcp_, const float *ulaw_, const float *fcw_,
                                                const float *fcb_, const float *fcf_, int lane)
  {
    rcp = rcp_;
    ulaw = ulaw_;
    fcw = fcw_;
    fcb = fcb_;
    fcf = fcf_;
    half = lane >> 5;
    hl = lane & 31;
    hb = 32 * half;
    ch2 = lane & 1;
    const int q = hl >> 1;
    qq = q < 15 ? q : 0;
    lvl_in = qq == 0 ? 0 : (qq < 3 ? 1 : (qq < 7 ? 2 : 3)); /* level of node qq+1 within 0..3 */
#pragma unroll
    for (int j = 0; j < NB; j++) w03[j] = fcw[(qq + 1) * 32 + ch2 * 16 + j];
    b03 = fcb[ch2 * 256 + qq + 1];
    f03 = fcf[ch2 * 256 + qq + 1];
  }

  /* factor*tanh(bias + w.x) of this lane, plus the other channel's term
   * (nnet.c:196-205: sum1 + sum2 through DPP quad_perm [1,0,3,2]).  FIN:
   * the node sum is known finite and below 2^60 (SampleArgs::fc_fin and
   * GRU_B states within [-2, 2]), tanh without its flush and NaN selects */
  template <bool FIN = false, bool HW = true>
  __device__ __forceinline__ float node_logit(float bias, float factor, const float *w, const float (&xv)[NB]) const
  {
    float sum = bias;
#pragma unroll
    for (int j = 0; j < NB; j++) sum = sum + w[j] * xv[j];
    return node_logit_tail<FIN, HW>(sum, factor);
  }

  /* the same from the finished dot product sum */
  /* HW: the hardware-reciprocal rcpps (proven equal to the Intel table
   * only); false: the LDS table (any host's rcpps, same-box parity) */
  template <bool FIN = false, bool HW = true>
  __device__ __forceinline__ float node_logit_tail(float sum, float factor) const
  {
    float v[1] = {sum};
    if constexpr (FIN)
      tanh_x86_fin_n<1, HW>(v, rcp);
    else
      tanh_x86_n<1, HW>(v, rcp);
    const float vv = factor * v[0];
    const float o = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(vv), 0xB1, 0xF, 0xF, false));
    return ch2 ? o + vv : vv + o;
  }
};

/* Result of one sample: excitation, output before de-emphasis, pred(n+1),
 * u-law indices of the next sample (lpcnet.c:252-261) and, when tracing,
 * the 8 pre-sampling logits along the path. */
struct WalkOut {
  int exc, su, pu;
  float pcm, pn;
  float lg[8];
};

/* The two thresholds a lane compares against (its node's level within
 * levels 0..3 and 4..7): thr = logit_table[byte] of this sample's two
 * kiss99 draws (nnet.c:178-184).  Off the critical path: called when the
 * draws are made. */
__device__ __forceinline__ void lane_thresholds(const FcLane &F, const float *logit_tab, uint32_t r0, uint32_t r1,
                                                float &t03, float &t47)
{
  t03 = logit_tab[(r0 >> (8 * F.lvl_in)) & 0xFF];
  t47 = logit_tab[(r1 >> (8 * F.lvl_in)) & 0xFF];
}

/* Decisions of one 4-level tree round from the lane's half of the ballot
 * (bit 2q = the q-th node of the round, both channel lanes of a node vote
 * alike): level b's node sits at lane pair (1 << b) - 1 + (the b bits
 * decided so far).  Three dependent 32-bit ops per level. */
__device__ __forceinline__ int walk_round(uint32_t m)
{
  int v = 0;
#pragma unroll
  for (int b = 0; b < 4; b++) v = (v << 1) | (int)__builtin_amdgcn_ubfe(m, 2 * v + 2 * ((1 << b) - 1), 1);
  return v;
}

/* this lane's half of a wave ballot */
__device__ __forceinline__ uint32_t half_bits(unsigned long long m, int half)
{
  return half ? (uint32_t)(m >> 32) : (uint32_t)m;
}

#ifndef WALK_INTERLEAVE
#define WALK_INTERLEAVE 1
#endif

/* phase-stamp hook of dual_fc_walk (diagnostic builds: mf_kernel -DMF_WALKFINE) */
struct WalkNoStamp {
  __device__ __forceinline__ void operator()(int, float) const {}
};

/* One sample of stream (half): t03/t47 = this lane's thresholds
 * (lane_thresholds), xv = GRU_B state, pred = pred(n), lsr/lpr = LPC
 * history and coefficients.  teach != nullptr:
 * teacher forcing with input *teach (lpcnet.c:256-259).  Uniform per half.
 * TRACE: also return the 8 logits along the path.
 *
 * Critical-path shape: round 1 (levels 0..3, all 15 nodes at once) ->
 * decisions -> round 2 (levels 4..7 under the prefix) with the 16
 * candidates' outputs computed beside it -> decisions -> one lane select.
 * Lanes hl and hl + 16 hold the same candidate c = hl & 15; the low 16
 * convert its output sample to u-law, the high 16 its pred(n+1), so one
 * lin2ulaw serves both indices. */
/* lprod[j] (j >= 1) = lsr[j - 1] * lpr[j]: the candidate-independent
 * products of pred(n+1) (lpcnet.c:252 after the history shift); the
 * reference multiplies and subtracts separately (no FMA), so a product
 * computed ahead -- before barrier Y, off the sampler chain -- is the same
 * float */
template <bool TRACE, bool FIN = false, bool HW = true, class ST = WalkNoStamp>
__device__ __forceinline__ WalkOut dual_fc_walk_p(const FcLane &F, float t03, float t47, const float (&xv)[NB], float pred,
                                                  const float (&lprod)[NLPC], const float (&lpr)[NLPC], const short *teach,
                                                  float deemph, ST st = ST())
{
  WalkOut R;
  int val;
  {
    const float l = F.node_logit<FIN, HW>(F.b03, F.f03, F.w03, xv);
    st(2, l);
    val = walk_round(half_bits(__ballot(t03 < l), F.half));
    if (TRACE) {
      int v = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const int nd = (1 << b) | v;
        R.lg[b] = __shfl(l, F.hb + 2 * (nd - 1));
        v = (v << 1) | ((val >> (3 - b)) & 1);
      }
    }
  }
  /* level 4..7 node of this lane under the chosen prefix */
  const int lvl = 4 + F.lvl_in;
  const int node = (1 << lvl) | (val << (lvl - 4)) | (F.qq + 1 - (1 << (lvl - 4)));
  const float b47 = F.fcb[F.ch2 * 256 + node], f47 = F.fcf[F.ch2 * 256 + node];
  float w47[NB];
  {
    const float4 *w4 = (const float4 *)(F.fcw + node * 32 + F.ch2 * 16);
#pragma unroll
    for (int j = 0; j < NB / 4; j++) {
      const float4 v = w4[j];
      w47[4 * j] = v.x; w47[4 * j + 1] = v.y; w47[4 * j + 2] = v.z; w47[4 * j + 3] = v.w;
    }
  }
  st(3, w47[NB - 1] + b47 + f47);
  /* candidate exc = 16*prefix + (hl & 15): output sample, pred(n+1) and one
   * u-law index (lpcnet.c:252-261), the reference's operations in order.
   * Its subtraction chain is pinned step for step beside round 2's dot
   * chain (two independent dependency chains interleaved); left to the
   * scheduler it runs before the w47 loads are even issued. */
  const float sp_pcm = pred + F.ulaw[(val << 4) | (F.hl & 15)];
  float p2 = 0.f - sp_pcm * lpr[0];
#if WALK_INTERLEAVE
  float sum = b47;
#pragma unroll
  for (int j = 0; j < NB; j++) {
    sum = sum + w47[j] * xv[j];
    if (j > 0) p2 = p2 - lprod[j];
    asm volatile("" : "+v"(sum), "+v"(p2));
  }
#else
  float sum = b47;
#pragma unroll
  for (int j = 0; j < NB; j++) sum = sum + w47[j] * xv[j];
#pragma unroll
  for (int j = 1; j < NLPC; j++) p2 = p2 - lprod[j];
#endif
  float sp_pred = p2;
  int sp_u = lin2ulaw_x86(F.hl < 16 ? sp_pcm : sp_pred);
  int low;
  {
    const float l = F.node_logit_tail<FIN, HW>(sum, f47);
    st(15, l);
    /* the speculation is needed only when not teaching: pin it before the
     * ballot, or the compiler sinks it into that branch, after the round */
    asm volatile("" : "+v"(sp_u), "+v"(sp_pred));
    low = walk_round(half_bits(__ballot(t47 < l), F.half));
    if (TRACE) {
      const int s = low;
      int v = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) {
        R.lg[4 + b] = __shfl(l, F.hb + 2 * ((1 << b) - 1 + v));
        v = (v << 1) | ((s >> (3 - b)) & 1);
      }
    }
  }
  R.exc = (val << 4) | low;
  if (teach != nullptr) {
    /* teacher forcing (lpcnet.c:256-259) */
    const float o_in = (float)*teach;
    const float pd = kPreemph * deemph;
    R.exc = lin2ulaw_x86((o_in - pd) - pred);
    R.pcm = o_in - pd;
    float q = 0.f - R.pcm * lpr[0];
#pragma unroll
    for (int j = 1; j < NLPC; j++) q = q - lprod[j];
    R.pn = q;
    R.su = lin2ulaw_x86(R.pcm);
    R.pu = lin2ulaw_x86(R.pn);
  } else {
    /* the chosen candidate's lane hb + low: its u-law pair (the pred
     * index comes over from lane + 16), output sample and pred(n+1) */
    const int pu = (int)__builtin_amdgcn_permlane16_swap((uint32_t)sp_u, (uint32_t)sp_u, false, false)[1];
    const int src = (F.hb + low) << 2;
    const int ic = __builtin_amdgcn_ds_bpermute(src, sp_u | (pu << 8));
    R.su = ic & 0xFF;
    R.pu = ic >> 8;
    R.pcm = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(sp_pcm)));
    R.pn = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(sp_pred)));
  }
  return R;
}

/* the same with the products formed here, beside round 1's dependent chain */
template <bool TRACE, bool FIN = false, bool HW = true, class ST = WalkNoStamp>
__device__ __forceinline__ WalkOut dual_fc_walk(const FcLane &F, float t03, float t47, const float (&xv)[NB], float pred,
                                                const float (&lsr)[NLPC], const float (&lpr)[NLPC], const short *teach,
                                                float deemph, ST st = ST())
{
  float lprod[NLPC];
  lprod[0] = 0.f;
#pragma unroll
  for (int j = 1; j < NLPC; j++) lprod[j] = lsr[j - 1] * lpr[j];
  return dual_fc_walk_p<TRACE, FIN, HW, ST>(F, t03, t47, xv, pred, lprod, lpr, teach, deemph, st);
}

}  // namespace lpcnet_mi355x

#endif
