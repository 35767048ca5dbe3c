/*
 * mf2_kernel.hip -- the matrix-core sample kernel for large batches: two
 * groups of S streams per 512-thread workgroup, half a sample apart
 * (lpcnet_synthesize_tail_impl, lpcnet.c:235-271; arithmetic term for term
 * mf_kernel's, which is the reference's).
 *
 * mf_kernel's per-sample recurrence splits into two halves that alternate
 * between its roles: the GRU_A waves gather the embedding rows and run the
 * GRU_A elementwise step (X -> Y) while the sampler waves wait, then the
 * samplers run GRU_B and the dual-FC walk (Y -> X) while the GRU_A waves
 * only have the recurrent product to do.  Each role idles for half the
 * sample.  Here the two groups A and B of a workgroup are staggered by one
 * half:
 *   phase A(t): GRU_A waves: gathers + elementwise of A's sample t, then the
 *               recurrent product of B's sample t;
 *               samplers:    GRU_B + walk of B's sample t-1 -> ix_B(t)
 *   phase B(t): GRU_A waves: gathers + elementwise of B's sample t, then the
 *               recurrent product of A's sample t+1;
 *               samplers:    GRU_B + walk of A's sample t -> ix_A(t+1)
 * one workgroup barrier per phase, so both roles work in every phase and the
 * GRU_A register tables and GRU_B tiles serve 2S streams.  Used for batches
 * of >= 2048 streams (a launch still fills every CU); preload, trace and
 * stamps take mf_kernel.  Samples t run over all frames of a
 * multi-frame launch (SampleArgs::nframes); the samplers write each output
 * sample straight to global memory.
 */
#include <hip/hip_runtime.h>

#include <type_traits>

#include "device_math.h"
#include "lpcnet_engine.h"
#include "mf_common.h"
#include "sampler.h"

namespace lpcnet_mi355x {

template <int S>
struct Mf2Lds {
  static constexpr int GS = 2 * S;
  static constexpr int x = GS * MF_XSTR;            /* quantized GRU_A state [2][S][MF_XSTR] */
  static constexpr int xb = GS * NB;                /* quantized GRU_B state [2][S][NB] */
  static constexpr int sb = GS * NB * 4;            /* float GRU_B state [2][S][NB] (walk broadcast) */
  static constexpr int ix = GS * 16;                /* sig/pred/exc row byte offsets [2][S] int4 */
  static constexpr int lpc = GS * NLPC * 4;         /* the frame's LPC [2][S][NLPC] */
  static constexpr int cnd = 2 * GA_ROWS * S * 4;   /* GRU_A conditioning [2][3][NA][S] */
  static constexpr int gbs = 2 * 2 * S * GB_ROWS * 4; /* GRU_B input seeds [sampler wave][2][S][48] */
  static constexpr int gbr = GB_ROWS * 4;           /* GRU_B recurrent seeds [48] */
  static constexpr int okw = 2 * 2 * 8 * 4;         /* range words [frame parity][group][GRU_A wave] */
  static constexpr int gbw = 3 * 64 * 16;           /* GRU_B recurrent A tiles [3][64] */
  static constexpr int total = x + xb + sb + ix + lpc + cnd + gbs + gbr + okw + gbw;
  static constexpr int part = 2 * 3 * (NA + 1) * S * 4; /* split models: hosted partial sums [group][3][NA + 1][S] */
};

int mf2_lds_bytes(int S, int split)
{
  return IMG_VAR + (S == 4 ? Mf2Lds<4>::total + (split ? Mf2Lds<4>::part : 0)
                           : Mf2Lds<2>::total + (split ? Mf2Lds<2>::part : 0));
}

/* SPLIT: models with block rows beyond the register tables (trained
 * Sparsify masks, engine.cpp mf_plan) -- each lane group also runs a hosted
 * piece of another row, whose partial sums reach the row's owner through
 * LDS: one buffer per group, added into by the group's recurrent product and
 * merged (then cleared) by its next elementwise step, a barrier apart */
template <int S, bool SPLIT, bool HWR>
__global__ __launch_bounds__(MF_THREADS) void mf2_kernel(SampleArgs A)
{
  extern __shared__ uint4 lds4[];
  unsigned char *lds = (unsigned char *)lds4;
  using L = Mf2Lds<S>;
  constexpr int GS = 2 * S;
  unsigned char *xa = lds; /* first: every x address fits the 16-bit offsets kept in registers */
  unsigned char *xb = xa + L::x;
  float *sbuf = (float *)(xb + L::xb);
  int *ix = (int *)((unsigned char *)sbuf + L::sb);
  float *lpcb = (float *)((unsigned char *)ix + L::ix);
  float *cnd = lpcb + GS * NLPC;
  int *gbs = (int *)(cnd + 2 * GA_ROWS * S);
  int *gbr = gbs + 2 * 2 * S * GB_ROWS;
  int *okw = gbr + GB_ROWS;
  v4i *gbw = (v4i *)(okw + 32);
  int *part = (int *)(gbw + 3 * 64); /* SPLIT: [2 groups][3][NA + 1][S / 2] 64-bit words */
  __shared__ uint4 img_s[IMG_VAR / 16];
  unsigned char *img = (unsigned char *)img_s;

  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int s0 = blockIdx.x * GS;
  const uint32_t *rcp = (const uint32_t *)(img + IMG_RCP);
  const int nfr = A.nframes > 1 ? A.nframes : 1;
  const int total = nfr * A.N;

  bool active[GS];
  bool any = false, bad = false;
  for (int s = 0; s < GS; s++) {
    const int sid = s0 + s;
    active[s] = sid < A.nstreams && frame_count_of(A, sid) > A.delay;
    any |= active[s];
  }
  if (nfr > 1) {
    const FrameCond *cl = A.cond + (size_t)(nfr - 1) * A.nstreams;
    for (int s = 0; s < GS; s++) {
      const int sid = s0 + s;
      bad |= sid < A.nstreams && (frame_count_of(A, cl, sid) > A.delay) != active[s];
    }
    if (bad && tid == 0 && A.status) A.status[0] = STATUS_ACTIVITY; /* plain vector store to the pinned host word */
  }
  if (!any || bad) {
    for (int e = tid; e < GS * total; e += MF_THREADS) {
      const int s = e / total, fn = e % total, f = fn / A.N, n = fn % A.N;
      if (s0 + s < A.nstreams) A.pcm[((size_t)f * A.nstreams + s0 + s) * A.N + n] = 0;
    }
    return;
  }
  for (int o = tid; o < IMG_VAR / 16; o += MF_THREADS) img_s[o] = A.image[o];

  if (wv < SAMPLE_WAVES) {
    /* ======================= GRU_A role ================================== */
    const int i = A.mf_unit[tid];
    const float bz = A.ga_par[i], br = A.ga_par[NA + i], bh = A.ga_par[2 * NA + i];
    const float dz = A.ga_par[3 * NA + i], dr = A.ga_par[4 * NA + i], dh = A.ga_par[5 * NA + i];
    const int wsz = A.ga_wsum[i], wsr = A.ga_wsum[NA + i], wsh = A.ga_wsum[2 * NA + i];
    float st[2][S];
    for (int g = 0; g < 2; g++)
      for (int s = 0; s < S; s++) st[g][s] = A.st[min(s0 + g * S + s, A.nstreams - 1)].gru_a_state[i];
    /* group g's inputs of a frame: its conditioning (lane-private LDS
     * entries) and this wave's range word */
    auto stage = [&](int g, const FrameCond *cf, int par) {
      bool in_range = true;
      float *cg = cnd + g * GA_ROWS * S;
      for (int s = 0; s < S; s++) {
        const int sid = min(s0 + g * S + s, A.nstreams - 1);
        const float *ca = gru_a_cond_of(cf, A, sid);
        const float cz = ca[i], cr = ca[NA + i], ch = ca[2 * NA + i];
        cg[tid * S + s] = cz;
        cg[(NA + tid) * S + s] = cr;
        cg[(2 * NA + tid) * S + s] = ch;
        in_range &= fabsf(st[g][s]) <= 2.f && fabsf(cz) <= A.mf_zr_bound && fabsf(cr) <= A.mf_zr_bound &&
                    fabsf(ch) <= A.mf_h_bound;
      }
      if (lane == 0) okw[(par * 2 + g) * 8 + wv] = __ballot(!in_range) == 0ull;
    };
    const FrameCond *cf = A.cond;
    stage(0, cf, 0);
    stage(1, cf, 0);
    if (tid < GB_ROWS) gbr[tid] = cvt_rne(A.gb_par[GB_ROWS + tid] * kScale) + A.gb_wsum[GB_ROWS + tid];
    uint32_t wz[MF_ZMAX], wr[MF_ZMAX], wh[MF_HMAX], oz[MF_ZMAX / 2], orr[MF_ZMAX / 2], oh[MF_HMAX / 2];
    {
      const uint32_t *mt = A.mf + (size_t)wv * MF_LANE_U32 * 64 + lane;
#pragma unroll
      for (int t = 0; t < MF_ZMAX; t++) {
        wz[t] = mt[t * 64];
        wr[t] = mt[(MF_ZMAX + t) * 64];
      }
#pragma unroll
      for (int t = 0; t < MF_HMAX; t++) wh[t] = mt[(2 * MF_ZMAX + t) * 64];
      uint32_t cw[MF_GA / 4];
#pragma unroll
      for (int k = 0; k < MF_GA / 4; k++) cw[k] = mt[(MF_GA + k) * 64];
      /* A operand of lane 4b+m = stream m of a group (lanes m >= S duplicate stream S-1) */
      const uint32_t mo = (uint32_t)min(lane & 3, S - 1) * MF_XSTR;
      auto off = [&](int t) -> uint32_t { return ((cw[t >> 2] >> (8 * (t & 3))) & 0xFF) * 4 + mo; };
#pragma unroll
      for (int t = 0; t < MF_ZMAX / 2; t++) {
        oz[t] = off(2 * t) | (off(2 * t + 1) << 16);
        orr[t] = off(MF_ZMAX + 2 * t) | (off(MF_ZMAX + 2 * t + 1) << 16);
      }
#pragma unroll
      for (int t = 0; t < MF_HMAX / 2; t++) oh[t] = off(2 * MF_ZMAX + 2 * t) | (off(2 * MF_ZMAX + 2 * t + 1) << 16);
    }
    const int nzr = A.mf_nzr[wv], nh = A.mf_nh[wv];
    const int nfzr = SPLIT ? A.mf_nfzr[wv] : 0, nfh = SPLIT ? A.mf_nfh[wv] : 0;
    /* split models: the rows of this lane's hosted pieces (9 bits per gate,
     * NA: none) and whether this thread's own unit has pieces to merge (bits
     * 27..29), as in mf_kernel */
    uint32_t frow = 0;
    if constexpr (SPLIT) {
      const uint32_t *fro = (const uint32_t *)A.mf_frow + tid;
      const uint32_t e0 = fro[0], e1 = fro[SAMPLE_THREADS], e2 = fro[2 * SAMPLE_THREADS];
      frow = (e0 & 0x1FF) | (e1 & 0x1FF) << 9 | (e2 & 0x1FF) << 18 | (e0 >> 16 & 1) << 27 | (e1 >> 16 & 1) << 28 |
             (e2 >> 16 & 1) << 29;
    }
    __syncthreads(); /* image in LDS */
    for (int g = 0; g < 2; g++)
      for (int s = 0; s < S; s++) xa[(g * S + s) * MF_XSTR + i] = (unsigned char)quant_s8_state(st[g][s]);
    if constexpr (SPLIT)
      for (int e = tid; e < 2 * 3 * (NA + 1) * S; e += SAMPLE_THREADS) part[e] = 0;
    __syncthreads(); /* initial q(h_A) of both groups, ix of both groups, seeds */

    /* one group's recurrent terms, for its next elementwise step */
    float az[S], ar[S]; /* the recurrent sums as exact floats (ga_elementwise) */
    float tz[S], tr[S], hpre[S];
    int iaz[S], iar[S], iah[S]; /* SPLIT: the own sums as int32 until the hosted partial sums are merged */
    auto recurrent = [&](auto gc) {
      constexpr int g = decltype(gc)::value;
      const unsigned char *xg = xa + g * S * MF_XSTR;
      v4i vz[1] = {{wsz, wsz, wsz, wsz}}, vr[1] = {{wsr, wsr, wsr, wsr}}, vh[2] = {{wsh, wsh, wsh, wsh}, {0, 0, 0, 0}};
      mf_opaque(oz);
      mf_opaque(orr);
      mf_opaque(oh);
      if constexpr (SPLIT) {
        /* own groups into v*, the hosted piece into f*, added into the
         * owner's row through this group's LDS buffer (exact int32 adds) */
        v4i fz = {0, 0, 0, 0}, fr = {0, 0, 0, 0}, fh[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
        uint32_t xz[4], xr[4], xh[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          xz[k] = mf_x(xg, oz, k);
          xr[k] = mf_x(xg, orr, k);
          xh[k] = mf_x(xg, oh, k);
        }
        mf_zr_split(xg, wz, wr, oz, orr, nzr, nfzr, xz, xr, vz[0], vr[0], fz, fr);
        uint32_t fp = frow;
        asm volatile("" : "+v"(fp));
        const int frz = (int)(fp & 0x1FF), frr = (int)((fp >> 9) & 0x1FF), frh = (int)((fp >> 18) & 0x1FF);
        int *pg = part + g * 3 * (NA + 1) * S;
        int pz[S], pr[S], ph[S];
        for (int s = 0; s < S; s++) {
          pz[s] = fz[s];
          pr[s] = fr[s];
        }
        /* the z/r adds go out before the h product and drain beside its
         * MFMAs (2048 streams: -0.9 % frame step; neutral on mf_kernel<4>) */
        /* branch-free: a lane of a hosting wave without a piece adds 0 to
         * its own row's words (skewed model: 2048 / 8192 streams -0.7 /
         * -0.9 %, three same-box rounds) */
        auto padd = [&](int gt, int fr_, int (&v)[S]) {
          const bool h = fr_ != NA;
          int vv[S];
          for (int s = 0; s < S; s++) vv[s] = h ? v[s] : 0;
          part_add<S, true>(pg, gt, h ? fr_ : i, vv);
        };
        if (nfzr > 0) {
          padd(0, frz, pz);
          padd(1, frr, pr);
        }
        mf_h_split(xg, wh, oh, nh, nfh, xh, vh, fh);
        for (int s = 0; s < S; s++) ph[s] = fh[0][s] + fh[1][s];
        if (nfh > 0) padd(2, frh, ph);
        for (int s = 0; s < S; s++) {
          iaz[s] = vz[0][s];
          iar[s] = vr[0][s];
          iah[s] = (vh[0][s] + vh[1][s]) + cvt_rne((bh + dh * st[g][s]) * kScale); /* int32 sums associate */
          tz[s] = bz + dz * st[g][s];
          tr[s] = br + dr * st[g][s];
        }
        return;
      }
      switch (nzr * 16 + nh) {
#define MF_CASE(Z, H)                                 \
  case Z * 16 + H:                                    \
    mf_zr<1>(xg, wz, wr, oz, orr, Z, vz, vr);         \
    mf_run<MF_HMAX, 2>(xg, wh, oh, H, vh);            \
    break;
#define MF_CASES(Z) MF_CASE(Z, 1) MF_CASE(Z, 2) MF_CASE(Z, 3) MF_CASE(Z, 4) MF_CASE(Z, 5) MF_CASE(Z, 6) MF_CASE(Z, 7) MF_CASE(Z, 8)
        MF_CASES(1)
        MF_CASES(2)
        MF_CASES(3)
        MF_CASES(4)
#undef MF_CASES
#undef MF_CASE
        default:
          mf_zr<1>(xg, wz, wr, oz, orr, nzr, vz, vr);
          mf_run<MF_HMAX, 2>(xg, wh, oh, nh, vh);
          break;
      }
      for (int s = 0; s < S; s++) {
        az[s] = (float)vz[0][s];
        ar[s] = (float)vr[0][s];
        tz[s] = bz + dz * st[g][s];
        tr[s] = br + dr * st[g][s];
        hpre[s] = (float)((vh[0][s] + vh[1][s]) + cvt_rne((bh + dh * st[g][s]) * kScale)) * kScale1;
      }
    };
    /* one group's GRU_A input gathers (nnet.c:484-491) and elementwise step */
    auto step = [&](auto gc, bool fast) {
      constexpr int g = decltype(gc)::value;
      float e[S][9];
      for (int s = 0; s < S; s++) {
        const int4 v = *(const int4 *)(ix + (g * S + s) * 4);
        uint32_t o1 = (uint32_t)tid * 4u + (uint32_t)v.x;
        uint32_t o2 = (uint32_t)tid * 4u + (uint32_t)v.y;
        uint32_t o3 = (uint32_t)tid * 4u + (uint32_t)v.z;
        asm volatile("" : "+v"(o1), "+v"(o2), "+v"(o3));
        const char *b1 = (const char *)A.mf_emb[0], *b2 = (const char *)A.mf_emb[1], *b3 = (const char *)A.mf_emb[2];
#pragma unroll
        for (uint32_t q = 0; q < 3; q++) {
          e[s][q] = *(const float *)(b1 + o1 + q * NA * 4u);
          e[s][3 + q] = *(const float *)(b2 + o2 + q * NA * 4u);
          e[s][6 + q] = *(const float *)(b3 + o3 + q * NA * 4u);
        }
      }
      if constexpr (SPLIT) {
        /* the hosted pieces' partial sums of this thread's rows (added by
         * the group's recurrent product a barrier ago), then cleared */
        uint32_t fp = frow;
        asm volatile("" : "+v"(fp));
        int *pg = part + g * 3 * (NA + 1) * S;
        /* every row reads its words (no branch waits on the reads; rows
         * without pieces read zeros): +3 % at 2048 streams */
        int zadd[S], radd[S], hadd[S];
        part_read<S, true>(pg, 0, i, zadd);
        part_read<S, true>(pg, 1, i, radd);
        part_read<S, true>(pg, 2, i, hadd);
        if (fp >> 27 & 1) part_clear<S, true>(pg, 0, i);
        if (fp >> 28 & 1) part_clear<S, true>(pg, 1, i);
        if (fp >> 29 & 1) part_clear<S, true>(pg, 2, i);
        for (int s = 0; s < S; s++) {
          iaz[s] += zadd[s];
          iar[s] += radd[s];
        }
        for (int s = 0; s < S; s++) {
          hpre[s] = (float)(iah[s] + hadd[s]) * kScale1;
          az[s] = (float)iaz[s];
          ar[s] = (float)iar[s];
        }
      }
      int stub = 0;
      auto nostamp = [&](int) { (void)stub; };
      const float *cg = cnd + g * GA_ROWS * S;
      if (__builtin_amdgcn_readfirstlane((int)fast))
        ga_elementwise<S, true, false>(st[g], e, cg, tid, az, ar, tz, tr, hpre, rcp, xa + g * S * MF_XSTR + i, false, nostamp);
      else
        ga_elementwise<S, false, false>(st[g], e, cg, tid, az, ar, tz, tr, hpre, rcp, xa + g * S * MF_XSTR + i, false, nostamp);
    };
    /* the range words of a frame are double-buffered by frame parity: a
     * frame boundary's staging never overwrites words still being read */
    auto group_fast = [&](int g, int par) {
      bool f = true;
      for (int w = 0; w < SAMPLE_WAVES; w++) f &= okw[(par * 2 + g) * 8 + w] != 0;
      return f;
    };
    using G0 = std::integral_constant<int, 0>;
    using G1 = std::integral_constant<int, 1>;
    recurrent(G0{});
    bool fast0 = true, fast1 = true;
    for (int t = 0; t < total; t++) {
      const int n = t % A.N, par = (t / A.N) & 1;
      __syncthreads(); /* phase A(t): ix_A(t) published, q(h_A) of B(t-1) complete */
      if (n == 0) fast0 = group_fast(0, par);
      step(G0{}, fast0);
      recurrent(G1{});
      __syncthreads(); /* phase B(t): ix_B(t) published, q(h_A) of A(t) complete */
      if (n == 0) fast1 = group_fast(1, par);
      step(G1{}, fast1);
      if (n == A.N - 1 && t + 1 < total) {
        /* the next frame's conditioning: lane-private entries (both groups'
         * last elementwise steps of this frame are done); the range words
         * are read after the next barrier */
        cf += A.nstreams;
        stage(0, cf, par ^ 1);
        stage(1, cf, par ^ 1);
      }
      if (t + 1 < total) recurrent(G0{});
    }
    __syncthreads(); /* extra phase: the samplers walk B's last sample */
    __syncthreads(); /* final */
    for (int g = 0; g < 2; g++)
      for (int s = 0; s < S; s++)
        if (active[g * S + s]) A.st[s0 + g * S + s].gru_a_state[i] = st[g][s];
  } else {
    /* ======================= sampler role ================================ */
    const float *logit_tab = (const float *)(img + IMG_LOGIT);
    const int sw = wv - SAMPLE_WAVES;
    const int half = lane >> 5, hl = lane & 31;
    const int ms = S == 4 ? 2 * sw + half : sw; /* this half's stream within a group */
    const bool samp = ms < S;
    const bool samp_w = samp && (S == 4 || half == 0);
    const int msc = samp ? ms : 0;
    /* GRU_B lanes: (stream gs, unit gu) = (lane / 16, lane % 16); states
     * as the MFMA A operand (row m = stream m/4), weight tiles as B: D
     * register 0 is unit gu of stream gs (mf_kernel) */
    const int gs = lane >> 4, gu = lane & 15, sl = min(gs, S - 1), sx = min(gu >> 2, S - 1);
    const bool gown = gs < S && (S == 4 ? (gs >> 1) : gs) == sw;

    float lsr[2][NLPC], pred[2], deemph[2], sbv[2];
    uint32_t rng[2][4];
    int last_exc[2];
    bool my_act[2], g_act[2];
    for (int g = 0; g < 2; g++) {
      const int sid = min(s0 + g * S + msc, A.nstreams - 1);
      const StreamState *p = &A.st[sid];
#pragma unroll
      for (int j = 0; j < NLPC; j++) lsr[g][j] = p->last_sig[j];
      deemph[g] = p->deemph_mem;
      last_exc[g] = p->last_exc & 0xFF;
      rng[g][0] = p->rng[0]; rng[g][1] = p->rng[1]; rng[g][2] = p->rng[2]; rng[g][3] = p->rng[3];
      my_act[g] = samp && active[g * S + msc];
      g_act[g] = gown && active[g * S + sl];
      sbv[g] = A.st[min(s0 + g * S + sl, A.nstreams - 1)].gru_b_state[gu];
    }

    /* GRU_B input tiles in registers, the recurrent ones in LDS */
    v4i wt[MF_GB_IN];
#pragma unroll
    for (int t = 0; t < MF_GB_IN; t++) {
      const uint4 u = A.mf_gb[t * 64 + lane];
      wt[t] = v4i{(int)u.x, (int)u.y, (int)u.z, (int)u.w};
    }
    if (sw == 0)
      for (int q = 0; q < 3; q++) {
        const uint4 u = A.mf_gb[(MF_GB_IN + q) * 64 + lane];
        gbw[q * 64 + lane] = v4i{(int)u.x, (int)u.y, (int)u.z, (int)u.w};
      }
    /* this wave's GRU_B input seeds of group g for a frame (nnet.c:347-356
     * with the offset-128 correction), and group g's LPC of that frame */
    int *myg = gbs + sw * 2 * S * GB_ROWS;
    auto stage_frame = [&](int g, const FrameCond *cf) {
      for (int e = lane; e < S * GB_ROWS; e += 64) {
        const int s = e / GB_ROWS, r = e % GB_ROWS;
        myg[g * S * GB_ROWS + e] =
            cvt_rne((A.gb_par[r] + gru_b_cond_of(cf, A, min(s0 + g * S + s, A.nstreams - 1))[r]) * kScale) + A.gb_wsum[r];
      }
      if (samp_w && hl < NLPC) lpcb[(g * S + ms) * NLPC + hl] = lpc_of(cf, A, min(s0 + g * S + ms, A.nstreams - 1))[hl];
    };
    auto ix_word = [](int su, int pu, int exc) { return make_int4(su * (GA_ROWS * 4), pu * (GA_ROWS * 4), exc * (GA_ROWS * 4), 0); };
    /* pred and the u-law indices of group g's next sample (lpcnet.c:252-254)
     * from the frame's LPC */
    auto restart = [&](int g) {
      float p2 = 0.f;
#pragma unroll
      for (int j = 0; j < NLPC; j++) p2 = p2 - lsr[g][j] * lpcb[(g * S + msc) * NLPC + j];
      pred[g] = p2;
      if (samp_w && hl == 0) *(int4 *)(ix + (g * S + ms) * 4) = ix_word(lin2ulaw_x86(lsr[g][0]), lin2ulaw_x86(pred[g]), last_exc[g]);
    };
    const FrameCond *cfr[2] = {A.cond, A.cond};
    stage_frame(0, cfr[0]);
    stage_frame(1, cfr[1]);
    __syncthreads(); /* image in LDS */
    FcLane F;
    F.init(img, lane);
    for (int g = 0; g < 2; g++)
      if (gown) xb[(g * S + gs) * NB + gu] = (unsigned char)quant_s8_state(sbv[g]);
    __builtin_amdgcn_wave_barrier();
    restart(0);
    restart(1);
    __syncthreads(); /* initial */
    __builtin_amdgcn_s_setprio(3);

    /* group g's GRU_B step and walk of sample t (lpcnet.c:244-270) */
    auto walk = [&](auto gc, int t) {
      constexpr int g = decltype(gc)::value;
      const int n = t % A.N, f = t / A.N;
      if (!samp) return;
      const uint32_t r0 = kiss99_next(rng[g][0], rng[g][1], rng[g][2], rng[g][3]);
      const uint32_t r1 = kiss99_next(rng[g][0], rng[g][1], rng[g][2], rng[g][3]);
      float t03, t47;
      lane_thresholds(F, logit_tab, r0, r1, t03, t47);
      /* GRU_B (nnet.c:345-361): recurrent product on q(h_B(t-1)), input
       * product on q(h_A(t)), all S streams of the group as MFMA columns */
      v4i acc[3], accr[3];
      const v4i xr = *(const v4i *)(xb + (g * S + sx) * NB); /* k 0..15; the tiles' other K chunks are zero */
#pragma unroll
      for (int q = 0; q < 3; q++) {
        acc[q] = v4i{myg[(g * S + sl) * GB_ROWS + 16 * q + gu], 0, 0, 0};
        accr[q] = v4i{gbr[16 * q + gu], 0, 0, 0};
      }
#pragma unroll
      for (int q = 0; q < 3; q++) accr[q] = mfma16(xr, gbw[q * 64 + lane], accr[q]);
      v4i xk[6];
#pragma unroll
      for (int kt = 0; kt < 6; kt++) xk[kt] = *(const v4i *)(xa + (g * S + sx) * MF_XSTR + 64 * kt + 16 * gs);
#pragma unroll
      for (int kt = 0; kt < 6; kt++)
#pragma unroll
        for (int q = 0; q < 2; q++) acc[q] = mfma16(xk[kt], wt[q * 6 + kt], acc[q]);
#pragma unroll
      for (int kt = 0; kt < 6; kt++) acc[2] = mfma16(xk[kt], wt[12 + kt], acc[2]);
      float zrb[2] = {(float)acc[0][0] * kScale1 + (float)accr[0][0] * kScale1,
                      (float)acc[1][0] * kScale1 + (float)accr[1][0] * kScale1};
      sigmoid_x86_fin_n<2, HWR>(zrb, rcp);
      float hh[1] = {(float)acc[2][0] * kScale1 + ((float)accr[2][0] * kScale1) * zrb[1]};
      tanh_x86_fin_n<1, HWR>(hh, rcp); /* |hh| < 2^19: int32 sums x 2^-14 */
      sbv[g] = zrb[0] * sbv[g] + (1.f - zrb[0]) * hh[0];
      if (gown) sbuf[(g * S + gs) * NB + gu] = sbv[g];
      __builtin_amdgcn_wave_barrier();
      float xv[NB];
      {
        const float4 *b4 = (const float4 *)(sbuf + (g * S + msc) * NB);
#pragma unroll
        for (int j = 0; j < NB / 4; j++) {
          const float4 v = b4[j];
          xv[4 * j] = v.x; xv[4 * j + 1] = v.y; xv[4 * j + 2] = v.z; xv[4 * j + 3] = v.w;
        }
      }
      float lpr[NLPC];
      {
        const float4 *l4 = (const float4 *)(lpcb + (g * S + msc) * NLPC);
#pragma unroll
        for (int j = 0; j < NLPC / 4; j++) {
          const float4 v = l4[j];
          lpr[4 * j] = v.x; lpr[4 * j + 1] = v.y; lpr[4 * j + 2] = v.z; lpr[4 * j + 3] = v.w;
        }
      }
      /* (the select-free walk of mf_kernel measured 1 % slower here) */
      const WalkOut R = dual_fc_walk<false, false, HWR>(F, t03, t47, xv, pred[g], lsr[g], lpr, nullptr, deemph[g]);
      if (samp_w && hl == 0) *(int4 *)(ix + (g * S + ms) * 4) = ix_word(R.su, R.pu, R.exc);
      /* bookkeeping (lpcnet.c:262-269) and the output sample */
#pragma unroll
      for (int j = NLPC - 1; j > 0; j--) lsr[g][j] = lsr[g][j - 1];
      lsr[g][0] = R.pcm;
      last_exc[g] = R.exc;
      pred[g] = R.pn;
      float o = R.pcm + kPreemph * deemph[g];
      deemph[g] = o;
      if (o < -32767) o = -32767;
      if (o > 32767) o = 32767;
      const int sid = s0 + g * S + ms;
      if (samp_w && hl == 0 && sid < A.nstreams)
        A.pcm[((size_t)f * A.nstreams + sid) * A.N + n] = my_act[g] ? (short)round_half_up(o) : (short)0;
      if (gown) xb[(g * S + gs) * NB + gu] = (unsigned char)quant_s8_state(sbv[g]);
      if (n == A.N - 1 && f + 1 < nfr) {
        /* frame boundary: the next frame's seeds and LPC, then pred and the
         * indices of its first sample, as at a launch start */
        cfr[g] += A.nstreams;
        stage_frame(g, cfr[g]);
        __builtin_amdgcn_wave_barrier();
        restart(g);
      }
    };
    using G0 = std::integral_constant<int, 0>;
    using G1 = std::integral_constant<int, 1>;
    for (int t = 0; t < total; t++) {
      __syncthreads(); /* phase A(t) */
      if (t > 0) walk(G1{}, t - 1);
      __syncthreads(); /* phase B(t) */
      walk(G0{}, t);
    }
    __syncthreads(); /* extra phase */
    walk(G1{}, total - 1);
    __syncthreads(); /* final */
    for (int g = 0; g < 2; g++) {
      if (samp_w && my_act[g] && hl == 0) {
        StreamState *p = &A.st[s0 + g * S + ms];
#pragma unroll
        for (int j = 0; j < NLPC; j++) p->last_sig[j] = lsr[g][j];
        p->deemph_mem = deemph[g];
        p->last_exc = last_exc[g];
        p->rng[0] = rng[g][0]; p->rng[1] = rng[g][1]; p->rng[2] = rng[g][2]; p->rng[3] = rng[g][3];
      }
      if (g_act[g]) A.st[s0 + g * S + gs].gru_b_state[gu] = sbv[g];
    }
  }
}

template <int S, bool SPLIT, bool HWR>
static int launch_mf2_t(const SampleArgs &a, hipStream_t stream)
{
  if (ensure_dyn_lds((const void *)mf2_kernel<S, SPLIT, HWR>, 160 * 1024 - IMG_VAR)) return -1;
  const int grid = (a.nstreams + 2 * S - 1) / (2 * S);
  hipLaunchKernelGGL((mf2_kernel<S, SPLIT, HWR>), dim3(grid), dim3(MF_THREADS), mf2_lds_bytes(S, SPLIT) - IMG_VAR, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <bool HWR>
static int launch_mf2_h(const SampleArgs &a, int S, hipStream_t st)
{
  if (a.mf_split) return S == 4 ? launch_mf2_t<4, true, HWR>(a, st) : launch_mf2_t<2, true, HWR>(a, st);
  return S == 4 ? launch_mf2_t<4, false, HWR>(a, st) : launch_mf2_t<2, false, HWR>(a, st);
}

int launch_mf2(const SampleArgs &a, int S, void *stream)
{
  hipStream_t st = (hipStream_t)stream;
  return a.rcp_hw ? launch_mf2_h<true>(a, S, st) : launch_mf2_h<false>(a, S, st);
}

}  // namespace lpcnet_mi355x
