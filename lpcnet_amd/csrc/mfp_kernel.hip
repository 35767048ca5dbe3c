/*
 * mfp_kernel.hip -- the two-group matrix-core sample kernel:
 * lpcnet_synthesize_tail_impl (lpcnet.c:235-271) for 4 streams per
 * 512-thread workgroup, as two groups of two streams running half a sample
 * apart.  Default for non-saturating int8 models at >= 1024 streams.
 *
 * Same roles, weights and arithmetic as mf_kernel (mf_kernel.hip): GRU_A
 * waves 0..5 (thread = unit) run the GRU_A input gathers, elementwise step
 * and the recurrent product on v_mfma_i32_4x4x4_16b_i8; sampler wave 6+g
 * runs GRU_B (v_mfma_i32_16x16x64_i8) and the dual-FC walk of group g
 * (streams 2g, 2g+1, one per 32-lane half).
 *
 * What changes is the schedule.  In mf_kernel all four streams step
 * together, so each sample costs X (GRU_A gathers + elementwise, VALU bound
 * on the SIMDs that carry two GRU_A waves) plus Y (GRU_B + walk, a latency
 * chain in the sampler waves), and each role idles through the other's
 * phase.  Here the GRU_A waves alternate between the groups:
 *     X(0,n)  MV(0,n)  X(1,n)  MV(1,n)  X(0,n+1) ...
 * while sampler 6 runs Y(0,n) during X(1,n) and sampler 7 runs Y(1,n)
 * during X(0,n+1).  The per-group cycle is X + Y of two streams; the GRU_A
 * waves' cycle is X + MV of both groups.  No workgroup barrier inside the
 * loop: LDS flags (lds_flags.h) carry each dependency --
 *   ixseq[g] = n+1    ix of group g's sample n published (sampler -> GRU_A)
 *   done[g][w] = n+1  wave w wrote q(h_A(n)) of group g (GRU_A -> all)
 * q(h_A) is double-buffered by sample parity: a GRU_A wave writing sample
 * n+1 can only pass ixseq once every wave finished X(g,n), which in each
 * wave's program order follows MV(g,n-1), the last reader of that buffer.
 */
#include <hip/hip_runtime.h>

#include <type_traits>

#include "device_math.h"
#include "lds_flags.h"
#include "lpcnet_engine.h"
#include "mf_common.h"
#include "sampler.h"

namespace lpcnet_mi355x {

namespace {

constexpr int MFP_S = 4;
constexpr int MFP_SYNC_IX = 0;    /* ixseq[2] */
constexpr int MFP_SYNC_ABORT = 2;
constexpr int MFP_SYNC_DONE = 8;  /* done[2][8] */

struct MfpLds {
  static constexpr int x = 2 * MFP_S * MF_XSTR; /* q(h_A) [parity][stream][MF_XSTR] (signed form) */
  static constexpr int xb = MFP_S * NB;          /* q(h_B) [stream][16] */
  static constexpr int sb = MFP_S * NB * 4;      /* float h_B [stream][16] (tree-walk broadcast) */
  static constexpr int ix = MFP_S * 16;          /* sig/pred/exc indices */
  static constexpr int sync = 32 * 4;            /* flags */
  static constexpr int pcm = ((MFP_S * FRAME * 2 + 15) / 16) * 16;
  static constexpr int cnd = GA_ROWS * MFP_S * 4; /* GRU_A conditioning [3][NA][stream] */
  static constexpr int gbs = MFP_S * GB_ROWS * 4; /* GRU_B input accumulator seeds [stream][48] */
  static constexpr int gbr = GB_ROWS * 4;         /* GRU_B recurrent accumulator seeds [48] */
  static constexpr int total = x + xb + sb + ix + sync + pcm + cnd + gbs + gbr;
};

template <int V>
using ic = std::integral_constant<int, V>;

}  // namespace

int mfp_lds_bytes() { return IMG_VAR + MfpLds::total; }

template <bool TRACE>
__global__ __launch_bounds__(MF_THREADS) void mfp_kernel(SampleArgs A)
{
  extern __shared__ uint4 lds4[];
  unsigned char *lds = (unsigned char *)lds4;
  using L = MfpLds;
  constexpr int S = MFP_S;
  unsigned char *xa = lds; /* first: every x address fits the 16-bit offsets kept in registers */
  unsigned char *xb = xa + L::x;
  float *sbuf = (float *)(xb + L::xb);
  int *ix = (int *)((unsigned char *)sbuf + L::sb);
  int *sync = (int *)((unsigned char *)ix + L::ix);
  short *pcmbuf = (short *)((unsigned char *)sync + L::sync);
  float *cnd = (float *)((unsigned char *)pcmbuf + L::pcm);
  int *gbs = (int *)((unsigned char *)cnd + L::cnd);
  int *gbr = gbs + S * GB_ROWS;
  unsigned char *img = lds + L::total;
  int *abort_w = sync + MFP_SYNC_ABORT;

  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int s0 = blockIdx.x * S;
  const uint32_t *rcp = (const uint32_t *)(img + IMG_RCP);

  bool active[S];
  bool any = false;
  for (int s = 0; s < S; s++) {
    const int sid = s0 + s;
    active[s] = sid < A.nstreams && A.st[sid].frame_count > FEATURES_DELAY;
    any |= active[s];
  }
  if (!any) {
    for (int e = tid; e < S * A.N; e += MF_THREADS) {
      const int s = e / A.N, n = e % A.N;
      if (s0 + s < A.nstreams) A.pcm[(size_t)(s0 + s) * A.N + n] = 0;
    }
    return;
  }
  {
    uint4 *img4 = (uint4 *)img;
    for (int o = tid; o < IMG_VAR / 16; o += MF_THREADS) img4[o] = A.image[o];
  }
  for (int e = tid; e < S * A.preload; e += MF_THREADS) {
    const int s = e / A.preload, n = e % A.preload;
    pcmbuf[s * FRAME + n] = A.pcm[(size_t)min(s0 + s, A.nstreams - 1) * A.N + n];
  }
  if (tid < 32) sync[tid] = tid < 2 ? 1 : 0; /* ix of sample 0 is written before the loop */

  const bool stamping = A.stamps != nullptr;
  unsigned long long stp[16] = {};
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

  if (wv < SAMPLE_WAVES) {
    /* ======================= GRU_A role ================================== */
    const int i = tid;
    const float bz = A.ga_par[i], br = A.ga_par[NA + i], bh = A.ga_par[2 * NA + i];
    const float dz = A.ga_par[3 * NA + i], dr = A.ga_par[4 * NA + i], dh = A.ga_par[5 * NA + i];
    const int wsz = A.ga_wsum[i], wsr = A.ga_wsum[NA + i], wsh = A.ga_wsum[2 * NA + i];
    float st[S];
    for (int s = 0; s < S; s++) {
      const StreamState *p = &A.st[min(s0 + s, A.nstreams - 1)];
      st[s] = p->gru_a_state[i];
      cnd[i * S + s] = p->gru_a_cond[i];
      cnd[(NA + i) * S + s] = p->gru_a_cond[NA + i];
      cnd[(2 * NA + i) * S + s] = p->gru_a_cond[2 * NA + i];
    }
    /* GRU_B accumulator seeds (nnet.c:347-356 with the offset-128 correction) */
    for (int e = tid; e < S * GB_ROWS; e += SAMPLE_THREADS) {
      const int s = e / GB_ROWS, r = e % GB_ROWS;
      gbs[e] = cvt_rne((A.gb_par[r] + A.st[min(s0 + s, A.nstreams - 1)].gru_b_cond[r]) * kScale) + A.gb_wsum[r];
    }
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
      /* A operand of lane 4b+m = stream m of the group (m >= 2 duplicate
       * stream 1; their D registers are never read) */
      const uint32_t mo = (uint32_t)min(lane & 3, 1) * MF_XSTR;
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
    __syncthreads(); /* image in LDS */
    /* q(h_A) before sample 0 goes to parity 1 ("sample -1") */
    for (int s = 0; s < S; s++) xa[(S + s) * MF_XSTR + i] = (unsigned char)quant_s8(st[s]);
    __syncthreads(); /* initial q(h_A), q(h_B), ix, seeds, flags */
    stamp_start();

    int az[S], ar[S];
    float tz[S], tr[S], hpre[S];
    /* W q(h_A) of group G from parity-P buffer, and the per-sample terms
     * that depend only on the state (nnet.c:431-440) */
    auto recurrent = [&](auto G, auto P) {
      constexpr int g = decltype(G)::value, p = decltype(P)::value;
      const unsigned char *xg = lds + (p * S + 2 * g) * MF_XSTR;
      v4i vz[2] = {{wsz, wsz, wsz, wsz}, {0, 0, 0, 0}}, vr[2] = {{wsr, wsr, wsr, wsr}, {0, 0, 0, 0}};
      v4i vh[4] = {{wsh, wsh, wsh, wsh}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
      mf_opaque(oz);
      mf_opaque(orr);
      mf_opaque(oh);
      mf_zr<2>(xg, wz, wr, oz, orr, nzr, vz, vr);
      mf_run<MF_HMAX, 4>(xg, wh, oh, nh, vh);
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const int s = 2 * g + k;
        az[s] = vz[0][k] + vz[1][k];
        ar[s] = vr[0][k] + vr[1][k];
        const int ah = (vh[0][k] + vh[1][k]) + (vh[2][k] + vh[3][k]);
        tz[s] = bz + dz * st[s];
        tr[s] = br + dr * st[s];
        hpre[s] = (float)(ah + cvt_rne((bh + dh * st[s]) * kScale)) * kScale1;
      }
    };
    /* X(G, n): GRU_A input gathers (nnet.c:484-491) and the compute_sparse_gru
     * elementwise step (nnet.c:431-447) for the group's two streams, into
     * parity P; then MV(G, n) for sample n+1 */
    auto xstep = [&](auto G, auto P, int n) {
      constexpr int g = decltype(G)::value, p = decltype(P)::value;
      constexpr int sa = 2 * g;
      flag_wait<1>(sync + MFP_SYNC_IX + g, n + 1, abort_w);
      stamp(5);
      typedef float v2f __attribute__((ext_vector_type(2)));
      float e[2][9];
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const int4 v = *(const int4 *)(ix + (sa + k) * 4);
        const float *e1 = A.emb_sig + (__builtin_amdgcn_readfirstlane(v.x) & 0xFF) * GA_ROWS;
        const float *e2 = A.emb_pred + (__builtin_amdgcn_readfirstlane(v.y) & 0xFF) * GA_ROWS;
        const float *e3 = A.emb_exc + (__builtin_amdgcn_readfirstlane(v.z) & 0xFF) * GA_ROWS;
#pragma unroll
        for (int q = 0; q < 3; q++) {
          e[k][q] = e1[q * NA + i];
          e[k][3 + q] = e2[q * NA + i];
          e[k][6 + q] = e3[q * NA + i];
        }
      }
      if (stamping) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < 2; k++)
#pragma unroll
          for (int q = 0; q < 9; q++) t += e[k][q];
        asm volatile("" ::"v"(t));
        stamp(10);
      }
      /* packed v_pk_add/mul_f32 over the stream pair: each lane of a packed
       * op is the scalar IEEE op, so the sums keep their order and bits */
      const v2f inz = ((*(const v2f *)(cnd + i * S + sa) + v2f{e[0][0], e[1][0]}) + v2f{e[0][3], e[1][3]}) +
                      v2f{e[0][6], e[1][6]};
      const v2f inr = ((*(const v2f *)(cnd + (NA + i) * S + sa) + v2f{e[0][1], e[1][1]}) + v2f{e[0][4], e[1][4]}) +
                      v2f{e[0][7], e[1][7]};
      const v2f inh = ((*(const v2f *)(cnd + (2 * NA + i) * S + sa) + v2f{e[0][2], e[1][2]}) + v2f{e[0][5], e[1][5]}) +
                      v2f{e[0][8], e[1][8]};
      const v2f qz = (v2f{tz[sa], tz[sa + 1]} + inz) * kScale;
      const v2f qr = (v2f{tr[sa], tr[sa + 1]} + inr) * kScale;
      const v2f fz = v2f{(float)(az[sa] + cvt_rne(qz.x)), (float)(az[sa + 1] + cvt_rne(qz.y))} * kScale1;
      const v2f fr = v2f{(float)(ar[sa] + cvt_rne(qr.x)), (float)(ar[sa + 1] + cvt_rne(qr.y))} * kScale1;
      float zrv[4] = {fz.x, fz.y, fr.x, fr.y};
      sigmoid_x86_n<4>(zrv, rcp);
      const v2f h2 = v2f{hpre[sa], hpre[sa + 1]} * v2f{zrv[2], zrv[3]} + inh;
      float hv[2] = {h2.x, h2.y};
      tanh_x86_n<2>(hv, rcp);
      const v2f z = v2f{zrv[0], zrv[1]};
      const v2f n2 = z * v2f{st[sa], st[sa + 1]} + (1.f - z) * v2f{hv[0], hv[1]};
      st[sa] = n2.x;
      st[sa + 1] = n2.y;
      xa[(p * S + sa) * MF_XSTR + i] = (unsigned char)quant_s8(st[sa]);
      xa[(p * S + sa + 1) * MF_XSTR + i] = (unsigned char)quant_s8(st[sa + 1]);
      stamp(0);
      flag_publish(sync + MFP_SYNC_DONE + 8 * g + wv, n + 1);
      if (n + 1 < A.N) {
        /* the recurrent product reads every wave's units of q(h_A(n)) */
        for (int w = 0; w < SAMPLE_WAVES; w++) flag_wait(sync + MFP_SYNC_DONE + 8 * g + w, n + 1, abort_w);
        stamp(3);
        recurrent(G, P);
        stamp(2);
      }
    };
    recurrent(ic<0>(), ic<1>());
    recurrent(ic<1>(), ic<1>());
    for (int n = 0; n < A.N; n += 2) {
      xstep(ic<0>(), ic<0>(), n);
      xstep(ic<1>(), ic<0>(), n);
      if (n + 1 < A.N) {
        xstep(ic<0>(), ic<1>(), n + 1);
        xstep(ic<1>(), ic<1>(), n + 1);
      }
    }
    stamp(4);
    __syncthreads(); /* final */
    stamp(5);
    for (int s = 0; s < S; s++)
      if (active[s]) A.st[s0 + s].gru_a_state[i] = st[s];
  } else {
    /* ======================= sampler role ================================ */
    const float *logit_tab = (const float *)(img + IMG_LOGIT);
    const int g = wv - SAMPLE_WAVES; /* group: streams 2g, 2g+1 */
    const int half = lane >> 5, hl = lane & 31;
    const int ms = 2 * g + half;     /* stream walked by this half */
    const bool my_active = s0 + ms < A.nstreams && A.st[s0 + ms].frame_count > FEATURES_DELAY;
    /* GRU_B: lane = (unit quad gq, column gs, gi); column gs carries stream
     * 2g + (gs & 1) (columns 2, 3 duplicate 0, 1); D register gi of this lane
     * holds row 4gq + gi.  gown: the lane's column is the stream's owner. */
    const int gq = lane >> 4, gs = (lane & 15) >> 2, gi = lane & 3, gu = 4 * gq + gi, sl = 2 * g + (gs & 1);
    const bool gown = gs < 2;
    const bool gact = gown && s0 + sl < A.nstreams && A.st[s0 + sl].frame_count > FEATURES_DELAY;

    float lsr[NLPC], lpr[NLPC];
    float pred = 0.f, deemph = 0.f;
    uint32_t rz = 0, rw = 0, rj = 0, rc = 0;
    int last_exc = 0;
    {
      const StreamState *p = &A.st[min(s0 + ms, A.nstreams - 1)];
#pragma unroll
      for (int j = 0; j < NLPC; j++) {
        lsr[j] = p->last_sig[j];
        lpr[j] = p->lpc[j];
      }
      deemph = p->deemph_mem;
      last_exc = p->last_exc;
      rz = p->rng[0]; rw = p->rng[1]; rj = p->rng[2]; rc = p->rng[3];
    }
    float sbv = A.st[min(s0 + sl, A.nstreams - 1)].gru_b_state[gu];
    v4i wt[MF_GB_TILES];
#pragma unroll
    for (int t = 0; t < MF_GB_TILES; t++) {
      const uint4 u = A.mf_gb[t * 64 + lane];
      wt[t] = v4i{(int)u.x, (int)u.y, (int)u.z, (int)u.w};
    }
    auto put_xb = [&]() {
      if (gown) xb[sl * NB + gu] = (unsigned char)quant_s8(sbv);
    };
    auto pick = [&](const v4i &a) -> int { return gi == 0 ? a[0] : (gi == 1 ? a[1] : (gi == 2 ? a[2] : a[3])); };
    __syncthreads(); /* image in LDS */
    FcLane F;
    F.init(img, lane);
    put_xb();
    {
      /* pred and the u-law indices of the first sample (lpcnet.c:252-254) */
      float p2 = 0.f;
#pragma unroll
      for (int j = 0; j < NLPC; j++) p2 = p2 - lsr[j] * lpr[j];
      pred = p2;
      if (hl == 0) *(int4 *)(ix + ms * 4) = make_int4(lin2ulaw_x86(lsr[0]), lin2ulaw_x86(pred), last_exc, 0);
    }
    __syncthreads(); /* initial q(h_A), q(h_B), ix, seeds, flags */
    stamp_start();
    /* the sampler chain is each group's critical path: issue first */
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
      if (hl == 0 && pend_n >= A.preload) pcmbuf[ms * FRAME + pend_n] = (short)round_half_up(o);
      put_xb();
      pend_n = -1;
    };
    for (int n = 0; n < A.N; n++) {
      stamp(4);
      finish();
      stamp(13);
      /* the two kiss99 draws of this sample and their thresholds (nnet.c:178-184) */
      const uint32_t r0 = kiss99_next(rz, rw, rj, rc);
      const uint32_t r1 = kiss99_next(rz, rw, rj, rc);
      lane_thresholds(F, logit_tab, r0, r1, t03, t47);
      /* GRU_B recurrent product (nnet.c:355-361): needs only q(h_B(n-1)) */
      v4i acc[3], accr[3];
      const v4i xr = *(const v4i *)(xb + sl * NB);
#pragma unroll
      for (int q = 0; q < 3; q++) {
        acc[q] = *(const v4i *)(gbs + sl * GB_ROWS + 16 * q + 4 * gq);
        accr[q] = *(const v4i *)(gbr + 16 * q + 4 * gq);
      }
#pragma unroll
      for (int q = 0; q < 3; q++) accr[q] = mfma16(wt[18 + q], xr, accr[q]);
      stamp(0);
      /* q(h_A(n)) of this group complete */
      for (int w = 0; w < SAMPLE_WAVES; w++) flag_wait(sync + MFP_SYNC_DONE + 8 * g + w, n + 1, abort_w);
      stamp(1);
      {
        /* GRU_B input product (nnet.c:345-353), 48 x 384 */
        const unsigned char *xs = xa + ((n & 1) * S + sl) * MF_XSTR;
        v4i xk[6];
#pragma unroll
        for (int kt = 0; kt < 6; kt++) xk[kt] = *(const v4i *)(xs + 64 * kt + 16 * gq);
#pragma unroll
        for (int kt = 0; kt < 6; kt++)
#pragma unroll
          for (int q = 0; q < 2; q++) acc[q] = mfma16(wt[q * 6 + kt], xk[kt], acc[q]);
#pragma unroll
        for (int kt = 0; kt < 6; kt++) acc[2] = mfma16(wt[12 + kt], xk[kt], acc[2]);
        stamp(10);
        /* GRU_B elementwise (nnet.c:362-371), unit gu of stream sl */
        float zrb[2] = {(float)pick(acc[0]) * kScale1 + (float)pick(accr[0]) * kScale1,
                        (float)pick(acc[1]) * kScale1 + (float)pick(accr[1]) * kScale1};
        sigmoid_x86_n<2>(zrb, rcp);
        float hh[1] = {(float)pick(acc[2]) * kScale1 + ((float)pick(accr[2]) * kScale1) * zrb[1]};
        stamp(14);
        tanh_x86_n<1>(hh, rcp);
        sbv = zrb[0] * sbv + (1.f - zrb[0]) * hh[0];
        if (gown) sbuf[sl * NB + gu] = sbv;
      }
      stamp(8);
      __builtin_amdgcn_wave_barrier();
      float xv[NB];
      {
        const float4 *b4 = (const float4 *)(sbuf + ms * NB);
#pragma unroll
        for (int j = 0; j < NB / 4; j++) {
          const float4 v = b4[j];
          xv[4 * j] = v.x; xv[4 * j + 1] = v.y; xv[4 * j + 2] = v.z; xv[4 * j + 3] = v.w;
        }
      }
      stamp(9);
      const WalkOut R = dual_fc_walk<TRACE>(F, t03, t47, xv, pred, lsr, lpr, n < A.preload ? pcmbuf + ms * FRAME + n : nullptr,
                                            deemph);
      stamp(11);
      if (n + 1 < A.N) {
        if (hl == 0) *(int4 *)(ix + ms * 4) = make_int4(R.su, R.pu, R.exc, 0);
        flag_publish(sync + MFP_SYNC_IX + g, n + 2);
      }
      if (TRACE && hl < 8 && my_active) {
        float v = R.lg[0];
#pragma unroll
        for (int b = 1; b < 8; b++) v = hl == b ? R.lg[b] : v;
        A.trace_logits[((size_t)(s0 + ms) * A.N + n) * 8 + hl] = v;
      }
      if (A.trace_exc && hl == 0 && my_active) A.trace_exc[(size_t)(s0 + ms) * A.N + n] = R.exc;
      pend_pcm = R.pcm;
      pend_pred = R.pn;
      pend_exc = R.exc;
      pend_n = n;
      stamp(12);
    }
    finish();
    stamp(4);
    __syncthreads(); /* final */
    stamp(5);
    if (my_active && hl == 0) {
      StreamState *p = &A.st[s0 + ms];
#pragma unroll
      for (int j = 0; j < NLPC; j++) p->last_sig[j] = lsr[j];
      p->deemph_mem = deemph;
      p->last_exc = last_exc;
      p->rng[0] = rz; p->rng[1] = rw; p->rng[2] = rj; p->rng[3] = rc;
    }
    if (gact) A.st[s0 + sl].gru_b_state[gu] = sbv;
  }
  if (stamping && lane == 0) {
    stp[6] = __builtin_amdgcn_s_memtime() - t_loop0;
    stp[7] = (unsigned long long)A.N;
    stp[15] = (unsigned long long)__hip_atomic_load(abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (int k = 0; k < 16; k++) A.stamps[((size_t)blockIdx.x * STAMP_WAVES + wv) * 16 + k] = stp[k];
  }
  for (int e = tid; e < S * A.N; e += MF_THREADS) {
    const int s = e / A.N, n = e % A.N;
    if (s0 + s < A.nstreams) A.pcm[(size_t)(s0 + s) * A.N + n] = active[s] ? pcmbuf[s * FRAME + n] : (short)0;
  }
}

template <bool TRACE>
static int launch_mfp_t(const SampleArgs &a, hipStream_t stream)
{
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void *)mfp_kernel<TRACE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
        hipSuccess)
      return -1;
    attr_set = true;
  }
  const int grid = (a.nstreams + MFP_S - 1) / MFP_S;
  hipLaunchKernelGGL((mfp_kernel<TRACE>), dim3(grid), dim3(MF_THREADS), mfp_lds_bytes(), stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_mfp(const SampleArgs &a, void *stream)
{
  hipStream_t st = (hipStream_t)stream;
  return a.trace_logits ? launch_mfp_t<true>(a, st) : launch_mfp_t<false>(a, st);
}

}  // namespace lpcnet_mi355x
