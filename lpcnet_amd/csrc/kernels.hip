/*
 * kernels.hip -- CDNA4 (gfx950) kernels of the LPCNet synthesis engine.
 *
 * Numerics contract: every float operation reproduces
 * the reference x86 AVX2 build bit for bit.  This file MUST be compiled with
 * -ffp-contract=off; explicit __builtin_fmaf appears exactly where the
 * reference issues _mm256_fmadd_ps, and _mm256_rcp_ps is emulated through the
 * 2048-entry table (rcp_x86 below).
 *
 * Kernels (frame_kernel.hip: the frame network; mf_kernel.hip: the
 * matrix-core sample kernel)
 *   sample_kernel -- lpcnet_synthesize_tail_impl (lpcnet.c:235-271) for one
 *                    frame: S streams per 384-thread workgroup, persistent over
 *                    the N samples.  Thread i owns GRU_A unit i (its z, r and h
 *                    rows) for all S streams; wave w owns GRU_B row block w;
 *                    wave s runs stream s's GRU_B update, dual-FC tree sampling
 *                    and the LPC/de-emphasis output.  GRU_A/GRU_B int8 blocks,
 *                    dual_fc weights and all tables live in LDS for the whole
 *                    frame; three workgroup barriers per sample.
 */
#include <hip/hip_runtime.h>

#include "device_math.h"
#include "lpcnet_engine.h"
#include "sampler.h"

namespace lpcnet_mi355x {

/* ------------------------------------------------------------------------ */
/* sample network                                                            */

/* LDS areas after the image (byte sizes for S streams). */
template <int S, int V>
struct SampleLds {
  static constexpr int xa = V == 0 ? 2 * (NA / 4) * S * 4 : 2 * (NA / 4) * S * 16; /* double-buffered GRU_A input */
  static constexpr int xb = V == 0 ? (NB / 4) * S * 4 : 0;                          /* quantized GRU_B state */
  static constexpr int sb = S * NB * 4;                                             /* float GRU_B state */
  static constexpr int zr = S * 2 * GB_ROWS * 4;                                    /* GRU_B gate sums, input|recurrent */
  static constexpr int cb = S * GB_ROWS * 4;                                        /* GRU_B conditioning */
  static constexpr int ix = S * 4 * 4;                                              /* sig/pred/exc indices */
  static constexpr int pcm = S * FRAME * 2;
  static constexpr int total = xa + xb + sb + zr + cb + ix + ((pcm + 15) / 16) * 16;
};

int sample_lds_bytes(int S, int variant, int image_bytes)
{
  int extra = 0;
#define CASE(s, v) if (S == s && variant == v) extra = SampleLds<s, v>::total;
  CASE(1, 0) CASE(2, 0) CASE(4, 0) CASE(1, 1) CASE(2, 1) CASE(4, 1)
#undef CASE
  return image_bytes + extra;
}

/* x quads of the S streams for one column block: S dot4 accumulations */
template <int S, bool SAT>
__device__ __forceinline__ void dot_streams(const unsigned char *xa, int off, uint32_t w, int *acc)
{
  if constexpr (S == 4) {
    uint4 xv = *(const uint4 *)(xa + off);
    acc[0] = dot4<SAT>(w, xv.x, acc[0]);
    acc[1] = dot4<SAT>(w, xv.y, acc[1]);
    acc[2] = dot4<SAT>(w, xv.z, acc[2]);
    acc[3] = dot4<SAT>(w, xv.w, acc[3]);
  } else if constexpr (S == 2) {
    uint2 xv = *(const uint2 *)(xa + off);
    acc[0] = dot4<SAT>(w, xv.x, acc[0]);
    acc[1] = dot4<SAT>(w, xv.y, acc[1]);
  } else {
    acc[0] = dot4<SAT>(w, *(const uint32_t *)(xa + off), acc[0]);
  }
}

/* x quad type for S streams of one column block */
template <int S> struct XQ { using T = uint32_t; };
template <> struct XQ<2> { using T = uint2; };
template <> struct XQ<4> { using T = uint4; };

template <int S, bool SAT>
__device__ __forceinline__ void dot_x(const typename XQ<S>::T &x, uint32_t w, int *acc)
{
  if constexpr (S == 4) {
    acc[0] = dot4<SAT>(w, x.x, acc[0]);
    acc[1] = dot4<SAT>(w, x.y, acc[1]);
    acc[2] = dot4<SAT>(w, x.z, acc[2]);
    acc[3] = dot4<SAT>(w, x.w, acc[3]);
  } else if constexpr (S == 2) {
    acc[0] = dot4<SAT>(w, x.x, acc[0]);
    acc[1] = dot4<SAT>(w, x.y, acc[1]);
  } else {
    acc[0] = dot4<SAT>(w, x, acc[0]);
  }
}

/* Quad-path gate: K4 groups of 4 slots.  Group g of this lane: its four
 * weight quads are one uint4 (wq[qoff + g*64 + lane]) and the four column
 * blocks one u32 shared by the 8 lanes of a row block (cq[coff + g*8 + rb]),
 * so the dependent LDS round trip (index -> x) is paid once per 4 slots. */
template <int S, bool SAT>
__device__ __forceinline__ void gate_quad(const unsigned char *xa, const uint4 *wq, const uint32_t *cq, int qoff,
                                          int coff, int K4, int lane, int *acc)
{
  using X = typename XQ<S>::T;
  const uint4 *wp = wq + qoff + lane;
  const uint32_t *cp = cq + coff + (lane >> 3);
#pragma unroll 2
  for (int g = 0; g < K4; g++) {
    const uint4 w = wp[g * 64];
    const uint32_t c = cp[g * 8];
    const X x0 = *(const X *)(xa + (c & 0xFF) * (S * 4));
    const X x1 = *(const X *)(xa + ((c >> 8) & 0xFF) * (S * 4));
    const X x2 = *(const X *)(xa + ((c >> 16) & 0xFF) * (S * 4));
    const X x3 = *(const X *)(xa + (c >> 24) * (S * 4));
    dot_x<S, SAT>(x0, w.x, acc);
    dot_x<S, SAT>(x1, w.y, acc);
    dot_x<S, SAT>(x2, w.z, acc);
    dot_x<S, SAT>(x3, w.w, acc);
  }
}

/* Sum over the 8 lanes {l ^ 8k} (xor 8, 16, 32) without LDS: DPP row_ror:8
 * inside each 16-lane row, then the gfx950 row-swap permutes.  Integer sums,
 * so the order is immaterial. */
__device__ __forceinline__ int sum_lanes_xor8_16_32(int x)
{
  x += __builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false);
  const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  x = (int)p[0] + (int)p[1];
  const auto q = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return (int)q[0] + (int)q[1];
}

/* The z, r and h quad groups of one wave as one software-pipelined stream
 * (they are contiguous in the image): the column word is loaded two groups
 * ahead and the x gathers one group ahead, so neither dependent LDS round
 * trip (column word -> x address -> x) sits on the chain of a group; the
 * dot4s of group g run while the gathers of g+1 are in flight.  Prefetches
 * past the end re-read the last group. */
template <int S, bool SAT>
__device__ __forceinline__ void gru_a_stream(const unsigned char *xa, const uint4 *wq, const uint32_t *cq, int qoff,
                                             int coff, int Kz, int Kr, int Kh, int lane, int *az, int *ar, int *ah)
{
  using X = typename XQ<S>::T;
  const int G = Kz + Kr + Kh;
  if (G == 0) return;
  const uint4 *wp = wq + qoff + lane;
  const uint32_t *cp = cq + coff + (lane >> 3);
  auto xat = [&](uint32_t c, int b) -> X { return *(const X *)(xa + ((c >> (8 * b)) & 0xFF) * (S * 4)); };
  const uint32_t c0 = cp[0];
  uint32_t c1 = cp[min(1, G - 1) * 8];
  uint4 w = wp[0];
  X x0 = xat(c0, 0), x1 = xat(c0, 1), x2 = xat(c0, 2), x3 = xat(c0, 3);
  int g = 0;
  auto step = [&](int *acc) {
    const int g1 = min(g + 1, G - 1), g2 = min(g + 2, G - 1);
    const uint32_t c2 = cp[g2 * 8];
    const uint4 wn = wp[g1 * 64];
    const X y0 = xat(c1, 0), y1 = xat(c1, 1), y2 = xat(c1, 2), y3 = xat(c1, 3);
    dot_x<S, SAT>(x0, w.x, acc);
    dot_x<S, SAT>(x1, w.y, acc);
    dot_x<S, SAT>(x2, w.z, acc);
    dot_x<S, SAT>(x3, w.w, acc);
    x0 = y0; x1 = y1; x2 = y2; x3 = y3;
    w = wn;
    c1 = c2;
    g++;
  };
  while (g < Kz) step(az);
  while (g < Kz + Kr) step(ar);
  while (g < G) step(ah);
}

template <int S, int V, bool SAT, bool REG>
__global__ __launch_bounds__(SAMPLE_THREADS) void sample_kernel(SampleArgs A)
{
  extern __shared__ uint4 lds4[];
  unsigned char *lds = (unsigned char *)lds4;
  using L = SampleLds<S, V>;
  unsigned char *xa_base = lds + A.image_bytes;
  unsigned char *xb = xa_base + L::xa;
  float *sbuf = (float *)(xb + L::xb);
  float *zr = sbuf + S * NB;
  float *condb = zr + S * 2 * GB_ROWS;
  int *ix = (int *)(condb + S * GB_ROWS);
  short *pcmbuf = (short *)(ix + S * 4);

  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6); /* wave-uniform */
  const int s0 = blockIdx.x * S;
  const uint32_t *rcp = (const uint32_t *)(lds + IMG_RCP);
  const float *ulaw = (const float *)(lds + IMG_ULAW);
  const float *logit_tab = (const float *)(lds + IMG_LOGIT);
  const float *fcw = (const float *)(lds + IMG_FCW);
  const float *fcb = (const float *)(lds + IMG_FCB);
  const float *fcf = (const float *)(lds + IMG_FCF);

  /* Which streams of this group synthesise this frame (lpcnet.c:239-243). */
  bool active[S];
  bool any = false;
  for (int s = 0; s < S; s++) {
    int sid = s0 + s;
    active[s] = sid < A.nstreams && A.st[sid].frame_count > FEATURES_DELAY;
    any |= active[s];
  }
  if (!any) {
    for (int e = tid; e < S * A.N; e += SAMPLE_THREADS) {
      int s = e / A.N, n = e % A.N;
      if (s0 + s < A.nstreams) A.pcm[(size_t)(s0 + s) * A.N + n] = 0;
    }
    return;
  }

  /* weights and tables -> LDS */
  for (int o = tid; o < A.image_bytes / 16; o += SAMPLE_THREADS) lds4[o] = A.image[o];

  const int K4z = REG ? A.ga_K4[wv][0] : 0, K4r = REG ? A.ga_K4[wv][1] : 0, K4h = REG ? A.ga_K4[wv][2] : 0;
  const uint4 *wq = (const uint4 *)lds;
  const uint32_t *cq = (const uint32_t *)lds;

  /* GRU_A unit state and constants: thread tid owns unit i = tid */
  const int i = tid;
  const float bz = A.ga_par[i], br = A.ga_par[NA + i], bh = A.ga_par[2 * NA + i];
  const float dz = A.ga_par[3 * NA + i], dr = A.ga_par[4 * NA + i], dh = A.ga_par[5 * NA + i];
  const int wsz = A.ga_wsum[i], wsr = A.ga_wsum[NA + i], wsh = A.ga_wsum[2 * NA + i];
  float st[S], cz[S], cr[S], ch[S];
  for (int s = 0; s < S; s++) {
    const StreamState *p = &A.st[min(s0 + s, A.nstreams - 1)];
    st[s] = p->gru_a_state[i];
    cz[s] = p->gru_a_cond[i];
    cr[s] = p->gru_a_cond[NA + i];
    ch[s] = p->gru_a_cond[2 * NA + i];
  }
  /* stream-serial state: wave s owns stream s (lanes 0..15 hold last_sig/lpc/GRU_B units) */
  /* last_sig / lpc are held as uniform register arrays by every lane of the
   * stream's wave, so the sequential pred chain needs no cross-lane traffic */
  float lsr[NLPC], lpr[NLPC];
  float sbv = 0.f, pred = 0.f, deemph = 0.f;
  uint32_t rz = 0, rw = 0, rj = 0, rc = 0, r0 = 0, r1 = 0;
  int last_exc = 0;
  const int my_s = wv;
  const bool stream_wave = my_s < S;
#pragma unroll
  for (int j = 0; j < NLPC; j++) { lsr[j] = 0.f; lpr[j] = 0.f; }
  if (stream_wave) {
    const StreamState *p = &A.st[min(s0 + my_s, A.nstreams - 1)];
#pragma unroll
    for (int j = 0; j < NLPC; j++) {
      lsr[j] = p->last_sig[j];
      lpr[j] = p->lpc[j];
    }
    sbv = p->gru_b_state[lane & (NB - 1)];
    for (int k = lane; k < GB_ROWS; k += 64) condb[my_s * GB_ROWS + k] = p->gru_b_cond[k];
    deemph = p->deemph_mem;
    last_exc = p->last_exc;
    rz = p->rng[0]; rw = p->rng[1]; rj = p->rng[2]; rc = p->rng[3];
  }
  __syncthreads(); /* image in LDS */

  /* initial quantized inputs: GRU_A state (buffer 0) and GRU_B state */
  if constexpr (V == 0) {
    for (int s = 0; s < S; s++) xa_base[(i >> 2) * S * 4 + s * 4 + (i & 3)] = (unsigned char)quant_s8(st[s]);
    if (stream_wave && lane < NB) {
      xb[(lane >> 2) * S * 4 + my_s * 4 + (lane & 3)] = (unsigned char)quant_s8(sbv);
      sbuf[my_s * NB + lane] = sbv;
    }
  } else {
    float *xf = (float *)xa_base;
    for (int s = 0; s < S; s++) xf[((i >> 2) * S + s) * 4 + (i & 3)] = st[s];
    if (stream_wave && lane < NB) sbuf[my_s * NB + lane] = sbv;
  }

  /* per-stream step between samples: pred and the u-law indices (lpcnet.c:252-254) */
  auto pre_sample = [&]() {
    /* pred = -sum last_sig[j]*lpc[j], sequential (lpcnet.c:252) */
    float p2 = 0.f;
#pragma unroll
    for (int j = 0; j < NLPC; j++) p2 = p2 - lsr[j] * lpr[j];
    pred = p2;
    const int su = lin2ulaw_x86(lsr[0]);
    const int pu = lin2ulaw_x86(pred);
    if (lane == 0) {
      ix[my_s * 4 + 0] = su;
      ix[my_s * 4 + 1] = pu;
      ix[my_s * 4 + 2] = last_exc;
    }
  };
  for (int e = tid; e < S * A.preload; e += SAMPLE_THREADS) {
    const int s = e / A.preload, n = e % A.preload;
    pcmbuf[s * FRAME + n] = A.pcm[(size_t)min(s0 + s, A.nstreams - 1) * A.N + n];
  }
  if (stream_wave) pre_sample();
  __syncthreads();

  const uint32_t *lds32 = (const uint32_t *)lds;
  const uint16_t *lds16 = (const uint16_t *)lds;
  const int j8 = lane >> 3;
  /* dual_fc nodes 1..15 (tree levels 0..3) never change lane: node qq+1,
   * channel lane&1 -> weights, bias and factor held in registers */
  float f03w[NB], f03b = 0.f, f03f = 0.f;
  {
    const int q0 = lane >> 1, node = (q0 < 15 ? q0 : 0) + 1, c2 = lane & 1;
#pragma unroll
    for (int j = 0; j < NB; j++) f03w[j] = stream_wave ? fcw[node * 32 + c2 * 16 + j] : 0.f;
    if (stream_wave) {
      f03b = fcb[c2 * 256 + node];
      f03f = fcf[c2 * 256 + node];
    }
  }
  /* frame-constant GRU_B accumulator seeds of this lane's row (nnet.c:347-356) */
  int gb_seed[S], gb_seedr = 0;
  if constexpr (V == 0) {
    const int row = wv * 8 + (lane & 7);
    for (int s = 0; s < S; s++)
      gb_seed[s] = cvt_rne((A.gb_par[row] + condb[s * GB_ROWS + row]) * kScale) + (SAT ? 0 : A.gb_wsum[row]);
    gb_seedr = cvt_rne(A.gb_par[GB_ROWS + row] * kScale) + (SAT ? 0 : A.gb_wsum[GB_ROWS + row]);
  }

  /* optional phase timing (diagnostics only): per wave, s_memtime sums of
   * [0] phase B work [1] barrier 1 wait [2] phase C [3] barrier 2 wait
   * [4] phase F [5] barrier 3 wait [6] total loop [7] samples */
  const bool stamping = A.stamps != nullptr;
  unsigned long long stp[16] = {};
  unsigned long long t_prev = stamping ? __builtin_amdgcn_s_memtime() : 0, t_loop0 = t_prev;
  auto stamp = [&](int k) {
    if (stamping) {
      unsigned long long t = __builtin_amdgcn_s_memtime();
      stp[k] += t - t_prev;
      t_prev = t;
    }
  };

  for (int n = 0; n < A.N; n++) {
    const int cur = n & 1;
    /* ---- phase B: GRU_A (nnet.c:484-491 + 410-448) ---------------------- */
    {
      /* the two kiss99 draws of this sample (sample_mdense, nnet.c:178-184) */
      if (stream_wave) {
        r0 = kiss99_next(rz, rw, rj, rc);
        r1 = kiss99_next(rz, rw, rj, rc);
      }
      /* embedding gathers issued first; consumed after the recurrent matvec */
      float e1z[S], e1r[S], e1h[S], e2z[S], e2r[S], e2h[S], e3z[S], e3r[S], e3h[S];
      for (int s = 0; s < S; s++) {
        const int sig = __builtin_amdgcn_readfirstlane(ix[s * 4 + 0]) & 0xFF;
        const int prd = __builtin_amdgcn_readfirstlane(ix[s * 4 + 1]) & 0xFF;
        const int exc = __builtin_amdgcn_readfirstlane(ix[s * 4 + 2]) & 0xFF;
        const float *e1 = A.emb_sig + sig * GA_ROWS, *e2 = A.emb_pred + prd * GA_ROWS, *e3 = A.emb_exc + exc * GA_ROWS;
        e1z[s] = e1[i]; e1r[s] = e1[NA + i]; e1h[s] = e1[2 * NA + i];
        e2z[s] = e2[i]; e2r[s] = e2[NA + i]; e2h[s] = e2[2 * NA + i];
        e3z[s] = e3[i]; e3r[s] = e3[NA + i]; e3h[s] = e3[2 * NA + i];
      }
      float gz[S], gr[S], gh[S], inh[S];
      if constexpr (V == 0) {
        /* integer part first: the seed (which needs the gathers) is added after,
         * int32 addition being associative */
        int az[S], ar[S], ah[S];
        for (int s = 0; s < S; s++) {
          az[s] = SAT ? 0 : wsz;
          ar[s] = SAT ? 0 : wsr;
          ah[s] = SAT ? 0 : wsh;
        }
        const unsigned char *xa = xa_base + cur * (NA / 4) * S * 4;
        if constexpr (REG) {
          gru_a_stream<S, SAT>(xa, wq, cq, A.ga_qoff[wv][0], A.ga_coff[wv][0], K4z, K4r, K4h, lane, az, ar, ah);
        } else {
          auto run_gate = [&](int g, int *acc) {
            const uint32_t *wp = lds32 + A.ga_woff[wv][g] + lane;
            const uint16_t *cp = lds16 + A.ga_coff[wv][g] + j8;
            const int K = A.ga_K[wv][g];
#pragma unroll 4
            for (int k = 0; k < K; k++) dot_streams<S, SAT>(xa, cp[k * 8] * (S * 4), wp[k * 64], acc);
          };
          run_gate(0, az);
          run_gate(1, ar);
          run_gate(2, ah);
        }
        for (int s = 0; s < S; s++) {
          const float inz = ((cz[s] + e1z[s]) + e2z[s]) + e3z[s];
          const float inr = ((cr[s] + e1r[s]) + e2r[s]) + e3r[s];
          inh[s] = ((ch[s] + e1h[s]) + e2h[s]) + e3h[s];
          gz[s] = (float)(az[s] + cvt_rne(((bz + dz * st[s]) + inz) * kScale)) * kScale1;
          gr[s] = (float)(ar[s] + cvt_rne(((br + dr * st[s]) + inr) * kScale)) * kScale1;
          gh[s] = (float)(ah[s] + cvt_rne((bh + dh * st[s]) * kScale)) * kScale1;
        }
      } else {
        for (int s = 0; s < S; s++) {
          const float inz = ((cz[s] + e1z[s]) + e2z[s]) + e3z[s];
          const float inr = ((cr[s] + e1r[s]) + e2r[s]) + e3r[s];
          inh[s] = ((ch[s] + e1h[s]) + e2h[s]) + e3h[s];
          gz[s] = (bz + dz * st[s]) + inz;
          gr[s] = (br + dr * st[s]) + inr;
          gh[s] = bh + dh * st[s];
        }
        const float4 *xf = (const float4 *)(xa_base + cur * (NA / 4) * S * 16);
        auto run_gate_f = [&](int g, float *y) {
          const float4 *wp = A.ga_wf + A.ga_woff[wv][g] + lane;
          const uint16_t *cp = lds16 + A.ga_coff[wv][g] + j8;
          const int K = A.ga_K[wv][g];
          for (int k = 0; k < K; k++) {
            int c = cp[k * 8];
            float4 w = wp[k * 64];
            if (c != 0xFFFF) {
              for (int s = 0; s < S; s++) {
                float4 x = xf[c * S + s];
                y[s] = __builtin_fmaf(w.x, x.x, y[s]);
                y[s] = __builtin_fmaf(w.y, x.y, y[s]);
                y[s] = __builtin_fmaf(w.z, x.z, y[s]);
                y[s] = __builtin_fmaf(w.w, x.w, y[s]);
              }
            }
          }
        };
        run_gate_f(0, gz);
        run_gate_f(1, gr);
        run_gate_f(2, gh);
      }
      const int nxt = cur ^ 1;
      for (int s = 0; s < S; s++) {
        float z = sigmoid_x86(gz[s], rcp);
        float r = sigmoid_x86(gr[s], rcp);
        float h = gh[s] * r + inh[s];
        h = tanh_x86(h, rcp);
        st[s] = z * st[s] + (1.f - z) * h;
        if constexpr (V == 0)
          xa_base[nxt * (NA / 4) * S * 4 + (i >> 2) * S * 4 + s * 4 + (i & 3)] = (unsigned char)quant_s8(st[s]);
        else
          ((float *)(xa_base + nxt * (NA / 4) * S * 16))[((i >> 2) * S + s) * 4 + (i & 3)] = st[s];
      }
    }
    stamp(0);
    __syncthreads();
    stamp(1);

    /* ---- phase C: GRU_B gate sums, wave w = row block w (nnet.c:345-361) --- */
    {
      const int nxt = cur ^ 1;
      const int rb = wv, r = lane & 7, ks = lane >> 3, row = rb * 8 + r;
      if constexpr (V == 0) {
        const unsigned char *xa = xa_base + nxt * (NA / 4) * S * 4;
        int acc[S], accr[S];
        for (int s = 0; s < S; s++) { acc[s] = 0; accr[s] = 0; }
        if constexpr (REG) {
          gru_a_stream<S, SAT>(xa, wq, cq, A.gb_qoff[rb], A.gb_coff[rb], REG_GB / 4, 0, 0, lane, acc, acc, acc);
        } else {
          const uint32_t *wp = lds32 + A.gb_woff[rb];
          const uint16_t *cp = lds16 + A.gb_coff[rb];
          const int nb = A.gb_nb[rb];
#pragma unroll 4
          for (int k = ks; k < nb; k += 8) dot_streams<S, SAT>(xa, cp[k] * (S * 4), wp[k * 8 + r], acc);
        }
        if (ks < NB / 4) {
          uint32_t w = ((const uint32_t *)(lds + A.gb_rec_off))[(rb * (NB / 4) + ks) * 8 + r];
          dot_streams<S, SAT>(xb, ks * S * 4, w, accr);
        }
        for (int s = 0; s < S; s++) {
          acc[s] = sum_lanes_xor8_16_32(acc[s]);
          accr[s] = sum_lanes_xor8_16_32(accr[s]);
        }
        if (ks == 0) {
          for (int s = 0; s < S; s++) {
            zr[s * 2 * GB_ROWS + row] = (float)(gb_seed[s] + acc[s]) * kScale1;
            zr[s * 2 * GB_ROWS + GB_ROWS + row] = (float)(gb_seedr + accr[s]) * kScale1;
          }
        }
      } else {
        /* fp32: one sequential FMA chain per (row, stream) in block order */
        const int s = lane >> 3;
        if (s < S) {
          const float4 *xf = (const float4 *)(xa_base + nxt * (NA / 4) * S * 16);
          const float4 *wp = (const float4 *)(lds + A.gb_woff[rb] * 4);
          const uint16_t *cp = lds16 + A.gb_coff[rb];
          const int nb = A.gb_nb[rb];
          float y = A.gb_par[row] + condb[s * GB_ROWS + row];
          for (int k = 0; k < nb; k++) {
            float4 w = wp[k * 8 + r];
            float4 x = xf[cp[k] * S + s];
            y = __builtin_fmaf(w.x, x.x, y);
            y = __builtin_fmaf(w.y, x.y, y);
            y = __builtin_fmaf(w.z, x.z, y);
            y = __builtin_fmaf(w.w, x.w, y);
          }
          float y2 = A.gb_par[GB_ROWS + row];
          for (int j = 0; j < NB; j++) y2 = __builtin_fmaf(A.gb_recf[j * GB_ROWS + row], sbuf[s * NB + j], y2);
          zr[s * 2 * GB_ROWS + row] = y;
          zr[s * 2 * GB_ROWS + GB_ROWS + row] = y2;
        }
      }
    }
    stamp(2);
    __syncthreads();
    stamp(3);

    /* ---- phase F: per-stream GRU_B update, dual-FC sampling, output -------- */
    if (stream_wave) {
      const int s = my_s;
      const float *zs = zr + s * 2 * GB_ROWS;
      /* GRU_B elementwise (nnet.c:362-371): every lane computes unit lane%16
       * (lanes >= 16 duplicate), so no exec masking on the serial path */
      {
        const int u = lane & (NB - 1);
        float z = sigmoid_x86(zs[u] + zs[GB_ROWS + u], rcp);
        float r = sigmoid_x86(zs[NB + u] + zs[GB_ROWS + NB + u], rcp);
        float h = zs[2 * NB + u] + zs[GB_ROWS + 2 * NB + u] * r;
        h = tanh_x86(h, rcp);
        sbv = z * sbv + (1.f - z) * h;
        if (lane < NB) sbuf[s * NB + lane] = sbv;
      }
      stamp(8);
      /* same-wave LDS exchange: the reads below follow the writes in this
       * wave's LDS queue */
      __builtin_amdgcn_wave_barrier();
      float xv[NB];
      {
        const float4 *sb4 = (const float4 *)(sbuf + s * NB);
#pragma unroll
        for (int j = 0; j < NB / 4; j++) {
          const float4 v = sb4[j];
          xv[4 * j] = v.x; xv[4 * j + 1] = v.y; xv[4 * j + 2] = v.z; xv[4 * j + 3] = v.w;
        }
      }
      /* dual_fc tree sampling (nnet.c:163-214): lane 2q+c computes channel c
       * of one node; each even lane compares its node's logit with its
       * level's threshold and the walk runs on the ballot mask in scalar ops */
      float thr[8];
#pragma unroll
      for (int b = 0; b < 4; b++) {
        thr[b] = logit_tab[(r0 >> (8 * b)) & 0xFF];
        thr[b + 4] = logit_tab[(r1 >> (8 * b)) & 0xFF];
      }
      stamp(9);
      const int q = lane >> 1, ch2 = lane & 1;
      const int qq = q < 15 ? q : 0;
      const int lvl_in = qq == 0 ? 0 : (qq < 3 ? 1 : (qq < 7 ? 2 : 3)); /* level of node qq+1 within 0..3 */
      auto node_logit_w = [&](float bias, float factor, const float *w) -> float {
        float sum = bias;
#pragma unroll
        for (int j = 0; j < NB; j++) sum = sum + w[j] * xv[j];
        const float v = factor * tanh_x86(sum, rcp);
        /* sum1 + sum2 (nnet.c:205); adjacent-lane swap through DPP quad_perm [1,0,3,2] */
        const float o = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
        return ch2 ? o + v : v + o;
      };
      auto node_logit = [&](int node) -> float {
        return node_logit_w(fcb[ch2 * 256 + node], fcf[ch2 * 256 + node], fcw + node * 32 + ch2 * 16);
      };
      const bool tracing = A.trace_logits != nullptr;
      float lg[8];
      int val = 0;
      {
        const float l = node_logit_w(f03b, f03f, f03w); /* levels 0..3: nodes 1..15, weights in registers */
        const float t = lvl_in == 0 ? thr[0] : (lvl_in == 1 ? thr[1] : (lvl_in == 2 ? thr[2] : thr[3]));
        const unsigned long long m = __ballot(t < l);
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int nd = (1 << b) | val;
          if (tracing) lg[b] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(l), 2 * (nd - 1)));
          val = (val << 1) | (int)((m >> (2 * (nd - 1))) & 1ull);
        }
      }
      stamp(10);
      {
        /* levels 4..7 under the chosen 4-bit prefix: 1 + 2 + 4 + 8 nodes */
        const int lvl = 4 + lvl_in;
        const int off = qq + 1 - (1 << (lvl - 4));
        const float l = node_logit((1 << lvl) | (val << (lvl - 4)) | off);
        const float t = lvl_in == 0 ? thr[4] : (lvl_in == 1 ? thr[5] : (lvl_in == 2 ? thr[6] : thr[7]));
        const unsigned long long m = __ballot(t < l);
#pragma unroll
        for (int b = 4; b < 8; b++) {
          const int qi = (1 << (b - 4)) - 1 + (val & ((1 << (b - 4)) - 1));
          if (tracing) lg[b] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(l), 2 * qi));
          val = (val << 1) | (int)((m >> (2 * qi)) & 1ull);
        }
      }
      stamp(11);
      int exc = val;
      /* output sample (lpcnet.c:256-269) */
      float pcm;
      if (n < A.preload) {
        /* teacher forcing: the caller's PCM replaces the sampled excitation */
        const float o_in = (float)pcmbuf[s * FRAME + n];
        const float pd = kPreemph * deemph;
        exc = lin2ulaw_x86((o_in - pd) - pred);
        pcm = o_in - pd;
      } else {
        pcm = pred + ulaw[exc];
      }
#pragma unroll
      for (int j = NLPC - 1; j > 0; j--) lsr[j] = lsr[j - 1];
      lsr[0] = pcm;
      last_exc = exc;
      float o = pcm + kPreemph * deemph;
      deemph = o;
      if (o < -32767) o = -32767;
      if (o > 32767) o = 32767;
      if (lane == 0 && n >= A.preload) pcmbuf[s * FRAME + n] = (short)round_half_up(o);
      if (tracing && lane < 8 && active[s]) {
        float v = lg[0];
#pragma unroll
        for (int b = 1; b < 8; b++) v = lane == b ? lg[b] : v;
        A.trace_logits[((size_t)(s0 + s) * A.N + n) * 8 + lane] = v;
      }
      if (A.trace_exc && lane == 0 && active[s]) A.trace_exc[(size_t)(s0 + s) * A.N + n] = exc;
      if constexpr (V == 0) {
        if (lane < NB) xb[(lane >> 2) * S * 4 + s * 4 + (lane & 3)] = (unsigned char)quant_s8(sbv);
      }
      stamp(12);
      if (n + 1 < A.N) pre_sample();
    }
    stamp(4);
    __syncthreads();
    stamp(5);
  }
  if (stamping && lane == 0) {
    stp[6] = __builtin_amdgcn_s_memtime() - t_loop0;
    stp[7] = (unsigned long long)A.N;
    for (int k = 0; k < 16; k++) A.stamps[((size_t)blockIdx.x * STAMP_WAVES + wv) * 16 + k] = stp[k];
  }

  /* ---- write back (only streams that synthesised this frame) ------------- */
  for (int s = 0; s < S; s++)
    if (active[s]) A.st[s0 + s].gru_a_state[i] = st[s];
  if (stream_wave && active[my_s]) {
    StreamState *p = &A.st[s0 + my_s];
    if (lane < NB) p->gru_b_state[lane] = sbv;
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < NLPC; j++) p->last_sig[j] = lsr[j];
    }
    if (lane == 0) {
      p->deemph_mem = deemph;
      p->last_exc = last_exc;
      p->rng[0] = rz; p->rng[1] = rw; p->rng[2] = rj; p->rng[3] = rc;
    }
  }
  for (int e = tid; e < S * A.N; e += SAMPLE_THREADS) {
    int s = e / A.N, n = e % A.N;
    if (s0 + s < A.nstreams) A.pcm[(size_t)(s0 + s) * A.N + n] = active[s] ? pcmbuf[s * FRAME + n] : (short)0;
  }
}

/* ------------------------------------------------------------------------ */
/* wave-per-stream sample network (large batches)                            */
/*
 * One wavefront runs one stream through all N samples with no workgroup
 * barrier after the image load: the NW waves of a workgroup share the LDS
 * weight image (same quad layout as sample_kernel) and overlap each other's
 * latency.  Lane l owns GRU_A units l + 64j (j = 0..5): pass j is exactly
 * chunk j of the quad image.  GRU_B: pass rb = row block rb, lane (row l%8,
 * k-slice l/8) with three quad groups, reduced across k-slices by shuffles.
 */
constexpr int WV_X = NA;              /* quantized GRU_A state, [96 column blocks] u32 */
constexpr int WV_XB = NB;             /* quantized GRU_B state */
constexpr int WV_ZR = 2 * GB_ROWS * 4;
constexpr int WV_SB = NB * 4;
constexpr int WV_PCM = FRAME * 2;
constexpr int WV_STRIDE = ((WV_X + WV_XB + WV_ZR + WV_SB + WV_PCM) + 15) / 16 * 16;

int wave_lds_bytes(int nw, int image_bytes) { return image_bytes + nw * WV_STRIDE; }

template <int NW, bool SAT>
__global__ __launch_bounds__(NW * 64) void wave_kernel(SampleArgs A)
{
  extern __shared__ uint4 lds4[];
  unsigned char *lds = (unsigned char *)lds4;
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6); /* wave-uniform */
  const int sid = blockIdx.x * NW + wv;
  const bool valid = sid < A.nstreams;
  const bool active = valid && A.st[sid].frame_count > FEATURES_DELAY;

  for (int o = tid; o < A.image_bytes / 16; o += NW * 64) lds4[o] = A.image[o];
  __syncthreads(); /* the only workgroup barrier */

  unsigned char *wbase = lds + A.image_bytes + wv * WV_STRIDE;
  unsigned char *xa = wbase;                 /* byte u = quantized unit u (XOR 0x80) */
  unsigned char *xb = wbase + WV_X;
  float *zr = (float *)(xb + WV_XB);
  float *sbuf = zr + 2 * GB_ROWS;
  short *pcmbuf = (short *)(sbuf + NB);
  if (!active) {
    if (valid)
      for (int n = lane; n < A.N; n += 64) A.pcm[(size_t)sid * A.N + n] = 0;
    return;
  }
  const uint32_t *rcp = (const uint32_t *)(lds + IMG_RCP);
  const float *ulaw = (const float *)(lds + IMG_ULAW);
  const float *logit_tab = (const float *)(lds + IMG_LOGIT);
  const float *fcw = (const float *)(lds + IMG_FCW);
  const float *fcb = (const float *)(lds + IMG_FCB);
  const float *fcf = (const float *)(lds + IMG_FCF);
  const uint4 *wq = (const uint4 *)lds;
  const uint32_t *cq = (const uint32_t *)lds;
  StreamState *P = &A.st[sid];

  /* GRU_A units of this lane */
  float st[6], cz[6], cr[6], ch[6];
#pragma unroll
  for (int j = 0; j < 6; j++) {
    const int u = 64 * j + lane;
    st[j] = P->gru_a_state[u];
    cz[j] = P->gru_a_cond[u];
    cr[j] = P->gru_a_cond[NA + u];
    ch[j] = P->gru_a_cond[2 * NA + u];
    xa[u] = (unsigned char)quant_s8(st[j]);
  }
  /* GRU_B: lane r = lane % 8 seeds rows 8*rb + r */
  const int r8 = lane & 7, ks = lane >> 3;
  float cbr[6];
#pragma unroll
  for (int rb = 0; rb < 6; rb++) cbr[rb] = P->gru_b_cond[rb * 8 + r8];
  float sbv = P->gru_b_state[lane & (NB - 1)];
  if (lane < NB) xb[lane] = (unsigned char)quant_s8(sbv);
  float lsr[NLPC], lpr[NLPC];
#pragma unroll
  for (int j = 0; j < NLPC; j++) {
    lsr[j] = P->last_sig[j];
    lpr[j] = P->lpc[j];
  }
  float deemph = P->deemph_mem;
  int last_exc = P->last_exc;
  uint32_t rz = P->rng[0], rw = P->rng[1], rj = P->rng[2], rc = P->rng[3];
  for (int e = lane; e < A.preload; e += 64) pcmbuf[e] = A.pcm[(size_t)sid * A.N + e];
  const bool tracing = A.trace_logits != nullptr;

  for (int n = 0; n < A.N; n++) {
    /* ---- per-stream scalars: pred, u-law indices, kiss99 draws ---------- */
    float pred = 0.f;
#pragma unroll
    for (int j = 0; j < NLPC; j++) pred = pred - lsr[j] * lpr[j];
    const int sig = lin2ulaw_x86(lsr[0]) & 0xFF, prd = lin2ulaw_x86(pred) & 0xFF, exc_in = last_exc & 0xFF;
    const uint32_t r0 = kiss99_next(rz, rw, rj, rc);
    const uint32_t r1 = kiss99_next(rz, rw, rj, rc);

    /* ---- GRU_A: gathers in flight during the integer matvec ------------- */
    const float *e1 = A.emb_sig + sig * GA_ROWS, *e2 = A.emb_pred + prd * GA_ROWS, *e3 = A.emb_exc + exc_in * GA_ROWS;
    float g1[18], g2[18], g3[18];
#pragma unroll
    for (int j = 0; j < 6; j++)
#pragma unroll
      for (int g = 0; g < 3; g++) {
        const int row = g * NA + 64 * j + lane;
        g1[3 * j + g] = e1[row];
        g2[3 * j + g] = e2[row];
        g3[3 * j + g] = e3[row];
      }
    int acc[18];
#pragma unroll
    for (int j = 0; j < 6; j++)
#pragma unroll
      for (int g = 0; g < 3; g++) {
        int a = SAT ? 0 : A.ga_wsum[g * NA + 64 * j + lane];
        const uint4 *wp = wq + A.ga_qoff[j][g] + lane;
        const uint32_t *cp = cq + A.ga_coff[j][g] + (lane >> 3);
        const int K4 = A.ga_K4[j][g];
        for (int k = 0; k < K4; k++) {
          const uint4 w = wp[k * 64];
          const uint32_t c = cp[k * 8];
          const uint32_t *x32 = (const uint32_t *)xa;
          a = dot4<SAT>(w.x, x32[c & 0xFF], a);
          a = dot4<SAT>(w.y, x32[(c >> 8) & 0xFF], a);
          a = dot4<SAT>(w.z, x32[(c >> 16) & 0xFF], a);
          a = dot4<SAT>(w.w, x32[c >> 24], a);
        }
        acc[3 * j + g] = a;
      }
#pragma unroll
    for (int j = 0; j < 6; j++) {
      const int u = 64 * j + lane;
      const float bz = A.ga_par[u], br = A.ga_par[NA + u], bh = A.ga_par[2 * NA + u];
      const float dz = A.ga_par[3 * NA + u], dr = A.ga_par[4 * NA + u], dh = A.ga_par[5 * NA + u];
      const float inz = ((cz[j] + g1[3 * j]) + g2[3 * j]) + g3[3 * j];
      const float inr = ((cr[j] + g1[3 * j + 1]) + g2[3 * j + 1]) + g3[3 * j + 1];
      const float inh = ((ch[j] + g1[3 * j + 2]) + g2[3 * j + 2]) + g3[3 * j + 2];
      const float gz = (float)(acc[3 * j] + cvt_rne(((bz + dz * st[j]) + inz) * kScale)) * kScale1;
      const float gr = (float)(acc[3 * j + 1] + cvt_rne(((br + dr * st[j]) + inr) * kScale)) * kScale1;
      const float gh = (float)(acc[3 * j + 2] + cvt_rne((bh + dh * st[j]) * kScale)) * kScale1;
      const float z = sigmoid_x86(gz, rcp);
      const float r = sigmoid_x86(gr, rcp);
      float h = gh * r + inh;
      h = tanh_x86(h, rcp);
      st[j] = z * st[j] + (1.f - z) * h;
    }
    /* every read of the old x is done (program order, in-order LDS queue) */
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < 6; j++) xa[64 * j + lane] = (unsigned char)quant_s8(st[j]);
    __builtin_amdgcn_wave_barrier();

    /* ---- GRU_B gate sums (nnet.c:345-361) -------------------------------- */
#pragma unroll
    for (int rb = 0; rb < 6; rb++) {
      int a = 0, ar = 0;
      const uint4 *wp = wq + A.gb_qoff[rb] + lane;
      const uint32_t *cp = cq + A.gb_coff[rb] + ks;
      const uint32_t *x32 = (const uint32_t *)xa;
#pragma unroll
      for (int k = 0; k < REG_GB / 4; k++) {
        const uint4 w = wp[k * 64];
        const uint32_t c = cp[k * 8];
        a = dot4<SAT>(w.x, x32[c & 0xFF], a);
        a = dot4<SAT>(w.y, x32[(c >> 8) & 0xFF], a);
        a = dot4<SAT>(w.z, x32[(c >> 16) & 0xFF], a);
        a = dot4<SAT>(w.w, x32[c >> 24], a);
      }
      if (ks < NB / 4)
        ar = dot4<SAT>(((const uint32_t *)(lds + A.gb_rec_off))[(rb * (NB / 4) + ks) * 8 + r8], ((const uint32_t *)xb)[ks], ar);
      a += __shfl_xor(a, 8);
      a += __shfl_xor(a, 16);
      a += __shfl_xor(a, 32);
      ar += __shfl_xor(ar, 8);
      ar += __shfl_xor(ar, 16);
      ar += __shfl_xor(ar, 32);
      if (ks == 0) {
        const int row = rb * 8 + r8;
        const int seed = cvt_rne((A.gb_par[row] + cbr[rb]) * kScale) + (SAT ? 0 : A.gb_wsum[row]);
        const int seedr = cvt_rne(A.gb_par[GB_ROWS + row] * kScale) + (SAT ? 0 : A.gb_wsum[GB_ROWS + row]);
        zr[row] = (float)(seed + a) * kScale1;
        zr[GB_ROWS + row] = (float)(seedr + ar) * kScale1;
      }
    }
    __builtin_amdgcn_wave_barrier();

    /* ---- GRU_B update, dual-FC tree sampling, output (as sample_kernel) -- */
    {
      const int u = lane & (NB - 1);
      const float z = sigmoid_x86(zr[u] + zr[GB_ROWS + u], rcp);
      const float r = sigmoid_x86(zr[NB + u] + zr[GB_ROWS + NB + u], rcp);
      float h = zr[2 * NB + u] + zr[GB_ROWS + 2 * NB + u] * r;
      h = tanh_x86(h, rcp);
      sbv = z * sbv + (1.f - z) * h;
      if (lane < NB) sbuf[lane] = sbv;
    }
    __builtin_amdgcn_wave_barrier();
    float xv[NB];
    {
      const float4 *sb4 = (const float4 *)sbuf;
#pragma unroll
      for (int j = 0; j < NB / 4; j++) {
        const float4 v = sb4[j];
        xv[4 * j] = v.x; xv[4 * j + 1] = v.y; xv[4 * j + 2] = v.z; xv[4 * j + 3] = v.w;
      }
    }
    float thr[8];
#pragma unroll
    for (int b = 0; b < 4; b++) {
      thr[b] = logit_tab[(r0 >> (8 * b)) & 0xFF];
      thr[b + 4] = logit_tab[(r1 >> (8 * b)) & 0xFF];
    }
    const int q = lane >> 1, ch2 = lane & 1;
    const int qq = q < 15 ? q : 0;
    const int lvl_in = qq == 0 ? 0 : (qq < 3 ? 1 : (qq < 7 ? 2 : 3));
    auto node_logit = [&](int node) -> float {
      float sum = fcb[ch2 * 256 + node];
      const float *w = fcw + node * 32 + ch2 * 16;
#pragma unroll
      for (int j = 0; j < NB; j++) sum = sum + w[j] * xv[j];
      const float v = fcf[ch2 * 256 + node] * tanh_x86(sum, rcp);
      const float o = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
      return ch2 ? o + v : v + o;
    };
    float lg[8];
    int val = 0;
    {
      const float l = node_logit(qq + 1);
      const float t = lvl_in == 0 ? thr[0] : (lvl_in == 1 ? thr[1] : (lvl_in == 2 ? thr[2] : thr[3]));
      const unsigned long long m = __ballot(t < l);
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const int nd = (1 << b) | val;
        if (tracing) lg[b] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(l), 2 * (nd - 1)));
        val = (val << 1) | (int)((m >> (2 * (nd - 1))) & 1ull);
      }
    }
    {
      const int lvl = 4 + lvl_in;
      const int off = qq + 1 - (1 << (lvl - 4));
      const float l = node_logit((1 << lvl) | (val << (lvl - 4)) | off);
      const float t = lvl_in == 0 ? thr[4] : (lvl_in == 1 ? thr[5] : (lvl_in == 2 ? thr[6] : thr[7]));
      const unsigned long long m = __ballot(t < l);
#pragma unroll
      for (int b = 4; b < 8; b++) {
        const int qi = (1 << (b - 4)) - 1 + (val & ((1 << (b - 4)) - 1));
        if (tracing) lg[b] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(l), 2 * qi));
        val = (val << 1) | (int)((m >> (2 * qi)) & 1ull);
      }
    }
    int exc = val;
    float pcm;
    if (n < A.preload) {
      const float o_in = (float)pcmbuf[n];
      const float pd = kPreemph * deemph;
      exc = lin2ulaw_x86((o_in - pd) - pred);
      pcm = o_in - pd;
    } else {
      pcm = pred + ulaw[exc];
    }
#pragma unroll
    for (int j = NLPC - 1; j > 0; j--) lsr[j] = lsr[j - 1];
    lsr[0] = pcm;
    last_exc = exc;
    float o = pcm + kPreemph * deemph;
    deemph = o;
    if (o < -32767) o = -32767;
    if (o > 32767) o = 32767;
    if (lane == 0 && n >= A.preload) pcmbuf[n] = (short)round_half_up(o);
    if (tracing && lane < 8) {
      float v = lg[0];
#pragma unroll
      for (int b = 1; b < 8; b++) v = lane == b ? lg[b] : v;
      A.trace_logits[((size_t)sid * A.N + n) * 8 + lane] = v;
    }
    if (A.trace_exc && lane == 0) A.trace_exc[(size_t)sid * A.N + n] = exc;
    if (lane < NB) xb[lane] = (unsigned char)quant_s8(sbv);
    __builtin_amdgcn_wave_barrier();
  }

  /* ---- write back ---------------------------------------------------------- */
#pragma unroll
  for (int j = 0; j < 6; j++) P->gru_a_state[64 * j + lane] = st[j];
  if (lane < NB) P->gru_b_state[lane] = sbv;
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < NLPC; j++) P->last_sig[j] = lsr[j];
    P->deemph_mem = deemph;
    P->last_exc = last_exc;
    P->rng[0] = rz; P->rng[1] = rw; P->rng[2] = rj; P->rng[3] = rc;
  }
  for (int e = lane; e < A.N; e += 64) A.pcm[(size_t)sid * A.N + e] = pcmbuf[e];
}

template <int NW, bool SAT>
static int launch_wave_t(const SampleArgs &a, int lds_bytes, hipStream_t stream)
{
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void *)wave_kernel<NW, SAT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
        hipSuccess)
      return -1;
    attr_set = true;
  }
  int grid = (a.nstreams + NW - 1) / NW;
  hipLaunchKernelGGL((wave_kernel<NW, SAT>), dim3(grid), dim3(NW * 64), lds_bytes, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_wave(const SampleArgs &a, int nw, int sat, int lds_bytes, void *stream)
{
  hipStream_t st = (hipStream_t)stream;
#define W(n) if (nw == n) return sat ? launch_wave_t<n, true>(a, lds_bytes, st) : launch_wave_t<n, false>(a, lds_bytes, st);
  W(1) W(2) W(4) W(8) W(16)
#undef W
  return -1;
}

/* ------------------------------------------------------------------------ */
/* ------------------------------------------------------------------------ */
/* pipe_kernel: fixed wave roles, the GRU_A recurrent product of sample n+1
 * overlapping the sampling of sample n.
 *
 * The recurrent part of GRU_A, W·q(h_A(n)) (sparse_sgemv_accum8x4 inside
 * compute_sparse_gru, nnet.c:441), depends on the GRU_A state only, not on
 * the excitation sampled at n (which enters sample n+1 through the embedding
 * gathers, nnet.c:484-491).  So while the sampler waves run GRU_B's update
 * and the dual-FC tree walk of sample n (nnet.c:362-371, 163-214), the six
 * GRU_A waves already accumulate W·q(h_A(n)) for sample n+1 in registers.
 * Per sample, three workgroup barriers:
 *   X  ix(n) (sig, pred, exc indices) published by the samplers
 *      GRU_A waves: embedding gathers + elementwise GRU_A(n) -> q(h_A(n))
 *      sampler waves: the two kiss99 draws and their logit thresholds
 *   Y  q(h_A(n)) complete
 *      GRU_A wave w: GRU_B gate sums of row block w (nnet.c:345-361)
 *   Z  GRU_B gate sums complete
 *      GRU_A waves: W·q(h_A(n)) for sample n+1
 *      sampler waves: GRU_B update, tree walk, output, pred(n+1) -> ix(n+1)
 * Same arithmetic as sample_kernel's quad path, term for term. */
template <int S>
struct PipeLds {
  static constexpr int x = (NA / 4) * S * 4;   /* quantized GRU_A state (single buffer) */
  static constexpr int xb = (NB / 4) * S * 4;  /* quantized GRU_B state */
  static constexpr int sb = S * NB * 4;        /* float GRU_B state */
  static constexpr int zr = S * 2 * GB_ROWS * 4;
  static constexpr int ix = S * 4 * 4;
  static constexpr int pcm = ((S * FRAME * 2 + 15) / 16) * 16;
  static constexpr int total = x + xb + sb + zr + ix + pcm;
};

/* LDS: [image | regions] */
int pipe_lds_bytes(int S, int image_bytes)
{
  return image_bytes + (S == 4 ? PipeLds<4>::total : (S == 2 ? PipeLds<2>::total : PipeLds<1>::total));
}

template <int S, bool SAT, bool TRACE>
__global__ __launch_bounds__(PIPE_THREADS) void pipe_kernel(SampleArgs A)
{
  extern __shared__ uint4 lds4[];
  unsigned char *lds = (unsigned char *)lds4;
  using L = PipeLds<S>;
  unsigned char *img = lds;
  unsigned char *xa = lds + A.image_bytes;
  unsigned char *xb = xa + L::x;
  float *sbuf = (float *)(xb + L::xb);
  float *zr = sbuf + S * NB;
  int *ix = (int *)(zr + S * 2 * GB_ROWS);
  short *pcmbuf = (short *)(ix + S * 4);

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
    for (int e = tid; e < S * A.N; e += PIPE_THREADS) {
      const int s = e / A.N, n = e % A.N;
      if (s0 + s < A.nstreams) A.pcm[(size_t)(s0 + s) * A.N + n] = 0;
    }
    return;
  }
  {
    uint4 *img4 = (uint4 *)img;
    const int n16 = A.image_bytes / 16;
    for (int o = tid; o < n16; o += PIPE_THREADS) img4[o] = A.image[o];
  }
  for (int e = tid; e < S * A.preload; e += PIPE_THREADS) {
    const int s = e / A.preload, n = e % A.preload;
    pcmbuf[s * FRAME + n] = A.pcm[(size_t)min(s0 + s, A.nstreams - 1) * A.N + n];
  }

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

  /* Roles (wave-uniform): waves 0..5 GRU_A (thread = unit), waves 6..7
   * samplers.  Each role runs its own sample loop with the same barrier
   * sequence (prologue, then X, Y, Z per sample, then one final), so the
   * registers of one role are not live in the other's code. */
  if (wv < SAMPLE_WAVES) {
    /* ======================= GRU_A role ================================== */
    const uint4 *wq = (const uint4 *)img;
    const uint32_t *cq = (const uint32_t *)img;
    const int i = tid;
    const int K4z = A.ga_K4[wv][0], K4r = A.ga_K4[wv][1], K4h = A.ga_K4[wv][2];
    const int qoff = A.ga_qoff[wv][0], coff = A.ga_coff[wv][0];
    const float bz = A.ga_par[i], br = A.ga_par[NA + i], bh = A.ga_par[2 * NA + i];
    const float dz = A.ga_par[3 * NA + i], dr = A.ga_par[4 * NA + i], dh = A.ga_par[5 * NA + i];
    const int wsz = A.ga_wsum[i], wsr = A.ga_wsum[NA + i], wsh = A.ga_wsum[2 * NA + i];
    const int rb = wv, r8 = lane & 7, ks = lane >> 3, row = rb * 8 + r8;
    float st[S], cz[S], cr[S], ch[S];
    int gb_seed[S];
    for (int s = 0; s < S; s++) {
      const StreamState *p = &A.st[min(s0 + s, A.nstreams - 1)];
      st[s] = p->gru_a_state[i];
      cz[s] = p->gru_a_cond[i];
      cr[s] = p->gru_a_cond[NA + i];
      ch[s] = p->gru_a_cond[2 * NA + i];
      gb_seed[s] = cvt_rne((A.gb_par[row] + p->gru_b_cond[row]) * kScale) + (SAT ? 0 : A.gb_wsum[row]);
    }
    const int gb_seedr = cvt_rne(A.gb_par[GB_ROWS + row] * kScale) + (SAT ? 0 : A.gb_wsum[GB_ROWS + row]);
    __syncthreads(); /* image in LDS */
    for (int s = 0; s < S; s++) xa[(i >> 2) * S * 4 + s * 4 + (i & 3)] = (unsigned char)quant_s8(st[s]);
    __syncthreads(); /* initial q(h_A), q(h_B), ix */
    stamp_start();

    int az[S], ar[S], ah[S];
    auto recurrent = [&]() {
      for (int s = 0; s < S; s++) {
        az[s] = SAT ? 0 : wsz;
        ar[s] = SAT ? 0 : wsr;
        ah[s] = SAT ? 0 : wsh;
      }
      gru_a_stream<S, SAT>(xa, wq, cq, qoff, coff, K4z, K4r, K4h, lane, az, ar, ah);
    };
    recurrent();
    for (int n = 0; n < A.N; n++) {
      stamp(4);
      __syncthreads(); /* X */
      stamp(5);
      {
        /* GRU_A input (nnet.c:484-491): all 9*S gathers in flight at once */
        float e[S][9];
        for (int s = 0; s < S; s++) {
          /* the indices are the same in every lane: scalar row addresses */
          const int4 v = *(const int4 *)(ix + s * 4);
          const float *e1 = A.emb_sig + (__builtin_amdgcn_readfirstlane(v.x) & 0xFF) * GA_ROWS;
          const float *e2 = A.emb_pred + (__builtin_amdgcn_readfirstlane(v.y) & 0xFF) * GA_ROWS;
          const float *e3 = A.emb_exc + (__builtin_amdgcn_readfirstlane(v.z) & 0xFF) * GA_ROWS;
#pragma unroll
          for (int g = 0; g < 3; g++) {
            e[s][g] = e1[g * NA + i];
            e[s][3 + g] = e2[g * NA + i];
            e[s][6 + g] = e3[g * NA + i];
          }
        }
        /* compute_sparse_gru elementwise (nnet.c:431-447) */
        float zrv[2 * S], hv[S], inh[S];
        for (int s = 0; s < S; s++) {
          const float inz = ((cz[s] + e[s][0]) + e[s][3]) + e[s][6];
          const float inr = ((cr[s] + e[s][1]) + e[s][4]) + e[s][7];
          inh[s] = ((ch[s] + e[s][2]) + e[s][5]) + e[s][8];
          zrv[s] = (float)(az[s] + cvt_rne(((bz + dz * st[s]) + inz) * kScale)) * kScale1;
          zrv[S + s] = (float)(ar[s] + cvt_rne(((br + dr * st[s]) + inr) * kScale)) * kScale1;
          hv[s] = (float)(ah[s] + cvt_rne((bh + dh * st[s]) * kScale)) * kScale1;
        }
        sigmoid_x86_n<2 * S>(zrv, rcp);
        for (int s = 0; s < S; s++) hv[s] = hv[s] * zrv[S + s] + inh[s];
        tanh_x86_n<S>(hv, rcp);
        for (int s = 0; s < S; s++) {
          st[s] = zrv[s] * st[s] + (1.f - zrv[s]) * hv[s];
          xa[(i >> 2) * S * 4 + s * 4 + (i & 3)] = (unsigned char)quant_s8(st[s]);
        }
      }
      stamp(0);
      __syncthreads(); /* Y */
      stamp(1);
      {
        /* GRU_B gate sums of row block rb (nnet.c:345-361) */
        int acc[S], accr[S];
        for (int s = 0; s < S; s++) { acc[s] = 0; accr[s] = 0; }
        gru_a_stream<S, SAT>(xa, wq, cq, A.gb_qoff[rb], A.gb_coff[rb], REG_GB / 4, 0, 0, lane, acc, acc, acc);
        if (ks < NB / 4) {
          const uint32_t w = ((const uint32_t *)(img + A.gb_rec_off))[(rb * (NB / 4) + ks) * 8 + r8];
          dot_streams<S, SAT>(xb, ks * S * 4, w, accr);
        }
        for (int s = 0; s < S; s++) {
          acc[s] = sum_lanes_xor8_16_32(acc[s]);
          accr[s] = sum_lanes_xor8_16_32(accr[s]);
        }
        if (ks == 0) {
          for (int s = 0; s < S; s++) {
            zr[s * 2 * GB_ROWS + row] = (float)(gb_seed[s] + acc[s]) * kScale1;
            zr[s * 2 * GB_ROWS + GB_ROWS + row] = (float)(gb_seedr + accr[s]) * kScale1;
          }
        }
      }
      stamp(2);
      __syncthreads(); /* Z */
      stamp(3);
      if (n + 1 < A.N) recurrent(); /* W q(h_A(n)) for sample n+1, beside the sampling of n */
    }
    stamp(4);
    __syncthreads(); /* final */
    stamp(5);
    for (int s = 0; s < S; s++)
      if (active[s]) A.st[s0 + s].gru_a_state[i] = st[s];
  } else {
    /* ======================= sampler role ================================ */
    const float *logit_tab = (const float *)(img + IMG_LOGIT);
    /* with S=4 a sampler wave carries two streams, one per 32-lane half */
    const int sw = wv - SAMPLE_WAVES;
    const int half = lane >> 5, hl = lane & 31;
    const int my_s = S == 4 ? 2 * sw + half : sw;
    const bool samp = my_s < S;                         /* wave-uniform */
    const bool samp_w = samp && (S == 4 || half == 0);  /* lanes owning the stream's outputs */
    const int ms = samp ? my_s : 0;
    const bool my_active = samp && s0 + ms < A.nstreams && A.st[s0 + ms].frame_count > FEATURES_DELAY;

    float lsr[NLPC], lpr[NLPC];
    float sbv = 0.f, pred = 0.f, deemph = 0.f;
    uint32_t rz = 0, rw = 0, rj = 0, rc = 0;
    int last_exc = 0;
    {
      const StreamState *p = &A.st[min(s0 + ms, A.nstreams - 1)];
#pragma unroll
      for (int j = 0; j < NLPC; j++) {
        lsr[j] = p->last_sig[j];
        lpr[j] = p->lpc[j];
      }
      sbv = p->gru_b_state[hl & (NB - 1)];
      deemph = p->deemph_mem;
      last_exc = p->last_exc;
      rz = p->rng[0]; rw = p->rng[1]; rj = p->rng[2]; rc = p->rng[3];
    }
    __syncthreads(); /* image in LDS */
    FcLane F;
    F.init(img, lane);
    if (samp_w && hl < NB) {
      xb[(hl >> 2) * S * 4 + ms * 4 + (hl & 3)] = (unsigned char)quant_s8(sbv);
      sbuf[ms * NB + hl] = sbv;
    }
    if (samp) {
      /* pred and the u-law indices of the first sample (lpcnet.c:252-254) */
      float p2 = 0.f;
#pragma unroll
      for (int j = 0; j < NLPC; j++) p2 = p2 - lsr[j] * lpr[j];
      pred = p2;
      if (samp_w && hl == 0) *(int4 *)(ix + ms * 4) = make_int4(lin2ulaw_x86(lsr[0]), lin2ulaw_x86(pred), last_exc, 0);
    }
    __syncthreads(); /* initial q(h_A), q(h_B), ix */
    stamp_start();

    float t03 = 0.f, t47 = 0.f;
    constexpr bool tracing = TRACE;
    /* Bookkeeping of sample n (lpcnet.c:260-270: LPC history shift,
     * de-emphasis, output, q(h_B)) is deferred into the X->Y interval of
     * sample n+1, where the sampler waves are otherwise idle; only the next
     * indices ix(n+1) stay on the per-sample critical path. */
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
      if (samp_w && hl == 0 && pend_n >= A.preload) pcmbuf[ms * FRAME + pend_n] = (short)round_half_up(o);
      if (samp_w && hl < NB) xb[(hl >> 2) * S * 4 + ms * 4 + (hl & 3)] = (unsigned char)quant_s8(sbv);
      pend_n = -1;
    };
    for (int n = 0; n < A.N; n++) {
      stamp(4);
      __syncthreads(); /* X */
      stamp(5);
      if (samp) {
        finish();
        stamp(13);
        /* the two kiss99 draws of this sample and their thresholds (nnet.c:178-184) */
        const uint32_t r0 = kiss99_next(rz, rw, rj, rc);
        const uint32_t r1 = kiss99_next(rz, rw, rj, rc);
        lane_thresholds(F, logit_tab, r0, r1, t03, t47);
      }
      stamp(0);
      __syncthreads(); /* Y */
      stamp(1);
      stamp(2);
      __syncthreads(); /* Z */
      stamp(3);
      if (!samp) continue;
      const int s = ms;
      const float *zs = zr + s * 2 * GB_ROWS;
      {
        /* GRU_B elementwise (nnet.c:362-371); lanes >= 16 of a half duplicate */
        const int u = hl & (NB - 1);
        float zrb[2] = {zs[u] + zs[GB_ROWS + u], zs[NB + u] + zs[GB_ROWS + NB + u]};
        sigmoid_x86_n<2>(zrb, rcp);
        float h[1] = {zs[2 * NB + u] + zs[GB_ROWS + 2 * NB + u] * zrb[1]};
        tanh_x86_n<1>(h, rcp);
        sbv = zrb[0] * sbv + (1.f - zrb[0]) * h[0];
        if (samp_w && hl < NB) sbuf[s * NB + hl] = sbv;
      }
      stamp(8);
      /* same-wave LDS exchange (measured faster than 32 v_readlane: gfx9
       * VALU ops read one SGPR each and SGPR hazards add wait states) */
      __builtin_amdgcn_wave_barrier();
      float xv[NB];
      {
        const float4 *sb4 = (const float4 *)(sbuf + s * NB);
#pragma unroll
        for (int j = 0; j < NB / 4; j++) {
          const float4 v = sb4[j];
          xv[4 * j] = v.x; xv[4 * j + 1] = v.y; xv[4 * j + 2] = v.z; xv[4 * j + 3] = v.w;
        }
      }
      stamp(9);
      const WalkOut R = dual_fc_walk<TRACE>(F, t03, t47, xv, pred, lsr, lpr, n < A.preload ? pcmbuf + s * FRAME + n : nullptr,
                                            deemph);
      stamp(11);
      if (samp_w && hl == 0 && n + 1 < A.N) *(int4 *)(ix + s * 4) = make_int4(R.su, R.pu, R.exc, 0);
      if (tracing && samp_w && hl < 8 && my_active) {
        float v = R.lg[0];
#pragma unroll
        for (int b = 1; b < 8; b++) v = hl == b ? R.lg[b] : v;
        A.trace_logits[((size_t)(s0 + s) * A.N + n) * 8 + hl] = v;
      }
      if (A.trace_exc && samp_w && hl == 0 && my_active) A.trace_exc[(size_t)(s0 + s) * A.N + n] = R.exc;
      pend_pcm = R.pcm;
      pend_pred = R.pn;
      pend_exc = R.exc;
      pend_n = n;
      stamp(12);
    }
    if (samp) finish();
    stamp(4);
    __syncthreads(); /* final */
    stamp(5);
    if (samp_w && my_active) {
      StreamState *p = &A.st[s0 + ms];
      if (hl < NB) p->gru_b_state[hl] = sbv;
      if (hl == 0) {
#pragma unroll
        for (int j = 0; j < NLPC; j++) p->last_sig[j] = lsr[j];
        p->deemph_mem = deemph;
        p->last_exc = last_exc;
        p->rng[0] = rz; p->rng[1] = rw; p->rng[2] = rj; p->rng[3] = rc;
      }
    }
  }
  if (stamping && lane == 0) {
    stp[6] = __builtin_amdgcn_s_memtime() - t_loop0;
    stp[7] = (unsigned long long)A.N;
    for (int k = 0; k < 16; k++) A.stamps[((size_t)blockIdx.x * STAMP_WAVES + wv) * 16 + k] = stp[k];
  }
  for (int e = tid; e < S * A.N; e += PIPE_THREADS) {
    const int s = e / A.N, n = e % A.N;
    if (s0 + s < A.nstreams) A.pcm[(size_t)(s0 + s) * A.N + n] = active[s] ? pcmbuf[s * FRAME + n] : (short)0;
  }
}

template <int S, bool SAT, bool TRACE>
static int launch_pipe_t(const SampleArgs &a, int lds_bytes, hipStream_t stream)
{
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void *)pipe_kernel<S, SAT, TRACE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return -1;
    attr_set = true;
  }
  const int grid = (a.nstreams + S - 1) / S;
  hipLaunchKernelGGL((pipe_kernel<S, SAT, TRACE>), dim3(grid), dim3(PIPE_THREADS), lds_bytes, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int S, bool SAT>
static int launch_pipe_s(const SampleArgs &a, int lds_bytes, hipStream_t st)
{
  return a.trace_logits ? launch_pipe_t<S, SAT, true>(a, lds_bytes, st) : launch_pipe_t<S, SAT, false>(a, lds_bytes, st);
}

int launch_pipe(const SampleArgs &a, int S, int sat, int lds_bytes, void *stream)
{
  hipStream_t st = (hipStream_t)stream;
  if (S == 4) return sat ? launch_pipe_s<4, true>(a, lds_bytes, st) : launch_pipe_s<4, false>(a, lds_bytes, st);
  if (S == 2) return sat ? launch_pipe_s<2, true>(a, lds_bytes, st) : launch_pipe_s<2, false>(a, lds_bytes, st);
  return sat ? launch_pipe_s<1, true>(a, lds_bytes, st) : launch_pipe_s<1, false>(a, lds_bytes, st);
}

template <int S, int V, bool SAT, bool REG>
static int launch_sample_t(const SampleArgs &a, int lds_bytes, hipStream_t stream)
{
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void *)sample_kernel<S, V, SAT, REG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return -1;
    attr_set = true;
  }
  int grid = (a.nstreams + S - 1) / S;
  hipLaunchKernelGGL((sample_kernel<S, V, SAT, REG>), dim3(grid), dim3(SAMPLE_THREADS), lds_bytes, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int S>
static int launch_s(const SampleArgs &a, int variant, int sat, int reg, int lds_bytes, hipStream_t st)
{
  if (variant == 1) return launch_sample_t<S, 1, false, false>(a, lds_bytes, st);
  if (sat) return reg ? launch_sample_t<S, 0, true, true>(a, lds_bytes, st) : launch_sample_t<S, 0, true, false>(a, lds_bytes, st);
  return reg ? launch_sample_t<S, 0, false, true>(a, lds_bytes, st) : launch_sample_t<S, 0, false, false>(a, lds_bytes, st);
}

int launch_sample(const SampleArgs &a, int S, int variant, int sat, int reg, int lds_bytes, void *stream)
{
  hipStream_t st = (hipStream_t)stream;
  if (S == 4) return launch_s<4>(a, variant, sat, reg, lds_bytes, st);
  if (S == 2) return launch_s<2>(a, variant, sat, reg, lds_bytes, st);
  return launch_s<1>(a, variant, sat, reg, lds_bytes, st);
}

}  // namespace lpcnet_mi355x
