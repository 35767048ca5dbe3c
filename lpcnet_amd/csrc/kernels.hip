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
  /* the image is copied to LDS whole, or -- models whose weight sections
   * do not fit (long block rows) -- only its fixed tables, the weights being
   * read from the global copy (same offsets) */
  const unsigned char *wimg = A.image_lds_bytes < A.image_bytes ? (const unsigned char *)A.image : lds;
  unsigned char *xa_base = lds + A.image_lds_bytes;
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
    active[s] = sid < A.nstreams && A.st[sid].frame_count > A.delay;
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
  for (int o = tid; o < A.image_lds_bytes / 16; o += SAMPLE_THREADS) lds4[o] = A.image[o];

  const int K4z = REG ? A.ga_K4[wv][0] : 0, K4r = REG ? A.ga_K4[wv][1] : 0, K4h = REG ? A.ga_K4[wv][2] : 0;
  const uint4 *wq = (const uint4 *)wimg;
  const uint32_t *cq = (const uint32_t *)wimg;

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
    last_exc = p->last_exc & 0xFF;
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

  const uint32_t *lds32 = (const uint32_t *)wimg;
  const uint16_t *lds16 = (const uint16_t *)wimg;
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
          uint32_t w = ((const uint32_t *)(wimg + A.gb_rec_off))[(rb * (NB / 4) + ks) * 8 + r];
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
          const float4 *wp = (const float4 *)(wimg + A.gb_woff[rb] * 4);
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

template <int S, int V, bool SAT, bool REG>
static int launch_sample_t(const SampleArgs &a, int lds_bytes, hipStream_t stream)
{
  if (ensure_dyn_lds((const void *)sample_kernel<S, V, SAT, REG>, 160 * 1024)) return -1;
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
