/*
 * lpcnet_oracle.c -- CPU restatement of the reference LPCNet synthesis path.
 * TEST INFRASTRUCTURE ONLY (see lpcnet_oracle.h).  Compile with
 * -ffp-contract=off: every float expression below is evaluated exactly in the
 * order the reference evaluates it, and explicit fmaf() appears only where the
 * reference issues _mm256_fmadd_ps.
 *
 * All citations are /root/reference/src/<file>:<line>.
 */
#include "lpcnet_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Model constants of the default LPCNet model (training_tf2/lpcnet.py:312-325,
 * train_lpcnet.py:82-101; generated into nnet_data.h by dump_lpcnet.py).     */
#define NB_FEATURES 20
#define EMBED_PITCH 64
#define FRAME_INPUT (NB_FEATURES + EMBED_PITCH) /* lpcnet.c:44 */
#define COND 128
#define NA 384
#define NB 16
#define CONV_K 3
#define FEATURES_DELAY 2 /* dump_lpcnet.py:442 default lookahead */
#define MAX_FEATURES_DELAY 4 /* train_lpcnet.py:273: lookahead <= 4 */
#define CONV1_DELAY 1    /* dump_lpcnet.py:306 (k-1)//2 */
#define LPC_ORDER 16
#define FRAME_SIZE 160
#define PREEMPH 0.85f /* lpcnet.c:40 */
#define NLEVELS 256
#define MAX_FEATURE_BUFFER_SIZE 4 /* lpcnet_private.h:26 */
#define NB_BANDS 18               /* freq.h:48 */
#define NB_BANDS_1 (NB_BANDS - 1) /* freq.h:49 */
#define NB_TOTAL_FEATURES 36      /* include/lpcnet.h:46 */

/* ------------------------------------------------------------------------ */
/* rcpps emulation.  The table holds _mm256_rcp_ps(1.m) for the 2048 values of
 * the top 11 mantissa bits (tabulated on the x86 host, tests/golden/rcp_x86.bin);
 * the instruction is exponent invariant and flushes denormal results to 0. */
static uint32_t g_rcp[2048];

void oracle_set_rcp_table(const uint32_t *tab) { memcpy(g_rcp, tab, sizeof(g_rcp)); }

static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

float oracle_rcp(float x)
{
  uint32_t u = f2u(x);
  uint32_t sign = u & 0x80000000u;
  int e = (int)((u >> 23) & 0xff);
  if (e == 0) return u2f(sign | 0x7f800000u);            /* 0 / denormal -> inf */
  if (e == 255) {
    if (u & 0x7fffff) return u2f(u | 0x00400000u);        /* NaN -> quiet NaN */
    return u2f(sign);                                     /* inf -> 0 */
  }
  uint32_t t = g_rcp[(u >> 12) & 0x7ff];
  int te = (int)((t >> 23) & 0xff) - (e - 127);
  if (te < 1) return u2f(sign);                            /* denormal result flushed */
  return u2f(sign | (t & 0x007fffffu) | ((uint32_t)te << 23));
}

/* _mm256_min_ps / _mm256_max_ps: second operand when unordered */
static float mm_min(float a, float b) { return a < b ? a : b; }
static float mm_max(float a, float b) { return a > b ? a : b; }

/* vec_avx.h:393-411 tanh8_approx */
float oracle_tanh(float X)
{
  const float N0 = 952.52801514f, N1 = 96.39235687f, N2 = 0.60863042f;
  const float D0 = 952.72399902f, D1 = 413.36801147f, D2 = 11.88600922f;
  float X2 = X * X;
  float num = fmaf(fmaf(N2, X2, N1), X2, N0);
  float den = fmaf(fmaf(D2, X2, D1), X2, D0);
  num = num * X;
  den = oracle_rcp(den);
  num = num * den;
  return mm_max(-1.f, mm_min(1.f, num));
}

/* vec_avx.h:421-440 sigmoid8_approx */
float oracle_sigmoid(float X)
{
  const float N0 = 238.13200378f, N1 = 6.02452230f, N2 = 0.00950985f;
  const float D0 = 952.72399902f, D1 = 103.34200287f, D2 = 0.74287558f;
  float X2 = X * X;
  float num = fmaf(fmaf(N2, X2, N1), X2, N0);
  float den = fmaf(fmaf(D2, X2, D1), X2, D0);
  num = num * X;
  den = oracle_rcp(den);
  num = fmaf(num, den, 0.5f);
  return mm_max(0.f, mm_min(1.f, num));
}

static void port_vec_tanh(float *y, const float *x, int n) { for (int i = 0; i < n; i++) y[i] = oracle_tanh(x[i]); }
static void port_vec_sigmoid(float *y, const float *x, int n) { for (int i = 0; i < n; i++) y[i] = oracle_sigmoid(x[i]); }

/* vec_avx.h:618-643 sgemv_accum16: y[i] = fma(w[j*stride+i], x[j], y[i]) for j ascending */
static void port_sgemv16(float *out, const float *w, int rows, int cols, int stride, const float *x)
{
  for (int i = 0; i < rows; i++) {
    float y = out[i];
    for (int j = 0; j < cols; j++) y = fmaf(w[j * stride + i], x[j], y);
    out[i] = y;
  }
}

/* _mm256_cvtps_epi32 (round to nearest even, out of range -> INT_MIN) */
static int32_t cvt_rne(float v)
{
  if (!(v >= -2147483648.f && v < 2147483648.f)) return INT32_MIN;
  return (int32_t)nearbyintf(v);
}

/* vec_avx.h:321-336 vector_ps_to_epi8: u8 = sat(cvt_rne(fma(x,127,127))) */
void oracle_quantize_u8(unsigned char *x, const float *xf, int n)
{
  for (int i = 0; i < n; i++) {
    int32_t v = cvt_rne(fmaf(xf[i], 127.f, 127.f));
    x[i] = (unsigned char)(v < 0 ? 0 : (v > 255 ? 255 : v));
  }
}

static int32_t sat16(int32_t v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

/* one 8x4 block: maddubs (u8 x s8 pair sums, int16 saturation) + madd(ones) */
static void block8x4(int32_t *acc, const int8_t *w, const unsigned char *xp)
{
  for (int r = 0; r < 8; r++) {
    int32_t p0 = sat16((int32_t)xp[0] * w[r * 4 + 0] + (int32_t)xp[1] * w[r * 4 + 1]);
    int32_t p1 = sat16((int32_t)xp[2] * w[r * 4 + 2] + (int32_t)xp[3] * w[r * 4 + 3]);
    acc[r] = (int32_t)((uint32_t)acc[r] + (uint32_t)(p0 + p1));
  }
}

#define SCALE (128.f * 127.f)          /* vec_avx.h:686 */
#define SCALE_1 (1.f / 128.f / 127.f)  /* vec_avx.h:687 */

/* vec_avx.h:790-858 sparse_sgemv_accum8x4 (DOT_PROD) */
static void port_sparse8x4_i8(float *out, const int8_t *w, int rows, int cols, const int *idx, const float *xf)
{
  unsigned char x[2048];
  oracle_quantize_u8(x, xf, cols);
  for (int i = 0; i < rows; i += 8) {
    int32_t acc[8];
    int nb = *idx++;
    for (int r = 0; r < 8; r++) acc[r] = cvt_rne(out[i + r] * SCALE);
    for (int k = 0; k < nb; k++) {
      int pos = *idx++;
      block8x4(acc, w, &x[pos]);
      w += 32;
    }
    for (int r = 0; r < 8; r++) out[i + r] = (float)acc[r] * SCALE_1;
  }
}

/* vec_avx.h:690-755 sgemv_accum8x4 (DOT_PROD, dense) */
static void port_dense8x4_i8(float *out, const int8_t *w, int rows, int cols, const float *xf)
{
  unsigned char x[2048];
  oracle_quantize_u8(x, xf, cols);
  for (int i = 0; i < rows; i += 8) {
    int32_t acc[8];
    for (int r = 0; r < 8; r++) acc[r] = cvt_rne(out[i + r] * SCALE);
    for (int j = 0; j < cols; j += 4) {
      block8x4(acc, w, &x[j]);
      w += 32;
    }
    for (int r = 0; r < 8; r++) out[i + r] = (float)acc[r] * SCALE_1;
  }
}

/* vec_avx.h:861-904 sparse_sgemv_accum8x4 (no DOT_PROD): block is [4 in][8 out] */
static void port_sparse8x4_f32(float *out, const float *w, int rows, const int *idx, const float *x)
{
  for (int i = 0; i < rows; i += 8) {
    float y[8];
    int nb = *idx++;
    for (int r = 0; r < 8; r++) y[r] = out[i + r];
    for (int k = 0; k < nb; k++) {
      int id = *idx++;
      for (int c = 0; c < 4; c++)
        for (int r = 0; r < 8; r++) y[r] = fmaf(w[c * 8 + r], x[id + c], y[r]);
      w += 32;
    }
    for (int r = 0; r < 8; r++) out[i + r] = y[r];
  }
}

/* common.h:18-33 log2_approx */
static float log2_approx(float x)
{
  int32_t integer;
  uint32_t i = f2u(x);
  integer = (int32_t)(i >> 23) - 127;
  i -= (uint32_t)integer << 23;
  float frac = u2f(i) - 1.5f;
  frac = -0.41445418f + frac * (0.95909232f + frac * (-0.33951290f + frac * 0.16541097f));
  return 1 + integer + frac;
}

#define LOG256 5.5451774445f
/* common.h:47-58 lin2ulaw */
static int port_lin2ulaw(float x)
{
  float u;
  float scale = 255.f / 32768.f;
  int s = x >= 0 ? 1 : -1;
  x = fabsf(x);
  u = (s * (128 * (0.69315f * log2_approx(1 + scale * x)) / LOG256));
  u = 128 + u;
  if (u < 0) u = 0;
  if (u > 255) u = 255;
  return (int)floor(.5 + u);
}

/* common.h:37-45 ulaw2lin */
static float port_ulaw2lin(float u)
{
  float s;
  float scale_1 = 32768.f / 255.f;
  u = u - 128.f;
  s = u >= 0.f ? 1.f : -1.f;
  u = fabsf(u);
  return s * scale_1 * (exp(u / 128. * LOG256) - 1);
}

/* kiss99.c:59-81 */
static uint32_t port_rng_rand(oracle_rng *r)
{
  uint32_t znew = 36969 * (r->z & 0xFFFF) + (r->z >> 16);
  uint32_t wnew = 18000 * (r->w & 0xFFFF) + (r->w >> 16);
  uint32_t mwc = (znew << 16) + wnew;
  uint32_t shr3 = r->jsr ^ (r->jsr << 13);
  shr3 ^= shr3 >> 17;
  shr3 ^= shr3 << 5;
  uint32_t cong = 69069 * r->jcong + 1234567;
  r->z = znew;
  r->w = wnew;
  r->jsr = shr3;
  r->jcong = cong;
  return (mwc ^ cong) + shr3;
}

/* kiss99.c:32-57 */
static void port_rng_srand(oracle_rng *r, const unsigned char *d, int n)
{
  int i;
  r->z = 362436069;
  r->w = 521288629;
  r->jsr = 123456789;
  r->jcong = 380116160;
  for (i = 3; i < n; i += 4) {
    r->z ^= d[i - 3];
    r->w ^= d[i - 2];
    r->jsr ^= d[i - 1];
    r->jcong ^= d[i];
    port_rng_rand(r);
  }
  if (i - 3 < n) r->z ^= d[i - 3];
  if (i - 2 < n) r->w ^= d[i - 2];
  if (i - 1 < n) r->jsr ^= d[i - 1];
  if (r->z == 0 || r->z == 0x9068FFFF) r->z++;
  if (r->w == 0 || r->w == 0x464FFFFF) r->w++;
  if (r->jsr == 0) r->jsr++;
}

/* ------------------------------------------------------------------------ */
/* lpc_from_cepstrum (freq.c:310-320) and its helpers.  The 320-point FFT is a
 * restatement of Opus' kiss_fft (kiss_fft.c:101-305, 518-586) with factors
 * {5,64,4,16,4,4,4,1}; twiddles, bit reversal and the DCT table are generated
 * exactly as kiss_fft.c:406-421/315-345 and dump_lpcnet_tables.c:88-95 do. */
#define NB_BANDS 18
#define WINDOW_SIZE 320
#define FREQ_SIZE 161
typedef struct { float r, i; } cpx;

static const short eband5ms[NB_BANDS] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28, 34, 40};
static const float compensation[NB_BANDS] = {0.8f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 0.666667f, 0.5f, 0.5f, 0.5f,
                                             0.333333f, 0.25f, 0.25f, 0.2f, 0.166667f, 0.173913f};
static cpx g_tw[WINDOW_SIZE];
static short g_bitrev[WINDOW_SIZE];
static float g_dct[NB_BANDS * NB_BANDS];
static int g_tables_ready;

static void bitrev_rec(int fout, short *f, int fstride, const short *factors)
{
  int p = factors[0], m = factors[1];
  if (m == 1) {
    for (int j = 0; j < p; j++) { *f = (short)(fout + j); f += fstride; }
  } else {
    for (int j = 0; j < p; j++) { bitrev_rec(fout, f, fstride * p, factors + 2); f += fstride; fout += m; }
  }
}

static const short g_factors[8] = {5, 64, 4, 16, 4, 4, 4, 1};

static void init_tables(void)
{
  if (g_tables_ready) return;
  for (int i = 0; i < WINDOW_SIZE; i++) {
    const double pi = 3.14159265358979323846264338327;
    double phase = (-2 * pi / WINDOW_SIZE) * i;
    g_tw[i].r = (float)cos(phase);
    g_tw[i].i = (float)sin(phase);
  }
  bitrev_rec(0, g_bitrev, 1, g_factors);
  for (int i = 0; i < NB_BANDS; i++)
    for (int j = 0; j < NB_BANDS; j++) {
      g_dct[i * NB_BANDS + j] = (float)cos((i + .5) * j * M_PI / NB_BANDS);
      if (j == 0) g_dct[i * NB_BANDS + j] *= sqrt(.5);
    }
  g_tables_ready = 1;
}

static void bfly4(cpx *Fout, int fstride, int m, int N, int mm)
{
  if (m == 1) {
    for (int i = 0; i < N; i++) {
      cpx s0, s1;
      s0.r = Fout[0].r - Fout[2].r; s0.i = Fout[0].i - Fout[2].i;
      Fout[0].r = Fout[0].r + Fout[2].r; Fout[0].i = Fout[0].i + Fout[2].i;
      s1.r = Fout[1].r + Fout[3].r; s1.i = Fout[1].i + Fout[3].i;
      Fout[2].r = Fout[0].r - s1.r; Fout[2].i = Fout[0].i - s1.i;
      Fout[0].r = Fout[0].r + s1.r; Fout[0].i = Fout[0].i + s1.i;
      s1.r = Fout[1].r - Fout[3].r; s1.i = Fout[1].i - Fout[3].i;
      Fout[1].r = s0.r + s1.i; Fout[1].i = s0.i - s1.r;
      Fout[3].r = s0.r - s1.i; Fout[3].i = s0.i + s1.r;
      Fout += 4;
    }
    return;
  }
  cpx *beg = Fout;
  for (int i = 0; i < N; i++) {
    Fout = beg + i * mm;
    const cpx *tw1 = g_tw, *tw2 = g_tw, *tw3 = g_tw;
    for (int j = 0; j < m; j++) {
      cpx s[6];
      s[0].r = Fout[m].r * tw1->r - Fout[m].i * tw1->i; s[0].i = Fout[m].r * tw1->i + Fout[m].i * tw1->r;
      s[1].r = Fout[2 * m].r * tw2->r - Fout[2 * m].i * tw2->i; s[1].i = Fout[2 * m].r * tw2->i + Fout[2 * m].i * tw2->r;
      s[2].r = Fout[3 * m].r * tw3->r - Fout[3 * m].i * tw3->i; s[2].i = Fout[3 * m].r * tw3->i + Fout[3 * m].i * tw3->r;
      s[5].r = Fout[0].r - s[1].r; s[5].i = Fout[0].i - s[1].i;
      Fout[0].r = Fout[0].r + s[1].r; Fout[0].i = Fout[0].i + s[1].i;
      s[3].r = s[0].r + s[2].r; s[3].i = s[0].i + s[2].i;
      s[4].r = s[0].r - s[2].r; s[4].i = s[0].i - s[2].i;
      Fout[2 * m].r = Fout[0].r - s[3].r; Fout[2 * m].i = Fout[0].i - s[3].i;
      tw1 += fstride; tw2 += fstride * 2; tw3 += fstride * 3;
      Fout[0].r = Fout[0].r + s[3].r; Fout[0].i = Fout[0].i + s[3].i;
      Fout[m].r = s[5].r + s[4].i; Fout[m].i = s[5].i - s[4].r;
      Fout[3 * m].r = s[5].r - s[4].i; Fout[3 * m].i = s[5].i + s[4].r;
      ++Fout;
    }
  }
}

static void bfly5(cpx *Fout, int fstride, int m, int N, int mm)
{
  cpx ya = g_tw[fstride * m], yb = g_tw[fstride * 2 * m];
  cpx *beg = Fout;
  for (int i = 0; i < N; i++) {
    cpx *F0 = beg + i * mm, *F1 = F0 + m, *F2 = F0 + 2 * m, *F3 = F0 + 3 * m, *F4 = F0 + 4 * m;
    for (int u = 0; u < m; ++u) {
      cpx s[13];
      const cpx *t1 = &g_tw[u * fstride], *t2 = &g_tw[2 * u * fstride], *t3 = &g_tw[3 * u * fstride], *t4 = &g_tw[4 * u * fstride];
      s[0] = *F0;
      s[1].r = F1->r * t1->r - F1->i * t1->i; s[1].i = F1->r * t1->i + F1->i * t1->r;
      s[2].r = F2->r * t2->r - F2->i * t2->i; s[2].i = F2->r * t2->i + F2->i * t2->r;
      s[3].r = F3->r * t3->r - F3->i * t3->i; s[3].i = F3->r * t3->i + F3->i * t3->r;
      s[4].r = F4->r * t4->r - F4->i * t4->i; s[4].i = F4->r * t4->i + F4->i * t4->r;
      s[7].r = s[1].r + s[4].r; s[7].i = s[1].i + s[4].i;
      s[10].r = s[1].r - s[4].r; s[10].i = s[1].i - s[4].i;
      s[8].r = s[2].r + s[3].r; s[8].i = s[2].i + s[3].i;
      s[9].r = s[2].r - s[3].r; s[9].i = s[2].i - s[3].i;
      F0->r = F0->r + (s[7].r + s[8].r);
      F0->i = F0->i + (s[7].i + s[8].i);
      s[5].r = s[0].r + ((s[7].r * ya.r) + (s[8].r * yb.r));
      s[5].i = s[0].i + ((s[7].i * ya.r) + (s[8].i * yb.r));
      s[6].r = (s[10].i * ya.i) + (s[9].i * yb.i);
      s[6].i = -((s[10].r * ya.i) + (s[9].r * yb.i));
      F1->r = s[5].r - s[6].r; F1->i = s[5].i - s[6].i;
      F4->r = s[5].r + s[6].r; F4->i = s[5].i + s[6].i;
      s[11].r = s[0].r + ((s[7].r * yb.r) + (s[8].r * ya.r));
      s[11].i = s[0].i + ((s[7].i * yb.r) + (s[8].i * ya.r));
      s[12].r = (s[9].i * ya.i) - (s[10].i * yb.i);
      s[12].i = (s[10].r * yb.i) - (s[9].r * ya.i);
      F2->r = s[11].r + s[12].r; F2->i = s[11].i + s[12].i;
      F3->r = s[11].r - s[12].r; F3->i = s[11].i - s[12].i;
      ++F0; ++F1; ++F2; ++F3; ++F4;
    }
  }
}

/* kiss_fft.c:566-586 opus_fft_c + :518-564 opus_fft_impl for nfft=320 */
static void fft320(const cpx *fin, cpx *fout)
{
  const float scale = 1.f / 320.f;
  for (int i = 0; i < WINDOW_SIZE; i++) {
    fout[g_bitrev[i]].r = scale * fin[i].r;
    fout[g_bitrev[i]].i = scale * fin[i].i;
  }
  bfly4(fout, 80, 1, 80, 4);
  bfly4(fout, 20, 4, 20, 16);
  bfly4(fout, 5, 16, 5, 64);
  bfly5(fout, 1, 64, 1, 1);
}

/* freq.c:299-308 */
static void port_lpc_weighting(float *lpc, float gamma)
{
  float gamma_i = gamma;
  for (int i = 0; i < LPC_ORDER; i++) {
    lpc[i] *= gamma_i;
    gamma_i *= gamma;
  }
}

/* freq.c:86-127 lpcn_lpc (float build) */
static float lpcn_lpc(float *lpc, float *rc, const float *ac, int p)
{
  float r, error = ac[0];
  memset(lpc, 0, p * sizeof(float));
  memset(rc, 0, p * sizeof(float));
  if (ac[0] != 0) {
    for (int i = 0; i < p; i++) {
      float rr = 0;
      for (int j = 0; j < i; j++) rr += lpc[j] * ac[i - j];
      rr += ac[i + 1];
      r = -rr / error;
      rc[i] = r;
      lpc[i] = r;
      for (int j = 0; j < (i + 1) >> 1; j++) {
        float tmp1 = lpc[j], tmp2 = lpc[i - 1 - j];
        lpc[j] = tmp1 + r * tmp2;
        lpc[i - 1 - j] = tmp2 + r * tmp1;
      }
      error = error - (r * r) * error;
      if (error < .001f * ac[0]) break;
    }
  }
  return error;
}

/* freq.c:310-320 (with idct :230-240, lpc_from_bands :275-297,
 * interp_band_gain :202-216, inverse_transform :256-273) */
static float port_lpc_from_cepstrum(float *lpc, const float *cepstrum)
{
  float Ex[NB_BANDS], tmp[NB_BANDS];
  init_tables();
  memcpy(tmp, cepstrum, sizeof(tmp));
  tmp[0] += 4;
  for (int i = 0; i < NB_BANDS; i++) {
    float sum = 0;
    for (int j = 0; j < NB_BANDS; j++) sum += tmp[j] * g_dct[i * NB_BANDS + j];
    Ex[i] = sum * sqrt(2. / NB_BANDS);
  }
  for (int i = 0; i < NB_BANDS; i++) Ex[i] = pow(10.f, Ex[i]) * compensation[i];
  /* lpc_from_bands */
  float Xr[FREQ_SIZE];
  for (int i = 0; i < NB_BANDS - 1; i++) {
    int band_size = (eband5ms[i + 1] - eband5ms[i]) * 4;
    for (int j = 0; j < band_size; j++) {
      float frac = (float)j / band_size;
      Xr[(eband5ms[i] * 4) + j] = (1 - frac) * Ex[i] + frac * Ex[i + 1];
    }
  }
  Xr[FREQ_SIZE - 1] = 0;
  cpx x[WINDOW_SIZE], y[WINDOW_SIZE];
  for (int i = 0; i < FREQ_SIZE; i++) { x[i].r = Xr[i]; x[i].i = 0; }
  for (int i = FREQ_SIZE; i < WINDOW_SIZE; i++) {
    x[i].r = x[WINDOW_SIZE - i].r;
    x[i].i = -x[WINDOW_SIZE - i].i;
  }
  fft320(x, y);
  float ac[LPC_ORDER + 1], rc[LPC_ORDER];
  ac[0] = WINDOW_SIZE * y[0].r;
  for (int i = 1; i < LPC_ORDER + 1; i++) ac[i] = WINDOW_SIZE * y[WINDOW_SIZE - i].r;
  ac[0] += ac[0] * 1e-4 + 320 / 12 / 38.;
  for (int i = 1; i < LPC_ORDER + 1; i++) ac[i] *= (1 - 6e-5 * i * i);
  return lpcn_lpc(lpc, rc, ac, LPC_ORDER);
}

static const oracle_kernels g_port = {
  port_vec_tanh, port_vec_sigmoid, oracle_tanh, port_sgemv16, port_sparse8x4_i8, port_dense8x4_i8,
  port_sparse8x4_f32, port_lin2ulaw, port_ulaw2lin, port_rng_srand, port_rng_rand,
  port_lpc_from_cepstrum, port_lpc_weighting,
};

const oracle_kernels *oracle_port_kernels(void) { return &g_port; }

/* ------------------------------------------------------------------------ */
/* Weight blob (nnet.h:54-61, parse_lpcnet_weights.c:36-113)                 */
typedef struct {
  char head[4];
  int version, type, size, block_size;
  char name[44];
} whead;

typedef struct {
  const char *name;
  int size;
  const void *data;
} warray;

static int parse_blob(warray *list, int cap, const unsigned char *data, int len)
{
  int n = 0;
  while (len > 0) {
    const whead *h = (const whead *)data;
    if (len < 64 || h->block_size < h->size || h->block_size > len - 64 || h->name[43] != 0 || h->size < 0) return -1;
    if (h->size > 0) {
      if (n >= cap) return -1;
      list[n].name = h->name;
      list[n].size = h->size;
      list[n].data = data + 64;
      n++;
    } else {
      return -1; /* parse_weights treats a zero-size record as an error */
    }
    data += h->block_size + 64;
    len -= h->block_size + 64;
  }
  return n;
}

static const void *find_arr(const warray *l, int n, const char *name, int size)
{
  for (int i = 0; i < n; i++)
    if (strcmp(l[i].name, name) == 0) return l[i].size == size ? l[i].data : NULL;
  return NULL;
}

static const int *find_idx(const warray *l, int n, const char *name, int nb_in, int nb_out, int *total)
{
  for (int i = 0; i < n; i++) {
    if (strcmp(l[i].name, name) != 0) continue;
    const int *idx = (const int *)l[i].data;
    int remain = l[i].size / (int)sizeof(int);
    *total = 0;
    while (remain > 0) {
      int nb = *idx++;
      /* nb < 0 and pos < 0: the reference's find_idx_check loops forever /
       * accepts an out-of-bounds block here; rejected */
      if (nb < 0 || remain < nb + 1) return NULL;
      for (int k = 0; k < nb; k++) {
        int pos = *idx++;
        if (pos + 3 >= nb_in || (pos & 3) || pos < 0) return NULL;
      }
      nb_out -= 8;
      remain -= nb + 1;
      *total += nb;
    }
    if (nb_out != 0) return NULL;
    return (const int *)l[i].data;
  }
  return NULL;
}

/* ------------------------------------------------------------------------ */
/* Synthesis state (lpcnet_private.h:28-48)                                  */
struct OracleState {
  const oracle_kernels *k;
  int variant;
  unsigned char *blob;
  /* model (pointers into blob) */
  const float *conv1_w, *conv1_b, *conv2_w, *conv2_b, *dense1_w, *dense1_b, *dense2_w, *dense2_b;
  const float *gadf_w, *gadf_b, *gbdf_w, *gbdf_b, *embed_pitch, *emb_sig, *emb_pred, *emb_exc;
  const float *ga_bias, *ga_subias, *ga_diag;
  const void *ga_w;
  const int *ga_idx;
  const float *gb_bias, *gb_subias;
  const void *gb_w, *gb_rec;
  const int *gb_idx;
  const float *fc_w, *fc_b, *fc_factor;
  float logit_table[256];
  /* model constants (nnet_data.h #defines, dump_lpcnet.py:423-446) */
  float lpc_gamma;
  int delay, end2end;
  oracle_rng rng;
  /* dynamic state (cleared by reset) */
  float conv1_mem[FRAME_INPUT * (CONV_K - 1)];
  float conv2_mem[COND * (CONV_K - 1)];
  float gru_a_state[NA];
  float gru_b_state[NB];
  int last_exc;
  float last_sig[LPC_ORDER];
  float old_lpc[MAX_FEATURES_DELAY][LPC_ORDER];
  float gru_a_cond[3 * NA];
  float gru_b_cond[3 * NB];
  int frame_count;
  float deemph_mem;
  float lpc[LPC_ORDER];
  float feature_buffer[NB_FEATURES * MAX_FEATURE_BUFFER_SIZE]; /* lpcnet_private.h:37-38 */
  int feature_buffer_fill;
  /* trace */
  float *t_logits;
  int *t_exc;
  uint32_t *t_rng;
  /* 1.6 kb/s decoder: codebooks (generated ceps_codebooks.c in the
   * reference, optional blob records here) and LPCNetDecState::vq_mem */
  const float *cb1, *cb2, *cb3, *cbd;
  float vq_mem[NB_BANDS];
};

OracleState *oracle_create(const unsigned char *blob, int len, int variant, const oracle_kernels *k)
{
  warray list[64];
  int tot;
  OracleState *st = (OracleState *)calloc(1, sizeof(OracleState));
  if (!st) return NULL;
  st->k = k ? k : &g_port;
  st->variant = variant;
  st->blob = (unsigned char *)malloc(len > 0 ? len : 1);
  memcpy(st->blob, blob, len);
  int n = parse_blob(list, 64, st->blob, len);
  int q = variant == ORACLE_FP32 ? 4 : 1; /* sizeof(qweight) */
  if (n < 0) goto fail;
#define F(dst, name, cnt) if (!(dst = (const float *)find_arr(list, n, name, (cnt) * 4))) goto fail
  F(st->conv1_w, "feature_conv1_weights", CONV_K * FRAME_INPUT * COND);
  F(st->conv1_b, "feature_conv1_bias", COND);
  F(st->conv2_w, "feature_conv2_weights", CONV_K * COND * COND);
  F(st->conv2_b, "feature_conv2_bias", COND);
  F(st->dense1_w, "feature_dense1_weights", COND * COND);
  F(st->dense1_b, "feature_dense1_bias", COND);
  F(st->dense2_w, "feature_dense2_weights", COND * COND);
  F(st->dense2_b, "feature_dense2_bias", COND);
  F(st->gadf_w, "gru_a_dense_feature_weights", COND * 3 * NA);
  F(st->gadf_b, "gru_a_dense_feature_bias", 3 * NA);
  F(st->gbdf_w, "gru_b_dense_feature_weights", COND * 3 * NB);
  F(st->gbdf_b, "gru_b_dense_feature_bias", 3 * NB);
  F(st->embed_pitch, "embed_pitch_weights", 256 * EMBED_PITCH);
  { const float *unused; F(unused, "embed_sig_weights", 256 * 128); (void)unused; }
  F(st->emb_sig, "gru_a_embed_sig_weights", 256 * 3 * NA);
  F(st->emb_pred, "gru_a_embed_pred_weights", 256 * 3 * NA);
  F(st->emb_exc, "gru_a_embed_exc_weights", 256 * 3 * NA);
  F(st->ga_bias, "sparse_gru_a_bias", 6 * NA);
  F(st->ga_subias, "sparse_gru_a_subias", 6 * NA);
  F(st->ga_diag, "sparse_gru_a_recurrent_weights_diag", 3 * NA);
  if (!(st->ga_idx = find_idx(list, n, "sparse_gru_a_recurrent_weights_idx", NA, 3 * NA, &tot))) goto fail;
  if (!(st->ga_w = find_arr(list, n, "sparse_gru_a_recurrent_weights", 32 * tot * q))) goto fail;
  F(st->gb_bias, "gru_b_bias", 6 * NB);
  F(st->gb_subias, "gru_b_subias", 6 * NB);
  if (!(st->gb_idx = find_idx(list, n, "gru_b_weights_idx", NA, 3 * NB, &tot))) goto fail;
  if (!(st->gb_w = find_arr(list, n, "gru_b_weights", 32 * tot * q))) goto fail;
  if (!(st->gb_rec = find_arr(list, n, "gru_b_recurrent_weights", 3 * NB * NB * q))) goto fail;
  F(st->fc_b, "dual_fc_bias", 2 * NLEVELS);
  F(st->fc_w, "dual_fc_weights", NB * 2 * NLEVELS);
  F(st->fc_factor, "dual_fc_factor", 2 * NLEVELS);
#undef F
  /* optional decoder codebooks (lpcnet_private.h:109-112; sizes lpcnet_enc.c:109-119, 709) */
  st->cb1 = (const float *)find_arr(list, n, "ceps_codebook1", 1024 * NB_BANDS_1 * 4);
  st->cb2 = (const float *)find_arr(list, n, "ceps_codebook2", 1024 * NB_BANDS_1 * 4);
  st->cb3 = (const float *)find_arr(list, n, "ceps_codebook3", 1024 * NB_BANDS_1 * 4);
  st->cbd = (const float *)find_arr(list, n, "ceps_codebook_diff4", 4096 * NB_BANDS * 4);
  st->lpc_gamma = 1.f;
  st->delay = FEATURES_DELAY;
  st->end2end = 0;
  /* lpcnet.c:188-191 */
  for (int i = 0; i < 256; i++) {
    float prob = .025f + .95f * i / 255.f;
    st->logit_table[i] = -log((1 - prob) / prob);
  }
  oracle_reset(st);
  return st;
fail:
  free(st->blob);
  free(st);
  return NULL;
}

void oracle_destroy(OracleState *st)
{
  if (!st) return;
  free(st->blob);
  free(st);
}

/* lpcnet.c:174-182 */
void oracle_reset(OracleState *st)
{
  memset(st->conv1_mem, 0, (char *)&st->t_logits - (char *)st->conv1_mem);
  st->last_exc = st->k->lin2ulaw(0.f);
  st->k->rng_srand(&st->rng, (const unsigned char *)"LPCNet", 6);
}

int oracle_set_constants(OracleState *st, float lpc_gamma, int features_delay, int end2end)
{
  if (features_delay < 0 || features_delay > MAX_FEATURES_DELAY || (end2end != 0 && end2end != 1)) return -1;
  st->lpc_gamma = lpc_gamma;
  st->delay = features_delay;
  st->end2end = end2end;
  return 0;
}

void oracle_set_trace(OracleState *st, float *logits8, int *exc, uint32_t *rng_words2)
{
  st->t_logits = logits8;
  st->t_exc = exc;
  st->t_rng = rng_words2;
}

void oracle_get_frame(const OracleState *st, float *a, float *b, float *lpc)
{
  if (a) memcpy(a, st->gru_a_cond, sizeof(st->gru_a_cond));
  if (b) memcpy(b, st->gru_b_cond, sizeof(st->gru_b_cond));
  if (lpc) memcpy(lpc, st->lpc, sizeof(st->lpc));
}

int oracle_frame_count(const OracleState *st) { return st->frame_count; }

void oracle_get_state(const OracleState *st, float *a, float *b)
{
  if (a) memcpy(a, st->gru_a_state, sizeof(st->gru_a_state));
  if (b) memcpy(b, st->gru_b_state, sizeof(st->gru_b_state));
}

/* nnet.c:122-135 _lpcnet_compute_dense (all row counts here are multiples of 16) */
static void dense(const OracleState *st, float *out, const float *w, const float *b, int nin, int nout, int tanh_act, const float *in)
{
  for (int i = 0; i < nout; i++) out[i] = b[i];
  st->k->sgemv16(out, w, nout, nin, nout, in);
  if (tanh_act) st->k->vec_tanh(out, out, nout);
}

/* nnet.c:452-470 compute_conv1d */
static void conv1d(const OracleState *st, float *out, float *mem, const float *w, const float *b, int nin, const float *in)
{
  float tmp[COND * CONV_K];
  memcpy(tmp, mem, nin * (CONV_K - 1) * sizeof(float));
  memcpy(&tmp[nin * (CONV_K - 1)], in, nin * sizeof(float));
  for (int i = 0; i < COND; i++) out[i] = b[i];
  st->k->sgemv16(out, w, COND, nin * CONV_K, COND, tmp);
  st->k->vec_tanh(out, out, COND);
  memcpy(mem, &tmp[nin], nin * (CONV_K - 1) * sizeof(float));
}

/* lpcnet.c:56-80 rc2lpc (END2END models), as written */
static void rc2lpc(float *lpc, const float *rc)
{
  float tmp[LPC_ORDER], ntmp[LPC_ORDER] = {0};
  memcpy(tmp, rc, sizeof(tmp));
  for (int i = 0; i < LPC_ORDER; i++) {
    for (int j = 0; j <= i - 1; j++) ntmp[j] = tmp[j] + tmp[i] * tmp[i - j - 1];
    for (int k = 0; k <= i - 1; k++) tmp[k] = ntmp[k];
  }
  for (int i = 0; i < LPC_ORDER; i++) lpc[i] = tmp[i];
}

/* lpcnet.c:82-120 run_frame_network */
static void run_frame_network(OracleState *st, float *gru_a_condition, float *gru_b_condition, float *lpc,
                              const float *features)
{
  float in[FRAME_INPUT], conv1_out[COND], conv2_out[COND], dense1_out[COND], condition[COND];
  int pitch = (int)floor(.1 + 50 * features[18] + 100);
  pitch = pitch > 255 ? 255 : (pitch < 33 ? 33 : pitch);
  memcpy(in, features, NB_FEATURES * sizeof(float));
  memcpy(&in[NB_FEATURES], &st->embed_pitch[pitch * EMBED_PITCH], EMBED_PITCH * sizeof(float));
  conv1d(st, conv1_out, st->conv1_mem, st->conv1_w, st->conv1_b, FRAME_INPUT, in);
  if (st->frame_count < CONV1_DELAY) memset(conv1_out, 0, sizeof(conv1_out));
  conv1d(st, conv2_out, st->conv2_mem, st->conv2_w, st->conv2_b, COND, conv1_out);
  if (st->frame_count < st->delay) memset(conv2_out, 0, sizeof(conv2_out));
  dense(st, dense1_out, st->dense1_w, st->dense1_b, COND, COND, 1, conv2_out);
  dense(st, condition, st->dense2_w, st->dense2_b, COND, COND, 1, dense1_out);
  dense(st, gru_a_condition, st->gadf_w, st->gadf_b, COND, 3 * NA, 0, condition);
  dense(st, gru_b_condition, st->gbdf_w, st->gbdf_b, COND, 3 * NB, 0, condition);
  if (st->end2end) {
    rc2lpc(lpc, condition); /* lpcnet.c:104,107-108: rc = condition[0..LPC_ORDER) */
  } else if (st->delay > 0) {   /* lpcnet.c:109-112 */
    memcpy(lpc, st->old_lpc[st->delay - 1], LPC_ORDER * sizeof(float));
    memmove(st->old_lpc[1], st->old_lpc[0], (st->delay - 1) * LPC_ORDER * sizeof(float));
    st->k->lpc_from_cepstrum(st->old_lpc[0], features);
  } else {                      /* lpcnet.c:113-114 */
    st->k->lpc_from_cepstrum(lpc, features);
  }
  st->k->lpc_weighting(lpc, st->lpc_gamma); /* lpcnet.c:116-118 */
  if (st->frame_count < 1000) st->frame_count++;
}

/* nnet.c:410-448 compute_sparse_gru */
static void sparse_gru(OracleState *st, float *state, const float *input)
{
  float recur[3 * NA];
  const float *bias = st->variant == ORACLE_INT8 ? &st->ga_subias[3 * NA] : &st->ga_bias[3 * NA];
  float *z = recur, *r = &recur[NA], *h = &recur[2 * NA];
  for (int k = 0; k < 2; k++)
    for (int i = 0; i < NA; i++) recur[k * NA + i] = bias[k * NA + i] + st->ga_diag[k * NA + i] * state[i] + input[k * NA + i];
  for (int i = 0; i < NA; i++) recur[2 * NA + i] = bias[2 * NA + i] + st->ga_diag[2 * NA + i] * state[i];
  if (st->variant == ORACLE_INT8)
    st->k->sparse8x4_i8(recur, (const int8_t *)st->ga_w, 3 * NA, NA, st->ga_idx, state);
  else
    st->k->sparse8x4_f32(recur, (const float *)st->ga_w, 3 * NA, st->ga_idx, state);
  st->k->vec_sigmoid(recur, recur, 2 * NA);
  for (int i = 0; i < NA; i++) h[i] = h[i] * r[i] + input[2 * NA + i];
  st->k->vec_tanh(h, h, NA);
  for (int i = 0; i < NA; i++) state[i] = z[i] * state[i] + (1 - z[i]) * h[i];
}

/* nnet.c:326-372 compute_gruB */
static void gru_b(OracleState *st, const float *cond, float *state, const float *input)
{
  float zrh[3 * NB], recur[3 * NB];
  float *z = zrh, *r = &zrh[NB], *h = &zrh[2 * NB];
  const float *b = st->variant == ORACLE_INT8 ? st->gb_subias : st->gb_bias;
  for (int i = 0; i < 3 * NB; i++) zrh[i] = b[i] + cond[i];
  if (st->variant == ORACLE_INT8)
    st->k->sparse8x4_i8(zrh, (const int8_t *)st->gb_w, 3 * NB, NA, st->gb_idx, input);
  else
    st->k->sparse8x4_f32(zrh, (const float *)st->gb_w, 3 * NB, st->gb_idx, input);
  for (int i = 0; i < 3 * NB; i++) recur[i] = b[3 * NB + i];
  if (st->variant == ORACLE_INT8)
    st->k->dense8x4_i8(recur, (const int8_t *)st->gb_rec, 3 * NB, NB, state);
  else
    st->k->sgemv16(recur, (const float *)st->gb_rec, 3 * NB, NB, 3 * NB, state);
  for (int i = 0; i < 2 * NB; i++) zrh[i] += recur[i];
  st->k->vec_sigmoid(zrh, zrh, 2 * NB);
  for (int i = 0; i < NB; i++) h[i] += recur[2 * NB + i] * r[i];
  st->k->vec_tanh(h, h, NB);
  for (int i = 0; i < NB; i++) h[i] = z[i] * state[i] + (1 - z[i]) * h[i];
  for (int i = 0; i < NB; i++) state[i] = h[i];
}

/* nnet.c:163-214 sample_mdense */
static int sample_mdense(OracleState *st, const float *input, float *logits_out, uint32_t *rng_out)
{
  float thresholds[8];
  int val = 0;
  for (int b = 0; b < 8; b += 4) {
    uint32_t r = st->k->rng_rand(&st->rng);
    if (rng_out) rng_out[b / 4] = r;
    thresholds[b] = st->logit_table[r & 0xFF];
    thresholds[b + 1] = st->logit_table[(r >> 8) & 0xFF];
    thresholds[b + 2] = st->logit_table[(r >> 16) & 0xFF];
    thresholds[b + 3] = st->logit_table[(r >> 24) & 0xFF];
  }
  for (int b = 0; b < 8; b++) {
    int i = (1 << b) | val;
    float sum1 = st->fc_b[i], sum2 = st->fc_b[i + NLEVELS];
    for (int j = 0; j < NB; j++) {
      sum1 += st->fc_w[i * 2 * NB + j] * input[j];
      sum2 += st->fc_w[i * 2 * NB + j + NB] * input[j];
    }
    sum1 = st->fc_factor[i] * st->k->tanh1(sum1);
    sum2 = st->fc_factor[NLEVELS + i] * st->k->tanh1(sum2);
    sum1 += sum2;
    if (logits_out) logits_out[b] = sum1;
    int bit = thresholds[b] < sum1;
    val = (val << 1) | bit;
  }
  return val;
}

/* lpcnet.c:146-167 run_sample_network */
static int run_sample_network(OracleState *st, int last_exc, int last_sig, int pred, float *logits, uint32_t *rngw)
{
  float gru_a_input[3 * NA], in_b[NA];
  const float *e1 = &st->emb_sig[last_sig * 3 * NA], *e2 = &st->emb_pred[pred * 3 * NA], *e3 = &st->emb_exc[last_exc * 3 * NA];
  for (int i = 0; i < 3 * NA; i++) gru_a_input[i] = st->gru_a_cond[i] + e1[i] + e2[i] + e3[i]; /* nnet.c:484-491 */
  sparse_gru(st, st->gru_a_state, gru_a_input);
  memcpy(in_b, st->gru_a_state, sizeof(in_b));
  gru_b(st, st->gru_b_cond, st->gru_b_state, in_b);
  return sample_mdense(st, st->gru_b_state, logits, rngw);
}

/* lpcnet.c:235-271 lpcnet_synthesize_tail_impl */
static void synthesize_tail(OracleState *st, short *output, int N, int preload)
{
  if (st->frame_count <= st->delay) {
    memset(output, 0, N * sizeof(short));
    return;
  }
  for (int i = 0; i < N; i++) {
    float pcm, pred = 0;
    int exc;
    for (int j = 0; j < LPC_ORDER; j++) pred -= st->last_sig[j] * st->lpc[j];
    int last_sig_ulaw = st->k->lin2ulaw(st->last_sig[0]);
    int pred_ulaw = st->k->lin2ulaw(pred);
    exc = run_sample_network(st, st->last_exc, last_sig_ulaw, pred_ulaw, st->t_logits ? &st->t_logits[8 * i] : NULL,
                             st->t_rng ? &st->t_rng[2 * i] : NULL);
    if (i < preload) {
      exc = st->k->lin2ulaw(output[i] - PREEMPH * st->deemph_mem - pred);
      pcm = output[i] - PREEMPH * st->deemph_mem;
    } else {
      pcm = pred + st->k->ulaw2lin(exc);
    }
    if (st->t_exc) st->t_exc[i] = exc;
    memmove(&st->last_sig[1], &st->last_sig[0], (LPC_ORDER - 1) * sizeof(float));
    st->last_sig[0] = pcm;
    st->last_exc = exc;
    pcm += PREEMPH * st->deemph_mem;
    st->deemph_mem = pcm;
    if (pcm < -32767) pcm = -32767;
    if (pcm > 32767) pcm = 32767;
    if (i >= preload) output[i] = (short)(int)floor(.5 + pcm);
  }
}

/* lpcnet.c:273-277 */
void oracle_synthesize(OracleState *st, const float *features, short *output, int N, int preload)
{
  run_frame_network(st, st->gru_a_cond, st->gru_b_cond, st->lpc, features);
  synthesize_tail(st, output, N, preload);
}

void oracle_synthesize_tail(OracleState *st, short *output, int N, int preload)
{
  synthesize_tail(st, output, N, preload);
}

/* lpcnet.c:122-132 run_frame_network_deferred; max_buffer_size = the two
 * 3-tap convolutions' kernel_size - 1 each = 4 */
void oracle_frame_deferred(OracleState *st, const float *features)
{
  const int max_buffer_size = (CONV_K - 1) + (CONV_K - 1);
  if (st->feature_buffer_fill == max_buffer_size)
    memmove(st->feature_buffer, &st->feature_buffer[NB_FEATURES], (max_buffer_size - 1) * NB_FEATURES * sizeof(float));
  else
    st->feature_buffer_fill++;
  memcpy(&st->feature_buffer[(st->feature_buffer_fill - 1) * NB_FEATURES], features, NB_FEATURES * sizeof(float));
}

/* lpcnet.c:134-144 run_frame_network_flush: outputs into locals */
void oracle_frame_flush(OracleState *st)
{
  for (int i = 0; i < st->feature_buffer_fill; i++) {
    float lpc[LPC_ORDER], gru_a_condition[3 * NA], gru_b_condition[3 * NB];
    run_frame_network(st, gru_a_condition, gru_b_condition, lpc, &st->feature_buffer[i * NB_FEATURES]);
  }
  st->feature_buffer_fill = 0;
}

/* lpcnet.c:226-233 lpcnet_reset_signal */
void oracle_reset_signal(OracleState *st)
{
  st->deemph_mem = 0;
  st->last_exc = st->k->lin2ulaw(0.f);
  memset(st->last_sig, 0, sizeof(st->last_sig));
  memset(st->gru_a_state, 0, sizeof(st->gru_a_state));
  memset(st->gru_b_state, 0, sizeof(st->gru_b_state));
}

/* The PLC's struct copies (lpcnet_plc.c:223,230): a snapshot of the whole
 * state into / out of caller memory of oracle_state_size() bytes. */
int oracle_state_size(void) { return (int)sizeof(OracleState); }
void oracle_state_save(const OracleState *st, void *buf) { memcpy(buf, st, sizeof(OracleState)); }
void oracle_state_restore(OracleState *st, const void *buf) { memcpy(st, buf, sizeof(OracleState)); }

/* ------------------------------------------------------------------------ */
/* 1.6 kb/s decoder.  Parity unpinned by a reference build: lpcnet_dec.c and
 * common.c include lpcnet_private.h -> the generated nnet_data.h, and the
 * codebooks are generated data (ceps_codebooks.c) absent from the tree. */

typedef struct {
  int byte_pos, bit_pos, max_bytes;
  const unsigned char *chars;
} unpacker;

/* lpcnet_dec.c:52-72 bits_unpack */
static unsigned bits_unpack(unpacker *bits, int nb_bits)
{
  unsigned d = 0;
  while (nb_bits) {
    if (bits->byte_pos == bits->max_bytes) return 0;
    d <<= 1;
    d |= (bits->chars[bits->byte_pos] >> (8 - 1 - bits->bit_pos)) & 1;
    bits->bit_pos++;
    if (bits->bit_pos == 8) {
      bits->bit_pos = 0;
      bits->byte_pos++;
    }
    nb_bits--;
  }
  return d;
}

/* common.c:36-56 single_interp */
static void single_interp(float *x, const float *left, const float *right, int id)
{
  float pred[3 * NB_BANDS];
  for (int i = 0; i < NB_BANDS; i++) pred[i] = .5f * (left[i] + right[i]);
  for (int i = 0; i < NB_BANDS; i++) pred[NB_BANDS + i] = left[i];
  for (int i = 0; i < NB_BANDS; i++) pred[2 * NB_BANDS + i] = right[i];
  for (int i = 0; i < NB_BANDS; i++) x[i] = pred[id * NB_BANDS + i];
}

/* common.c:58-65 perform_double_interp */
static void perform_double_interp(float features[4][NB_TOTAL_FEATURES], const float *mem, int best_id)
{
  best_id += (best_id >= 7); /* FORBIDDEN_INTERP, lpcnet_private.h:23 */
  int id0 = best_id / 3, id1 = best_id % 3;
  single_interp(features[0], mem, features[1], id0);
  single_interp(features[2], features[1], features[3], id1);
}

/* lpcnet_dec.c:81-156 decode_packet.  -1 if the model has no codebooks. */
int oracle_decode_packet(OracleState *st, const unsigned char *buf, float *feat /* [4][NB_TOTAL_FEATURES] */)
{
  float(*features)[NB_TOTAL_FEATURES] = (float(*)[NB_TOTAL_FEATURES])feat;
  if (!st->cb1 || !st->cb2 || !st->cb3 || !st->cbd) return -1;
  unpacker bits = {0, 0, 8, buf};
  int c0_id = bits_unpack(&bits, 7);
  int main_pitch = bits_unpack(&bits, 6);
  int modulation = bits_unpack(&bits, 3);
  int corr_id = bits_unpack(&bits, 2);
  int vq_end[3];
  vq_end[0] = bits_unpack(&bits, 10);
  vq_end[1] = bits_unpack(&bits, 10);
  vq_end[2] = bits_unpack(&bits, 10);
  int vq_mid = bits_unpack(&bits, 13);
  int interp_id = bits_unpack(&bits, 3);
  int voiced = 1;
  float frame_corr, sign;
  for (int i = 0; i < 4; i++) memset(features[i], 0, NB_TOTAL_FEATURES * sizeof(float));
  modulation -= 4;
  if (modulation == -4) {
    voiced = 0;
    modulation = 0;
  }
  if (voiced) frame_corr = 0.3875f + .175f * corr_id;
  else frame_corr = 0.0375f + .075f * corr_id;
  for (int sub = 0; sub < 4; sub++) {
    float p = pow(2.f, main_pitch / 21.) * 32; /* PITCH_MIN_PERIOD, lpcnet_private.h:14 */
    p *= 1.f + modulation / 16.f / 7.f * (2 * sub - 3);
    p = (255 < (33 > p ? 33 : p) ? 255 : (33 > p ? 33 : p)); /* MIN16(255, MAX16(33, p)) */
    features[sub][NB_BANDS] = .02f * (p - 100.f);
    features[sub][NB_BANDS + 1] = frame_corr - .5f;
  }
  features[3][0] = (c0_id - 64) / 4.f;
  for (int i = 0; i < NB_BANDS_1; i++)
    features[3][i + 1] = st->cb1[vq_end[0] * NB_BANDS_1 + i] + st->cb2[vq_end[1] * NB_BANDS_1 + i] +
                         st->cb3[vq_end[2] * NB_BANDS_1 + i];
  sign = 1;
  if (vq_mid >= 4096) {
    vq_mid -= 4096;
    sign = -1;
  }
  for (int i = 0; i < NB_BANDS; i++) features[1][i] = sign * st->cbd[vq_mid * NB_BANDS + i];
  if ((vq_mid & 3) < 2) {
    for (int i = 0; i < NB_BANDS; i++) features[1][i] += .5f * (st->vq_mem[i] + features[3][i]);
  } else if ((vq_mid & 3) == 2) {
    for (int i = 0; i < NB_BANDS; i++) features[1][i] += st->vq_mem[i];
  } else {
    for (int i = 0; i < NB_BANDS; i++) features[1][i] += features[3][i];
  }
  perform_double_interp(features, st->vq_mem, interp_id);
  memcpy(st->vq_mem, &features[3][0], NB_BANDS * sizeof(float));
  return 0;
}

/* lpcnet.c:310-319 lpcnet_decode */
int oracle_decode(OracleState *st, const unsigned char *buf, short *pcm /* [4 * FRAME_SIZE] */)
{
  float features[4][NB_TOTAL_FEATURES];
  if (oracle_decode_packet(st, buf, &features[0][0])) return -1;
  for (int k = 0; k < 4; k++) oracle_synthesize(st, features[k], &pcm[k * FRAME_SIZE], FRAME_SIZE, 0);
  return 0;
}
