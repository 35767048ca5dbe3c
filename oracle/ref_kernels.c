/*
 * ref_kernels.c -- exposes the reference's OWN arithmetic kernels through the
 * oracle_kernels table.  TEST INFRASTRUCTURE ONLY; built by oracle/Makefile
 * into oracle/_ref/libref_kernels.so against the unmodified sources in
 * /root/reference/src (vec_avx.h, common.h, kiss99.c, freq.c, kiss_fft.c,
 * lpcnet_tables.c, pitch.c, burg.c).  Nothing is copied: the reference headers
 * are included from their own directory and the .c files compiled in place.
 *
 * This file holds only thin adapters; every arithmetic operation executed
 * through it is the reference's compiled code (or, for rcpps, the host CPU).
 */
#include <immintrin.h>
#include <string.h>

#include "vec_avx.h" /* /root/reference/src/vec_avx.h (DOT_PROD int8 build) */
#include "common.h"  /* /root/reference/src/common.h (lin2ulaw / ulaw2lin) */
#include "kiss99.h"
#include "freq.h"

#include "lpcnet_oracle.h"

/* from ref_kernels_fp32.c (vec_avx.h compiled with DISABLE_DOT_PROD) */
void ref_sparse8x4_f32(float *out, const float *w, int rows, const int *idx, const float *x);

static void r_vec_tanh(float *y, const float *x, int n) { vec_tanh(y, x, n); }
static void r_vec_sigmoid(float *y, const float *x, int n) { vec_sigmoid(y, x, n); }
static float r_tanh1(float x) { return tanh_approx(x); }
static void r_sgemv16(float *out, const float *w, int rows, int cols, int stride, const float *x)
{
  sgemv_accum16(out, w, rows, cols, stride, x);
}
static void r_sparse8x4_i8(float *out, const int8_t *w, int rows, int cols, const int *idx, const float *x)
{
  sparse_sgemv_accum8x4(out, (const qweight *)w, rows, cols, idx, x);
}
static void r_dense8x4_i8(float *out, const int8_t *w, int rows, int cols, const float *x)
{
  sgemv_accum8x4(out, (const qweight *)w, rows, cols, 3 * rows, x);
}
static int r_lin2ulaw(float x) { return lin2ulaw(x); }
static float r_ulaw2lin(float u) { return ulaw2lin(u); }

/* oracle_rng and kiss99_ctx have the same four uint32 fields in the same order */
static void r_srand(oracle_rng *r, const unsigned char *d, int n) { kiss99_srand((kiss99_ctx *)r, d, n); }
static uint32_t r_rand(oracle_rng *r) { return kiss99_rand((kiss99_ctx *)r); }

static const oracle_kernels g_ref = {
  r_vec_tanh, r_vec_sigmoid, r_tanh1, r_sgemv16, r_sparse8x4_i8, r_dense8x4_i8, ref_sparse8x4_f32,
  r_lin2ulaw, r_ulaw2lin, r_srand, r_rand, lpc_from_cepstrum, lpc_weighting,
};

const oracle_kernels *ref_kernels(void) { return &g_ref; }

/* Tabulates this CPU's rcpps over the 2048 top-11-bit mantissa prefixes of
 * [1,2); returns the number of mantissas that violate the 11-bit property. */
int ref_rcp_table(uint32_t *tab)
{
  int bad = 0;
  for (uint32_t m = 0; m < (1u << 23); m++) {
    uint32_t u = 0x3f800000u | m, r;
    float x;
    memcpy(&x, &u, 4);
    float o[8];
    _mm256_storeu_ps(o, _mm256_rcp_ps(_mm256_set1_ps(x)));
    memcpy(&r, &o[0], 4);
    if ((m & 0xfff) == 0) tab[m >> 12] = r;
    else if (tab[m >> 12] != r) bad++;
  }
  return bad;
}

/* This CPU's rcpps of every float in [1, 2): tab[m] = rcpps(1.m), 2^23
 * entries (the full mantissa table, for hosts whose rcpps is not a function
 * of the top 11 mantissa bits). */
void ref_rcp_full(uint32_t *tab)
{
  for (uint32_t m = 0; m < (1u << 23); m += 8) {
    uint32_t u[8];
    for (int k = 0; k < 8; k++) u[k] = 0x3f800000u | (m + k);
    __m256 v = _mm256_rcp_ps(_mm256_loadu_ps((const float *)u));
    _mm256_storeu_ps((float *)&tab[m], v);
  }
}

/* Single rcpps on this CPU (for spot checks of the emulation). */
float ref_rcp(float x)
{
  float o[8];
  _mm256_storeu_ps(o, _mm256_rcp_ps(_mm256_set1_ps(x)));
  return o[0];
}

/* vector_ps_to_epi8 of the DOT_PROD build */
void ref_quantize_u8(unsigned char *x, const float *xf, int n) { vector_ps_to_epi8(x, xf, n); }
