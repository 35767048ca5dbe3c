/*
 * ref_kernels_fp32.c -- the reference's fp32 block-sparse kernel
 * (vec_avx.h:861-904, selected by --disable-dot-product / DISABLE_DOT_PROD).
 * TEST INFRASTRUCTURE ONLY; compiled by oracle/Makefile against
 * /root/reference/src/vec_avx.h.
 */
#define DISABLE_DOT_PROD
#include "vec_avx.h"

void ref_sparse8x4_f32(float *out, const float *w, int rows, const int *idx, const float *x)
{
  sparse_sgemv_accum8x4(out, w, rows, 0, idx, x);
}
