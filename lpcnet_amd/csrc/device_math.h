/*
 * device_math.h -- exact x86 AVX2 numerics of the LPCNet synthesis path as
 * CDNA4 device functions, shared by every sample-network kernel.
 * Contract: SURVEY.md Appendix A.  Translation units including this header
 * MUST be compiled with -ffp-contract=off.
 */
#ifndef LPCNET_DEVICE_MATH_H
#define LPCNET_DEVICE_MATH_H

#include <hip/hip_runtime.h>

#include "lpcnet_engine.h"

namespace lpcnet_mi355x {

/* ------------------------------------------------------------------------ */
/* numerics helpers                                                          */

/* rcpps of a Pade denominator from its device table entry T = t + (127 << 23)
 * (kRcpBias; t = rcpps(1.m), see rcp_x86): ldexp(t, 127 - e) as one integer
 * subtraction of the exponent field, flushed to +0 below 2^-126 (a borrow
 * into the sign reads negative).  Identical to the ldexp form for every den
 * in [952.72, +inf] (oracle/checks/exact_identities.c (5)). */
__device__ __forceinline__ float rcp_x86_fix(float x, uint32_t T)
{
  const int q = (int)(T - (__float_as_uint(x) & 0x7f800000u));
  return q < 0x00800000 ? 0.f : __int_as_float(q);
}

/* clamp with _mm256_max_ps(lo, _mm256_min_ps(hi, v)) semantics: NaN stays
 * NaN (the intrinsics return their second operand when unordered) */
__device__ __forceinline__ float clamp_x86(float v, float lo, float hi)
{
  return v != v ? v : __builtin_amdgcn_fmed3f(v, lo, hi);
}

/* rcpps of a Pade denominator in [2^9, 2^126), without the table: the x86
 * entry for mantissa prefix i (11 bits) is 1/(1 + (i + 1/2)/2048) rounded to
 * 12 significant bits (checked against every entry of tests/golden/
 * rcp_x86.bin).  On gfx950, round12(v_rcp_f32(m)) with m = the prefix
 * followed by 0x7FF and the rounding increment 0x3FF reproduces the table
 * (times the exponent) for every prefix and every exponent of that range
 * (tools/probes/rcp12_probe.hip, exhaustive; tests/test_gpu_numerics.py
 * pins it).  Four VALU ops, no LDS read on the activation's critical path. */
__device__ __forceinline__ float rcp12_hw(float den)
{
  const float m = __uint_as_float((__float_as_uint(den) & 0xFFFFF000u) | 0x7FFu);
  return __uint_as_float((__float_as_uint(__builtin_amdgcn_rcpf(m)) + 0x3FFu) & 0xFFFFF800u);
}

/* the same for every Pade denominator: den >= 2^126 (rcpps result below
 * 2^-126, flushed), +inf and NaN (sign bit set or not: the unsigned compare
 * catches both) give +0, as rcp_x86_fix does */
__device__ __forceinline__ float rcp_x86_hw(float den)
{
  return __float_as_uint(den) >= 0x7E800000u ? 0.f : rcp12_hw(den);
}

/* rcpps from the LDS table or (HW) from rcp_x86_hw.  The table costs an
 * LDS read with bank conflicts (random index) and its latency; the hardware
 * form costs a transcendental issue slot and three more VALU ops: HW wins on
 * latency-bound chains (the samplers, one stream per lane), the table on
 * VALU-throughput-bound ones (GRU_A elementwise over 2-4 streams per lane). */
template <bool HW = false>
__device__ __forceinline__ float rcp_x86(float x, const uint32_t *tab)
{
  if constexpr (HW) return rcp_x86_hw(x);
  /* _mm256_rcp_ps of a Pade denominator (its only use, tanh8_approx and
   * sigmoid8_approx): den = fma(fma(D2,X2,D1),X2,D0) with positive D's and
   * X2 = X*X lies in [952.72, +inf] or is NaN.  rcpps there is the
   * table of the top RCP_TABLE_BITS mantissa bits, rebiased; results below
   * 2^-126 (and rcp(+inf)) are +0.  ldexp + flush reproduces it for every
   * such den (oracle/checks/exact_identities.c (4)); a NaN den only occurs
   * with a NaN numerator, whose product stays NaN.  The table load is pinned
   * (empty asm) so the select stays branch-free. */
  uint32_t t = tab[__builtin_amdgcn_ubfe(__float_as_uint(x), 23 - RCP_TABLE_BITS, RCP_TABLE_BITS)];
  asm volatile("" : "+v"(t));
  return rcp_x86_fix(x, t);
}

/* _mm256_min_ps / _mm256_max_ps return the second operand when unordered */
__device__ __forceinline__ float mm_min(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float mm_max(float a, float b) { return a > b ? a : b; }

/* vec_avx.h:393-411 tanh8_approx */
template <bool HW = false>
__device__ __forceinline__ float tanh_x86(float X, const uint32_t *tab)
{
  float X2 = X * X;
  float num = __builtin_fmaf(__builtin_fmaf(0.60863042f, X2, 96.39235687f), X2, 952.52801514f);
  float den = __builtin_fmaf(__builtin_fmaf(11.88600922f, X2, 413.36801147f), X2, 952.72399902f);
  num = num * X;
  den = rcp_x86<HW>(den, tab);
  num = num * den;
  return clamp_x86(num, -1.f, 1.f);
}

/* vec_avx.h:421-440 sigmoid8_approx */
template <bool HW = false>
__device__ __forceinline__ float sigmoid_x86(float X, const uint32_t *tab)
{
  float X2 = X * X;
  float num = __builtin_fmaf(__builtin_fmaf(0.00950985f, X2, 6.02452230f), X2, 238.13200378f);
  float den = __builtin_fmaf(__builtin_fmaf(0.74287558f, X2, 103.34200287f), X2, 952.72399902f);
  num = num * X;
  den = rcp_x86<HW>(den, tab);
  num = __builtin_fmaf(num, den, 0.5f);
  return clamp_x86(num, 0.f, 1.f);
}

/* N independent rcp_x86: all N table reads are issued before any is pinned,
 * so their LDS latencies overlap (rcp_x86's pin alone serialises a chain).
 * TB: the table's index bits.  11 reads a 2,048-entry table of the x86
 * entries themselves (kRcpTable, 11-bit prefixes: mfw_kernel's split form,
 * whose models run with that table only), the default 12 the device table
 * of every other kernel (RCP_ENTRIES, any host's). */
template <int N, bool HW = false, int TB = RCP_TABLE_BITS>
__device__ __forceinline__ void rcp_x86_n(float (&x)[N], const uint32_t *tab)
{
  if constexpr (HW) {
#pragma unroll
    for (int k = 0; k < N; k++) x[k] = rcp_x86_hw(x[k]);
    return;
  }
  uint32_t t[N];
#pragma unroll
  for (int k = 0; k < N; k++) t[k] = tab[__builtin_amdgcn_ubfe(__float_as_uint(x[k]), 23 - TB, TB)];
#pragma unroll
  for (int k = 0; k < N; k++) asm volatile("" : "+v"(t[k]));
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = rcp_x86_fix(x[k], t[k]);
}

/* N sigmoid8_approx / tanh8_approx lanes with one batched rcp (same
 * arithmetic as sigmoid_x86 / tanh_x86, term for term) */
template <int N, bool HW = false>
__device__ __forceinline__ void sigmoid_x86_n(float (&X)[N], const uint32_t *tab)
{
  float num[N], den[N];
#pragma unroll
  for (int k = 0; k < N; k++) {
    const float X2 = X[k] * X[k];
    num[k] = __builtin_fmaf(__builtin_fmaf(0.00950985f, X2, 6.02452230f), X2, 238.13200378f);
    den[k] = __builtin_fmaf(__builtin_fmaf(0.74287558f, X2, 103.34200287f), X2, 952.72399902f);
    num[k] = num[k] * X[k];
  }
  rcp_x86_n<N, HW>(den, tab);
#pragma unroll
  for (int k = 0; k < N; k++) X[k] = clamp_x86(__builtin_fmaf(num[k], den[k], 0.5f), 0.f, 1.f);
}

/* sigmoid8_approx for inputs of the form (float)(int32) * kScale1 (+ another
 * such term): |X| < 2^18, so X2 < 2^36, the Pade denominator lies in
 * [952.72, 2^73) and the numerator is finite.  rcpps of such a denominator
 * never reaches the flush-to-zero range (exponent field <= 200 < 253, see
 * rcp_x86_fix) and no NaN can arise, so the result is rcp_x86 / clamp_x86
 * without the flush select and the NaN select: identical to sigmoid_x86_n
 * for every such input.  Used for the int8 products' z / r gates. */
template <int N, bool HW = false, int TB = RCP_TABLE_BITS>
__device__ __forceinline__ void sigmoid_x86_fin_n(float (&X)[N], const uint32_t *tab)
{
  float num[N], den[N];
  if constexpr (HW) {
#pragma unroll
    for (int k = 0; k < N; k++) {
      const float X2 = X[k] * X[k];
      num[k] = __builtin_fmaf(__builtin_fmaf(0.00950985f, X2, 6.02452230f), X2, 238.13200378f);
      den[k] = __builtin_fmaf(__builtin_fmaf(0.74287558f, X2, 103.34200287f), X2, 952.72399902f);
      num[k] = num[k] * X[k];
    }
#pragma unroll
    for (int k = 0; k < N; k++) X[k] = __builtin_amdgcn_fmed3f(__builtin_fmaf(num[k], rcp12_hw(den[k]), 0.5f), 0.f, 1.f);
    return;
  }
  uint32_t t[N];
#pragma unroll
  for (int k = 0; k < N; k++) {
    const float X2 = X[k] * X[k];
    num[k] = __builtin_fmaf(__builtin_fmaf(0.00950985f, X2, 6.02452230f), X2, 238.13200378f);
    den[k] = __builtin_fmaf(__builtin_fmaf(0.74287558f, X2, 103.34200287f), X2, 952.72399902f);
    num[k] = num[k] * X[k];
    t[k] = tab[__builtin_amdgcn_ubfe(__float_as_uint(den[k]), 23 - TB, TB)];
  }
#pragma unroll
  for (int k = 0; k < N; k++) asm volatile("" : "+v"(t[k]));
#pragma unroll
  for (int k = 0; k < N; k++) {
    const float r = __int_as_float((int)(t[k] - (__float_as_uint(den[k]) & 0x7f800000u)));
    X[k] = __builtin_amdgcn_fmed3f(__builtin_fmaf(num[k], r, 0.5f), 0.f, 1.f);
  }
}

template <int N, bool HW = false, int TB = RCP_TABLE_BITS>
__device__ __forceinline__ void tanh_x86_n(float (&X)[N], const uint32_t *tab)
{
  float num[N], den[N];
#pragma unroll
  for (int k = 0; k < N; k++) {
    const float X2 = X[k] * X[k];
    num[k] = __builtin_fmaf(__builtin_fmaf(0.60863042f, X2, 96.39235687f), X2, 952.52801514f);
    den[k] = __builtin_fmaf(__builtin_fmaf(11.88600922f, X2, 413.36801147f), X2, 952.72399902f);
    num[k] = num[k] * X[k];
  }
  rcp_x86_n<N, HW, TB>(den, tab);
#pragma unroll
  for (int k = 0; k < N; k++) X[k] = clamp_x86(num[k] * den[k], -1.f, 1.f);
}

/* tanh8_approx for finite inputs below 2^60 in magnitude: the Pade
 * denominator lies in [952.72, 2^125), so rcpps never flushes and no NaN
 * arises: rcp_x86 / clamp_x86 without their flush and NaN selects, identical
 * to tanh_x86_n for every such input (mf_kernel's bounded-input path). */
template <int N, bool HW = false, int TB = RCP_TABLE_BITS>
__device__ __forceinline__ void tanh_x86_fin_n(float (&X)[N], const uint32_t *tab)
{
  float num[N], den[N];
#pragma unroll
  for (int k = 0; k < N; k++) {
    const float X2 = X[k] * X[k];
    num[k] = __builtin_fmaf(__builtin_fmaf(0.60863042f, X2, 96.39235687f), X2, 952.52801514f);
    den[k] = __builtin_fmaf(__builtin_fmaf(11.88600922f, X2, 413.36801147f), X2, 952.72399902f);
    num[k] = num[k] * X[k];
  }
  if constexpr (HW) {
#pragma unroll
    for (int k = 0; k < N; k++) X[k] = __builtin_amdgcn_fmed3f(num[k] * rcp12_hw(den[k]), -1.f, 1.f);
    return;
  }
  uint32_t t[N];
#pragma unroll
  for (int k = 0; k < N; k++) t[k] = tab[__builtin_amdgcn_ubfe(__float_as_uint(den[k]), 23 - TB, TB)];
#pragma unroll
  for (int k = 0; k < N; k++) asm volatile("" : "+v"(t[k]));
#pragma unroll
  for (int k = 0; k < N; k++) {
    const float r = __int_as_float((int)(t[k] - (__float_as_uint(den[k]) & 0x7f800000u)));
    X[k] = __builtin_amdgcn_fmed3f(num[k] * r, -1.f, 1.f);
  }
}

/* cvt_rne for |v| < 2^31 (finite): v_cvt_i32_f32 of the rounded value */
__device__ __forceinline__ int cvt_rne_fin(float v)
{
  const float r = __builtin_rintf(v);
  int c;
  asm("v_cvt_i32_f32 %0, %1" : "=v"(c) : "v"(r));
  return c;
}

/* _mm256_cvtps_epi32: round to nearest even, out of range / NaN -> INT_MIN.
 * v_cvt_i32_f32 saturates (-big -> INT_MIN, +big -> INT_MAX) and maps NaN
 * to 0: only r >= 2^31 and NaN need the fix, and both fail r < 2^31. */
__device__ __forceinline__ int cvt_rne(float v)
{
  const float r = __builtin_rintf(v);
  int c;
  asm("v_cvt_i32_f32 %0, %1" : "=v"(c) : "v"(r));
  return r < 2147483648.f ? c : (int)0x80000000u;
}

/* vector_ps_to_epi8 (vec_avx.h:321-336) -> u8, returned XOR 0x80 (= u8-128,
 * the signed form the int8 products consume): cvtps_epi32 then two unsigned
 * saturating packs, i.e. 0 for NaN / r >= 2^31 (INT_MIN) and r <= 0,
 * min(r, 255) otherwise. */
__device__ __forceinline__ uint32_t quant_s8(float x)
{
  /* v_cvt_pk_u8_f32 = min(255, max(0, rne(v))), NaN -> 0 (measured over
   * every 1/64 step of [-4, 258], the halves and the specials:
   * tools/probes/cvt_u8_probe.hip); only v >= 2^31 (-> 255 here, 0 on x86)
   * needs the select */
  const float v = __builtin_fmaf(x, 127.f, 127.f);
  const uint32_t q = __builtin_amdgcn_cvt_pk_u8_f32(v, 0, 0u);
  return (v < 2147483648.f ? q : 0u) ^ 0x80u;
}

/* quant_s8 for GRU states: |x| <= 1 (+ rounding) or NaN by construction
 * (convex combinations of states and tanh outputs; lpcnet_batch_restore_state
 * refuses snapshots outside [-2, 2]), so v = 127 x + 127 < 2^31 and the
 * out-of-range select of quant_s8 is dead: identical for every such x */
__device__ __forceinline__ uint32_t quant_s8_state(float x)
{
  return __builtin_amdgcn_cvt_pk_u8_f32(__builtin_fmaf(x, 127.f, 127.f), 0, 0u) ^ 0x80u;
}

constexpr float kScale = 128.f * 127.f;          /* vec_avx.h:686 */
constexpr float kScale1 = 1.f / 128.f / 127.f;   /* vec_avx.h:687 */
constexpr float kLog256 = 5.5451774445f;         /* common.h:17 */
constexpr float kRcpLog256 = 1.f / kLog256;       /* RN(1/log 256), see lin2ulaw_x86 */
constexpr float kPreemph = 0.85f;                /* lpcnet.c:40 */

/* common.h:18-33, 47-58 lin2ulaw */
__device__ __forceinline__ int lin2ulaw_x86(float x)
{
  const float scale = 255.f / 32768.f;
  int s = x >= 0 ? 1 : -1;
  x = fabsf(x);
  float y = 1 + scale * x;
  uint32_t bits = __float_as_uint(y);
  int integer = (int)(bits >> 23) - 127;
  bits -= (uint32_t)integer << 23;
  float frac = __uint_as_float(bits) - 1.5f;
  frac = -0.41445418f + frac * (0.95909232f + frac * (-0.33951290f + frac * 0.16541097f));
  float l2 = (float)(1 + integer) + frac;
  /* RN(v / log(256)) by one FMA-corrected product: exact for every v in
   * [2^-10, 2^15) (oracle/checks/exact_identities.c); v here is in
   * [0.0395, 11500] */
  const float v = 128.f * (0.69315f * l2);
  const float q0 = v * kRcpLog256;
  const float q = __builtin_fmaf(__builtin_fmaf(-q0, kLog256, v), kRcpLog256, q0);
  float u = (float)s * q;
  u = 128.f + u;
  if (u < 0) u = 0;
  if (u > 255) u = 255;
  /* (int)floor(.5 + (double)u) for u in [0, 255] (exact_identities.c) */
  const int k = (int)u;
  return k + (u - (float)k >= .5f ? 1 : 0);
}

/* (int)floor(.5 + (double)o) for |o| <= 32767 (exact_identities.c) */
__device__ __forceinline__ int round_half_up(float o)
{
  const float k = floorf(o);
  return (int)k + (o - k >= .5f ? 1 : 0);
}

/* kiss99.c:59-81 */
__device__ __forceinline__ uint32_t kiss99_next(uint32_t &z, uint32_t &w, uint32_t &jsr, uint32_t &jcong)
{
  uint32_t znew = 36969u * (z & 0xFFFF) + (z >> 16);
  uint32_t wnew = 18000u * (w & 0xFFFF) + (w >> 16);
  uint32_t mwc = (znew << 16) + wnew;
  uint32_t shr3 = jsr ^ (jsr << 13);
  shr3 ^= shr3 >> 17;
  shr3 ^= shr3 << 5;
  uint32_t cong = 69069u * jcong + 1234567u;
  z = znew; w = wnew; jsr = shr3; jcong = cong;
  return (mwc ^ cong) + shr3;
}

/* maddubs(u8 x, s8 w) pair sums with int16 saturation + madd(ones) for one
 * 4-input group; x given in the XOR-0x80 signed form. */
__device__ __forceinline__ int dot4_sat(uint32_t w, uint32_t xs)
{
  uint32_t xu = xs ^ 0x80808080u;
  int x0 = xu & 0xff, x1 = (xu >> 8) & 0xff, x2 = (xu >> 16) & 0xff, x3 = xu >> 24;
  int w0 = (int)(int8_t)(w & 0xff), w1 = (int)(int8_t)((w >> 8) & 0xff);
  int w2 = (int)(int8_t)((w >> 16) & 0xff), w3 = (int)(int8_t)(w >> 24);
  int p0 = min(max(x0 * w0 + x1 * w1, -32768), 32767);
  int p1 = min(max(x2 * w2 + x3 * w3, -32768), 32767);
  return p0 + p1;
}

template <bool SAT>
__device__ __forceinline__ int dot4(uint32_t w, uint32_t xs, int acc)
{
  if constexpr (SAT) return acc + dot4_sat(w, xs);
  else return __builtin_amdgcn_sdot4((int)w, (int)xs, acc, false);
}

/* rc2lpc (lpcnet.c:56-80, END2END models): the reference's recursion as
 * written, one thread, float products and sums separately rounded (this TU
 * is compiled with -ffp-contract=off). */
__device__ __forceinline__ void rc2lpc_dev(float (&lpc)[NLPC], const float (&rc)[NLPC])
{
  float tmp[NLPC], ntmp[NLPC];
#pragma unroll
  for (int k = 0; k < NLPC; k++) {
    tmp[k] = rc[k];
    ntmp[k] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < NLPC; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) ntmp[j] = tmp[j] + tmp[i] * tmp[i - j - 1];
#pragma unroll
    for (int k = 0; k < i; k++) tmp[k] = ntmp[k];
  }
#pragma unroll
  for (int k = 0; k < NLPC; k++) lpc[k] = tmp[k];
}

/* lpc_weighting (freq.c:299-308) of coefficient k: lpc[k] * gamma^(k+1),
 * the power built as the reference's running float product */
__device__ __forceinline__ float lpc_weight(float v, int k, float gamma)
{
  float gi = gamma;
  for (int m = 0; m < k; m++) gi *= gamma;
  return v * gi;
}

}  // namespace lpcnet_mi355x

#endif
