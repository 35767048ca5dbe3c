/*
 * mf_common.h -- matrix-core building blocks shared by the two int8 sample
 * kernels (mf_kernel.hip, mfp_kernel.hip): register-resident GRU_A weight
 * slots driven through v_mfma_i32_4x4x4_16b_i8 with LDS x words addressed by
 * packed 16-bit offsets, and the v_mfma_i32_16x16x64_i8 GRU_B tiles.
 */
#ifndef LPCNET_MF_COMMON_H
#define LPCNET_MF_COMMON_H

#include <hip/hip_runtime.h>

#include "device_math.h"
#include "lpcnet_engine.h"

namespace lpcnet_mi355x {

typedef int v4i __attribute__((ext_vector_type(4)));

/* Keep packed offsets packed: without this the compiler hoists every
 * unpacked 16-bit offset out of the sample loop (one VGPR per slot). */
template <int N>
__device__ __forceinline__ void mf_opaque(uint32_t (&o)[N])
{
#pragma unroll
  for (int k = 0; k < N; k++) asm volatile("" : "+v"(o[k]));
}

/* x word of slot t: the packed 16-bit LDS byte offsets o[t/2] */
template <int NO>
__device__ __forceinline__ uint32_t mf_x(const unsigned char *lds, const uint32_t (&o)[NO], int t)
{
  return *(const uint32_t *)(lds + ((o[t >> 1] >> (16 * (t & 1))) & 0xFFFF));
}

/* v_mfma_i32_4x4x4_16b_i8, 16 blocks: block b = lanes 4b..4b+3.
 * A (src0) lane 4b+m: 4 int8 of row m (= stream m's x quad of the block's
 * column block); B (src1) lane 4b+n: 4 int8 of column n (= weight row n);
 * D lane 4b+n, register m: sum over k of A[m][k] B[k][n] (exact int32).
 * Layout measured on gfx950 (tools/probes/mfma_i8_probe.hip). */
__device__ __forceinline__ v4i mfma4(uint32_t x, uint32_t w, v4i acc)
{
  return __builtin_amdgcn_mfma_i32_4x4x4i8((int)x, (int)w, acc, 0, 0, 0);
}

/* an optional scheduling fence between a group's next-x reads and its
 * MFMAs (-DMF_SCHED): without it the scheduler may sink the reads below the
 * products.  Measured (same box, alternating): mf_kernel<4> at 1024 streams
 * 3 % slower fenced, mf2_kernel unchanged, so it is off here; mfw_kernel
 * fences its own loops (MFW_FENCE, 1.5-1.7 % faster). */
#ifdef MF_SCHED
#define MF_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define MF_FENCE() do { } while (0)
#endif

/* GRU_A z and r products over ng 4-slot groups (wave-uniform ng): the two
 * gates interleave, each over NC independent accumulators (slot k -> chain
 * k % NC; int32 sums, so any split is the same exact result), x words of
 * group g+1 are read from LDS while the MFMAs of group g run. */
template <int NC>
__device__ __forceinline__ void mf_zr(const unsigned char *lds, const uint32_t (&wz)[MF_ZMAX],
                                      const uint32_t (&wr)[MF_ZMAX], const uint32_t (&oz)[MF_ZMAX / 2],
                                      const uint32_t (&orr)[MF_ZMAX / 2], int ng, v4i (&az)[NC], v4i (&ar)[NC])
{
  uint32_t xz[4], xr[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    xz[k] = mf_x(lds, oz, k);
    xr[k] = mf_x(lds, orr, k);
  }
#pragma unroll
  for (int g = 0; g < MF_ZMAX / 4; g++) {
    if (g < ng) {
      uint32_t nz[4], nr[4];
      if (g + 1 < MF_ZMAX / 4 && g + 1 < ng) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
          nz[k] = mf_x(lds, oz, 4 * (g + 1) + k);
          nr[k] = mf_x(lds, orr, 4 * (g + 1) + k);
        }
      }
      MF_FENCE();
#pragma unroll
      for (int k = 0; k < 4; k++) {
        az[k % NC] = mfma4(xz[k], wz[4 * g + k], az[k % NC]);
        ar[k % NC] = mfma4(xr[k], wr[4 * g + k], ar[k % NC]);
      }
      MF_FENCE();
#pragma unroll
      for (int k = 0; k < 4; k++) {
        xz[k] = nz[k];
        xr[k] = nr[k];
      }
    }
  }
}

/* NS-slot product over ng 4-slot groups over NC accumulators (slot k ->
 * chain k % NC) */
template <int NS, int NC>
__device__ __forceinline__ void mf_run(const unsigned char *lds, const uint32_t (&w)[NS], const uint32_t (&o)[NS / 2],
                                       int ng, v4i (&a)[NC])
{
  uint32_t x[4];
#pragma unroll
  for (int k = 0; k < 4; k++) x[k] = mf_x(lds, o, k);
#pragma unroll
  for (int g = 0; g < NS / 4; g++) {
    if (g < ng) {
      uint32_t n[4];
      if (g + 1 < NS / 4 && g + 1 < ng) {
#pragma unroll
        for (int k = 0; k < 4; k++) n[k] = mf_x(lds, o, 4 * (g + 1) + k);
      }
      MF_FENCE();
#pragma unroll
      for (int k = 0; k < 4; k++) a[k % NC] = mfma4(x[k], w[4 * g + k], a[k % NC]);
      MF_FENCE();
#pragma unroll
      for (int k = 0; k < 4; k++) x[k] = n[k];
    }
  }
}

/* Split models (engine.cpp mf_plan): the z and r products over NO own
 * groups into az / ar and NF hosted groups (a piece of another row) into
 * fz / fr, compile-time counts (a runtime own/hosted choice per group makes
 * the compiler issue the next group's LDS reads only after the current
 * group's MFMAs have drained: measured ~1.7K extra cycles per sample).  x
 * words of group 0 come preloaded in xz / xr; those of group g+1 are read
 * while group g's MFMAs run. */
template <int NO, int NF>
__device__ __forceinline__ void mf_zr_ct(const unsigned char *lds, const uint32_t (&wz)[MF_ZMAX],
                                         const uint32_t (&wr)[MF_ZMAX], const uint32_t (&oz)[MF_ZMAX / 2],
                                         const uint32_t (&orr)[MF_ZMAX / 2], uint32_t (&xz)[4], uint32_t (&xr)[4],
                                         v4i &az, v4i &ar, v4i &fz, v4i &fr)
{
  static_assert(NO + NF <= MF_ZMAX / 4, "z/r groups");
#pragma unroll
  for (int g = 0; g < NO + NF; g++) {
    uint32_t nz[4], nr[4];
    if (g + 1 < NO + NF) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        nz[k] = mf_x(lds, oz, 4 * (g + 1) + k);
        nr[k] = mf_x(lds, orr, 4 * (g + 1) + k);
      }
    }
    MF_FENCE();
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (g < NO) {
        az = mfma4(xz[k], wz[4 * g + k], az);
        ar = mfma4(xr[k], wr[4 * g + k], ar);
      } else {
        fz = mfma4(xz[k], wz[4 * g + k], fz);
        fr = mfma4(xr[k], wr[4 * g + k], fr);
      }
    }
    MF_FENCE();
    if (g + 1 < NO + NF) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        xz[k] = nz[k];
        xr[k] = nr[k];
      }
    }
  }
}

/* the same for the h gate: NO own groups over two chains a[], NF hosted
 * groups over two chains f[] */
template <int NO, int NF>
__device__ __forceinline__ void mf_h_ct(const unsigned char *lds, const uint32_t (&w)[MF_HMAX],
                                        const uint32_t (&o)[MF_HMAX / 2], uint32_t (&x)[4], v4i (&a)[2], v4i (&f)[2])
{
  static_assert(NO + NF <= MF_HMAX / 4, "h groups");
#pragma unroll
  for (int g = 0; g < NO + NF; g++) {
    uint32_t n[4];
    if (g + 1 < NO + NF) {
#pragma unroll
      for (int k = 0; k < 4; k++) n[k] = mf_x(lds, o, 4 * (g + 1) + k);
    }
    MF_FENCE();
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (g < NO)
        a[k & 1] = mfma4(x[k], w[4 * g + k], a[k & 1]);
      else
        f[k & 1] = mfma4(x[k], w[4 * g + k], f[k & 1]);
    }
    MF_FENCE();
    if (g + 1 < NO + NF) {
#pragma unroll
      for (int k = 0; k < 4; k++) x[k] = n[k];
    }
  }
}

/* Split models: a hosted piece's int32 partial sums go to its row's owner
 * through LDS adds into pg: PACK false, [3 gates][NA + 1][S] int32 words (a row's S streams
 * contiguous: one 16-byte read and clear per gate at S = 4); PACK (S even):
 * two streams per 64-bit add ([3][NA + 1][S / 2] words of hi * 2^32 + lo, lo
 * sign-extended).  Summed in 64-bit two's complement over
 * the pieces that is (sum hi) * 2^32 + (sum lo) exactly, and a row's
 * products stay below 384 * 255 * 128 < 2^24 in magnitude, so the low word
 * read as int32 is sum lo and the rest is sum hi: half the LDS atomics of
 * one add per stream.  Measured (three alternating same-box rounds, skewed
 * model): mf2_kernel at 2048 streams 0.6 % faster packed, mf_kernel<4> at
 * 1024 streams 3.5 % slower, so only mf2_kernel packs. */
/* PACK word q of a row: [3 gates][NA + 1][S / 2], a row's words contiguous
 * (one 16-byte read and clear per gate at S = 4: mf2_kernel at 2048 streams
 * -1.1 % against [3][S / 2][NA + 1]) */
#define PIDX(gate, q, row) (((gate) * (NA + 1) + (row)) * (S / 2) + (q))
template <int S, bool PACK>
__device__ __forceinline__ void part_add(int *pg, int gate, int row, const int (&v)[S])
{
  if constexpr (S % 2 == 0 && PACK) {
    unsigned long long *p = (unsigned long long *)pg;
#pragma unroll
    for (int q = 0; q < S / 2; q++)
      atomicAdd(&p[PIDX(gate, q, row)],
                ((unsigned long long)(uint32_t)v[2 * q + 1] << 32) + (unsigned long long)(long long)v[2 * q]);
  } else {
#pragma unroll
    for (int s = 0; s < S; s++) atomicAdd(&pg[(gate * (NA + 1) + row) * S + s], v[s]);
  }
}

/* the owner's side, in two parts so that no branch waits on the reads: the
 * row's hosted sums (v[s]; a row without pieces reads its words, which no
 * piece ever adds to, as 0), then -- only where the row has pieces -- the
 * words cleared for the next sample */
template <int S, bool PACK>
__device__ __forceinline__ void part_read(const int *pg, int gate, int row, int (&v)[S])
{
  if constexpr (S % 2 == 0 && PACK) {
    const unsigned long long *p = (const unsigned long long *)pg;
#pragma unroll
    for (int q = 0; q < S / 2; q++) {
      const unsigned long long t = p[PIDX(gate, q, row)];
      const int lo = (int)(uint32_t)t;
      v[2 * q] = lo;
      v[2 * q + 1] = (int)((long long)(t - (unsigned long long)(long long)lo) >> 32);
    }
  } else if constexpr (S == 4) {
    const int4 t = *(const int4 *)&pg[(gate * (NA + 1) + row) * 4];
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else if constexpr (S == 2) {
    const int2 t = *(const int2 *)&pg[(gate * (NA + 1) + row) * 2];
    v[0] = t.x; v[1] = t.y;
  } else {
#pragma unroll
    for (int s = 0; s < S; s++) v[s] = pg[(gate * (NA + 1) + row) * S + s];
  }
}

template <int S, bool PACK>
__device__ __forceinline__ void part_clear(int *pg, int gate, int row)
{
  if constexpr (S % 2 == 0 && PACK) {
    unsigned long long *p = (unsigned long long *)pg;
#pragma unroll
    for (int q = 0; q < S / 2; q++) p[PIDX(gate, q, row)] = 0;
  } else if constexpr (S == 4) {
    *(int4 *)&pg[(gate * (NA + 1) + row) * 4] = make_int4(0, 0, 0, 0);
  } else if constexpr (S == 2) {
    *(int2 *)&pg[(gate * (NA + 1) + row) * 2] = make_int2(0, 0);
  } else {
#pragma unroll
    for (int s = 0; s < S; s++) pg[(gate * (NA + 1) + row) * S + s] = 0;
  }
}

/* runtime (no, nf) -> the compile-time forms (every count the plan allows) */
__device__ __forceinline__ void mf_zr_split(const unsigned char *lds, const uint32_t (&wz)[MF_ZMAX],
                                            const uint32_t (&wr)[MF_ZMAX], const uint32_t (&oz)[MF_ZMAX / 2],
                                            const uint32_t (&orr)[MF_ZMAX / 2], int no, int nf, uint32_t (&xz)[4],
                                            uint32_t (&xr)[4], v4i &az, v4i &ar, v4i &fz, v4i &fr)
{
  switch (no * 8 + nf) {
#define MF_ZC(O, F)                                                   \
  case O * 8 + F:                                                     \
    mf_zr_ct<O, F>(lds, wz, wr, oz, orr, xz, xr, az, ar, fz, fr);     \
    break;
    MF_ZC(0, 1) MF_ZC(0, 2) MF_ZC(0, 3) MF_ZC(0, 4)
    MF_ZC(1, 0) MF_ZC(1, 1) MF_ZC(1, 2) MF_ZC(1, 3)
    MF_ZC(2, 0) MF_ZC(2, 1) MF_ZC(2, 2)
    MF_ZC(3, 0) MF_ZC(3, 1)
    MF_ZC(4, 0)
#undef MF_ZC
    default: break;
  }
}

__device__ __forceinline__ void mf_h_split(const unsigned char *lds, const uint32_t (&w)[MF_HMAX],
                                           const uint32_t (&o)[MF_HMAX / 2], int no, int nf, uint32_t (&x)[4],
                                           v4i (&a)[2], v4i (&f)[2])
{
  switch (no * 16 + nf) {
#define MF_HC(O, F)                                \
  case O * 16 + F:                                 \
    mf_h_ct<O, F>(lds, w, o, x, a, f);             \
    break;
    MF_HC(0, 1) MF_HC(0, 2) MF_HC(0, 3) MF_HC(0, 4) MF_HC(0, 5) MF_HC(0, 6) MF_HC(0, 7) MF_HC(0, 8)
    MF_HC(1, 0) MF_HC(1, 1) MF_HC(1, 2) MF_HC(1, 3) MF_HC(1, 4) MF_HC(1, 5) MF_HC(1, 6) MF_HC(1, 7)
    MF_HC(2, 0) MF_HC(2, 1) MF_HC(2, 2) MF_HC(2, 3) MF_HC(2, 4) MF_HC(2, 5) MF_HC(2, 6)
    MF_HC(3, 0) MF_HC(3, 1) MF_HC(3, 2) MF_HC(3, 3) MF_HC(3, 4) MF_HC(3, 5)
    MF_HC(4, 0) MF_HC(4, 1) MF_HC(4, 2) MF_HC(4, 3) MF_HC(4, 4)
    MF_HC(5, 0) MF_HC(5, 1) MF_HC(5, 2) MF_HC(5, 3)
    MF_HC(6, 0) MF_HC(6, 1) MF_HC(6, 2)
    MF_HC(7, 0) MF_HC(7, 1)
    MF_HC(8, 0)
#undef MF_HC
    default: break;
  }
}

/* compute_sparse_gru elementwise (nnet.c:431-447) of one GRU_A unit for S
 * streams, from the gathered rows e (nnet.c:484-491 sums in the reference's
 * order), the recurrent sums faz/far, the state terms tz/tr and the recurrent
 * h-gate value hpre; FAST: the range-guarded select-free forms.
 *
 * faz/far are the int32 recurrent sums as floats: a sum over at most 384
 * u8 x s8 products is below 384 * 255 * 128 < 2^24, so the float is exact,
 * and with the seed r = rint((t + in) * SCALE) below 0.99 * 2^31 (the FAST
 * range guard) the int32 sum az + r cannot wrap, so (float)(az + (int)r)
 * = RNE(az + r) = faz + r as one float add: vec_avx.h:804-806,852-854's
 * cvtps_epi32 / add_epi32 / cvtepi32_ps in two VALU ops fewer.  Scalar
 * float ops only: packed v_pk_add/mul_f32 (explicit or SLP-formed -- this
 * file is built with -fno-slp-vectorize) cost more SIMD issue cycles than
 * the scalar pairs, and waves 0/4 and 1/5 share one SIMD's VALU here
 * (measured: 7,450 -> 7,240 cycles per sample at 1024 streams). */
template <int S, bool FAST, bool HW, int TB = RCP_TABLE_BITS, typename Stamp>
__device__ __forceinline__ void ga_elementwise(float (&st)[S], const float (&e)[S][9], const float *cnd, int tid,
                                               const float (&faz)[S], const float (&far)[S], const float (&tz)[S],
                                               const float (&tr)[S], const float (&hpre)[S], const uint32_t *rcp,
                                               unsigned char *xa_i, bool stamping, Stamp &stamp)
{
  (void)stamping;
  (void)stamp;
  float zrv[2 * S], hv[S], inh[S];
  for (int s = 0; s < S; s++) {
    const float inz = ((cnd[tid * S + s] + e[s][0]) + e[s][3]) + e[s][6];
    const float inr = ((cnd[(NA + tid) * S + s] + e[s][1]) + e[s][4]) + e[s][7];
    inh[s] = ((cnd[(2 * NA + tid) * S + s] + e[s][2]) + e[s][5]) + e[s][8];
    if (FAST) {
      zrv[s] = (faz[s] + __builtin_rintf((tz[s] + inz) * kScale)) * kScale1;
      zrv[S + s] = (far[s] + __builtin_rintf((tr[s] + inr) * kScale)) * kScale1;
    } else {
      /* x86's INT_MIN for out-of-range / NaN seeds and the wrapping add */
      zrv[s] = (float)((int)faz[s] + cvt_rne((tz[s] + inz) * kScale)) * kScale1;
      zrv[S + s] = (float)((int)far[s] + cvt_rne((tr[s] + inr) * kScale)) * kScale1;
    }
    hv[s] = hpre[s];
  }
#ifdef MF_FINE
  if (stamping) { float g = 0.f; for (int k = 0; k < 2 * S; k++) g += zrv[k]; asm volatile("" ::"v"(g)); stamp(11); }
#endif
  sigmoid_x86_fin_n<2 * S, HW, TB>(zrv, rcp);
#ifdef MF_FINE
  if (stamping) { float g = 0.f; for (int k = 0; k < 2 * S; k++) g += zrv[k]; asm volatile("" ::"v"(g)); stamp(12); }
#endif
  for (int s = 0; s < S; s++) hv[s] = hv[s] * zrv[S + s] + inh[s];
  if (FAST)
    tanh_x86_fin_n<S, HW, TB>(hv, rcp);
  else
    tanh_x86_n<S, HW, TB>(hv, rcp);
  for (int s = 0; s < S; s++) st[s] = zrv[s] * st[s] + (1.f - zrv[s]) * hv[s];
#ifdef MF_FINE
  if (stamping) { float g = 0.f; for (int k = 0; k < S; k++) g += st[k]; asm volatile("" ::"v"(g)); stamp(13); }
#endif
  for (int s = 0; s < S; s++) xa_i[s * MF_XSTR] = (unsigned char)quant_s8_state(st[s]);
}

/* v_mfma_i32_16x16x64_i8: A (src0) lane l = row l%16, B (src1) lane l =
 * column l%16, the 16 bytes of both = k 16(l/16) + 0..15 (any k permutation
 * common to A and B is the same product); D lane l register i = row
 * 4(l/16)+i, column l%16 (tools/probes/mfma16_probe.hip). */
__device__ __forceinline__ v4i mfma16(const v4i &w, const v4i &x, v4i acc)
{
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(w, x, acc, 0, 0, 0);
}


}  // namespace lpcnet_mi355x

#endif
