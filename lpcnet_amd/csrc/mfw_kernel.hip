/*
 * mfw_kernel.hip -- the wide-batch matrix-core sample kernel: three groups of
 * four streams per 896-thread workgroup, three dedicated roles
 * (lpcnet_synthesize_tail_impl, lpcnet.c:235-271; arithmetic term for term
 * mf_kernel's, which is the reference's).
 *
 * mf_kernel / mf2_kernel give one wave the GRU_A unit's whole sample: the
 * embedding gathers, the elementwise step (VALU) and the recurrent product
 * (matrix cores, x words from LDS) run back to back on the same six waves,
 * so at most one of the three resources works at a time and the SIMDs see
 * one or two VALU-issuing waves each (mf2: ~5.1 K cycles per 4-stream phase,
 * ~1.28 K CU-cycles per stream-sample, the ~465 M samples/s plateau).  Here
 * each of the three jobs has waves of its own and a workgroup carries three
 * 4-stream groups one phase apart:
 *   E waves 0..5   (thread = GRU_A unit, mf_unit): gathers + elementwise of
 *                  group p % 3 (nnet.c:484-491, 431-447) -> q(h_A)
 *   S waves 6..7   (one 32-lane half per stream): GRU_B + dual-FC walk of
 *                  group (p - 1) % 3 (nnet.c:326-372, 163-214; lpcnet.c
 *                  244-270) -> the group's next gather indices, PCM out
 *   R waves 8..13  (GRU_A unit rows of wave r = wv - 8, weights in
 *                  registers): W q(h_A) of group (p - 2) % 3 for its next
 *                  sample (nnet.c:441, v_mfma_i32_4x4x4_16b_i8) -> int32
 *                  sums to LDS for the E waves of the next phase
 * one workgroup barrier per phase p; a group's sample takes three phases and
 * every role works on some group in every phase.  Waves sit on SIMDs w % 4:
 * SIMDs 0/1 carry E, E, R, R; SIMDs 2/3 carry E, S, R, so the VALU-heavy E
 * waves are spread 2-2-1-1 and the latency-critical samplers share their
 * SIMD with one E wave only.
 *
 * The R waves run one straight-line instance per (z/r, h) slot-group count
 * (mfw_r_role<Z, H>): weight and column registers sized to the wave's own
 * plan (896 threads leave 128 VGPRs per wave).  The rcpps table is not in
 * LDS (the budget is taken by three groups' conditioning and the R -> E
 * sums): every activation uses the hardware reciprocal, proven equal to the
 * Intel table on every Pade denominator (device_math.h), so models with
 * another host's table, split (long-row) models, preload, trace and stamps
 * run mf2 / mf_kernel (identical results).
 */
#include <hip/hip_runtime.h>

#include <type_traits>

#include "device_math.h"
#include "lpcnet_engine.h"
#include "mf_common.h"
#include "sampler.h"

namespace lpcnet_mi355x {

constexpr int MFW_S = 4;                 /* streams per group */
constexpr int MFW_THREADS = 64 * 14;     /* 6 E + 2 S + 6 R waves */
constexpr int MFW_THREADS_SPLIT = 64 * 16; /* split form: + 2 host waves (MFW_H_WAVES) */
/* split form: the host waves' partial sums [phase parity][gate][MFW_PART_ROWS][S / 2]
 * 64-bit words (two streams each, see mfw_r_role) */
constexpr int MFW_PRT = 2 * 3 * MFW_PART_ROWS * MFW_S * 4;
constexpr int MFW_S_WAVE0 = 6, MFW_R_WAVE0 = 8;

/* MFW_G groups of MFW_S streams per workgroup (2 or 3, see the header) */
template <int MFW_G>
struct MfwLds {
  static constexpr int MFW_GS = MFW_S * MFW_G;                  /* streams per workgroup */
  static constexpr int x = MFW_GS * MF_XSTR;                    /* q(h_A) [group][stream][MF_XSTR] (signed) */
  static constexpr int xb = MFW_GS * NB;                        /* q(h_B) [group][stream][16] */
  static constexpr int sb = MFW_GS * NB * 4;                    /* float h_B [group][stream][16] (walk broadcast) */
  static constexpr int ix = MFW_GS * 16;                        /* gather row byte offsets [group][stream] int4 */
  static constexpr int lpc = MFW_GS * NLPC * 4;                 /* the frame's LPC [group][stream][16] */
  static constexpr int lsr = MFW_GS * NLPC * 4;                 /* last_sig history [group][stream][16] */
  static constexpr int cnd = MFW_G * GA_ROWS * MFW_S * 4;       /* GRU_A conditioning [group][3][NA][S] */
  static constexpr int trm = 2 * 3 * SAMPLE_THREADS * MFW_S * 4;/* R -> E int32 sums [phase parity][gate][lane][S] */
  static constexpr int gbs = MFW_G * MFW_S * GB_ROWS * 4;       /* GRU_B input seeds [group][stream][48] */
  static constexpr int gbr = GB_ROWS * 4;                       /* GRU_B recurrent seeds [48] */
  static constexpr int okw = 2 * MFW_G * 8 * 4;                 /* range words [frame parity][group][E wave] */
  static constexpr int gbw = MF_GB_TILES * 64 * 16;             /* GRU_B A tiles [input 18 | recurrent 3][64] */
  static constexpr int sst = MFW_GS * 8 * 4;                    /* sampler state [group][stream]: kiss99 x4,
                                                                   de-emphasis, pred, last excitation, active */
  static constexpr int pcm = MFW_GS * 16 * 2;                  /* output samples [group][stream][n % 16] */
  static constexpr int total = x + xb + sb + ix + lpc + lsr + cnd + trm + gbs + gbr + okw + gbw + sst + pcm;
};
/* the image sections without the rcpps table: u-law, logit, dual_fc */
constexpr int MFW_IMG = IMG_VAR - IMG_ULAW;
static_assert(MfwLds<3>::total + MFW_IMG <= 160 * 1024, "mfw_kernel LDS");
/* two groups leave room for the rcpps table too: the E waves' activations
 * read it (the VALU-cheaper form mf_kernel<4> / mf2_kernel use at 4
 * streams per lane) instead of the hardware reciprocal */
static_assert(MfwLds<2>::total + IMG_VAR <= 160 * 1024, "mfw_kernel LDS (two groups, table)");

/* split form (two groups): the part area, and the rcpps table in its
 * 2,048-entry form (the x86 entries of the 11-bit prefixes, MFW_RC11 bytes;
 * the split form runs with that table only, see choose_kernel) instead of
 * the device's 4,096 entries.  -DMFW_SPLIT_TAB=0 (A/B): the hardware
 * reciprocal, no table */
#ifndef MFW_SPLIT_TAB
#define MFW_SPLIT_TAB 1
#endif
constexpr int MFW_RC11 = MFW_SPLIT_TAB ? 2048 * 4 : 0;
static_assert(MfwLds<2>::total + MFW_PRT + MFW_IMG + MFW_RC11 <= 160 * 1024, "mfw_kernel LDS (two groups, split)");

int mfw_lds_bytes(int groups, int split)
{
  if (split) return groups == 2 ? MfwLds<2>::total + MFW_PRT + MFW_IMG + MFW_RC11 : 1 << 30;
  return groups == 2 ? MfwLds<2>::total + IMG_VAR : MfwLds<3>::total + MFW_IMG;
}

template <int G>
__device__ __forceinline__ int modg(int p) { return (p % G + G) % G; }

/* keeps the next group's / K tile's LDS reads ahead of the current MFMAs
 * (the scheduler otherwise sinks them to their use) */
#ifdef MFW_NOFENCE
#define MFW_FENCE() do { } while (0)
#else
#define MFW_FENCE() __builtin_amdgcn_sched_barrier(0)
#endif

/* diagnostics (MFW_STAMPS builds only, tools/ab_build.sh): per wave of
 * workgroup 0, the s_memtime cycles spent working vs waiting at the phase
 * barriers over the whole loop, printed by lane 0 */
#ifdef MFW_STAMPS
#define MFW_BAR()                                                  \
  do {                                                             \
    const unsigned long long t0_ = __builtin_amdgcn_s_memtime();   \
    __syncthreads();                                               \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime();   \
    if (st_last) st_work += t0_ - st_last;                         \
    st_wait += t1_ - t0_;                                          \
    st_last = t1_;                                                 \
  } while (0)
#define MFW_STAMP_DECL unsigned long long st_last = 0, st_work = 0, st_wait = 0
/* sections of the S walk: cycles since the previous mark, summed */
#define MFW_SEC_DECL unsigned long long sec_t = 0, sec[6] = {0, 0, 0, 0, 0, 0}
#define MFW_SEC(k)                                                 \
  do {                                                             \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime();    \
    if ((k) > 0) sec[k] += n_ - sec_t;                             \
    sec_t = n_;                                                    \
  } while (0)
#define MFW_SEC_PRINT()                                                                                       \
  do {                                                                                                        \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0)                                                           \
      printf("mfw wave %d S sections per walk: rng+thr %.0f gru_b %.0f act+loads %.0f walk %.0f book %.0f\n", \
             (int)(threadIdx.x >> 6), sec[1] / (double)total, sec[2] / (double)total, sec[3] / (double)total, \
             sec[4] / (double)total, sec[5] / (double)total);                                                \
  } while (0)
#define MFW_STAMP_PRINT(role)                                                                                 \
  do {                                                                                                        \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0)                                                           \
      printf("mfw wave %d %s: work %llu wait %llu per phase %.0f / %.0f\n", (int)(threadIdx.x >> 6), role,   \
             st_work, st_wait, (double)st_work / (MFW_G * total + 1.0), (double)st_wait / (MFW_G * total + 1.0)); \
  } while (0)
#else
#define MFW_BAR() __syncthreads()
#define MFW_STAMP_DECL
#define MFW_STAMP_PRINT(role) do { } while (0)
#define MFW_SEC_DECL
#define MFW_SEC(k) do { } while (0)
#define MFW_SEC_PRINT() do { } while (0)
#endif

/* x word of slot t of a gate whose column quads are packed 4 per word in cw
 * (the mf table's own packing): quad * 4 + the lane's stream offset */
template <int N>
__device__ __forceinline__ uint32_t mfw_x(const unsigned char *xg, const uint32_t (&cw)[N], int t, uint32_t mo)
{
  return *(const uint32_t *)(xg + ((__builtin_amdgcn_ubfe(cw[t >> 2], 8 * (t & 3), 8) << 2) + mo));
}

/* x words of 4-slot groups in flight ahead of the MFMAs (the R waves' LDS
 * reads; -DMFW_XD=n for A/B) */
#ifndef MFW_XD
#define MFW_XD 1
#endif
/* issue priority of the R waves (s_setprio; the S waves run at 3) */
#ifndef MFW_R_PRIO
#define MFW_R_PRIO 0
#endif
/* two groups: the E waves' activations through the LDS rcpps table (1) or
 * the hardware reciprocal (0) */
#ifndef MFW_TAB
#define MFW_TAB 1
#endif
/* split form: host waves on SIMDs 0 / 1 instead of 2 / 3 (A/B) */
#ifndef MFW_H_LOW
#define MFW_H_LOW 0
#endif
/* issue priority of the S waves */
#ifndef MFW_S_PRIO
#define MFW_S_PRIO 3
#endif
/* issue priority of the E waves (split form: MFW_E_PRIO_SPLIT, beside the
 * host waves' 1: +0.8 %, profiles/r06/split_prio_ab_8192.json) */
#ifndef MFW_E_PRIO
#define MFW_E_PRIO 0
#endif
#ifndef MFW_E_PRIO_SPLIT
#define MFW_E_PRIO_SPLIT 1
#endif
/* split form: issue priority of the host waves, the longest role (they
 * share SIMDs 2 / 3 with the S waves at 3 and the R waves at 0): skewed
 * 8,192 streams 464 -> 482 M at 1 or 2 (profiles/r06/split_prio_ab_8192.json) */
#ifndef MFW_HOST_PRIO
#define MFW_HOST_PRIO 1
#endif

/* one gate's product over NG 4-slot groups, NC accumulators (slot k -> k %
 * NC; exact int32, any split), the x words of group g + MFW_XD read while
 * group g's MFMAs run (mf_common.h mf_run with compile-time counts) */
template <int NG, int NC>
__device__ __forceinline__ void mfw_gate(const unsigned char *xg, const uint32_t (&w)[4 * NG],
                                         const uint32_t (&cw)[NG], uint32_t mo, v4i (&a)[NC])
{
  uint32_t x[NG][4];
#pragma unroll
  for (int d = 0; d < MFW_XD && d < NG; d++)
#pragma unroll
    for (int k = 0; k < 4; k++) x[d][k] = mfw_x(xg, cw, 4 * d + k, mo);
#pragma unroll
  for (int g = 0; g < NG; g++) {
    if (g + MFW_XD < NG) {
#pragma unroll
      for (int k = 0; k < 4; k++) x[g + MFW_XD][k] = mfw_x(xg, cw, 4 * (g + MFW_XD) + k, mo);
    }
    /* the next groups' reads stay ahead of this group's products (the
     * scheduler otherwise sinks them below, one exposed LDS round trip per
     * group) */
    MFW_FENCE();
#pragma unroll
    for (int k = 0; k < 4; k++) a[k % NC] = mfma4(x[g][k], w[4 * g + k], a[k % NC]);
    MFW_FENCE();
  }
}

/* z and r interleaved (one chain each), as mf_zr<1> */
template <int NG>
__device__ __forceinline__ void mfw_zr(const unsigned char *xg, const uint32_t (&wz)[4 * NG], const uint32_t (&wr)[4 * NG],
                                       const uint32_t (&cz)[NG], const uint32_t (&cr)[NG], uint32_t mo, v4i &az, v4i &ar)
{
  uint32_t xz[NG][4], xr[NG][4];
#pragma unroll
  for (int d = 0; d < MFW_XD && d < NG; d++)
#pragma unroll
    for (int k = 0; k < 4; k++) {
      xz[d][k] = mfw_x(xg, cz, 4 * d + k, mo);
      xr[d][k] = mfw_x(xg, cr, 4 * d + k, mo);
    }
#pragma unroll
  for (int g = 0; g < NG; g++) {
    if (g + MFW_XD < NG) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        xz[g + MFW_XD][k] = mfw_x(xg, cz, 4 * (g + MFW_XD) + k, mo);
        xr[g + MFW_XD][k] = mfw_x(xg, cr, 4 * (g + MFW_XD) + k, mo);
      }
    }
    MFW_FENCE(); /* as mfw_gate */
#pragma unroll
    for (int k = 0; k < 4; k++) {
      az = mfma4(xz[g][k], wz[4 * g + k], az);
      ar = mfma4(xr[g][k], wr[4 * g + k], ar);
    }
    MFW_FENCE();
  }
}

/* ---- R role: GRU_A recurrent products (nnet.c:441) ------------------------ */
/* HOST (split form, r = 6, 7: the host waves): the lane's piece of another
 * unit's row, accumulated from 0, its int32 partial sums added into that
 * row's part words (prt) instead of stored to trm */
template <int MFW_G, int Z, int H, bool SPLIT = false, bool HOST = false>
__device__ __forceinline__ void mfw_r_role(const SampleArgs &A, unsigned char *xa, int *trm, int r, int lane, int total,
                                           int *prt = nullptr)
{
  /* this lane's weight words and packed column quads (engine.cpp mf tables:
   * z slots 0..15, r 16..31, h 32..63, quads 4 per word after them) */
  uint32_t wz[4 * Z], wr[4 * Z], wh[4 * H], cz[Z], cr[Z], ch[H];
  const uint32_t *mt = (SPLIT ? A.mfw_tab : A.mf) + (size_t)r * MF_LANE_U32 * 64 + lane;
#pragma unroll
  for (int t = 0; t < 4 * Z; t++) {
    wz[t] = mt[t * 64];
    wr[t] = mt[(MF_ZMAX + t) * 64];
  }
#pragma unroll
  for (int t = 0; t < 4 * H; t++) wh[t] = mt[(2 * MF_ZMAX + t) * 64];
#pragma unroll
  for (int k = 0; k < Z; k++) {
    cz[k] = mt[(MF_GA + k) * 64];
    cr[k] = mt[(MF_GA + MF_ZMAX / 4 + k) * 64];
  }
#pragma unroll
  for (int k = 0; k < H; k++) ch[k] = mt[(MF_GA + 2 * MF_ZMAX / 4 + k) * 64];
  int wsz = 0, wsr = 0, wsh = 0;
  uint32_t tgt = 0; /* HOST: part rows of the lane's pieces, 9 bits per gate */
  if constexpr (HOST) {
    const int *fr = A.mfw_frow + SAMPLE_THREADS + (r - SAMPLE_WAVES) * 64 + lane;
    constexpr int FS = SAMPLE_THREADS + 64 * MFW_H_WAVES;
    tgt = (uint32_t)fr[0] | (uint32_t)fr[FS] << 9 | (uint32_t)fr[2 * FS] << 18;
  } else {
    const int i = (SPLIT ? A.mfw_unit : A.mf_unit)[r * 64 + lane];
    wsz = A.ga_wsum[i];
    wsr = A.ga_wsum[NA + i];
    wsh = A.ga_wsum[2 * NA + i];
  }
  /* A operand of lane 4b+m = stream m of the group */
  const uint32_t mo = (uint32_t)(lane & 3) * MF_XSTR;
  const int row = r * 64 + lane;
  __syncthreads(); /* image in LDS */
  __syncthreads(); /* initial q(h_A) of every group */
#if MFW_R_PRIO > 0
  /* the R waves' few VALU ops (x addresses) ahead of the E waves' stream on
   * the shared SIMDs: the MFMAs then run beside the elementwise step */
  __builtin_amdgcn_s_setprio(MFW_R_PRIO);
#endif
#if MFW_HOST_PRIO > 0
  if constexpr (HOST) __builtin_amdgcn_s_setprio(MFW_HOST_PRIO);
#endif
  MFW_STAMP_DECL;
  /* group (p - (G - 1)) mod G: three groups, the group E left two phases
   * ago (S walks it in between); two groups, the group S walks beside */
  for (int p = -1; p <= MFW_G * total; p++) {
    const int g = modg<MFW_G>(p - (MFW_G - 1)), tn = (p - (MFW_G - 1) - g) / MFW_G + 1; /* group, sample whose sums these are */
    if (p >= 0) MFW_BAR(); /* phase p */
    if (tn < 0 || tn >= total) continue;
    const unsigned char *xg = xa + g * MFW_S * MF_XSTR;
    /* keep the column quads packed: otherwise every slot's address is
     * hoisted out of the phase loop (one VGPR per slot, as mf_opaque notes) */
    mf_opaque(cz);
    mf_opaque(cr);
    mf_opaque(ch);
    /* one accumulator per gate: a 4x4x4 MFMA issues every ~13 cycles
     * whether its accumulator chains or not (tools/probes/mfma_timing.hip) */
    v4i vz = {wsz, wsz, wsz, wsz}, vr = {wsr, wsr, wsr, wsr}, vh[1] = {{wsh, wsh, wsh, wsh}};
    mfw_zr<Z>(xg, wz, wr, cz, cr, mo, vz, vr);
    if constexpr (HOST) {
      /* exact LDS adds into the owners' part words, two streams per 64-bit
       * add (hi 2^32 + lo, lo sign-extended: mf_common.h part_add PACK); one
       * piece per lane and gate, lanes without one skip.  z / r go out
       * before the h product, so their adds complete under its MFMAs */
      uint32_t tq = tgt;
      asm volatile("" : "+v"(tq));
      unsigned long long *pp = (unsigned long long *)prt + (p & 1) * 3 * MFW_PART_ROWS * (MFW_S / 2);
      auto padd = [&](int q, const v4i &v) {
        const int t = (int)((tq >> (9 * q)) & 0x1FF);
        if (t != MFW_NOROW)
#pragma unroll
          for (int k = 0; k < MFW_S / 2; k++)
            atomicAdd(&pp[(q * MFW_PART_ROWS + t) * (MFW_S / 2) + k],
                      ((unsigned long long)(uint32_t)v[2 * k + 1] << 32) + (unsigned long long)(long long)v[2 * k]);
      };
      padd(0, vz);
      padd(1, vr);
      mfw_gate<H, 1>(xg, wh, ch, mo, vh);
      padd(2, vh[0]);
    } else {
      mfw_gate<H, 1>(xg, wh, ch, mo, vh);
    }
    if constexpr (HOST) {
    } else {
      /* the sums' LDS address from an opaque row (not hoisted per parity) */
      int rq = row;
      asm volatile("" : "+v"(rq));
      int *tp = trm + (p & 1) * 3 * SAMPLE_THREADS * MFW_S + rq * MFW_S;
      *(int4 *)&tp[0 * SAMPLE_THREADS * MFW_S] = make_int4(vz[0], vz[1], vz[2], vz[3]);
      *(int4 *)&tp[1 * SAMPLE_THREADS * MFW_S] = make_int4(vr[0], vr[1], vr[2], vr[3]);
      *(int4 *)&tp[2 * SAMPLE_THREADS * MFW_S] = make_int4(vh[0][0], vh[0][1], vh[0][2], vh[0][3]);
    }
  }
  __syncthreads(); /* final */
  MFW_STAMP_PRINT("R");
}

template <bool HWR, int MFW_G, bool SPLIT = false>
__global__ __launch_bounds__(SPLIT ? MFW_THREADS_SPLIT : MFW_THREADS) void mfw_kernel(SampleArgs A)
{
  /* the rcpps table in LDS for the E waves: two groups, unsplit, the
   * device table (TAB); the split form, its 2,048-entry form beside the part
   * area (STAB, see mfw_lds_bytes) */
  constexpr bool TAB = MFW_G == 2 && MFW_TAB && !SPLIT;
  constexpr bool STAB = SPLIT && MFW_SPLIT_TAB;
  constexpr int TB = STAB ? 11 : RCP_TABLE_BITS;
  constexpr int NT = SPLIT ? MFW_THREADS_SPLIT : MFW_THREADS;
  static_assert(!SPLIT || MFW_G == 2, "split form: two groups");
  static_assert(HWR, "mfw_kernel: hardware reciprocal only (no rcpps table in LDS)");
  static_assert(MFW_G == 2 || MFW_G == 3, "two or three groups");
  extern __shared__ uint4 lds4[];
  unsigned char *lds = (unsigned char *)lds4;
  using L = MfwLds<MFW_G>;
  constexpr int MFW_GS = L::MFW_GS;
  constexpr int S = MFW_S;
  unsigned char *xa = lds; /* first: every x address fits 16 bits */
  unsigned char *xb = xa + L::x;
  float *sbuf = (float *)(xb + L::xb);
  int *ix = (int *)((unsigned char *)sbuf + L::sb);
  float *lpcb = (float *)((unsigned char *)ix + L::ix);
  float *lsrb = lpcb + MFW_GS * NLPC;
  float *cnd = lsrb + MFW_GS * NLPC;
  int *trm = (int *)(cnd + MFW_G * GA_ROWS * S);
  int *gbs = trm + 2 * 3 * SAMPLE_THREADS * S;
  int *gbr = gbs + MFW_G * S * GB_ROWS;
  int *okw = gbr + GB_ROWS;
  v4i *gbw = (v4i *)(okw + 2 * MFW_G * 8);
  uint32_t *sst = (uint32_t *)(gbw + MF_GB_TILES * 64);
  short *pcms = (short *)(sst + MFW_GS * 8);
  int *prt = (int *)((unsigned char *)pcms + L::pcm); /* split form only (MFW_PRT bytes) */
  constexpr int IMG0 = TAB ? 0 : IMG_ULAW; /* first image byte held in LDS */
  __shared__ uint4 img_s[(IMG_VAR - IMG0) / 16];
  const unsigned char *img = (const unsigned char *)img_s - IMG0; /* section offsets as in the full image */
  const float *ulaw = (const float *)(img + IMG_ULAW);
  __shared__ uint32_t rc11[STAB ? 2048 : 1];
  const uint32_t *rcpt = TAB ? (const uint32_t *)(img + IMG_RCP) : STAB ? rc11 : nullptr;
  const float *logit_tab = ulaw + 256;
  const float *fcw = logit_tab + 256;
  const float *fcb = fcw + 256 * 32;
  const float *fcf = fcb + 512;
  (void)img;

  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int s0 = blockIdx.x * MFW_GS;
  const int nfr = A.nframes > 1 ? A.nframes : 1;
  const int total = nfr * A.N;

  bool active[MFW_GS];
  bool any = false, bad = false;
#pragma unroll
  for (int s = 0; s < MFW_GS; s++) {
    const int sid = s0 + s;
    active[s] = sid < A.nstreams && frame_count_of(A, sid) > A.delay;
    any |= active[s];
  }
  /* a stream's activity by a lane-dependent id (no private-array index) */
  auto active_bit = [&](int sid) { return frame_count_of(A, sid) > A.delay; };
  if (nfr > 1) {
    const FrameCond *cl = A.cond + (size_t)(nfr - 1) * A.nstreams;
#pragma unroll
    for (int s = 0; s < MFW_GS; s++) {
      const int sid = s0 + s;
      bad |= sid < A.nstreams && (frame_count_of(A, cl, sid) > A.delay) != active[s];
    }
    if (bad && tid == 0 && A.status) A.status[0] = STATUS_ACTIVITY; /* plain vector store to the pinned host word */
  }
  if (!any || bad) {
    for (int e = tid; e < MFW_GS * total; e += NT) {
      const int s = e / total, fn = e % total, f = fn / A.N, n = fn % A.N;
      if (s0 + s < A.nstreams) A.pcm[((size_t)f * A.nstreams + s0 + s) * A.N + n] = 0;
    }
    return;
  }
  for (int o = tid; o < (IMG_VAR - IMG0) / 16; o += NT) img_s[o] = A.image[IMG0 / 16 + o];
  if constexpr (STAB) {
    /* entry i of the 11-bit table = the device table's entries 2i, 2i + 1 */
    const uint32_t *dev = (const uint32_t *)A.image + IMG_RCP / 4;
    for (int o = tid; o < 2048; o += NT) rc11[o] = dev[2 * o];
  }

  if (wv >= MFW_R_WAVE0) {
    /* ======================= R role ====================================== */
    int r = wv - MFW_R_WAVE0;
#if MFW_H_LOW
    /* A/B: the host waves on hardware waves 12 / 13 (SIMDs 0 / 1, beside R
     * waves 0 / 1), R waves 4 / 5 on 14 / 15 (SIMDs 2 / 3, beside the
     * samplers) */
    if (SPLIT && r >= 4) r = r < 6 ? r + 2 : r - 2;
#endif
    if constexpr (SPLIT) {
      if (r >= SAMPLE_WAVES) {
        /* ===================== host waves (split form) ===================== */
        switch (A.mfw_nzr[r] * 16 + A.mfw_nh[r]) {
#define MFW_HCASE(Z, H) \
  case Z * 16 + H: mfw_r_role<MFW_G, Z, H, true, true>(A, xa, trm, r, lane, total, prt); break;
#define MFW_HCASES(Z) MFW_HCASE(Z, 1) MFW_HCASE(Z, 2) MFW_HCASE(Z, 3) MFW_HCASE(Z, 4) MFW_HCASE(Z, 5) MFW_HCASE(Z, 6) MFW_HCASE(Z, 7) MFW_HCASE(Z, 8)
          MFW_HCASES(1)
          MFW_HCASES(2)
          MFW_HCASES(3)
          MFW_HCASES(4)
#undef MFW_HCASES
#undef MFW_HCASE
          default: mfw_r_role<MFW_G, MF_ZMAX / 4, MF_HMAX / 4, true, true>(A, xa, trm, r, lane, total, prt); break;
        }
        return;
      }
    }
    const int *nzr_ = SPLIT ? A.mfw_nzr : A.mf_nzr, *nh_ = SPLIT ? A.mfw_nh : A.mf_nh;
    switch (nzr_[r] * 16 + nh_[r]) {
#define MFW_CASE(Z, H) \
  case Z * 16 + H: mfw_r_role<MFW_G, Z, H, SPLIT>(A, xa, trm, r, lane, total); break;
#define MFW_CASES(Z) MFW_CASE(Z, 1) MFW_CASE(Z, 2) MFW_CASE(Z, 3) MFW_CASE(Z, 4) MFW_CASE(Z, 5) MFW_CASE(Z, 6) MFW_CASE(Z, 7) MFW_CASE(Z, 8)
      MFW_CASES(1)
      MFW_CASES(2)
      MFW_CASES(3)
      MFW_CASES(4)
#undef MFW_CASES
#undef MFW_CASE
      default: mfw_r_role<MFW_G, MF_ZMAX / 4, MF_HMAX / 4, SPLIT>(A, xa, trm, r, lane, total); break;
    }
    return;
  }

  if (wv < MFW_S_WAVE0) {
    /* ======================= E role ====================================== */
    const int i = (SPLIT ? A.mfw_unit : A.mf_unit)[tid];
    const float bz = A.ga_par[i], br = A.ga_par[NA + i], bh = A.ga_par[2 * NA + i];
    const float dz = A.ga_par[3 * NA + i], dr = A.ga_par[4 * NA + i], dh = A.ga_par[5 * NA + i];
    float st[MFW_G][S];
#pragma unroll
    for (int g = 0; g < MFW_G; g++)
#pragma unroll
      for (int s = 0; s < S; s++) st[g][s] = A.st[min(s0 + g * S + s, A.nstreams - 1)].gru_a_state[i];
    /* group g's inputs of a frame: its conditioning (lane-private LDS
     * entries) and this wave's range word */
    auto stage = [&](int g, const FrameCond *cf, int par) {
      bool in_range = true;
      float *cg = cnd + g * GA_ROWS * S;
#pragma unroll
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
      if (lane == 0) okw[(par * MFW_G + g) * 8 + wv] = __ballot(!in_range) == 0ull;
    };
#pragma unroll
    for (int g = 0; g < MFW_G; g++) stage(g, A.cond, 0);
    /* split form: this thread's part rows (9 bits per gate) and whether its
     * unit has pieces there (bits 27..29), one register for the launch */
    uint32_t frow = 0;
    if constexpr (SPLIT) {
      constexpr int FS = SAMPLE_THREADS + 64 * MFW_H_WAVES;
      const int *fro = A.mfw_frow + tid;
      const uint32_t e0 = fro[0], e1 = fro[FS], e2 = fro[2 * FS];
      frow = (e0 & 0x1FF) | (e1 & 0x1FF) << 9 | (e2 & 0x1FF) << 18 | (e0 >> 16 & 1) << 27 | (e1 >> 16 & 1) << 28 |
             (e2 >> 16 & 1) << 29;
      for (int e = tid; e < MFW_PRT / 4; e += SAMPLE_THREADS) prt[e] = 0;
    }
    __syncthreads(); /* image in LDS */
#pragma unroll
    for (int g = 0; g < MFW_G; g++)
#pragma unroll
      for (int s = 0; s < S; s++) xa[(g * S + s) * MF_XSTR + i] = (unsigned char)quant_s8_state(st[g][s]);
    __syncthreads(); /* initial q(h_A) of every group */
    if constexpr ((SPLIT ? MFW_E_PRIO_SPLIT : MFW_E_PRIO) > 0) __builtin_amdgcn_s_setprio(SPLIT ? MFW_E_PRIO_SPLIT : MFW_E_PRIO);
    bool fast[MFW_G];
#pragma unroll
    for (int g = 0; g < MFW_G; g++) fast[g] = true;
    MFW_STAMP_DECL;
    /* one group's gathers (nnet.c:484-491) and elementwise step (nnet.c:431-447) */
    auto step = [&](auto gc, int t, int p) {
      constexpr int g = decltype(gc)::value;
      /* addresses formed per step from an opaque thread id (not hoisted
       * into registers for all three groups) */
      int tid = threadIdx.x;
      asm volatile("" : "+v"(tid));
      const int n = t % A.N, par = (t / A.N) & 1;
      if (n == 0) {
        bool f = true;
        for (int w = 0; w < MFW_S_WAVE0; w++) f &= okw[(par * MFW_G + g) * 8 + w] != 0;
        fast[g] = f;
      }
      float e[S][9];
#pragma unroll
      for (int s = 0; s < S; s++) {
        const int4 v = *(const int4 *)(ix + (g * S + s) * 4);
        uint32_t o1 = (uint32_t)tid * 4u + (uint32_t)v.x;
        uint32_t o2 = (uint32_t)tid * 4u + (uint32_t)v.y;
        uint32_t o3 = (uint32_t)tid * 4u + (uint32_t)v.z;
        asm volatile("" : "+v"(o1), "+v"(o2), "+v"(o3));
        const float *const *emb = SPLIT ? A.mfw_emb : A.mf_emb;
        const char *b1 = (const char *)emb[0], *b2 = (const char *)emb[1], *b3 = (const char *)emb[2];
#pragma unroll
        for (uint32_t q = 0; q < 3; q++) {
          e[s][q] = *(const float *)(b1 + o1 + q * NA * 4u);
          e[s][3 + q] = *(const float *)(b2 + o2 + q * NA * 4u);
          e[s][6 + q] = *(const float *)(b3 + o3 + q * NA * 4u);
        }
      }
      /* the R waves' sums of this group (written in the previous phase) */
      const int *tp = trm + ((p - 1) & 1) * 3 * SAMPLE_THREADS * S;
      const int4 iz = *(const int4 *)&tp[(0 * SAMPLE_THREADS + tid) * S];
      const int4 ir = *(const int4 *)&tp[(1 * SAMPLE_THREADS + tid) * S];
      const int4 ih = *(const int4 *)&tp[(2 * SAMPLE_THREADS + tid) * S];
      int vz[4] = {iz.x, iz.y, iz.z, iz.w}, vr[4] = {ir.x, ir.y, ir.z, ir.w}, vh[4] = {ih.x, ih.y, ih.z, ih.w};
      if constexpr (SPLIT) {
        /* the host waves' partial sums of this unit's rows (same phase
         * parity as the R waves' sums), read then cleared for the next use
         * of the parity; exact int32 adds */
        uint32_t fp = frow;
        asm volatile("" : "+v"(fp));
        unsigned long long *pp = (unsigned long long *)prt + ((p - 1) & 1) * 3 * MFW_PART_ROWS * (S / 2);
        int *vg[3] = {vz, vr, vh};
#pragma unroll
        for (int q = 0; q < 3; q++)
          if (fp >> (27 + q) & 1) {
            unsigned long long *w2 = pp + (q * MFW_PART_ROWS + (int)((fp >> (9 * q)) & 0x1FF)) * (S / 2);
#pragma unroll
            for (int k = 0; k < S / 2; k++) {
              /* sum over pieces of hi 2^32 + lo: lo is the low word, the
               * rest hi (|row sums| < 2^24) */
              const unsigned long long t = w2[k];
              const int lo = (int)(uint32_t)t;
              vg[q][2 * k] += lo;
              vg[q][2 * k + 1] += (int)((long long)(t - (unsigned long long)(long long)lo) >> 32);
              w2[k] = 0ull;
            }
          }
      }
      float az[S], ar[S], tz[S], tr[S], hpre[S];
#pragma unroll
      for (int s = 0; s < S; s++) {
        az[s] = (float)vz[s];
        ar[s] = (float)vr[s];
        tz[s] = bz + dz * st[g][s];
        tr[s] = br + dr * st[g][s];
        hpre[s] = (float)(vh[s] + cvt_rne((bh + dh * st[g][s]) * kScale)) * kScale1;
      }
      int stub = 0;
      auto nostamp = [&](int) { (void)stub; };
      const float *cg = cnd + g * GA_ROWS * S;
      if (__builtin_amdgcn_readfirstlane((int)fast[g]))
        ga_elementwise<S, true, !(TAB || STAB), TB>(st[g], e, cg, tid, az, ar, tz, tr, hpre, rcpt, xa + g * S * MF_XSTR + i, false, nostamp);
      else
        ga_elementwise<S, false, !(TAB || STAB), TB>(st[g], e, cg, tid, az, ar, tz, tr, hpre, rcpt, xa + g * S * MF_XSTR + i, false, nostamp);
    };
    using G0 = std::integral_constant<int, 0>;
    using G1 = std::integral_constant<int, 1>;
    using G2 = std::integral_constant<int, 2>;
    for (int p = -1; p <= MFW_G * total; p++) {
      if (p >= 0) MFW_BAR(); /* phase p */
      const int g = modg<MFW_G>(p), t = (p - g) / MFW_G;
      if (p < 0 || t >= total) continue;
      if (g == 0)
        step(G0{}, t, p);
      else if (MFW_G == 2 || g == 1)
        step(G1{}, t, p);
      else if constexpr (MFW_G > 2)
        step(G2{}, t, p);
      if (t % A.N == A.N - 1 && t + 1 < total) {
        /* the next frame's conditioning of this group (its last elementwise
         * step of the frame is done); range words by frame parity, read at
         * the group's next sample */
        const int f = t / A.N;
        stage(g, A.cond + (size_t)(f + 1) * A.nstreams, (f & 1) ^ 1);
      }
    }
    __syncthreads(); /* final */
    MFW_STAMP_PRINT("E");
#pragma unroll
    for (int g = 0; g < MFW_G; g++)
#pragma unroll
      for (int s = 0; s < S; s++)
        if (active[g * S + s]) A.st[s0 + g * S + s].gru_a_state[i] = st[g][s];
    return;
  }

  /* ======================= S role ====================================== */
  /* 128 VGPRs: a stream's sampler state between its samples lives in LDS
   * (history, kiss99, de-emphasis, pred, last excitation), only the GRU_B
   * state (one unit per lane) stays in registers */
  const int sw = wv - MFW_S_WAVE0;
  const int half = lane >> 5, hl = lane & 31;
  const int ms = 2 * sw + half; /* this half's stream within a group */
  /* GRU_B lanes: (stream gs, unit gu) = (lane / 16, lane % 16); states as
   * the MFMA A operand (row m = stream m/4), weight tiles as B: D register 0
   * is unit gu of stream gs (mf_kernel) */
  const int gs = lane >> 4, gu = lane & 15;
  const bool gown = (gs >> 1) == sw;
  float sbv[MFW_G];
#pragma unroll
  for (int g = 0; g < MFW_G; g++) {
    const int sid = min(s0 + g * S + ms, A.nstreams - 1);
    const StreamState *p = &A.st[sid];
    if (hl < NLPC) lsrb[(g * S + ms) * NLPC + hl] = p->last_sig[hl];
    uint32_t *ss = sst + (g * S + ms) * 8;
    if (hl < 4) ss[hl] = p->rng[hl];
    if (hl == 4) ss[4] = __float_as_uint(p->deemph_mem);
    if (hl == 6) ss[6] = (uint32_t)(p->last_exc & 0xFF);
    if (hl == 7) ss[7] = s0 + g * S + ms < A.nstreams && active_bit(s0 + g * S + ms);
    sbv[g] = A.st[min(s0 + g * S + gs, A.nstreams - 1)].gru_b_state[gu];
  }
  /* GRU_B tiles (input 18 then recurrent 3) into LDS, the recurrent seeds */
  for (int e = sw * 64 + lane; e < MF_GB_TILES * 64; e += 128) {
    const uint4 u = A.mf_gb[e];
    gbw[e] = v4i{(int)u.x, (int)u.y, (int)u.z, (int)u.w};
  }
  if (sw == 0 && lane < GB_ROWS) gbr[lane] = cvt_rne(A.gb_par[GB_ROWS + lane] * kScale) + A.gb_wsum[GB_ROWS + lane];
  /* group g's GRU_B input seeds of a frame (nnet.c:347-356 with the
   * offset-128 correction) and its LPC.  Each sampler wave stages its own
   * two streams' seeds: the other wave may still be reading the group's
   * previous ones, and a wave's GRU_B lanes of the other wave's streams are
   * never used (gown) */
  auto stage_frame = [&](int g, const FrameCond *cf) {
    for (int e = lane; e < S * GB_ROWS; e += 64) {
      const int s = e / GB_ROWS, rr = e % GB_ROWS;
      if ((s >> 1) != sw) continue;
      gbs[g * S * GB_ROWS + e] =
          cvt_rne((A.gb_par[rr] + gru_b_cond_of(cf, A, min(s0 + g * S + s, A.nstreams - 1))[rr]) * kScale) + A.gb_wsum[rr];
    }
    if (hl < NLPC) lpcb[(g * S + ms) * NLPC + hl] = lpc_of(cf, A, min(s0 + g * S + ms, A.nstreams - 1))[hl];
  };
  auto ix_word = [](int su, int pu, int exc) { return make_int4(su * (GA_ROWS * 4), pu * (GA_ROWS * 4), exc * (GA_ROWS * 4), 0); };
  /* pred and the u-law indices of group g's next sample (lpcnet.c:252-254)
   * from the history and the frame's LPC */
  auto restart = [&](int g) {
    const float *ls = lsrb + (g * S + ms) * NLPC, *lp = lpcb + (g * S + ms) * NLPC;
    uint32_t *ss = sst + (g * S + ms) * 8;
    float p2 = 0.f;
#pragma unroll
    for (int j = 0; j < NLPC; j++) p2 = p2 - ls[j] * lp[j];
    const int le = (int)ss[6];
    __builtin_amdgcn_wave_barrier();
    if (hl == 0) {
      ss[5] = __float_as_uint(p2);
      *(int4 *)(ix + (g * S + ms) * 4) = ix_word(lin2ulaw_x86(ls[0]), lin2ulaw_x86(p2), le);
    }
  };
#pragma unroll
  for (int g = 0; g < MFW_G; g++) stage_frame(g, A.cond);
  __syncthreads(); /* image in LDS */
#pragma unroll
  for (int g = 0; g < MFW_G; g++)
    if (gown) xb[(g * S + gs) * NB + gu] = (unsigned char)quant_s8_state(sbv[g]);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int g = 0; g < MFW_G; g++) restart(g);
  __syncthreads(); /* initial */
  __builtin_amdgcn_s_setprio(MFW_S_PRIO);

  MFW_SEC_DECL;
  /* group g's GRU_B step and walk of sample t (lpcnet.c:244-270) */
  auto walk = [&](auto gc, int t) {
    constexpr int g = decltype(gc)::value;
    const int n = t % A.N;
    /* the lane's ids from an opaque copy of the lane number: every LDS
     * address below is formed here, per sample, instead of three groups'
     * worth of them hoisted out of the loop into live registers (128 VGPRs:
     * they spilled) */
    int lnq = lane;
    asm volatile("" : "+v"(lnq));
    const int hl = lnq & 31, ms = 2 * sw + (lnq >> 5), gs = lnq >> 4, gu = lnq & 15, sx = gu >> 2;
    const bool gown = (gs >> 1) == sw;
    uint32_t *ss = sst + (g * S + ms) * 8;
    /* this lane's dual-FC round-1 node and weights, read from LDS per
     * sample (registers for the whole loop do not fit 128) */
    MFW_SEC(0);
    FcLane F;
    F.init_sections(nullptr, ulaw, fcw, fcb, fcf, lane);
    uint32_t rz = ss[0], rw = ss[1], rj = ss[2], rc = ss[3];
    const uint32_t r0 = kiss99_next(rz, rw, rj, rc);
    const uint32_t r1 = kiss99_next(rz, rw, rj, rc);
    float t03, t47;
    lane_thresholds(F, logit_tab, r0, r1, t03, t47);
    MFW_SEC(1);
    /* GRU_B (nnet.c:345-361): recurrent product on q(h_B(t-1)), input
     * product on q(h_A(t)), the group's 4 streams as MFMA columns */
    float hh[1], zrb[2];
    {
      v4i acc[3], accr[3];
      const v4i xr = *(const v4i *)(xb + (g * S + sx) * NB); /* k 0..15; the tiles' other K chunks are zero */
#pragma unroll
      for (int q = 0; q < 3; q++) {
        acc[q] = v4i{gbs[(g * S + gs) * GB_ROWS + 16 * q + gu], 0, 0, 0};
        accr[q] = v4i{gbr[16 * q + gu], 0, 0, 0};
      }
#pragma unroll
      for (int q = 0; q < 3; q++) accr[q] = mfma16(xr, gbw[(MF_GB_IN + q) * 64 + lane], accr[q]);
      /* K tile by K tile: its x and three weight tiles from LDS, three
       * MFMAs, tile kt + 1's loads in flight under tile kt's products; the
       * memory clobber keeps the compiler from hoisting all 18 weight tiles
       * (72 VGPRs) ahead of the products */
      const unsigned char *xk0 = xa + (g * S + sx) * MF_XSTR + 16 * gs;
      v4i xk = *(const v4i *)xk0;
      v4i wk[3] = {gbw[lnq], gbw[6 * 64 + lnq], gbw[12 * 64 + lnq]};
#pragma unroll
      for (int kt = 0; kt < 6; kt++) {
        v4i xn, wn[3];
        if (kt + 1 < 6) {
          xn = *(const v4i *)(xk0 + 64 * (kt + 1));
#pragma unroll
          for (int q = 0; q < 3; q++) wn[q] = gbw[(6 * q + kt + 1) * 64 + lnq];
        }
        MFW_FENCE();
#pragma unroll
        for (int q = 0; q < 3; q++) acc[q] = mfma16(xk, wk[q], acc[q]);
        asm volatile("" ::: "memory");
        MFW_FENCE();
        if (kt + 1 < 6) {
          xk = xn;
#pragma unroll
          for (int q = 0; q < 3; q++) wk[q] = wn[q];
        }
      }
      zrb[0] = (float)acc[0][0] * kScale1 + (float)accr[0][0] * kScale1;
      zrb[1] = (float)acc[1][0] * kScale1 + (float)accr[1][0] * kScale1;
      sigmoid_x86_fin_n<2, true>(zrb, nullptr);
      hh[0] = (float)acc[2][0] * kScale1 + ((float)accr[2][0] * kScale1) * zrb[1];
    }
    MFW_SEC(2);
    tanh_x86_fin_n<1, true>(hh, nullptr); /* |hh| < 2^19: int32 sums x 2^-14 */
    sbv[g] = zrb[0] * sbv[g] + (1.f - zrb[0]) * hh[0];
    if (gown) sbuf[(g * S + gs) * NB + gu] = sbv[g];
    float *ls = lsrb + (g * S + ms) * NLPC;
    const float *lp = lpcb + (g * S + ms) * NLPC;
    /* the history shift of lpcnet.c:262-263 in LDS: every lane reads its
     * predecessor's entry before any lane writes (in order within the
     * wave); entry 0 takes the sample after the walk */
    const float lprev = hl >= 1 && hl < NLPC ? ls[hl - 1] : 0.f;
    float xv[NB], lpr[NLPC], lprod[NLPC];
    __builtin_amdgcn_wave_barrier();
    {
      const float4 *b4 = (const float4 *)(sbuf + (g * S + ms) * NB);
      const float4 *s4 = (const float4 *)ls;
      const float4 *l4 = (const float4 *)lp;
      float lsr[NLPC];
#pragma unroll
      for (int j = 0; j < NB / 4; j++) {
        const float4 v = b4[j], u = s4[j], w = l4[j];
        xv[4 * j] = v.x; xv[4 * j + 1] = v.y; xv[4 * j + 2] = v.z; xv[4 * j + 3] = v.w;
        lsr[4 * j] = u.x; lsr[4 * j + 1] = u.y; lsr[4 * j + 2] = u.z; lsr[4 * j + 3] = u.w;
        lpr[4 * j] = w.x; lpr[4 * j + 1] = w.y; lpr[4 * j + 2] = w.z; lpr[4 * j + 3] = w.w;
      }
      lprod[0] = 0.f;
#pragma unroll
      for (int j = 1; j < NLPC; j++) lprod[j] = lsr[j - 1] * lpr[j];
    }
    __builtin_amdgcn_wave_barrier();
    if (hl >= 1 && hl < NLPC) ls[hl] = lprev;
    const float pred = __uint_as_float(ss[5]), deemph0 = __uint_as_float(ss[4]);
    MFW_SEC(3);
    const WalkOut R = dual_fc_walk_p<false, false, true>(F, t03, t47, xv, pred, lprod, lpr, nullptr, deemph0);
    MFW_SEC(4);
    /* bookkeeping (lpcnet.c:262-269) and the output sample */
    float o = R.pcm + kPreemph * deemph0;
    const float dn = o;
    if (o < -32767) o = -32767;
    if (o > 32767) o = 32767;
    if (hl == 0) {
      *(int4 *)(ix + (g * S + ms) * 4) = ix_word(R.su, R.pu, R.exc);
      ls[0] = R.pcm;
      ss[0] = rz; ss[1] = rw; ss[2] = rj; ss[3] = rc;
      ss[4] = __float_as_uint(dn);
      ss[5] = __float_as_uint(R.pn);
      ss[6] = (uint32_t)R.exc;
      /* staged in LDS, stored 16 samples at a time (flush): the global
       * store's address math and kernel-argument reloads sat on every
       * sample's critical path; activity from the state word */
      pcms[(g * S + ms) * 16 + (n & 15)] = ss[7] ? (short)round_half_up(o) : (short)0;
    }
    if (gown) xb[(g * S + gs) * NB + gu] = (unsigned char)quant_s8_state(sbv[g]);
    MFW_SEC(5);
  };
  /* group g's staged samples n0 .. n0 + cnt - 1 of frame f out of LDS,
   * this wave's two streams */
  auto flush = [&](int g, int f, int n0, int cnt) {
    __builtin_amdgcn_wave_barrier();
    const int m = 2 * sw + (lane >> 4), j = lane & 15, sid = s0 + g * S + m;
    if (lane < 32 && j < cnt && sid < A.nstreams) A.pcm[((size_t)f * A.nstreams + sid) * A.N + n0 + j] = pcms[(g * S + m) * 16 + j];
  };
  /* frame boundary of group g after its last sample of frame f: the next
   * frame's seeds and LPC, then pred and the indices of its first sample, as
   * at a launch start (outside walk: inlined there it raised the loop's
   * register pressure past 128) */
  auto boundary = [&](int g, int f) {
    __builtin_amdgcn_wave_barrier();
    stage_frame(g, A.cond + (size_t)(f + 1) * A.nstreams);
    __builtin_amdgcn_wave_barrier();
    restart(g);
  };
  using G0 = std::integral_constant<int, 0>;
  using G1 = std::integral_constant<int, 1>;
  using G2 = std::integral_constant<int, 2>;
  MFW_STAMP_DECL;
  for (int p = -1; p <= MFW_G * total; p++) {
    if (p >= 0) MFW_BAR(); /* phase p */
    const int g = modg<MFW_G>(p - 1), t = (p - 1 - g) / MFW_G;
    if (p < 1 || t >= total) continue;
    if (g == 0)
      walk(G0{}, t);
    else if (MFW_G == 2 || g == 1)
      walk(G1{}, t);
    else if constexpr (MFW_G > 2)
      walk(G2{}, t);
    const int n = t % A.N;
    if ((n & 15) == 15 || n == A.N - 1) flush(g, t / A.N, n & ~15, (n & 15) + 1);
    if (n == A.N - 1 && t / A.N + 1 < nfr) boundary(g, t / A.N);
  }
  __syncthreads(); /* final */
  MFW_STAMP_PRINT("S");
  MFW_SEC_PRINT();
#pragma unroll
  for (int g = 0; g < MFW_G; g++) {
    const int sid = s0 + g * S + ms;
    if (hl == 0 && sid < A.nstreams && active_bit(sid)) {
      StreamState *p = &A.st[sid];
      const uint32_t *ss = sst + (g * S + ms) * 8;
#pragma unroll
      for (int j = 0; j < NLPC; j++) p->last_sig[j] = lsrb[(g * S + ms) * NLPC + j];
      p->deemph_mem = __uint_as_float(ss[4]);
      p->last_exc = (int)ss[6];
      p->rng[0] = ss[0]; p->rng[1] = ss[1]; p->rng[2] = ss[2]; p->rng[3] = ss[3];
    }
    const int gsid = s0 + g * S + gs;
    if (gown && gsid < A.nstreams && active_bit(gsid)) A.st[gsid].gru_b_state[gu] = sbv[g];
  }
}

template <int G, bool SPLIT = false>
static int launch_mfw_g(const SampleArgs &a, void *stream)
{
  using L = MfwLds<G>;
  const int bytes = L::total + (SPLIT ? MFW_PRT : 0);
  if (ensure_dyn_lds((const void *)mfw_kernel<true, G, SPLIT>, bytes)) return -1;
  const int grid = (a.nstreams + L::MFW_GS - 1) / L::MFW_GS;
  hipLaunchKernelGGL((mfw_kernel<true, G, SPLIT>), dim3(grid), dim3(SPLIT ? MFW_THREADS_SPLIT : MFW_THREADS), bytes,
                     (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_mfw(const SampleArgs &a, int groups, void *stream)
{
  if (!a.rcp_hw || a.preload || a.trace_logits || a.stamps) return -1;
  if (a.mf_split) {
    /* split models: the host-wave form, two groups, where its tables exist */
    if (!a.mfw_split || groups != 2) return -1;
    return launch_mfw_g<2, true>(a, stream);
  }
  if (groups == 2) return launch_mfw_g<2>(a, stream);
  if (groups == 3) return launch_mfw_g<3>(a, stream);
  return -1;
}

}  // namespace lpcnet_mi355x
