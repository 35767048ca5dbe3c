/*
 * mf_kernel.hip -- the matrix-core sample kernel: lpcnet_synthesize_tail_impl
 * (lpcnet.c:235-271) for S <= 4 streams per 512-thread workgroup, persistent
 * over the N samples of one frame, or of several frames in one launch
 * (SampleArgs::nframes: no ~10 us dispatch gap and prologue per frame).
 * Default for non-saturating int8 models.
 *
 * Both int8 products run on the matrix cores, from register-resident weights,
 * with exact int32 accumulation (bit-identical to maddubs/madd whenever no
 * u8 x s8 pair can saturate int16 -- checked when the model is loaded):
 *   GRU_A waves 0..5 (thread = unit): the recurrent product of
 *     compute_sparse_gru (nnet.c:441, sparse_sgemv_accum8x4 vec_avx.h:790-858)
 *     on v_mfma_i32_4x4x4_16b_i8 -- 16 independent 4x4x4 blocks per
 *     instruction = 16 row groups x 4 streams of one 8x4-block slot;
 *   sampler waves 6..7: both GRU_B products of compute_gruB (nnet.c:345-361)
 *     on v_mfma_i32_16x16x64_i8 -- 3 gate tiles x 6 K tiles plus 3 recurrent
 *     tiles, dense (zeros where the block-sparse index has no block), all S
 *     streams as the N columns; each sampler wave computes them redundantly
 *     and keeps the GRU_B state in registers, so no barrier separates the
 *     GRU_B step from the sampling.
 * Per sample n, two workgroup barriers:
 *   X  ix(n) published: GRU_A waves gather the embedding rows and run the
 *      GRU_A elementwise step -> q(h_A(n)); samplers: deferred bookkeeping of
 *      n-1, kiss99 draws
 *   Y  q(h_A(n)) complete: GRU_A waves: W q(h_A(n)) for sample n+1;
 *      samplers: GRU_B products + update, dual-FC tree walk -> ix(n+1)
 * The arithmetic is term for term the reference's (see device_math.h).
 */
#include <hip/hip_runtime.h>

#include "device_math.h"
#include "lpcnet_engine.h"
#include "l2_warm.h"
#include "mf_common.h"
#include "sampler.h"

namespace lpcnet_mi355x {

template <int S>
struct MfLds {
  static constexpr int x = S * MF_XSTR;      /* quantized GRU_A state [S][MF_XSTR] (signed form) */
  static constexpr int xb = S * NB;          /* quantized GRU_B state [S][16] */
  static constexpr int sb = S * NB * 4;      /* float GRU_B state [S][16] (tree-walk broadcast) */
  static constexpr int ix = S * 16;          /* sig/pred/exc indices */
  static constexpr int pcm = ((S * FRAME * 2 + 15) / 16) * 16;
  static constexpr int cnd = GA_ROWS * S * 4; /* GRU_A conditioning [3][NA][S] */
  static constexpr int gbs = S * GB_ROWS * 4; /* GRU_B input accumulator seeds [S][48] */
  static constexpr int gbr = GB_ROWS * 4;     /* GRU_B recurrent accumulator seeds [48] */
  static constexpr int okw = 8 * 4;           /* per-GRU_A-wave "inputs in range" words */
  static constexpr int gbw = 3 * 64 * 16;     /* GRU_B recurrent A tiles [3][64 lanes] (LDS, not registers) */
  static constexpr int total = x + xb + sb + ix + pcm + cnd + gbs + gbr + okw + gbw;
  static constexpr int part = 3 * (NA + 1) * S * 4; /* split models: hosted partial sums [3][NA + 1][S] (row NA: none) */
};

int mf_lds_bytes(int S, int split)
{
  const int base = S == 4 ? MfLds<4>::total : (S == 2 ? MfLds<2>::total : MfLds<1>::total);
  const int part = S == 4 ? MfLds<4>::part : (S == 2 ? MfLds<2>::part : MfLds<1>::part);
  return IMG_VAR + base + (split ? part : 0);
}

/* DIAG: 0 the production kernel, 1 with the per-sample logit / excitation
 * trace (SampleArgs::trace_logits), 2 with the s_memtime phase stamps
 * (SampleArgs::stamps): the plain kernel carries no diagnostic branch */
template <int S, int DIAG, bool SPLIT, bool HWR>
__global__ __launch_bounds__(MF_THREADS) void mf_kernel(SampleArgs A)
{
  constexpr bool TRACE = DIAG == 1;
  extern __shared__ uint4 lds4[];
  unsigned char *lds = (unsigned char *)lds4;
  using L = MfLds<S>;
  unsigned char *xa = lds; /* first: every x address fits the 16-bit offsets kept in registers */
  unsigned char *xb = xa + L::x;
  float *sbuf = (float *)(xb + L::xb);
  int *ix = (int *)((unsigned char *)sbuf + L::sb);
  short *pcmbuf = (short *)((unsigned char *)ix + L::ix);
  float *cnd = (float *)((unsigned char *)pcmbuf + L::pcm);
  int *gbs = (int *)((unsigned char *)cnd + L::cnd);
  int *gbr = gbs + S * GB_ROWS;
  int *okw = gbr + GB_ROWS;
  v4i *gbw = (v4i *)(okw + 8);
  int *part = (int *)(gbw + 3 * 64); /* SPLIT: [3][NA + 1][S] (a row's streams contiguous: one 16-byte read per gate at S = 4) */
  /* fixed image sections (rcpps / u-law / logit tables, dual_fc) in static
   * LDS: addresses into dynamic LDS carry an extra add of its base per
   * access, on the activation and walk chains */
  __shared__ uint4 img_s[IMG_VAR / 16];
  unsigned char *img = (unsigned char *)img_s;

  if (l2_warm_role(A.mf_emb, (A.nstreams + S - 1) / S)) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int s0 = blockIdx.x * S;
  const uint32_t *rcp = (const uint32_t *)(img + IMG_RCP);
  /* GRU_A elementwise: one stream per lane is latency-bound (hardware rcp),
   * 2-4 streams per lane are VALU-bound (LDS table) */
  constexpr bool kHwA = S == 1 && HWR;
  constexpr bool kGbwLds = S == 4;

  bool active[S];
  bool any = false;
  for (int s = 0; s < S; s++) {
    const int sid = s0 + s;
    active[s] = sid < A.nstreams && frame_count_of(A, sid) > A.delay;
    any |= active[s];
  }
  /* multi-frame launches (A.nframes > 1): frame f reads cond + f B and
   * writes pcm + f B N, the states stay in registers from frame to frame,
   * the GRU_A waves stage the next frame's inputs (GRU_A conditioning, GRU_B
   * seeds, range words) after the last sample's barrier Y, and one extra
   * barrier separates the frames.  Activity (lpcnet.c:265-268: the first
   * `delay` (FEATURES_DELAY) frames of a stream give zeros and leave its state alone)
   * must be the same in every frame of the launch: the host splits runs at
   * that transition; a launch that sees one anyway reports STATUS_ACTIVITY. */
  const int nfr = A.nframes > 1 ? A.nframes : 1;
  const int total = nfr * A.N;
  bool bad = false;
  if (nfr > 1) {
    const FrameCond *cl = A.cond + (size_t)(nfr - 1) * A.nstreams;
    for (int s = 0; s < S; s++) {
      const int sid = s0 + s;
      bad |= sid < A.nstreams && (frame_count_of(A, cl, sid) > A.delay) != active[s];
    }
    if (bad && tid == 0 && A.status) A.status[0] = STATUS_ACTIVITY; /* plain vector store to the pinned host word */
  }
  if (!any || bad) {
    for (int e = tid; e < S * total; e += MF_THREADS) {
      const int s = e / total, fn = e % total, f = fn / A.N, n = fn % A.N;
      if (s0 + s < A.nstreams) A.pcm[((size_t)f * A.nstreams + s0 + s) * A.N + n] = 0;
    }
    return;
  }
  for (int o = tid; o < IMG_VAR / 16; o += MF_THREADS) img_s[o] = A.image[o];
  for (int e = tid; e < S * A.preload; e += MF_THREADS) {
    const int s = e / A.preload, n = e % A.preload;
    pcmbuf[s * FRAME + n] = A.pcm[(size_t)min(s0 + s, A.nstreams - 1) * A.N + n];
  }

  constexpr bool stamping = DIAG == 2;
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
    /* this lane's GRU_A unit (the host deals 8-unit blocks to the waves for
     * MFMA balance); the embedding tables' columns are stored in lane order */
    const int i = A.mf_unit[tid];
    const float bz = A.ga_par[i], br = A.ga_par[NA + i], bh = A.ga_par[2 * NA + i];
    const float dz = A.ga_par[3 * NA + i], dr = A.ga_par[4 * NA + i], dh = A.ga_par[5 * NA + i];
    const int wsz = A.ga_wsum[i], wsr = A.ga_wsum[NA + i], wsh = A.ga_wsum[2 * NA + i];
    float st[S];
    for (int s = 0; s < S; s++) st[s] = A.st[min(s0 + s, A.nstreams - 1)].gru_a_state[i];
    /* a frame's inputs: the conditioning in LDS by lane
     * position (conflict-free [gate][lane][stream] reads, from the unit's
     * column; read by this thread only: one buffer), the range word of this
     * wave and the GRU_B accumulator seeds (nnet.c:347-356 with the
     * offset-128 correction: cvt_rne((bias + cond) * SCALE) + 128 rowsum(w)) */
    auto stage = [&](const FrameCond *cf) {
      bool in_range = true;
      for (int s = 0; s < S; s++) {
        const int sid = min(s0 + s, A.nstreams - 1);
        const float *ca = gru_a_cond_of(cf, A, sid);
        const float cz = ca[i], cr = ca[NA + i], ch = ca[2 * NA + i];
        cnd[tid * S + s] = cz;
        cnd[(NA + tid) * S + s] = cr;
        cnd[(2 * NA + tid) * S + s] = ch;
        /* NaN fails every compare: such a workgroup takes the exact path */
        in_range &= fabsf(st[s]) <= 2.f && fabsf(cz) <= A.mf_zr_bound && fabsf(cr) <= A.mf_zr_bound &&
                    fabsf(ch) <= A.mf_h_bound;
      }
      if (lane == 0) okw[wv] = __ballot(!in_range) == 0ull;
      for (int e = tid; e < S * GB_ROWS; e += SAMPLE_THREADS) {
        const int s = e / GB_ROWS, r = e % GB_ROWS;
        gbs[e] =
            cvt_rne((A.gb_par[r] + gru_b_cond_of(cf, A, min(s0 + s, A.nstreams - 1))[r]) * kScale) + A.gb_wsum[r];
      }
    };
    const FrameCond *cf = A.cond;
    stage(cf);
    short *pcm_out = A.pcm; /* frame of the next write-out */
    if (tid < GB_ROWS) gbr[tid] = cvt_rne(A.gb_par[GB_ROWS + tid] * kScale) + A.gb_wsum[GB_ROWS + tid];
    /* this lane's GRU_A weight rows and x offsets, for all N samples */
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
      /* A operand of lane 4b+m = stream m (lanes m >= S duplicate stream S-1) */
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
    /* split models: this lane's hosted groups and the rows their partial
     * sums belong to (NA: none) */
    const int nfzr = SPLIT ? A.mf_nfzr[wv] : 0, nfh = SPLIT ? A.mf_nfh[wv] : 0;
    /* split models: the rows this lane's hosted pieces belong to (NA: none),
     * 9 bits per gate, and per gate whether this thread's own unit has
     * hosted pieces to merge (bits 27..29), in one register for the whole
     * launch */
    uint32_t frow = 0;
    if constexpr (SPLIT) {
      const uint32_t *fro = (const uint32_t *)A.mf_frow + tid;
      const uint32_t e0 = fro[0], e1 = fro[SAMPLE_THREADS], e2 = fro[2 * SAMPLE_THREADS];
      frow = (e0 & 0x1FF) | (e1 & 0x1FF) << 9 | (e2 & 0x1FF) << 18 | (e0 >> 16 & 1) << 27 | (e1 >> 16 & 1) << 28 |
             (e2 >> 16 & 1) << 29;
    }

    __syncthreads(); /* image in LDS */
    bool fast = true;
    for (int s = 0; s < S; s++) xa[s * MF_XSTR + i] = (unsigned char)quant_s8_state(st[s]);
    if constexpr (SPLIT)
      for (int e = tid; e < 3 * (NA + 1) * S; e += SAMPLE_THREADS) part[e] = 0;
    __syncthreads(); /* initial q(h_A), q(h_B), ix, seeds */
    stamp_start();
#ifdef MF_PRIO45
    /* waves 4/5 share SIMDs with the older waves 0/1 and lose every VALU
     * arbitration at equal priority */
    if (wv >= 4) __builtin_amdgcn_s_setprio(MF_PRIO45);
#endif

    /* per-sample terms that depend only on the state and the recurrent sums,
     * computed right after the recurrent product (off the X->Y critical path):
     * az/ar, the (subias + diag*state) terms of z and r, and the whole
     * recurrent h-gate value (nnet.c:431-440) */
    int az[S], ar[S], ah[S];
    float faz[S], far[S]; /* az / ar as exact floats (ga_elementwise) */
    float tz[S], tr[S], hpre[S];
    auto recurrent = [&]() {
      v4i vz[1] = {{wsz, wsz, wsz, wsz}}, vr[1] = {{wsr, wsr, wsr, wsr}}, vh[2] = {{wsh, wsh, wsh, wsh}, {0, 0, 0, 0}};
      mf_opaque(oz);
      mf_opaque(orr);
      mf_opaque(oh);
      if constexpr (SPLIT) {
        /* own groups into v*, the hosted piece into f*, whose partial sums
         * go to their row's owner through LDS (exact int32 adds, any order);
         * the owners add them after barrier X.  Group 0's x words of both
         * products are read first: the h product's are in flight while the
         * z/r MFMAs run (the two switches break the prefetch chain) */
        v4i fz = {0, 0, 0, 0}, fr = {0, 0, 0, 0}, fh[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
        uint32_t xz[4], xr[4], xh[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          xz[k] = mf_x(lds, oz, k);
          xr[k] = mf_x(lds, orr, k);
          xh[k] = mf_x(lds, oh, k);
        }
        mf_zr_split(lds, wz, wr, oz, orr, nzr, nfzr, xz, xr, vz[0], vr[0], fz, fr);
        uint32_t fp = frow;
        asm volatile("" : "+v"(fp)); /* unpacked here, not hoisted into three registers */
        const int frz = (int)(fp & 0x1FF), frr = (int)((fp >> 9) & 0x1FF), frh = (int)((fp >> 18) & 0x1FF);
        /* only lanes hosting a piece add (a shared dummy row would
         * serialise every other lane's atomic on one LDS address) */
        int pz[S], pr[S], ph[S];
        for (int s = 0; s < S; s++) {
          pz[s] = fz[s];
          pr[s] = fr[s];
        }
        /* S < 4: branch-free, a lane without a piece adds 0 to its own row's
         * words (same box, skewed model: 1 and 256 streams -1 to -2 %); S = 4
         * keeps the branches (+1 % branch-free) */
        auto padd = [&](int g, int fr_, int (&v)[S]) {
          if constexpr (S < 4) {
            const bool h = fr_ != NA;
            int vv[S];
            for (int s = 0; s < S; s++) vv[s] = h ? v[s] : 0;
            part_add<S, false>(part, g, h ? fr_ : i, vv);
          } else if (fr_ != NA) {
            part_add<S, false>(part, g, fr_, v);
          }
        };
        mf_h_split(lds, wh, oh, nh, nfh, xh, vh, fh);
        for (int s = 0; s < S; s++) ph[s] = fh[0][s] + fh[1][s];
        /* gate by gate: z of every stream, then r, then h (wave-uniform skips) */
        if (nfzr > 0) {
          padd(0, frz, pz);
          padd(1, frr, pr);
        }
        if (nfh > 0) padd(2, frh, ph);
      } else if (TRACE) {
        mf_zr<1>(lds, wz, wr, oz, orr, nzr, vz, vr);
        mf_run<MF_HMAX, 2>(lds, wh, oh, nh, vh);
      } else {
        /* straight-line code for this wave's group counts: with runtime
         * counts the per-group branches make the compiler copy the x
         * prefetch registers and wait for the next group's LDS reads
         * before each group's last MFMA (measured: ~48 -> ~26 cycles per
         * MFMA on a wave's own SIMD half) */
        switch (nzr * 16 + nh) {
#define MF_CASE(Z, H)                                 \
  case Z * 16 + H:                                    \
    mf_zr<1>(lds, wz, wr, oz, orr, Z, vz, vr);        \
    mf_run<MF_HMAX, 2>(lds, wh, oh, H, vh);           \
    break;
#define MF_CASES(Z) MF_CASE(Z, 1) MF_CASE(Z, 2) MF_CASE(Z, 3) MF_CASE(Z, 4) MF_CASE(Z, 5) MF_CASE(Z, 6) MF_CASE(Z, 7) MF_CASE(Z, 8)
          MF_CASES(1)
          MF_CASES(2)
          MF_CASES(3)
          MF_CASES(4)
#undef MF_CASES
#undef MF_CASE
          default:
            mf_zr<1>(lds, wz, wr, oz, orr, nzr, vz, vr);
            mf_run<MF_HMAX, 2>(lds, wh, oh, nh, vh);
            break;
        }
      }
      for (int s = 0; s < S; s++) {
        az[s] = vz[0][s];
        ar[s] = vr[0][s];
        faz[s] = (float)vz[0][s];
        far[s] = (float)vr[0][s];
        ah[s] = vh[0][s] + vh[1][s];
        tz[s] = bz + dz * st[s];
        tr[s] = br + dr * st[s];
        if constexpr (SPLIT)
          ah[s] += cvt_rne((bh + dh * st[s]) * kScale); /* the seed now: int32 sums associate */
        else
          hpre[s] = (float)(ah[s] + cvt_rne((bh + dh * st[s]) * kScale)) * kScale1;
      }
    };
    recurrent();
    for (int f = 0; f < nfr; f++) {
      if (f > 0) {
        __syncthreads(); /* frame start: inputs staged, the previous frame's PCM complete */
        for (int e = tid; e < S * A.N; e += SAMPLE_THREADS) {
          const int s = e / A.N, k = e % A.N;
          if (s0 + s < A.nstreams) pcm_out[(size_t)(s0 + s) * A.N + k] = active[s] ? pcmbuf[s * FRAME + k] : (short)0;
        }
        pcm_out += (size_t)A.nstreams * A.N;
      }
      /* every input of this frame within the host's range bounds
       * (SampleArgs::mf_zr_bound): the elementwise step's range selects are
       * dead, take the select-free forms (uniform per workgroup) */
      fast = true;
      for (int w = 0; w < SAMPLE_WAVES; w++) fast &= okw[w] != 0;
      for (int n = 0; n < A.N; n++) {
        stamp(4);
        __syncthreads(); /* X */
        stamp(5);
        {
          /* GRU_A input (nnet.c:484-491): all 9*S gathers in flight at once */
          float e[S][9];
          if constexpr (S > 1) {
            /* split form: every stream's indices read before the first
             * gather (one LDS wait instead of one per stream: skewed model at
             * 1024 streams -2.6 %; the unsplit form and mf2_kernel lose
             * 0.2-1 % with it, so they read stream by stream) */
            int4 ixv[S];
            if constexpr (SPLIT)
              for (int s = 0; s < S; s++) ixv[s] = *(const int4 *)(ix + s * 4);
            for (int s = 0; s < S; s++) {
              /* table base in SGPRs, row + lane offset in one 32-bit VGPR: the
               * global_load saddr form with no scalar address chain per row
               * (gathers 1,520 -> 1,435 cycles at 4 streams; neutral at 1) */
              const int4 v = SPLIT ? ixv[s] : *(const int4 *)(ix + s * 4);
              uint32_t o1 = (uint32_t)tid * 4u + (uint32_t)v.x;
              uint32_t o2 = (uint32_t)tid * 4u + (uint32_t)v.y;
              uint32_t o3 = (uint32_t)tid * 4u + (uint32_t)v.z;
              asm volatile("" : "+v"(o1), "+v"(o2), "+v"(o3));
              const char *b1 = (const char *)A.mf_emb[0], *b2 = (const char *)A.mf_emb[1], *b3 = (const char *)A.mf_emb[2];
#pragma unroll
              for (uint32_t g = 0; g < 3; g++) {
                e[s][g] = *(const float *)(b1 + o1 + g * NA * 4u);
                e[s][3 + g] = *(const float *)(b2 + o2 + g * NA * 4u);
                e[s][6 + g] = *(const float *)(b3 + o3 + g * NA * 4u);
              }
            }
          } else {
            for (int s = 0; s < S; s++) {
              /* the indices are the same in every lane: scalar row addresses */
              const int4 v = *(const int4 *)(ix + s * 4);
              const float *e1 = A.mf_emb[0] + (__builtin_amdgcn_readfirstlane(v.x) & 0xFF) * GA_ROWS;
              const float *e2 = A.mf_emb[1] + (__builtin_amdgcn_readfirstlane(v.y) & 0xFF) * GA_ROWS;
              const float *e3 = A.mf_emb[2] + (__builtin_amdgcn_readfirstlane(v.z) & 0xFF) * GA_ROWS;
              /* scalar row base + unsigned 32-bit lane offset + immediate: the
               * global_load saddr form, no vector address arithmetic per row */
              uint32_t ub = (uint32_t)tid * 4u;
              asm volatile("" : "+v"(ub)); /* opaque per row: not reassociated into table + lane pairs */
              const char *b1 = (const char *)e1, *b2 = (const char *)e2, *b3 = (const char *)e3;
#pragma unroll
              for (uint32_t g = 0; g < 3; g++) {
                e[s][g] = *(const float *)(b1 + ub + g * NA * 4u);
                e[s][3 + g] = *(const float *)(b2 + ub + g * NA * 4u);
                e[s][6 + g] = *(const float *)(b3 + ub + g * NA * 4u);
              }
            }
          }
          if constexpr (SPLIT) {
            /* the hosted pieces' partial sums of this thread's rows (written
             * between barriers Y and X), then cleared for the next sample;
             * only rows that have pieces (LDS bandwidth: all six waves do
             * this at once, on the critical path) */
            uint32_t fp = frow;
            asm volatile("" : "+v"(fp));
            /* only the rows with pieces read (mf2_kernel reads every row
             * unconditionally instead: +3 % there, -0.8 % here) */
            int zadd[S], radd[S], hadd[S];
            for (int s = 0; s < S; s++) zadd[s] = radd[s] = hadd[s] = 0;
            if (S < 4) fp |= 7u << 27; /* S < 4: every row, branch-free (-4 to -5 % at 1 and 256 streams) */
            if (fp >> 27 & 1) {
              part_read<S, false>(part, 0, i, zadd);
              part_clear<S, false>(part, 0, i);
            }
            if (fp >> 28 & 1) {
              part_read<S, false>(part, 1, i, radd);
              part_clear<S, false>(part, 1, i);
            }
            if (fp >> 29 & 1) {
              part_read<S, false>(part, 2, i, hadd);
              part_clear<S, false>(part, 2, i);
            }
            for (int s = 0; s < S; s++) {
              az[s] += zadd[s];
              ar[s] += radd[s];
            }
            for (int s = 0; s < S; s++) {
              hpre[s] = (float)(ah[s] + hadd[s]) * kScale1;
              faz[s] = (float)az[s];
              far[s] = (float)ar[s];
            }
          }
          if (stamping) {
            /* diagnostic only: wait for every gather before the stamp */
            float g = 0.f;
            for (int s = 0; s < S; s++)
#pragma unroll
              for (int k = 0; k < 9; k++) g += e[s][k];
            asm volatile("" ::"v"(g));
            stamp(10);
          }
          /* compute_sparse_gru elementwise (nnet.c:431-447): one uniform
           * branch per sample into straight-line code for all S streams */
          if (__builtin_amdgcn_readfirstlane((int)fast))
            ga_elementwise<S, true, kHwA>(st, e, cnd, tid, faz, far, tz, tr, hpre, rcp, xa + i, stamping, stamp);
          else
            ga_elementwise<S, false, kHwA>(st, e, cnd, tid, faz, far, tz, tr, hpre, rcp, xa + i, stamping, stamp);
        }
        stamp(0);
        __syncthreads(); /* Y */
        stamp(1);
        if (n + 1 < A.N || f + 1 < nfr) recurrent(); /* W q(h_A(n)) for sample n+1, beside GRU_B and the sampling of n */
        stamp(2);
      }
      if (f + 1 < nfr) {
        /* next frame's inputs, read after the frame-start barrier */
        cf += A.nstreams;
        stage(cf);
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
    /* tree walk: with S=4 a sampler wave carries two streams, one per 32-lane half */
    const int sw = wv - SAMPLE_WAVES;
    const int half = lane >> 5, hl = lane & 31;
    const int my_s = S == 4 ? 2 * sw + half : sw;
    const bool samp = my_s < S;                         /* wave-uniform */
    const bool samp_w = samp && (S == 4 || half == 0);  /* lanes owning the stream's outputs */
    const int ms = samp ? my_s : 0;
    const bool my_active = samp && s0 + ms < A.nstreams && frame_count_of(A, s0 + ms) > A.delay;
    /* GRU_B: lane = (stream gs, unit gu) = (lane / 16, lane % 16).  The
     * quantised states are the MFMA A operand (row m = stream m/4 of the
     * group: rows 4gs .. 4gs+3 are stream gs), the weight tiles the B
     * operand (column n = GRU_B row n of the gate), so D register 0 of this
     * lane is row 4gs, column gu: unit gu of stream gs, no register pick.
     * gown: stream gs is one of this wave's. */
    const int gs = lane >> 4, gu = lane & 15, sl = min(gs, S - 1), sx = min(gu >> 2, S - 1);
    const bool gown = gs < S && (S == 4 ? (gs >> 1) : gs) == sw;
    const bool gact = gown && s0 + gs < A.nstreams && frame_count_of(A, s0 + gs) > A.delay;

    float lsr[NLPC], lpr[NLPC];
    float pred = 0.f, deemph = 0.f;
    uint32_t rz = 0, rw = 0, rj = 0, rc = 0;
    int last_exc = 0;
    {
      const StreamState *p = &A.st[min(s0 + ms, A.nstreams - 1)];
#pragma unroll
      for (int j = 0; j < NLPC; j++) {
        lsr[j] = p->last_sig[j];
        lpr[j] = lpc_of(A, min(s0 + ms, A.nstreams - 1))[j];
      }
      deemph = p->deemph_mem;
      last_exc = p->last_exc & 0xFF; /* the gathers index 256-row tables: never out of bounds (restore_state also rejects such snapshots) */
      rz = p->rng[0]; rw = p->rng[1]; rj = p->rng[2]; rc = p->rng[3];
    }
    float sbv = A.st[min(s0 + sl, A.nstreams - 1)].gru_b_state[gu];
    /* the walk's select-free tanh: dual-FC node sums bounded by the model
     * (fc_fin) for GRU_B states within [-2, 2]; int8 GRU_B updates keep a
     * state there (convex combinations of it and tanh outputs), so the
     * launch-time check covers the launch */
    const bool walk_fin = A.fc_fin && __builtin_amdgcn_readfirstlane((int)(__ballot(!(fabsf(sbv) <= 2.f)) == 0ull));
    /* GRU_B weight tiles in registers; with 4 streams the 3 recurrent
     * tiles live in LDS instead (read in the samplers' slack before barrier
     * Y: 12 registers fewer, no spill) */
    constexpr int kRegTiles = kGbwLds ? MF_GB_IN : MF_GB_TILES;
    v4i wt[kRegTiles];
#pragma unroll
    for (int t = 0; t < kRegTiles; t++) {
      const uint4 u = A.mf_gb[t * 64 + lane];
      wt[t] = v4i{(int)u.x, (int)u.y, (int)u.z, (int)u.w};
    }
    if (kGbwLds && sw == 0)
      for (int g = 0; g < 3; g++) {
        const uint4 u = A.mf_gb[(MF_GB_IN + g) * 64 + lane];
        gbw[g * 64 + lane] = v4i{(int)u.x, (int)u.y, (int)u.z, (int)u.w};
      }
    auto put_xb = [&]() {
      if (gown) xb[gs * NB + gu] = (unsigned char)quant_s8_state(sbv);
    };
    __syncthreads(); /* image in LDS */
    FcLane F;
    F.init(img, lane);
    put_xb();
    /* the sig/pred/exc indices as the GRU_A waves consume them: at S > 1
     * the byte offsets of the three embedding rows (the gathers add the lane
     * offset only), at S = 1 the indices */
    auto ix_word = [](int su, int pu, int exc) {
      return S > 1 ? make_int4(su * (GA_ROWS * 4), pu * (GA_ROWS * 4), exc * (GA_ROWS * 4), 0) : make_int4(su, pu, exc, 0);
    };
    if (samp) {
      /* pred and the u-law indices of the first sample (lpcnet.c:252-254) */
      float p2 = 0.f;
#pragma unroll
      for (int j = 0; j < NLPC; j++) p2 = p2 - lsr[j] * lpr[j];
      pred = p2;
      if (samp_w && hl == 0) *(int4 *)(ix + ms * 4) = ix_word(lin2ulaw_x86(lsr[0]), lin2ulaw_x86(pred), last_exc);
    }
    __syncthreads(); /* initial q(h_A), q(h_B), ix, seeds */
    stamp_start();
    /* the sampler chain is the per-sample critical path; the GRU_A waves
     * sharing these SIMDs have slack: issue the samplers' instructions first */
    __builtin_amdgcn_s_setprio(3);

    float t03 = 0.f, t47 = 0.f;
    constexpr bool tracing = TRACE;
    /* bookkeeping of sample n deferred into the X->Y interval of n+1 */
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
      put_xb();
      pend_n = -1;
    };
    const FrameCond *cf = A.cond;
    for (int f = 0; f < nfr; f++) {
      if (f > 0) __syncthreads(); /* frame start */
      for (int n = 0; n < A.N; n++) {
        stamp(4);
        __syncthreads(); /* X */
        stamp(5);
        v4i acc[3], accr[3];
        float lpd[NLPC];
        if (samp) {
          finish();
          /* pred(n+1)'s candidate-independent products, off the chain */
          lpd[0] = 0.f;
#pragma unroll
          for (int j = 1; j < NLPC; j++) lpd[j] = lsr[j - 1] * lpr[j];
          stamp(13);
          /* the two kiss99 draws of this sample and their thresholds (nnet.c:178-184) */
          const uint32_t r0 = kiss99_next(rz, rw, rj, rc);
          const uint32_t r1 = kiss99_next(rz, rw, rj, rc);
          lane_thresholds(F, logit_tab, r0, r1, t03, t47);
          /* GRU_B recurrent product (nnet.c:355-361) needs only q(h_B(n-1)):
           * before barrier Y.  Seeds are the accumulator inputs. */
          const v4i xr = *(const v4i *)(xb + sx * NB); /* k 0..15; the tiles' other K chunks are zero */
#pragma unroll
          for (int g = 0; g < 3; g++) {
            acc[g] = v4i{gbs[sl * GB_ROWS + 16 * g + gu], 0, 0, 0};
            accr[g] = v4i{gbr[16 * g + gu], 0, 0, 0};
          }
#pragma unroll
          for (int g = 0; g < 3; g++) accr[g] = mfma16(xr, kGbwLds ? gbw[g * 64 + lane] : wt[(MF_GB_IN + g) % kRegTiles], accr[g]);
        }
        stamp(0);
        __syncthreads(); /* Y */
        stamp(1);
        if (!samp) continue;
        {
          /* GRU_B input product (nnet.c:345-353), 48 x 384, all S streams */
          v4i xk[6];
#pragma unroll
          for (int kt = 0; kt < 6; kt++) xk[kt] = *(const v4i *)(xa + sx * MF_XSTR + 64 * kt + 16 * gs);
          /* z and r tiles first: their sigmoids overlap the h tile's MFMAs */
#pragma unroll
          for (int kt = 0; kt < 6; kt++)
#pragma unroll
            for (int g = 0; g < 2; g++) acc[g] = mfma16(xk[kt], wt[g * 6 + kt], acc[g]);
#pragma unroll
          for (int kt = 0; kt < 6; kt++) acc[2] = mfma16(xk[kt], wt[12 + kt], acc[2]);
          stamp(10);
          /* GRU_B elementwise (nnet.c:362-371), unit gu of stream sl */
          float zrb[2] = {(float)acc[0][0] * kScale1 + (float)accr[0][0] * kScale1,
                          (float)acc[1][0] * kScale1 + (float)accr[1][0] * kScale1};
          sigmoid_x86_fin_n<2, HWR>(zrb, rcp);
          float hh[1] = {(float)acc[2][0] * kScale1 + ((float)accr[2][0] * kScale1) * zrb[1]};
          stamp(14);
          tanh_x86_fin_n<1, HWR>(hh, rcp); /* |hh| < 2^19: int32 sums x 2^-14 */
          sbv = zrb[0] * sbv + (1.f - zrb[0]) * hh[0];
          if (gown) sbuf[gs * NB + gu] = sbv;
        }
        stamp(8);
        /* same-wave LDS exchange: the half of stream ms reads its 16 GRU_B units */
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
#ifdef MF_WALKFINE
        auto wst = [&](int k, float v) {
          if (stamping) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const int u = __builtin_amdgcn_readfirstlane(__float_as_int(v));
            asm volatile("" ::"s"(u));
            stamp(k);
          }
        };
        const WalkOut R = walk_fin ? dual_fc_walk_p<TRACE, true, HWR>(F, t03, t47, xv, pred, lpd, lpr, n < A.preload ? pcmbuf + ms * FRAME + n : nullptr,
                                                                 deemph, wst)
                                   : dual_fc_walk_p<TRACE, false, HWR>(F, t03, t47, xv, pred, lpd, lpr, n < A.preload ? pcmbuf + ms * FRAME + n : nullptr,
                                                                  deemph, wst);
#else
        const short *teach = n < A.preload ? pcmbuf + ms * FRAME + n : nullptr;
        const WalkOut R = walk_fin ? dual_fc_walk_p<TRACE, true, HWR>(F, t03, t47, xv, pred, lpd, lpr, teach, deemph)
                                   : dual_fc_walk_p<TRACE, false, HWR>(F, t03, t47, xv, pred, lpd, lpr, teach, deemph);
#endif
        stamp(11);
        if (samp_w && hl == 0 && n + 1 < A.N) *(int4 *)(ix + ms * 4) = ix_word(R.su, R.pu, R.exc);
        if (tracing && samp_w && hl < 8 && my_active) {
          float v = R.lg[0];
#pragma unroll
          for (int b = 1; b < 8; b++) v = hl == b ? R.lg[b] : v;
          A.trace_logits[((size_t)(s0 + ms) * A.N + n) * 8 + hl] = v;
        }
        if (A.trace_exc && samp_w && hl == 0 && my_active) A.trace_exc[(size_t)(s0 + ms) * A.N + n] = R.exc;
        pend_pcm = R.pcm;
        pend_pred = R.pn;
        pend_exc = R.exc;
        pend_n = n;
        stamp(12);
      }
      if (f + 1 < nfr) {
        /* frame boundary (multi-frame launches): the last sample's
         * bookkeeping, then the next frame's LPC, pred and u-law indices as
         * at a launch start */
        finish(); /* the GRU_A waves write the frame's PCM out after the frame-start barrier */
        cf += A.nstreams;
        /* the lane's stream from an opaque copy of the lane id: the address
         * is formed here, not hoisted out of the loop into live registers */
        int lf = lane;
        asm volatile("" : "+v"(lf));
        const int msf = S == 4 ? 2 * sw + (lf >> 5) : sw;
        const float *lp = lpc_of(cf, A, min(s0 + msf, A.nstreams - 1));
#pragma unroll
        for (int j = 0; j < NLPC; j++) lpr[j] = lp[j];
        float p2 = 0.f;
#pragma unroll
        for (int j = 0; j < NLPC; j++) p2 = p2 - lsr[j] * lpr[j];
        pred = p2;
        if (samp_w && hl == 0) *(int4 *)(ix + ms * 4) = ix_word(lin2ulaw_x86(lsr[0]), lin2ulaw_x86(pred), last_exc);
      }
    }
    if (samp) finish();
    stamp(4);
    __syncthreads(); /* final */
    stamp(5);
    if (samp_w && my_active && hl == 0) {
      StreamState *p = &A.st[s0 + ms];
#pragma unroll
      for (int j = 0; j < NLPC; j++) p->last_sig[j] = lsr[j];
      p->deemph_mem = deemph;
      p->last_exc = last_exc;
      p->rng[0] = rz; p->rng[1] = rw; p->rng[2] = rj; p->rng[3] = rc;
    }
    if (gact) A.st[s0 + gs].gru_b_state[gu] = sbv;
  }
  if (stamping && lane == 0) {
    stp[6] = __builtin_amdgcn_s_memtime() - t_loop0;
    stp[7] = (unsigned long long)total;
    for (int k = 0; k < 16; k++) A.stamps[((size_t)blockIdx.x * STAMP_WAVES + wv) * 16 + k] = stp[k];
  }
  short *pcm_last = A.pcm + (size_t)(nfr - 1) * A.nstreams * A.N;
  for (int e = tid; e < S * A.N; e += MF_THREADS) {
    const int s = e / A.N, n = e % A.N;
    if (s0 + s < A.nstreams) pcm_last[(size_t)(s0 + s) * A.N + n] = active[s] ? pcmbuf[s * FRAME + n] : (short)0;
  }
}

template <int S, int DIAG, bool SPLIT, bool HWR = true>
static int launch_mf_t(const SampleArgs &a, int lds_bytes, hipStream_t stream)
{
  if (ensure_dyn_lds((const void *)mf_kernel<S, DIAG, SPLIT, HWR>, 160 * 1024 - IMG_VAR)) return -1;
  const int grid = warm_grid((a.nstreams + S - 1) / S, a.nstreams);
  /* lds_bytes counts the static image too (mf_lds_bytes) */
  hipLaunchKernelGGL((mf_kernel<S, DIAG, SPLIT, HWR>), dim3(grid), dim3(MF_THREADS), lds_bytes - IMG_VAR, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int S>
static int launch_mf_s(const SampleArgs &a, int lds_bytes, hipStream_t st)
{
  if (!a.rcp_hw) {
    /* another host's rcpps table: every activation through it (production
     * and trace forms; no stamped build) */
    if (a.stamps) return -1;
    if (a.mf_split)
      return a.trace_logits ? launch_mf_t<S, 1, true, false>(a, lds_bytes, st) : launch_mf_t<S, 0, true, false>(a, lds_bytes, st);
    return a.trace_logits ? launch_mf_t<S, 1, false, false>(a, lds_bytes, st) : launch_mf_t<S, 0, false, false>(a, lds_bytes, st);
  }
  if (a.mf_split)
    return a.trace_logits ? launch_mf_t<S, 1, true>(a, lds_bytes, st)
           : a.stamps     ? launch_mf_t<S, 2, true>(a, lds_bytes, st)
                          : launch_mf_t<S, 0, true>(a, lds_bytes, st);
  /* a trace takes precedence over the stamps (never requested together) */
  return a.trace_logits ? launch_mf_t<S, 1, false>(a, lds_bytes, st)
         : a.stamps     ? launch_mf_t<S, 2, false>(a, lds_bytes, st)
                        : launch_mf_t<S, 0, false>(a, lds_bytes, st);
}

int launch_mf(const SampleArgs &a, int S, int lds_bytes, void *stream)
{
  hipStream_t st = (hipStream_t)stream;
  if (S == 4) return launch_mf_s<4>(a, lds_bytes, st);
  if (S == 2) return launch_mf_s<2>(a, lds_bytes, st);
  return launch_mf_s<1>(a, lds_bytes, st);
}

}  // namespace lpcnet_mi355x
