/*
 * chunk_kernel.hip -- run_frame_network (lpcnet.c:82-120) for every frame of
 * a chunk of up to LPC_CHUNK frames at once, on the f32 matrix cores.
 *
 * The frame network never reads the sample network's outputs: frame f's
 * inputs are the features of frames f-2..f (conv1), conv1's outputs of
 * frames f-2..f (conv2) and the LPC of frame f-2.  So a chunk of frames is
 * one batch of columns (stream, frame) through the five layers, and every
 * weight is fetched once per 64 columns instead of once per 4.
 *
 * Numerics: v_mfma_f32_16x16x4_f32 computes
 *   D = fma(a3, b3, fma(a2, b2, fma(a1, b1, fma(a0, b0, C))))
 * in k order, one rounding per product (cdna_hip_programming.md, FP32-input
 * MFMA) -- the sequential fmaf chain of sgemv_accum16 (vec_avx.h:618-643)
 * started from the bias, so a row chained over its inputs 4 at a time is the
 * per-frame frame_kernel's result bit for bit.  tanh is the Pade form with
 * rcpps from the hardware reciprocal (rcp_x86_hw, proven equal to the x86
 * table: device_math.h), no table read from memory.
 *
 * Workgroup = SC streams x NFR frames = 64 columns (80 / 96 for 20 / 24
 * frames x 4 streams, see launch_chunk) (frames
 * >= nframes are computed on zero inputs and never stored); 8 waves.
 * Layers with 128 rows: wave w owns row tile w for all column tiles (one
 * weight fragment feeds one MFMA per column tile).  Projections (1200 rows = 75 tiles): wave w
 * owns tiles w, w + 8, ...  Activations live in LDS as [column][input] rows
 * whose stride makes the B-operand reads (16 columns x 4 inputs per
 * wave-instruction) bank-conflict free; weights stream from L2 in the blob's
 * [in][out] layout, PD steps ahead (the device copies carry FRAME_PREFETCH
 * zero input rows, so the prefetch needs no clamp).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "device_math.h"
#include "lpcnet_engine.h"

namespace lpcnet_mi355x {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int CK_THREADS = 512;
constexpr int CK_RS = COND + 4;   /* row stride of 128-wide activation rows: 4c + k banks */
constexpr int CK_PROJ = GA_ROWS + GB_ROWS;
constexpr int CK_PROJ_TILES = CK_PROJ / 16;
static_assert(CK_PROJ % 16 == 0 && GA_ROWS % 16 == 0 && COND == 8 * 16, "row tiles");

/* smallest stride >= v that is 32 mod 64 floats: a 16-column tile that spans
 * two streams (NFR = 8) then reads 64 distinct banks */
constexpr int ck_stride32(int v) { return v + ((32 - v % 64) + 64) % 64; }
/* stream stride of the conv windows: one-frame launches put 16 streams in a
 * column tile, lane (r, g) reading stream r's input 4 kk + g -- a stride of
 * 4 mod 64 floats gives the 64 lanes 64 distinct banks (at 32 mod 64 they
 * fell on 8: ~250 cycles per conv k step stamped, against ~100 for the dense
 * layers' 132-float rows) */
constexpr int ck_sstride(int v, int nfr) { return nfr == 1 ? v + ((4 - v % 64) + 64) % 64 : ck_stride32(v); }
constexpr int ck_max(int a, int b) { return a > b ? a : b; }

template <int NFR, int SC_>
struct CkGeom {
  static constexpr int SC = SC_;                           /* streams per workgroup */
  static constexpr int COLS = SC * NFR;                    /* (stream, frame) columns */
  static constexpr int NCT = COLS / 16;                    /* column tiles */
  static_assert(COLS % 16 == 0, "whole column tiles");
  static constexpr int INF = NFR + 2;                      /* frames -2 .. NFR-1 */
  static constexpr int IN_SS = ck_sstride(INF * FIN, NFR);   /* conv1 inputs: stream stride */
  static constexpr int C1_SS = ck_sstride(INF * CK_RS, NFR); /* conv1 outputs: stream stride */
  static constexpr int R0 = ck_max(SC * IN_SS, COLS * CK_RS); /* conv1 inputs, then dense1 outputs */
  static constexpr int R1 = SC * C1_SS;
  static constexpr int R2 = COLS * CK_RS;                  /* conv2, then dense2 outputs */
  static constexpr int FLOATS = R0 + R1 + R2;
};

/* T row tiles of a layer for the column tiles (T > 1: the projection's
 * tiles of one wave side by side, independent chains that share every x
 * read):
 *   acc[t][j][i] = bias[row] + sum_k W[k][row] * X(col, k),  row = 16 rt_t + 4 g + i,
 * col = 16 j + (lane & 15), each chain in k order (sgemv_accum16's
 * sequential fmaf, bit for bit).  X(col, k) = xs[xb[j] + (k / SEG) * SST +
 * k % SEG]: a column's inputs as segments of SEG values SST apart (conv
 * windows over padded frame rows), read XL k steps ahead.
 * Weights: each row tile's re-tiled copy (FrameArgs::ck_*, one float4 per
 * lane = 4 k steps) through a ring of PQ quads in registers; for T = 1 the
 * ring streams the wave's whole sequence of row tiles (conv1, conv2, dense1,
 * dense2, its projection tiles), so the next tile's first quads and bias are
 * in flight while this tile's chain runs.  Quad counts are multiples of PQ,
 * so the ring's phase is 0 at every tile start.
 * Stamped (CK_STAMPS, one-frame launch, 16 streams per workgroup): with one
 * quad of x lookahead and one projection tile at a time the LDS reads and
 * the dependent MFMA chains left ~300 cycles per k step. */
template <int T, int PQ>
struct CkRing {
  float4 w[PQ][T];
  float4 b[T]; /* the current tiles' bias quads (rows 16 rt + 4 g ..) */
};

template <int T, int PQ>
__device__ __forceinline__ void ck_prime(CkRing<T, PQ> &R, const float4 *const (&tile)[T], const float *const (&bias)[T])
{
#pragma unroll
  for (int d = 0; d < PQ; d++)
#pragma unroll
    for (int t = 0; t < T; t++) R.w[d][t] = tile[t][(size_t)d * 64];
#pragma unroll
  for (int t = 0; t < T; t++) R.b[t] = *(const float4 *)bias[t];
}

template <int K, int SEG, int SST, int NCT, int T, int PQ, int XL>
__device__ __forceinline__ void ck_tiles(CkRing<T, PQ> &R, const float4 *const (&cur)[T], const float4 *nxt,
                                         const float *nbias, const float *xs, const int (&xb)[NCT],
                                         f32x4 (&acc)[T][NCT])
{
  static_assert(K % 4 == 0 && SEG % 4 == 0, "k quads stay inside a segment");
  constexpr int KS = K / 4;
  constexpr int NQ = (KS + 3) / 4;
  static_assert(NQ % PQ == 0, "ring phase 0 at every tile start");
  static_assert(T == 1 || PQ <= NQ, "multi-tile: no streaming into a next tile");
  const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int t = 0; t < T; t++)
#pragma unroll
    for (int j = 0; j < NCT; j++) acc[t][j] = f32x4{R.b[t].x, R.b[t].y, R.b[t].z, R.b[t].w};
  if (T == 1 && nbias) R.b[0] = *(const float4 *)nbias; /* the next tile's bias, in flight beside this chain */
  auto xoff = [](int kk) { return ((4 * kk) / SEG) * SST + (4 * kk) % SEG; };
  float xv[XL][NCT];
#pragma unroll
  for (int d = 0; d < XL; d++)
    if (d < KS)
#pragma unroll
      for (int j = 0; j < NCT; j++) xv[d][j] = xs[xb[j] + g + xoff(d)];
#pragma unroll
  for (int kk = 0; kk < KS; kk++) {
    const int q = kk / 4;
    float a[T];
#pragma unroll
    for (int t = 0; t < T; t++) {
      const float4 &wq = R.w[q % PQ][t];
      a[t] = (kk & 3) == 0 ? wq.x : (kk & 3) == 1 ? wq.y : (kk & 3) == 2 ? wq.z : wq.w;
    }
    float xc[NCT];
#pragma unroll
    for (int j = 0; j < NCT; j++) xc[j] = xv[kk % XL][j];
    if (kk + XL < KS)
#pragma unroll
      for (int j = 0; j < NCT; j++) xv[kk % XL][j] = xs[xb[j] + g + xoff(kk + XL)];
#pragma unroll
    for (int t = 0; t < T; t++)
#pragma unroll
      for (int j = 0; j < NCT; j++) acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], xc[j], acc[t][j], 0, 0, 0);
    if ((kk & 3) == 3 || kk + 1 == KS) {
      /* quad q consumed: its slot takes quad q + PQ of the tile(s), past the
       * tile's end (T = 1) the next tile's first quads */
#pragma unroll
      for (int t = 0; t < T; t++) {
        if (q + PQ < NQ)
          R.w[q % PQ][t] = cur[t][(size_t)(q + PQ) * 64];
        else if (T == 1 && nxt)
          R.w[q % PQ][t] = nxt[(size_t)(q + PQ - NQ) * 64];
      }
    }
    /* k step boundary: without it the scheduler sinks every x read and ring
     * refill to its use (ds_read; s_waitcnt lgkmcnt(0); mfma -- the ~235
     * cycles per k step CK_STAMPS measured); not at 5-6 column tiles, whose
     * lookahead is one step and whose registers are full */
    if constexpr (NCT <= 4) __builtin_amdgcn_sched_barrier(0);
  }
}

/* quads per row tile of a re-tiled K-input matrix, padding included */
constexpr int ck_tq(int K) { return (K / 4 + 3) / 4 + CK_WPAD; }

/* per column-tile count: x lookahead, weight ring depth, projection tiles
 * per pass (registers: 4 T NCT accumulators + 4 PQ T ring + XL NCT x) */
constexpr int ck_xl(int nct) { return nct <= 2 ? 8 : (nct <= 4 ? 2 : 1); }
constexpr int ck_pq(int nct) { return nct <= 4 ? 8 : 2; }
constexpr int ck_tp(int nct) { return nct == 1 ? 10 : (nct == 2 ? 5 : (nct <= 4 ? 2 : 1)); }
constexpr int ck_pqp(int tp, int nct) { return tp >= 5 ? 2 : (tp >= 2 ? 4 : ck_pq(nct)); }

/* frame_count before frame f's update, given its value fc0 at the chunk start
 * (lpcnet.c:119: incremented while below 1000) */
__device__ __forceinline__ int ck_fc(int fc0, int f) { return fc0 >= 1000 ? fc0 : min(fc0 + f, 1000); }

/* diagnostics (CK_STAMPS builds only, tools/ab_build.sh): s_memtime at the
 * phase boundaries of workgroup 0, wave 0, printed once per launch */
#ifdef CK_STAMPS
#define CK_T(k) do { if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) ck_t[k] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define CK_T(k) do { } while (0)
#endif

/* a one-frame launch's L2 warm-up: the workgroups of an XCD (workgroup b
 * runs on XCD b % 8, tools/probes/xcc_probe.hip) split every re-tiled weight
 * matrix and touch each 128-byte line of their share once; the XOR of the
 * values only keeps the loads alive (placement changes speed, never
 * results) */
__device__ __forceinline__ uint32_t ck_warm_weights(const FrameArgs &A, int tid)
{
  const int x = blockIdx.x % 8, nx = ((int)gridDim.x - 1 - x) / 8 + 1, k = blockIdx.x / 8;
  const uint32_t *m[5] = {(const uint32_t *)A.ck_conv1, (const uint32_t *)A.ck_conv2, (const uint32_t *)A.ck_dense1,
                          (const uint32_t *)A.ck_dense2, (const uint32_t *)A.ck_proj};
  const int lines[5] = {8 * ck_tq(3 * FIN) * 64 * 16 / 128, 8 * ck_tq(3 * COND) * 64 * 16 / 128,
                        8 * ck_tq(COND) * 64 * 16 / 128, 8 * ck_tq(COND) * 64 * 16 / 128,
                        CK_PROJ_TILES * ck_tq(COND) * 64 * 16 / 128};
  uint32_t acc = 0;
#pragma unroll
  for (int t = 0; t < 5; t++)
#pragma unroll 4
    for (int o = k * CK_THREADS + tid; o < lines[t]; o += nx * CK_THREADS) acc ^= m[t][(size_t)o * 32];
  return acc;
}

/* PS > 1 (one-frame launches without per-frame outputs): each 16-stream
 * group runs as PS workgroups ("slices", consecutive blockIdx) that each
 * compute the frame network up to dense2 and the projection row tiles
 * rt = PS k + slice -- the projection (75 row tiles, issue-bound on the f32
 * matrix cores: 19.2 K cycles per SIMD at one slice) spread over PS CUs
 * instead of one.  The stream state (conv memories, LPC ring, frame_count)
 * is read by every slice and written by the last one only, after the
 * others have counted their arrival in ck_sync[group] past their prologue
 * reads: the writer has the highest blockIdx of its group, so the slices
 * it waits for were dispatched before it and the wait ends. */
template <int NFR, int SC, bool HWR, int PS = 1>
__global__ __launch_bounds__(CK_THREADS) void chunk_kernel(FrameArgs A)
{
  static_assert(PS == 1 || NFR == 1, "row slices: one-frame launches only");
#ifdef CK_STAMPS
  unsigned long long ck_t[10] = {};
#endif
  CK_T(0);
  using G = CkGeom<NFR, SC>;
  constexpr int NCT = G::NCT;
  extern __shared__ float4 lds4_[];
  float *lds = (float *)lds4_;
  float *inl = lds;          /* [SC][IN_SS]: frame inputs, row f + 2 = frame f (FIN values) */
  float *yb = lds;           /* [64][CK_RS]: dense1 outputs (inl is dead by then) */
  float *c1 = lds + G::R0;   /* [SC][C1_SS]: conv1 outputs, row f + 2 = frame f (stride CK_RS) */
  float *ya = c1 + G::R1;    /* [64][CK_RS]: conv2, then dense2 outputs */
  __shared__ int fcs[G::SC];
  __shared__ float olpc[G::SC][MAX_FEATURES_DELAY][NLPC];
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, g = l >> 4, r = l & 15;
  const int grp = PS > 1 ? (int)blockIdx.x / PS : (int)blockIdx.x;
  const int slice = PS > 1 ? (int)blockIdx.x % PS : 0;
  const bool writer = slice == PS - 1; /* workgroup-uniform */
  const int s0 = grp * G::SC;
  const int n = A.nframes, B = A.nstreams;
  const uint32_t *rcp = A.rcp;
  const int D = A.mc.delay;
  const float gamma = A.mc.lpc_gamma;

  /* inputs (lpcnet.c:91-99): frames -2, -1 from the conv1 memory, then
   * features | pitch embedding of each frame of the chunk; the conv2
   * memory, the LPC ring, frame_count.  Every global read that depends on
   * nothing goes out in one batch into registers (the lane of a pitch
   * embedding element reads its frame's pitch feature itself, no pitch
   * pass and barrier), then the embedding rows, then the LDS stores:
   * stamped (CK_STAMPS), the pass-by-pass form of a one-frame launch took
   * ~15 K cycles of dependent round trips here. */
  constexpr int NIN = (G::SC * G::INF * FIN + CK_THREADS - 1) / CK_THREADS;
  constexpr int NC2 = (G::SC * 2 * COND + CK_THREADS - 1) / CK_THREADS;
  float vin[NIN], vc2[NC2];
#pragma unroll
  for (int q = 0; q < NIN; q++) {
    const int e = q * CK_THREADS + tid;
    float v = 0.f;
    if (e < G::SC * G::INF * FIN) {
      const int s = e / (G::INF * FIN), rem = e % (G::INF * FIN);
      const int fr = rem / FIN - 2, j = rem % FIN, sid = s0 + s;
      if (sid < B) {
        if (fr < 0)
          v = A.st[sid].conv1_mem[(fr + 2) * FIN + j];
        else if (fr < n)
          v = A.features[((size_t)fr * B + sid) * NF + (j < NF ? j : 18)];
        /* deferred LPC: the frame's features for the lpc_kernel that runs
         * after the sample kernel (the host may refill its buffer by then) */
        if (NFR == 1 && writer && A.lpc_feat && fr == 0 && j < NF) A.lpc_feat[(size_t)sid * NF + j] = v;
      }
    }
    vin[q] = v;
  }
#pragma unroll
  for (int q = 0; q < NC2; q++) {
    const int e = q * CK_THREADS + tid, sid = s0 + e / (2 * COND);
    vc2[q] = e < G::SC * 2 * COND && sid < B ? A.st[sid].conv2_mem[e % (2 * COND)] : 0.f;
  }
  /* -DCK_WARM (A/B only): one-frame launches first read the weights into
   * each XCD's L2 (one load per 128-byte line, values discarded), beside the
   * inputs -- stamped, the inputs phase grew by ~6 K cycles and the layers
   * did not move (their k steps were bank-conflict bound, see CkGeom) */
  uint32_t warm = 0;
#ifdef CK_WARM
  if constexpr (NFR == 1) warm = ck_warm_weights(A, tid);
#endif
  /* this frame's lpc_from_cepstrum output, for the LPC ring after the
   * projection (read now: behind the projection's stores it waits for them) */
  __shared__ float nlpc[NFR == 1 ? G::SC * NLPC : 1];
  if constexpr (NFR == 1) {
    if (!A.mc.end2end && !A.lpc_defer && tid < G::SC * NLPC) {
      const int sid = s0 + tid / NLPC;
      nlpc[tid] = sid < B ? A.lpc_new[(size_t)sid * NLPC + tid % NLPC] : 0.f;
    }
  }
#pragma unroll
  for (int q = 0; q < NIN; q++) {
    const int e = q * CK_THREADS + tid;
    if (e < G::SC * G::INF * FIN) {
      const int s = e / (G::INF * FIN), rem = e % (G::INF * FIN);
      const int fr = rem / FIN - 2, j = rem % FIN, sid = s0 + s;
      if (sid < B && fr >= 0 && fr < n && j >= NF) {
        /* lpcnet.c:93-94: the 0.1 avoids rounding issues */
        int pitch = (int)floor(.1 + (double)(50.f * vin[q]) + 100);
        pitch = min(255, max(33, pitch));
        vin[q] = A.embed_pitch[pitch * EP + (j - NF)];
      }
      inl[s * G::IN_SS + rem] = vin[q];
    }
  }
  /* conv1 outputs of frames -2, -1: the conv2 memory */
#pragma unroll
  for (int q = 0; q < NC2; q++) {
    const int e = q * CK_THREADS + tid;
    if (e < G::SC * 2 * COND) {
      const int s = e / (2 * COND), j = e % (2 * COND);
      c1[s * G::C1_SS + (j / COND) * CK_RS + j % COND] = vc2[q];
    }
  }
  /* (a loop: 16-32 streams x FEATURES_DELAY 4 x 16 exceed the 512 threads) */
  for (int e = tid; e < G::SC * D * NLPC; e += CK_THREADS) {
    const int s = e / (D * NLPC), q = e % (D * NLPC), sid = s0 + s;
    olpc[s][q / NLPC][q % NLPC] = sid < B ? A.st[sid].old_lpc[q / NLPC][q % NLPC] : 0.f;
  }
  if (tid < G::SC) fcs[tid] = s0 + tid < B ? A.st[s0 + tid].frame_count : 1000;
  asm volatile("" ::"v"(warm)); /* the warming loads land before the weights are used */
  __syncthreads();
  CK_T(1);
  if constexpr (PS > 1) {
    /* every state read of this slice has landed (LDS / registers) */
    /* relaxed: the reads completed (their values are in LDS past the
     * barrier); a release fence here (buffer_wbl2) cost wave 0 ~10 K cycles */
    if (!writer && tid == 0) __hip_atomic_fetch_add(&A.ck_sync[grp], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  /* this lane's column of each column tile */
  int cs[NCT], cf[NCT];
#pragma unroll
  for (int j = 0; j < NCT; j++) {
    cs[j] = (16 * j + r) / NFR;
    cf[j] = (16 * j + r) % NFR;
  }
  int xb[NCT];
  /* this wave's weight stream: conv1, conv2, dense1, dense2 row tile `wave`
   * (one ring), then its projection tiles wave, wave + 8, ... TP at a time */
  const int l64 = tid & 63;
  constexpr int XL = ck_xl(NCT), PQ = ck_pq(NCT), TP = ck_tp(NCT), PQP = ck_pqp(TP, NCT);
  /* sliced: this slice's copy of the layer weights (same values) */
  const float4 *t_c1 = A.ck_conv1 + (size_t)slice * A.ck_rep[0] + (size_t)wave * ck_tq(3 * FIN) * 64 + l64;
  const float4 *t_c2 = A.ck_conv2 + (size_t)slice * A.ck_rep[1] + (size_t)wave * ck_tq(3 * COND) * 64 + l64;
  const float4 *t_d1 = A.ck_dense1 + (size_t)slice * A.ck_rep[2] + (size_t)wave * ck_tq(COND) * 64 + l64;
  const float4 *t_d2 = A.ck_dense2 + (size_t)slice * A.ck_rep[3] + (size_t)wave * ck_tq(COND) * 64 + l64;
  auto t_pj = [&](int rt) { return A.ck_proj + (size_t)rt * ck_tq(COND) * 64 + l64; };
  const int bo = 16 * wave + 4 * g; /* this lane's bias quad in a 128-row layer */
  CkRing<1, PQ> R;
  {
    const float4 *const t0[1] = {t_c1};
    const float *const b0[1] = {A.conv1_b + bo};
    ck_prime(R, t0, b0);
  }
  f32x4 acc1[1][NCT];
  f32x4 (&acc)[NCT] = acc1[0];

  /* conv1 (nnet.c:452-470): 252 inputs -> 128, tanh; cleared while frame_count < 1 (lpcnet.c:99) */
#pragma unroll
  for (int j = 0; j < NCT; j++) xb[j] = cs[j] * G::IN_SS + cf[j] * FIN; /* window = frames f-2..f */
  {
    const float4 *const c[1] = {t_c1};
    ck_tiles<3 * FIN, 3 * FIN, 3 * FIN, NCT, 1, PQ, XL>(R, c, t_c2, A.conv2_b + bo, inl, xb, acc1);
  }
#pragma unroll
  for (int j = 0; j < NCT; j++) {
    const bool clr = ck_fc(fcs[cs[j]], cf[j]) < 1;
    float4 t;
    t.x = clr ? 0.f : tanh_x86<HWR>(acc[j][0], rcp);
    t.y = clr ? 0.f : tanh_x86<HWR>(acc[j][1], rcp);
    t.z = clr ? 0.f : tanh_x86<HWR>(acc[j][2], rcp);
    t.w = clr ? 0.f : tanh_x86<HWR>(acc[j][3], rcp);
    *(float4 *)&c1[cs[j] * G::C1_SS + (cf[j] + 2) * CK_RS + 16 * wave + 4 * g] = t;
  }
  __syncthreads();

  CK_T(2);
  if constexpr (PS > 1) {
    /* the writer: the other slices have read the state (bounded wait: on a
     * timeout the status word reports the call invalid) */
    if (writer) {
      if (tid == 0) {
        int polls = 0;
        /* relaxed polls: the state stores below issue after the loop exits */
        while (__hip_atomic_load(&A.ck_sync[grp], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < PS - 1) {
          if (++polls > (1 << 22)) {
            A.status[0] = STATUS_SLICE_TIMEOUT; /* plain vector store to the pinned host word */
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        __hip_atomic_exchange(&A.ck_sync[grp], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
    }
  }
  /* the conv1 memory after the chunk: inputs of frames n-2, n-1 (nnet.c:469) */
  for (int e = tid; writer && e < G::SC * 2 * FIN; e += CK_THREADS) {
    const int s = e / (2 * FIN), j = e % (2 * FIN), sid = s0 + s;
    if (sid < B) A.st[sid].conv1_mem[j] = inl[s * G::IN_SS + n * FIN + j];
  }
  /* conv2: 384 inputs -> 128, tanh; cleared while frame_count < FEATURES_DELAY (lpcnet.c:101) */
#pragma unroll
  for (int j = 0; j < NCT; j++) xb[j] = cs[j] * G::C1_SS + cf[j] * CK_RS;
  {
    const float4 *const c[1] = {t_c2};
    ck_tiles<3 * COND, COND, CK_RS, NCT, 1, PQ, XL>(R, c, t_d1, A.dense1_b + bo, c1, xb, acc1);
  }
#pragma unroll
  for (int j = 0; j < NCT; j++) {
    const bool clr = ck_fc(fcs[cs[j]], cf[j]) < D;
    float4 t;
    t.x = clr ? 0.f : tanh_x86<HWR>(acc[j][0], rcp);
    t.y = clr ? 0.f : tanh_x86<HWR>(acc[j][1], rcp);
    t.z = clr ? 0.f : tanh_x86<HWR>(acc[j][2], rcp);
    t.w = clr ? 0.f : tanh_x86<HWR>(acc[j][3], rcp);
    *(float4 *)&ya[(16 * j + r) * CK_RS + 16 * wave + 4 * g] = t;
  }
  __syncthreads();

  CK_T(3);
  /* dense1, dense2 (lpcnet.c:104-105) */
#pragma unroll
  for (int j = 0; j < NCT; j++) xb[j] = (16 * j + r) * CK_RS;
  {
    const float4 *const c[1] = {t_d1};
    ck_tiles<COND, COND, CK_RS, NCT, 1, PQ, XL>(R, c, t_d2, A.dense2_b + bo, ya, xb, acc1);
  }
#pragma unroll
  for (int j = 0; j < NCT; j++)
    *(float4 *)&yb[(16 * j + r) * CK_RS + 16 * wave + 4 * g] =
        make_float4(tanh_x86<HWR>(acc[j][0], rcp), tanh_x86<HWR>(acc[j][1], rcp), tanh_x86<HWR>(acc[j][2], rcp),
                    tanh_x86<HWR>(acc[j][3], rcp));
  __syncthreads();
  {
    const float4 *const c[1] = {t_d2};
    ck_tiles<COND, COND, CK_RS, NCT, 1, PQ, XL>(R, c, nullptr, nullptr, yb, xb, acc1);
  }
#pragma unroll
  for (int j = 0; j < NCT; j++)
    *(float4 *)&ya[(16 * j + r) * CK_RS + 16 * wave + 4 * g] =
        make_float4(tanh_x86<HWR>(acc[j][0], rcp), tanh_x86<HWR>(acc[j][1], rcp), tanh_x86<HWR>(acc[j][2], rcp),
                    tanh_x86<HWR>(acc[j][3], rcp));
  __syncthreads();

  CK_T(4);
  /* END2END models (lpcnet.c:104,107-108): each frame's LPC = rc2lpc of the
   * first LPC_ORDER conditioning values, weighted by LPC_GAMMA; one lane per
   * (stream, frame) column */
  if (A.mc.end2end && tid < G::COLS) {
    const int s = tid / NFR, f = tid % NFR, sid = s0 + s;
    if (sid < B && f < n) {
      float rc[NLPC], lp[NLPC];
#pragma unroll
      for (int k = 0; k < NLPC; k++) rc[k] = ya[tid * CK_RS + k];
      rc2lpc_dev(lp, rc);
      float gi = gamma;
#pragma unroll
      for (int k = 0; k < NLPC; k++) {
        lp[k] = lp[k] * gi;
        gi *= gamma;
      }
      if (A.cond) {
        FrameCond *q = &A.cond[(size_t)f * B + sid];
#pragma unroll
        for (int k = 0; k < NLPC; k++) q->lpc[k] = lp[k];
      }
      if (f == n - 1 && writer)
#pragma unroll
        for (int k = 0; k < NLPC; k++) A.st[sid].lpc[k] = lp[k];
    }
  }

  /* conditioning projections (lpcnet.c:106-107), linear: gadf | gbdf as one
   * [128][1200] matrix, 75 row tiles over the 8 waves; frame f's outputs go
   * to cond[f], the last frame's also to the stream state */
  /* TP of this wave's tiles per pass (wave + 8 t, t < 10: the last pass of
   * waves 3..7 carries one tile past the 75th, computed on a clamped copy
   * and not stored) */
  /* sliced: this slice's tiles rt = PS lt + slice, lt = wave + 8 t */
  constexpr int WV = CK_THREADS / 64, NTS = (CK_PROJ_TILES + PS - 1) / PS, NT = (NTS + WV - 1) / WV;
  constexpr int TPS = PS > 1 ? NT : TP; /* all of a slice's tiles in one pass */
#pragma unroll 1
  for (int t0 = 0; t0 < NT; t0 += TPS) {
    const float4 *cur[TPS];
    const float *bia[TPS];
    int rts[TPS];
#pragma unroll
    for (int t = 0; t < TPS; t++) {
      const int rt = (wave + WV * (t0 + t)) * PS + slice;
      rts[t] = rt;
      const int rc = rt < CK_PROJ_TILES ? rt : slice; /* clamped: in bounds, result dropped */
      cur[t] = t_pj(rc);
      bia[t] = A.proj_b + 16 * rc + 4 * g;
    }
    constexpr int PQS = PS > 1 ? ck_pqp(TPS, NCT) : PQP;
    CkRing<TPS, PQS> RP;
    ck_prime(RP, cur, bia);
    f32x4 pacc[TPS][NCT];
    ck_tiles<COND, COND, CK_RS, NCT, TPS, PQS, XL>(RP, cur, nullptr, nullptr, ya, xb, pacc);
#pragma unroll
    for (int t = 0; t < TPS; t++) {
      if (rts[t] >= CK_PROJ_TILES) continue;
#pragma unroll
      for (int j = 0; j < NCT; j++) {
        const int sid = s0 + cs[j], f = cf[j];
        if (sid >= B || f >= n) continue;
        StreamState *p = &A.st[sid];
        /* this lane's 4 consecutive rows as one 16-byte store: the 4 lanes of
         * a column write its 16 rows as one 64-byte run (GA_ROWS is a multiple
         * of 16, so a row quad never straddles the two arrays) */
        const int row = 16 * rts[t] + 4 * g;
        const float4 v = make_float4(pacc[t][j][0], pacc[t][j][1], pacc[t][j][2], pacc[t][j][3]);
        if (A.cond) {
          FrameCond *q = &A.cond[(size_t)f * B + sid];
          float *qd = row < GA_ROWS ? q->gru_a_cond + row : q->gru_b_cond + (row - GA_ROWS);
          *(float4 *)qd = v;
        }
        if (f == n - 1) *(float4 *)(row < GA_ROWS ? p->gru_a_cond + row : p->gru_b_cond + (row - GA_ROWS)) = v;
      }
    }
  }

  CK_T(5);
  /* lpc_from_cepstrum of frame t of the chunk (one-frame launches: t = 0,
   * staged in LDS by the prologue) */
  auto lpcn = [&](int t, int s, int sid, int k) {
    if constexpr (NFR == 1) return nlpc[s * NLPC + k];
    else return A.lpc_new[((size_t)t * B + sid) * NLPC + k];
  };
  /* per frame: the LPC it synthesises with (lpcnet.c:110-118: the ring's
   * oldest slot, i.e. lpc_from_cepstrum of frame f - FEATURES_DELAY, then
   * lpc_weighting; END2END: written above) and frame_count after its update */
  for (int e = tid; writer && A.cond && e < G::SC * NFR * (NLPC + 1); e += CK_THREADS) {
    const int s = e / (NFR * (NLPC + 1)), rem = e % (NFR * (NLPC + 1));
    const int f = rem / (NLPC + 1), k = rem % (NLPC + 1), sid = s0 + s;
    if (sid >= B || f >= n) continue;
    FrameCond *q = &A.cond[(size_t)f * B + sid];
    if (k == NLPC) {
      const int fc = ck_fc(fcs[s], f);
      q->frame_count = fc < 1000 ? fc + 1 : fc;
    } else if (!A.mc.end2end) {
      const int t = f - D;
      q->lpc[k] = lpc_weight(t >= 0 ? lpcn(t, s, sid, k) : olpc[s][-1 - t][k], k, gamma);
    }
  }
  /* the stream state after the chunk: conv2 memory = conv1 outputs of frames
   * n-2, n-1; LPC ring; lpc of the last frame; frame_count */
  for (int e = tid; writer && e < G::SC * 2 * COND; e += CK_THREADS) {
    const int s = e / (2 * COND), j = e % (2 * COND), sid = s0 + s;
    if (sid < B) A.st[sid].conv2_mem[j] = c1[s * G::C1_SS + (n + j / COND) * CK_RS + j % COND];
  }
  if (!A.mc.end2end && writer && tid < G::SC * NLPC) {
    const int s = tid / NLPC, k = tid % NLPC, sid = s0 + s;
    if (sid < B) {
      auto L = [&](int t) { return t >= 0 ? lpcn(t, s, sid, k) : olpc[s][-1 - t][k]; };
      StreamState *p = &A.st[sid];
      p->lpc[k] = lpc_weight(L(n - 1 - D), k, gamma);
      /* deferred LPC (one frame, D >= 1): the frame read the ring's oldest
       * slot; lpc_kernel pushes this frame's LPC after the sample kernel */
      if (NFR != 1 || !A.lpc_defer)
        for (int j = 0; j < D; j++) p->old_lpc[j][k] = L(n - 1 - j);
    }
  }
  if (writer && tid < G::SC && s0 + tid < B) A.st[s0 + tid].frame_count = ck_fc(fcs[tid], n);
#ifdef CK_STAMPS
  CK_T(6);
  if (blockIdx.x == 0 && tid == 0)
    printf("ck<%d,%d> grid %d: inputs %llu conv1 %llu conv2 %llu dense %llu proj %llu epi %llu total %llu\n", NFR, SC,
           (int)gridDim.x, ck_t[1] - ck_t[0], ck_t[2] - ck_t[1], ck_t[3] - ck_t[2], ck_t[4] - ck_t[3], ck_t[5] - ck_t[4],
           ck_t[6] - ck_t[5], ck_t[6] - ck_t[0]);
#endif
}

template <int NFR, int SC, bool HWR, int PS = 1>
static int launch_chunk_t(const FrameArgs &a, void *stream)
{
  using G = CkGeom<NFR, SC>;
  /* sliced launches (one workgroup per CU at most 4 x 64 groups): more than
   * half the CU's LDS, so the dispatcher cannot pack two workgroups on one
   * CU -- two would share each SIMD's f32 matrix pipe, whose issue rate
   * bounds the layers (LPCNET_CK_PACK=1: the plain size, A/B) */
  static const bool pack = getenv("LPCNET_CK_PACK") && atoi(getenv("LPCNET_CK_PACK")) != 0;
  const int bytes = PS > 1 && !pack ? std::max(G::FLOATS * 4, 81 * 1024) : G::FLOATS * 4;
  if (ensure_dyn_lds((const void *)chunk_kernel<NFR, SC, HWR, PS>, bytes)) return -1;
  const int grid = (a.nstreams + G::SC - 1) / G::SC * PS;
  hipLaunchKernelGGL((chunk_kernel<NFR, SC, HWR, PS>), dim3(grid), dim3(CK_THREADS), bytes, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <bool HWR>
static int launch_chunk_h(const FrameArgs &a, void *stream)
{
  /* a workgroup's time grows with its column tiles, and the grid runs in
   * rounds of one workgroup per CU: 17..24 frames as 20 or 24 frames x 4
   * streams (5 or 6 column tiles) when that turns two rounds of 32 x 2 into
   * one (at 1024 streams: 20 frames 247 -> ~155 us) */
  const int cus = current_device_cus();
  /* estimated time: rounds of workgroups x column tiles per workgroup */
  auto cost = [&](int sc, int nct) { return ((a.nstreams + sc - 1) / sc + cus - 1) / cus * nct; };
  /* one frame (the per-frame host-I/O path of large batches: a live server's
   * 10 ms tick): stream-only columns, 16 or 32 streams per workgroup -- a
   * workgroup's time is mostly its pass over the 1.08 MB of weights, so the
   * smaller tile while the grid fits two rounds */
  if (a.nframes == 1) {
    /* row slices while the groups leave CUs idle (1024 streams: 64 groups x 4
     * slices = one workgroup per CU) */
    const int groups = (a.nstreams + 15) / 16;
    static const int ps_env = getenv("LPCNET_CK_SLICES") ? atoi(getenv("LPCNET_CK_SLICES")) : -1;
    const int ps = !a.ck_sync || !a.status || a.cond ? 1
                   : ps_env >= 1 ? ps_env
                   : 4 * groups <= cus ? 4 : 2 * groups <= cus ? 2 : 1;
    static_assert(CK_SLICES_MAX >= 4, "weight copies per slice");
    if (ps >= 4) return launch_chunk_t<1, 16, HWR, 4>(a, stream);
    if (ps == 2) return launch_chunk_t<1, 16, HWR, 2>(a, stream);
    return groups <= 2 * cus ? launch_chunk_t<1, 16, HWR>(a, stream) : launch_chunk_t<1, 32, HWR>(a, stream);
  }
  if (a.nframes <= 8) return launch_chunk_t<8, 8, HWR>(a, stream);
  if (a.nframes <= 16) return launch_chunk_t<16, 4, HWR>(a, stream);
  if (a.nframes <= 20 && cost(4, 5) < cost(2, 4)) return launch_chunk_t<20, 4, HWR>(a, stream);
  if (a.nframes <= 24 && cost(4, 6) < cost(2, 4)) return launch_chunk_t<24, 4, HWR>(a, stream);
  return launch_chunk_t<32, 2, HWR>(a, stream);
}

int launch_chunk(const FrameArgs &a, void *stream)
{
  /* one-frame launches may run without per-frame outputs (cond null): the
   * stream state carries the frame's conditioning, LPC and frame_count, and
   * the sample kernel reads them from there */
  if (a.nframes < 1 || a.nframes > LPC_CHUNK || (!a.cond && a.nframes != 1)) return -1;
  /* tanh through the hardware reciprocal, or through the LDS table when the
   * batch carries another host's rcpps (same-box parity) */
  return a.rcp_hw ? launch_chunk_h<true>(a, stream) : launch_chunk_h<false>(a, stream);
}

}  // namespace lpcnet_mi355x
