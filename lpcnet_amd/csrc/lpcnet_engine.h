/*
 * lpcnet_engine.h -- internal declarations of the MI355X LPCNet engine.
 * Shared by the host engine (engine.cpp) and the HIP kernels (kernels.hip).
 */
#ifndef LPCNET_ENGINE_H
#define LPCNET_ENGINE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lpcnet_mi355x {

/* Default model dimensions (training_tf2/lpcnet.py:312-325; the reference
 * bakes them into the generated nnet_data.h). */
constexpr int NA = 384;        /* GRU_A units */
constexpr int NB = 16;         /* GRU_B units */
constexpr int COND = 128;      /* conditioning size */
constexpr int NF = 20;         /* NB_FEATURES */
constexpr int EP = 64;         /* pitch embedding */
constexpr int FIN = NF + EP;   /* lpcnet.c:44 FRAME_INPUT_SIZE */
constexpr int NLPC = 16;       /* LPC_ORDER */
constexpr int FRAME = 160;     /* samples per frame */
constexpr int NBANDS = 18;     /* freq.h:48 NB_BANDS (cepstral bands of the 1.6 kb/s decoder) */
constexpr int GA_ROWS = 3 * NA;
constexpr int GB_ROWS = 3 * NB;
/* Model constants the reference bakes into the generated nnet_data.h
 * (dump_lpcnet.py:423-446, from train_lpcnet.py --lookahead / --lpc-gamma /
 * --end2end); here load-time parameters of a model (ModelConst). */
constexpr int DEFAULT_FEATURES_DELAY = 2; /* dump_lpcnet.py:441 default lookahead */
constexpr int MAX_FEATURES_DELAY = 4;     /* train_lpcnet.py:273 trims (4 - lookahead) frames: lookahead <= 4 */
constexpr int SAMPLE_THREADS = 384; /* one thread per GRU_A unit */
constexpr int SAMPLE_WAVES = SAMPLE_THREADS / 64;
constexpr int STAMP_WAVES = 8;      /* stamps are [workgroup][STAMP_WAVES][16] */
constexpr int FRAME_STREAMS = 4;    /* streams per frame-network workgroup */
constexpr int FRAME_PREFETCH = 64;  /* zero input rows padding each frame-network weight matrix */
constexpr int REG_GB = 12;          /* GRU_B input slots per lane: block k = ks + 8*j, j < 12 */
/* Matrix-core kernel (mf_kernel.hip).
 * GRU_A (v_mfma_i32_4x4x4_16b_i8): per-lane register tables, one u32 word
 * per slot.  Lane l of GRU_A wave w = (row group l/4 of the wave's 64 units,
 * row l%4 of the group); word k of the table holds
 *   [0, 16)   z-gate weight rows, slot t  (4 int8 = one row of an 8x4 block)
 *   [16, 32)  r-gate weight rows
 *   [32, 64)  h-gate weight rows
 *   [64, 80)  column-block bytes of those 64 slots (4 per word)
 * Unused slots hold zero weights and column block 0.
 * GRU_B (v_mfma_i32_16x16x64_i8, sampler waves): dense int8 A tiles, lane l
 * = row 16g + l%16, bytes k = 64kt + 16(l/16) + 0..15: tiles [g*6 + kt]
 * (input, 3 gates x 6 K tiles) then [18 + g] (recurrent, K = 16 in lanes
 * 0..15), [MF_GB_TILES][64 lanes] uint4. */
constexpr int MF_ZMAX = 16;         /* z / r slots per lane */
constexpr int MF_HMAX = 32;         /* h slots per lane */
constexpr int MF_GA = 2 * MF_ZMAX + MF_HMAX;
constexpr int MF_LANE_U32 = MF_GA + MF_GA / 4; /* 80 */
/* mfw_kernel split form (engine.cpp mfw_split_tables): two host waves after
 * the six R waves carry the pieces of block rows beyond the register caps */
constexpr int MFW_H_WAVES = 2;
constexpr int MFW_TAB_WAVES = 6 + MFW_H_WAVES; /* SAMPLE_WAVES R waves + the host waves */
constexpr int MFW_NOROW = 0x1FF;               /* frow entry: no part row */
constexpr int MFW_PART_ROWS = 128;             /* part rows per gate: 16 unit blocks x 8 */
constexpr int MF_GB_IN = 3 * 6;                 /* GRU_B input tiles (3 gates x 6 K tiles) */
constexpr int MF_GB_TILES = MF_GB_IN + 3;        /* + the 3 recurrent tiles */
constexpr int MF_XSTR = 416;        /* LDS bytes per stream of the quantized GRU_A state (stream-major):
                                       104 dwords = 8 banks (mod 32) apart, so the 4 streams of
                                       input quad c occupy banks c + {0, 8, 16, 24} (mod 32) */
constexpr int MF_THREADS = 512;     /* 6 GRU_A waves + 2 sampler waves */
/* fp32 latency kernel (fp_kernel.hip), one stream per workgroup.
 * GRU_A per-lane tables (lane l of wave w = unit 64w + l = row l%8 of row
 * block 8w + l/8 of each gate; slot t = the t-th 8x4 block of that row block,
 * as the float4 of this row's 4 columns):
 *   fp_zr [wave][2][FP_ZF][64] float4: slot t as packed (z, r) pairs,
 *         [z.x r.x z.y r.y] then [z.z r.z z.w r.w] (registers)
 *   fp_h  [wave][FP_HF][64] float4: h slots (streamed from L2 every sample)
 *   fp_off [wave][FP_OFF_WORDS][64] u32: column-quad bytes, 4 per word, of
 *         the z, r and h slots
 * Unused slots hold -0.0 weights and column quad NA/4, which the kernel
 * keeps at +0.0: fma(-0, +0, y) = y for every y, NaN and -0 included.
 * fp_gb [NA/4][GB_ROWS] float4: dense GRU_B input weights (column quad,
 * row), copied to LDS. */
constexpr int FP_ZF = 16;           /* z / r slots per lane */
constexpr int FP_HF = 32;           /* h slots per lane */
constexpr int FP_OFF_WORDS = (2 * FP_ZF + FP_HF) / 4;
constexpr int FP_THREADS = 448;     /* 6 GRU_A waves + 1 sampler wave */

/* Per-stream synthesis state in device memory (lpcnet_private.h:28-48). */
struct alignas(16) StreamState {
  float gru_a_state[NA];
  float gru_a_cond[GA_ROWS];
  float gru_b_cond[GB_ROWS];
  float gru_b_state[NB];
  float last_sig[NLPC];
  float lpc[NLPC];
  float old_lpc[MAX_FEATURES_DELAY][NLPC]; /* lpc_from_cepstrum ring, first `delay` rows used */
  float conv1_mem[FIN * 2];
  float conv2_mem[COND * 2];
  float deemph_mem;
  int last_exc;
  int frame_count;
  uint32_t rng[4];
  /* LPCNetDecState::vq_mem (lpcnet_private.h:50-53): the previous packet's
   * last cepstrum, read by decode_packet (lpcnet_dec.c:81-156); zero after
   * a reset (lpcnet_decoder_init memsets the decoder state) */
  float vq_mem[NBANDS];
  int pad[3];
};

/* The device rcpps table holds t + kRcpBias (device_math.h rcp_x86_fix),
 * indexed by the top RCP_TABLE_BITS mantissa bits of the Pade denominator:
 * 12, so one table format holds both the Intel build host's rcpps (a
 * function of the top 11 bits: each entry twice) and the AMD EPYC GPU-box
 * host's (a function of the top 12 bits, profiles/r03/box_rcpps.json). */
constexpr uint32_t kRcpBias = 127u << 23;
constexpr int RCP_TABLE_BITS = 12;
constexpr int RCP_ENTRIES = 1 << RCP_TABLE_BITS;

/* Fixed sections of the sample kernel's LDS image (byte offsets). */
constexpr int IMG_RCP = 0;                       /* RCP_ENTRIES u32 rcpps table */
constexpr int IMG_ULAW = IMG_RCP + RCP_ENTRIES * 4; /* 256 f32 ulaw2lin */
constexpr int IMG_LOGIT = IMG_ULAW + 256 * 4;    /* 256 f32 sampling logit table */
constexpr int IMG_FCW = IMG_LOGIT + 256 * 4;     /* dual_fc weights [256][2][16] f32 */
constexpr int IMG_FCB = IMG_FCW + 256 * 32 * 4;  /* dual_fc bias [2][256] */
constexpr int IMG_FCF = IMG_FCB + 512 * 4;       /* dual_fc factor [2][256] */
constexpr int IMG_VAR = IMG_FCF + 512 * 4;       /* start of the variable sections */

/* What one frame step hands from the frame kernel to the sample kernel,
 * double-buffered by the overlapped multi-frame path (frame kernel f+1 runs
 * beside sample kernel f): the conditioning vectors, the LPC of this frame
 * and frame_count after this frame's update. */
constexpr int ZC_FEAT_MAX = 4096; /* host-I/O ticks up to this size read the features from mapped host memory */
constexpr int TICK_SPIN_MS = 20;  /* a host-I/O tick polls its end this long before a blocking wait */
constexpr int TICK_POLL_PAUSE = 0; /* x86 pause instructions between two polls */
constexpr int OVERLAP_MAX_STREAMS = 128; /* batches up to this size get the overlapped multi-frame path (sample + frame workgroups fit the 256 CUs) */

struct alignas(16) FrameCond {
  float gru_a_cond[GA_ROWS];
  float gru_b_cond[GB_ROWS];
  float lpc[NLPC];
  int frame_count;
  int pad[3];
};

/* FEATURES_DELAY (lookahead frames: the LPC ring depth, the conv2 clear and
 * the silent first frames, lpcnet.c:101,109-112,239), LPC_GAMMA
 * (lpc_weighting, lpcnet.c:116-118) and END2END (LPC from the frame
 * network's rc outputs, lpcnet.c:56-80,107-108) of a model. */
struct ModelConst {
  float lpc_gamma;
  int delay;
  int end2end;
};

struct FrameArgs {
  StreamState *st;
  ModelConst mc;
  int nstreams;
  const float *features; /* [B][NF] for this frame */
  const float *lpc_new;  /* [B][NLPC] lpc_from_cepstrum(features) (lpc_kernel) */
  const float *conv1_w, *conv1_b, *conv2_w, *conv2_b;
  const float *dense1_w, *dense1_b, *dense2_w, *dense2_b;
  const float *gadf_w, *gadf_b, *gbdf_w, *gbdf_b;
  const float *proj_w, *proj_b; /* gadf | gbdf as one [COND][GA_ROWS + GB_ROWS] matrix, bias */
  const float *embed_pitch;
  const uint32_t *rcp; /* RCP_ENTRIES-entry table in global memory */
  unsigned long long *stamps; /* optional diagnostics [grid][16] s_memtime per phase */
  /* chunk_kernel only: features = [nframes][B][NF], lpc_new = [nframes][B][NLPC],
   * outputs of frame f into cond[f * B .. f * B + B) */
  int nframes;
  FrameCond *cond;
  /* frame_kernel: 1 = run_frame_network into the caller's locals, as
   * run_frame_network_flush does (lpcnet.c:134-144): conv memories, LPC ring
   * and frame_count advance, the state's conditioning and lpc stay */
  int keep_cond;
  int rcp_hw; /* chunk_kernel: hardware-reciprocal tanh allowed (see SampleArgs::rcp_hw) */
  /* chunk_kernel: the same five weight matrices re-tiled for 16-byte
   * per-lane loads (ck_tile_weights): [row tile][k quad][64 lanes] float4,
   * lane l = (g, r) = (l / 16, l % 16), element j of quad q = W[4 (4q + j) +
   * g][16 rt + r] (0 past K), CK_WPAD zero quads after each row tile's last */
  const float4 *ck_conv1, *ck_conv2, *ck_dense1, *ck_dense2, *ck_proj;
  /* conv1 .. dense2 are stored CK_SLICES_MAX times: copy k at + k ck_rep[i]
   * float4s (projection slice k of the one-frame kernel reads copy k) */
  int ck_rep[4];
  /* one-frame chunk_kernel, deferred LPC (FEATURES_DELAY >= 1): the frame's
   * LPC comes from the ring only, the ring is advanced later by lpc_kernel
   * (launch_lpc with a ring), and the frame's features are copied to
   * lpc_feat ([B][NF], device memory) for it when non-null */
  int lpc_defer;
  float *lpc_feat;
  /* one-frame chunk_kernel with its projection split over row slices
   * (launch_chunk picks the slice count): per 16-stream group an arrival
   * counter (zeroed, [groups]); a timed-out wait sets STATUS_SLICE_TIMEOUT
   * in *status (the batch's status word) */
  int *ck_sync;
  int *status;
};
constexpr int CK_SLICES_MAX = 4; /* projection slices of the one-frame chunk kernel */
constexpr int CK_WPAD = 8; /* chunk_kernel: k quads in flight per wave (zero padding of each row tile) */

struct SampleArgs {
  StreamState *st;
  int delay;             /* FEATURES_DELAY: a stream synthesises once frame_count > delay (lpcnet.c:239) */
  const FrameCond *cond; /* optional [B]: read the frame's outputs here instead of st */
  int nstreams;
  int N;                 /* samples to produce (<= FRAME) */
  int nframes;           /* mf_kernel: frames per launch (0 = 1).  Frame f reads cond + f B and
                            writes pcm + f B N; needs cond, preload 0, no trace, and every
                            stream active in all or none of the frames (the host splits a run
                            at the `delay` transition, STATUS_ACTIVITY otherwise) */
  short *pcm;            /* [B][N] */
  int preload;           /* samples 0..preload-1 are teacher-forced from pcm (lpcnet.c:256-259) */
  const float *emb_sig, *emb_pred, *emb_exc; /* [256][GA_ROWS] */
  const float *ga_par;   /* [6][NA]: recurrent bias z,r,h then diag z,r,h */
  const int *ga_wsum;    /* [3][NA]: 128*rowsum(int8 w) (non-saturating int8 path) */
  const float *gb_par;   /* [2][GB_ROWS]: input bias, recurrent bias */
  const int *gb_wsum;    /* [2][GB_ROWS] */
  const uint4 *image;    /* LDS image */
  int image_bytes;
  int image_lds_bytes;   /* lockstep kernel: bytes of the image copied to LDS (image_bytes, or IMG_VAR
                            when the weight sections stay in global memory) */
  int ga_K[SAMPLE_WAVES][3];   /* blocks per lane for wave w, gate g (padded) */
  int ga_woff[SAMPLE_WAVES][3];/* weight chunk offset (u32 units in image / float4 units in ga_wf) */
  int ga_coff[SAMPLE_WAVES][3];/* column-block index chunk offset (u16 units in image) */
  int gb_nb[GB_ROWS / 8];      /* blocks per GRU_B row block */
  int gb_woff[GB_ROWS / 8];    /* u32 units in image [k][8] / float4 [k][8][2] in gb_wf */
  int gb_coff[GB_ROWS / 8];    /* u16 units in image */
  int gb_rec_off;              /* byte offset of GRU_B recurrent int8 weights in image */
  /* quad int8 path (LDS image): per wave w / GRU_B row block, group of 4 slots gi:
   * weights [gi][64 lanes] uint4 at *_qoff (uint4 units), column blocks
   * [gi][8] u32 (4 x u8, one per lane octet) at *_coff (u32 units) */
  int ga_K4[SAMPLE_WAVES][3];
  int ga_qoff[SAMPLE_WAVES][3];
  int gb_qoff[GB_ROWS / 8];
  /* matrix-core kernel: GRU_A per-lane register tables [wave][MF_LANE_U32][64
   * lanes], 4-slot groups per wave (z/r padded to a common count, h); GRU_B
   * A tiles [MF_GB_TILES][64] */
  const uint32_t *mf;
  const int *mf_unit;                /* [SAMPLE_WAVES * 64]: GRU_A unit of each lane */
  float mf_zr_bound;                 /* |GRU_A z/r conditioning| below this (and finite) for a workgroup's
                                        streams: the elementwise step's range selects are dead (mf_kernel);
                                        negative: never */
  float mf_h_bound;                  /* the same for the h gate's conditioning (tanh range) */
  int fc_fin;                        /* every dual-FC node sum |bias| + 2 sum|w| is finite and below
                                        2^59: with GRU_B states within [-2, 2] (int8 models keep them
                                        there; checked per launch) the walk's tanh takes the
                                        select-free form */
  const float *mf_emb[3];            /* sig/pred/exc tables with columns in lane order:
                                        [256][3][SAMPLE_WAVES * 64], column p = unit mf_unit[p] */
  int mf_nzr[SAMPLE_WAVES];          /* own 4-slot groups per GRU_A wave: z and r */
  int mf_nh[SAMPLE_WAVES];           /* h */
  /* split models (rows longer than the own cap, engine.cpp mf_plan): hosted
   * 4-slot groups after the own ones, the row each lane's hosted partial
   * sums belong to [3 gates][SAMPLE_WAVES * 64] (NA: none) */
  int mf_split;
  int mf_nfzr[SAMPLE_WAVES];
  int mf_nfh[SAMPLE_WAVES];
  const int *mf_frow;
  /* mfw_kernel's split form: [MFW_TAB_WAVES][MF_LANE_U32][64] tables (R
   * waves own rows to the full caps, host waves the pieces), group counts,
   * frow [3][SAMPLE_THREADS + 64 MFW_H_WAVES] (see mfw_split_tables) */
  int mfw_split;
  const uint32_t *mfw_tab;
  const int *mfw_frow;
  const int *mfw_unit;      /* [SAMPLE_THREADS]: the split form's own unit of each E / R lane */
  const float *mfw_emb[3];  /* embedding tables in the split form's lane order (as mf_emb) */
  int mfw_nzr[MFW_TAB_WAVES];
  int mfw_nh[MFW_TAB_WAVES];
  const uint4 *mf_gb;
  const float4 *fp_zr, *fp_h, *fp_gb; /* fp_kernel tables (see FP_ZF) */
  const uint32_t *fp_off;
  int fp_nzr[SAMPLE_WAVES];    /* slots of the z/r chains per GRU_A wave */
  int fp_nh[SAMPLE_WAVES];     /* slots of the h chains */
  /* fp_kernel long form (block rows beyond FP_ZF / FP_HF): every slot
   * streamed, [wave][slot][64 lanes]: z/r packed pairs (2 float4), h float4,
   * offsets (z quad | r quad << 8 for fpl_kz slots, then h quads) */
  int fp_long;
  int fpl_kz, fpl_kh;
  const float4 *fpl_zr, *fpl_h;
  const uint32_t *fpl_off;
  const float4 *ga_wf;   /* fp32 variant: GRU_A blocks [chunk][k][64] float4 */
  const float4 *gb_wf;   /* fp32 variant: GRU_B blocks [rb][k][8 rows][2] float4 (in c) */
  const float *gb_recf;  /* fp32 variant: GRU_B recurrent [NB][GB_ROWS] */
  unsigned long long *stamps; /* optional diagnostics [grid][STAMP_WAVES][16] s_memtime sums */
  float *trace_logits;   /* optional [B][N][8] */
  int *trace_exc;        /* optional [B][N] */
  int rcp_hw;            /* 1: the latency chains may use the hardware-reciprocal rcpps (equal to the
                            default Intel table only); 0: every activation through the LDS table
                            (lpcnet_batch_set_rcp_table with another host's table) */
  int *status;           /* device view of the batch's pinned status word: a
                            kernel that aborts sets bits (STATUS_*), the host
                            checks after every sync */
  int spin_limit;        /* polls before an LDS flag wait aborts (FLAG_SPIN_LIMIT_DEFAULT) */
};

constexpr int FLAG_SPIN_LIMIT_DEFAULT = 1 << 20; /* lpcnet_batch_set_spin_limit */
constexpr int FLAG_SPIN_LIMIT_MAX = 1 << 30;     /* larger requests are clamped (int poll counters) */
/* Status bits a sample kernel reports to the host (SampleArgs::status). */
constexpr int STATUS_FLAG_TIMEOUT = 1; /* an LDS flag wait exceeded spin_limit: output invalid */
constexpr int STATUS_ACTIVITY = 2;     /* a multi-frame launch saw a stream become active mid-launch */
constexpr int STATUS_SLICE_TIMEOUT = 4; /* a sliced chunk_kernel's writer waited too long for its siblings */

/* The frame step's outputs as a sample kernel reads them: the FrameCond
 * copy when the launch has one, else the stream state. */
#if defined(__HIP__) || defined(__HIPCC__)
/* the same with the frame's conditioning array given (multi-frame launches) */
__device__ __forceinline__ int frame_count_of(const SampleArgs &A, const FrameCond *cf, int sid)
{
  return cf ? cf[sid].frame_count : A.st[sid].frame_count;
}
__device__ __forceinline__ const float *gru_a_cond_of(const FrameCond *cf, const SampleArgs &A, int sid)
{
  return cf ? cf[sid].gru_a_cond : A.st[sid].gru_a_cond;
}
__device__ __forceinline__ const float *gru_b_cond_of(const FrameCond *cf, const SampleArgs &A, int sid)
{
  return cf ? cf[sid].gru_b_cond : A.st[sid].gru_b_cond;
}
__device__ __forceinline__ const float *lpc_of(const FrameCond *cf, const SampleArgs &A, int sid)
{
  return cf ? cf[sid].lpc : A.st[sid].lpc;
}
__device__ __forceinline__ int frame_count_of(const SampleArgs &A, int sid)
{
  return A.cond ? A.cond[sid].frame_count : A.st[sid].frame_count;
}
__device__ __forceinline__ const float *gru_a_cond_of(const SampleArgs &A, int sid)
{
  return A.cond ? A.cond[sid].gru_a_cond : A.st[sid].gru_a_cond;
}
__device__ __forceinline__ const float *gru_b_cond_of(const SampleArgs &A, int sid)
{
  return A.cond ? A.cond[sid].gru_b_cond : A.st[sid].gru_b_cond;
}
__device__ __forceinline__ const float *lpc_of(const SampleArgs &A, int sid)
{
  return A.cond ? A.cond[sid].lpc : A.st[sid].lpc;
}
#endif

/* Host helpers shared by the launchers (engine.cpp), thread-safe and keyed
 * by the current HIP device: raise a kernel's dynamic-LDS limit to `bytes`
 * once per (kernel, device); the CU count of the current device. */
int ensure_dyn_lds(const void *kernel, int bytes);
int current_device_cus();

/* Kernel launchers (kernels.hip).  variant: 0 int8, 1 fp32. sat: int8 pairs
 * may saturate. lds_bytes from sample_lds_bytes(). */
int sample_lds_bytes(int S, int variant, int image_bytes);
int launch_frame(const FrameArgs &a, void *stream);
constexpr int FK_ONE_STREAM_MAX = 256; /* frame kernel: one stream per workgroup up to this batch */
int frame_groups(int nstreams);        /* frame kernel workgroups (stamp rows) for a batch */
/* copy the frame step's outputs of every stream into cond[B] */
int launch_cond_copy(const StreamState *st, FrameCond *cond, int nstreams, void *stream);
/* dst[dmap ? dmap[k] : k] = src[smap ? smap[k] : k], k < n (device index maps) */
int launch_state_copy(StreamState *dst, const StreamState *src, const int *dmap, const int *smap, int n, void *stream);
int launch_sample(const SampleArgs &a, int S, int variant, int sat, int reg, int lds_bytes, void *stream);

/* Frame network of up to LPC_CHUNK frames in one launch (chunk_kernel.hip):
 * f32 matrix cores, 64 (stream, frame) columns per workgroup. */
int launch_chunk(const FrameArgs &a, void *stream);
constexpr int CHUNK_MIN_FRAMES = 4; /* shorter runs use the per-frame kernel */
/* Matrix-core kernel (non-saturating int8 models within the MF_* limits):
 * GRU_A recurrent product on v_mfma_i32_4x4x4_16b_i8 in the GRU_A waves,
 * GRU_B products on v_mfma_i32_16x16x64_i8 in the sampler waves, two
 * workgroup barriers per sample. */
int mf_lds_bytes(int S, int split);
int launch_mf(const SampleArgs &a, int S, int lds_bytes, void *stream);
/* Large batches: two groups of S streams per workgroup, half a sample
 * apart (mf2_kernel.hip); no preload / trace / stamps. */
constexpr int MF2_MIN_STREAMS = 2048; /* automatic choice of mf2_kernel from this batch size */
int mf2_lds_bytes(int S, int split);
int launch_mf2(const SampleArgs &a, int S, void *stream);
/* wide-batch kernel (mfw_kernel.hip): 2 or 3 four-stream groups per
 * 896-thread workgroup with dedicated gather/elementwise, recurrent and
 * sampler waves (split models: two groups, 1,024 threads with two host
 * waves); int8 models with the default (Intel) rcpps, no preload / trace /
 * stamps (-1 otherwise) */
/* mfw_kernel runs in rounds of one workgroup per CU.  Per stream at whole
 * rounds (24,576 streams, same box, profiles/r05): two groups 7.07 ms per
 * frame, three 7.36 (per-phase time 1.04x), mf2_kernel 8.02 -- so two
 * groups replace mf2_kernel wherever both apply (same 8-stream rounds), and
 * three groups are taken where their 12-stream rounds save more than the 4 %
 * (3,072 streams: one round against two).  Above 4 streams per CU only:
 * below, mf_kernel's one-group latency wins. */
constexpr double MFW_G3_PHASE = 1.08; /* 1.04 before two groups took the LDS rcpps table (-3.4 %) */
/* 0 (batch within one mf_kernel<4> round), 2 or 3 */
int mfw_groups(int B, int cus);
int mfw_lds_bytes(int groups, int split = 0);
int launch_mfw(const SampleArgs &a, int groups, void *stream);
/* fp32 latency kernel: one stream per workgroup, LDS flags instead of
 * workgroup barriers (fp32 models within the FP_* limits, dense GRU_B). */
int fp_lds_bytes();
int launch_fp(const SampleArgs &a, void *stream);

/* lpc_from_cepstrum on the device (lpc_kernel.hip).  Constant tables built
 * once per batch on the host (engine.cpp build_lpc_tables): the idct matrix
 * (freq.c dct_table), the 320-point kiss FFT twiddles and input permutation
 * (kiss_fft.c, lpcnet_tables.c), the band index and interpolation fraction of
 * every spectrum bin (freq.c:202-216), the compensation factors (freq.c:50). */
constexpr int LPC_NBANDS = NBANDS;
constexpr int LPC_WIN = 320;
constexpr int LPC_ORDER1 = NLPC + 1;
constexpr int LPC_CHUNK = 32;     /* frames per batched lpc_kernel launch (lpcnet_batch_synthesize_frames) */
/* FFT input slot i (after kiss_fft's digit reversal): spectrum bin
 * k = perm[i] (mirrored to 320 - k above 160), interpolated between band
 * energies `band` and band + 1 with fraction `frac` (band = NB_BANDS - 1 for
 * the zero bin 160), imaginary part -0.f for the mirrored (conjugate) bins. */
struct LpcSlot {
  float frac;
  unsigned char band, conj, pad[2];
};
struct LpcTables {
  double sqrt_2_18;               /* sqrt(2./NB_BANDS) (freq.c:238) */
  float scale;                    /* 1/320, kiss_fft's inverse scaling */
  float dct[LPC_NBANDS * LPC_NBANDS];
  float comp[LPC_NBANDS];
  float twr[LPC_WIN], twi[LPC_WIN];
  LpcSlot slot[LPC_WIN];
};
/* features [nstreams][NF] -> lpc_out [nstreams][NLPC] */
/* read-only matrices an idle-time kernel touches once per 128-byte line in
 * every XCD's L2 (the deferred lpc_kernel warms the one-frame chunk
 * kernel's weights for the next tick) */
struct L2Warm {
  const uint32_t *m[5];
  int lines[5];
};
int launch_lpc(const float *features, float *lpc_out, int nstreams, const LpcTables *tables, void *stream,
               StreamState *ring = nullptr, int ring_depth = 0, const L2Warm *warm = nullptr);

/* decode_packet (lpcnet_dec.c:81-156) on the device (decode_kernel.hip):
 * packets [npackets][nstreams][8] -> features [4 npackets][nstreams][NF],
 * each stream's vq_mem in st carried from packet to packet. */
struct DecodeArgs {
  const unsigned char *packets;
  int npackets, nstreams;
  StreamState *st;
  const float *cb1, *cb2, *cb3; /* ceps_codebook1..3 [1024][NBANDS - 1] */
  const float *cbd;             /* ceps_codebook_diff4 [4096][NBANDS] */
  const float *pitch;           /* [64]: (float)(pow(2.f, m / 21.) * PITCH_MIN_PERIOD) (lpcnet_dec.c:118) */
  float *features;
};
constexpr int DEC_MAX_PACKETS = LPC_CHUNK / 4; /* packets per decode launch (the frames of one chunk) */
int launch_decode(const DecodeArgs &a, void *stream);

}  // namespace lpcnet_mi355x

#endif
