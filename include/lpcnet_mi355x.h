/*
 * lpcnet_mi355x.h -- batch extension and tooling of liblpcnet_mi355x.so.
 *
 * The reference has no batch API (one LPCNetState = one stream on one core,
 * SURVEY.md section 8b).  A batch owns B independent streams, each with
 * exactly the semantics of one reference LPCNetState; stream s of a batch is
 * PCM-identical to the same stream run alone through lpcnet_synthesize().
 * Streams shard across GPUs with no collective (one batch per device).
 */
#ifndef LPCNET_MI355X_H
#define LPCNET_MI355X_H

#include "lpcnet.h"
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct LPCNetBatch LPCNetBatch;

/* Weight-blob variants (chosen from the array sizes of the blob). */
#define LPCNET_VARIANT_INT8 0 /* reference AVX2 build: DOT_PROD int8 GRU weights */
#define LPCNET_VARIANT_FP32 1 /* reference --disable-dot-product build */

typedef struct {
  int variant;          /* LPCNET_VARIANT_* */
  int gru_a_blocks;     /* 8x4 blocks in sparse_gru_a_recurrent_weights */
  int gru_b_blocks;     /* 8x4 blocks in gru_b_weights */
  int may_saturate;     /* 1 if an int8 pair can saturate the int16 maddubs sum */
  double bytes_shared_per_frame;  /* algorithmic weight bytes read once per frame step */
  double bytes_shared_per_sample; /* algorithmic weight bytes read once per sample step (SURVEY 8d;
                                     add bytes_shared_per_frame / 160 for the whole step) */
  double bytes_per_stream_sample; /* per-stream bytes per sample (3 embedding rows, dual_fc path,
                                     conditioning/features/PCM share; SURVEY 8d: 15,009) */
  double ops_per_sample;          /* 2*MAC per stream per sample */
  int streams_per_workgroup;      /* streams per sample-kernel workgroup */
  int quad_path;                  /* sample kernel: 0 lockstep (per-slot LDS layout), 1 lockstep (quad
                                     LDS layout), 4 mf_kernel (matrix cores), 5 fp_kernel (fp32),
                                     6 mf2_kernel (matrix cores, two staggered 4-stream groups per
                                     workgroup; batches >= 2048; launches with preload or trace
                                     take mf_kernel), 7 mfw_kernel (two or three 4-stream groups per
                                     workgroup, chosen by cost -- two in the common case -- with dedicated
                                     gather/elementwise, recurrent and sampler waves; batches above one
                                     mf_kernel<4> round (> 4 streams per CU, i.e. > 1024 streams),
                                     non-split models, default rcpps; the same launches as 6) */
  int lds_bytes;                  /* dynamic LDS of the sample kernel */
  double mfma_ops_per_group_sample; /* int8 matrix-core ops issued per workgroup per sample
                                       (mf_kernel; padding included), 0 otherwise */
  /* model constants (see lpcnet_batch_set_model_constants) */
  float lpc_gamma;
  int features_delay;
  int end2end;
  /* 1: block rows longer than the fast kernels' register tables (trained
   * Sparsify masks): mf_kernel runs its split form, fp_kernel its streamed
   * (long) form */
  int long_rows;
  /* 1: the blob carries the 1.6 kb/s decoder's codebooks (ceps_codebook1..3,
   * ceps_codebook_diff4), so lpcnet_decode / lpcnet_batch_decode* accept it */
  int has_codebooks;
  /* 1: the fast kernels may use the hardware reciprocal for rcpps (the
   * default Intel table); 0: a custom table is set and they run their
   * table-only forms (the `HWR` template argument rocprofv3 shows) */
  int rcp_hw;
} LPCNetModelInfo;

/* Create a batch of nb_streams streams on HIP device `device`.
 * Returns NULL if the device is unavailable or nb_streams < 1. */
LPCNET_EXPORT LPCNetBatch *lpcnet_batch_create(int nb_streams, int device);
LPCNET_EXPORT void lpcnet_batch_destroy(LPCNetBatch *b);
/* 0 on success, -1 on a missing / mis-sized array (lpcnet_load_model rules). */
LPCNET_EXPORT int lpcnet_batch_load_model(LPCNetBatch *b, const unsigned char *data, int len);
LPCNET_EXPORT int lpcnet_batch_model_info(const LPCNetBatch *b, LPCNetModelInfo *info);
/* Sample-kernel selection: 0 automatic (default; env LPCNET_KERNEL),
 * 1 the lockstep kernel (every model: the fallback for saturating int8 models
 * and fp32 models with a sparse GRU_B), 4 mf_kernel (both int8 products on
 * the matrix cores; non-saturating int8 models whose blocks fit its register
 * tables), 5 fp_kernel (fp32 models with a dense GRU_B whose blocks fit its
 * tables).  Automatic: 5 where it applies, else 4 where it applies, else 1;
 * a forced mode the model cannot run falls back to 1.  Results are
 * identical; only speed differs.  Returns -1 for any other mode. */
LPCNET_EXPORT int lpcnet_batch_set_kernel(LPCNetBatch *b, int mode);
/* The model constants the reference compiles in from the generated
 * nnet_data.h (training_tf2/dump_lpcnet.py:423-446): LPC_GAMMA
 * (lpc_weighting of the frame's LPC, lpcnet.c:116-118), FEATURES_DELAY (the
 * lookahead: depth of the lpc_from_cepstrum ring, conv2 clear and silent
 * first frames, lpcnet.c:101,109-114,239; 0..4) and END2END (LPC from the
 * frame network's rc outputs via rc2lpc, lpcnet.c:56-80,107-108).
 * lpcnet_batch_load_model / lpcnet_load_model take them from optional blob
 * records named LPC_GAMMA (one float), FEATURES_DELAY and END2END (one int
 * each) -- the reference's parser skips records it does not bind -- else
 * the dump defaults (1.0, 2, 0); the environment variables LPCNET_LPC_GAMMA,
 * LPCNET_FEATURES_DELAY and LPCNET_END2END override both at load time.  This
 * setter changes them for the loaded model (until the next load).  Returns
 * -1 without a model or for an unsupported value. */
LPCNET_EXPORT int lpcnet_batch_set_model_constants(LPCNetBatch *b, float lpc_gamma, int features_delay, int end2end);
/* lpcnet_reset() on every stream / on one stream. */
LPCNET_EXPORT void lpcnet_batch_reset(LPCNetBatch *b);
LPCNET_EXPORT int lpcnet_batch_reset_stream(LPCNetBatch *b, int stream);
LPCNET_EXPORT int lpcnet_batch_nb_streams(const LPCNetBatch *b);

/* One frame for every stream, host buffers: features [B][NB_FEATURES],
 * pcm [B][N], N <= 160.  Equivalent to lpcnet_synthesize() on each stream.
 * Returns 0, or -1 on error (no model, bad N). */
LPCNET_EXPORT int lpcnet_batch_synthesize(LPCNetBatch *b, const float *features, short *pcm, int N);

/* The batch's own host-addressable buffers for a live server's tick
 * (features [B][NB_FEATURES], PCM [B][160]; allocated on first use, freed
 * with the batch, NULL on error).  lpcnet_batch_synthesize with these
 * pointers skips its host staging copies: the kernels read the features
 * where they are, and the sample kernel stores the PCM into the (mapped,
 * pinned) PCM buffer itself where its write-out is coalesced -- no
 * device-to-host copy.  The feature buffer is host-visible device memory on
 * a large-BAR device (write it from the host; reads back are slow uncached
 * PCIe reads; LPCNET_FEAT_VRAM=0: mapped pinned host memory instead).  The
 * PCM buffer holds a frame's output until the next synthesis call. */
LPCNET_EXPORT float *lpcnet_batch_host_features(LPCNetBatch *b);
LPCNET_EXPORT short *lpcnet_batch_host_pcm(LPCNetBatch *b);

/* lpcnet_synthesize_impl (src/lpcnet.c:273-277, the PLC entry point): as
 * above, but the first `preload` samples of every stream are teacher-forced
 * from pcm (input), exactly as lpcnet.c:256-259; pcm[s][preload..N) is output.
 * N == 0 runs only the frame network (run_frame_network_flush, lpcnet.c:134). */
LPCNET_EXPORT int lpcnet_batch_synthesize_impl(LPCNetBatch *b, const float *features, short *pcm, int N, int preload);

/* lpcnet_synthesize_tail_impl (src/lpcnet.c:235-271, declared at
 * lpcnet_private.h:131): N samples of every stream from the conditioning and
 * LPC already in its state (no frame network); the first `preload` samples
 * teacher-forced from pcm as above. */
LPCNET_EXPORT int lpcnet_batch_synthesize_tail_impl(LPCNetBatch *b, short *pcm, int N, int preload);

/* run_frame_network (src/lpcnet.c:82-120) of one frame per stream, no samples.
 * update_conditions = 1: into the state's conditioning and LPC, as
 * lpcnet_synthesize_impl(..., N = 0) does; 0: into locals, as
 * run_frame_network_flush does (lpcnet.c:134-144) -- conv memories, the
 * lpc_from_cepstrum ring and frame_count advance, the conditioning and LPC
 * the next tail_impl reads stay. */
LPCNET_EXPORT int lpcnet_batch_run_frame_network(LPCNetBatch *b, const float *features, int update_conditions);

/* lpcnet_reset_signal (src/lpcnet.c:226-233) on one stream. */
LPCNET_EXPORT int lpcnet_batch_reset_signal(LPCNetBatch *b, int stream);

/* 1.6 kb/s decoder (lpcnet_decode, src/lpcnet.c:310-319): one 8-byte packet
 * per stream (decode_packet, lpcnet_dec.c:81-156, on the device) -> 4 frames
 * synthesised.  Needs a model blob with the codebook records
 * (LPCNetModelInfo.has_codebooks).  Each stream's vq_mem is part of its state
 * (reset to zero by lpcnet_batch_reset / _reset_stream, as
 * lpcnet_decoder_init does; saved and restored with it).
 * Host I/O: packets [B][8] -> pcm [B][4 * 160]. */
LPCNET_EXPORT int lpcnet_batch_decode(LPCNetBatch *b, const unsigned char *packets, short *pcm);
/* Device-resident: d_packets [npackets][B][8] -> d_pcm [4 npackets][B][160]
 * (the frames-major layout of lpcnet_batch_synthesize_frames); the decoded
 * features stay in device memory.  Enqueued; lpcnet_batch_sync waits. */
LPCNET_EXPORT int lpcnet_batch_decode_frames(LPCNetBatch *b, const unsigned char *d_packets, short *d_pcm, int npackets);

/* Snapshot / restore of one stream's complete synthesis state (the struct
 * copies lpcnet_plc.c:223,230 make for speculation).  buf holds
 * lpcnet_batch_state_size() bytes. */
LPCNET_EXPORT int lpcnet_batch_state_size(void);
LPCNET_EXPORT int lpcnet_batch_save_state(LPCNetBatch *b, int stream, void *buf);
LPCNET_EXPORT int lpcnet_batch_restore_state(LPCNetBatch *b, int stream, const void *buf);

/* nframes consecutive frames for every stream with device-resident I/O:
 * d_features [nframes][B][NB_FEATURES] and d_pcm [nframes][B][N] are device
 * pointers on the batch's device.  h_features is ignored (it may be NULL;
 * lpc_from_cepstrum runs on the device since round 2 -- kept for ABI
 * compatibility).  Work is enqueued on the batch's HIP stream; the call
 * returns once every frame has been enqueued (use lpcnet_batch_sync to wait). */
LPCNET_EXPORT int lpcnet_batch_synthesize_frames(LPCNetBatch *b, const float *h_features, const float *d_features,
                                                 short *d_pcm, int nframes, int N);
/* Wait for every enqueued frame.  Returns 0, or -1 (lpcnet_mi355x_last_error)
 * on a HIP error or a device-side abort (see lpcnet_batch_set_spin_limit). */
LPCNET_EXPORT int lpcnet_batch_sync(LPCNetBatch *b);

/* Bound on the polls of one LDS flag wait inside the barrier-free sample
 * kernel (fp_kernel).  A wait that exceeds it means a protocol fault: the
 * kernel finishes early instead of hanging the device, and the next
 * synchronising call (lpcnet_batch_synthesize / _impl / _sync) returns -1
 * with lpcnet_mi355x_last_error() set -- never silent wrong PCM.  0 restores
 * the default (2^20 polls); tiny values exist to test the reporting. */
LPCNET_EXPORT int lpcnet_batch_set_spin_limit(LPCNetBatch *b, int polls);

/* Multi-frame path for batches above 128 streams with the matrix-core or
 * fp32 sample kernel: the frame network of each run of up to 32 frames
 * (>= 4) is computed in one launch before their sample kernels (chunk_kernel,
 * f32 matrix cores; identical outputs).  enable = 0 selects the per-frame
 * frame kernel instead (A/B and parity tests); default 1. */
LPCNET_EXPORT int lpcnet_batch_set_frame_chunking(LPCNetBatch *b, int enable);

/* Device memory helpers (so callers need no HIP headers). */
LPCNET_EXPORT void *lpcnet_batch_device_alloc(LPCNetBatch *b, size_t bytes);
LPCNET_EXPORT int lpcnet_batch_device_free(LPCNetBatch *b, void *p);
LPCNET_EXPORT int lpcnet_batch_memcpy_h2d(LPCNetBatch *b, void *dst, const void *src, size_t bytes);
LPCNET_EXPORT int lpcnet_batch_memcpy_d2h(LPCNetBatch *b, void *dst, const void *src, size_t bytes);

/* Kernel timing (HIP events on the batch's stream, recorded around every
 * launch since the last reset_timers): which = 0 sample-network kernel,
 * 1 frame-network kernel (per-frame frame kernel, or chunk_kernel once per
 * run of frames).  Returns total ms and the number of launches.
 * enable: 0 off, 1 events around the sample kernel only, 2 (or more) around
 * both kernels. */
LPCNET_EXPORT void lpcnet_batch_reset_timers(LPCNetBatch *b, int enable);
LPCNET_EXPORT double lpcnet_batch_kernel_ms(LPCNetBatch *b, int which, int *launches);
/* Frames covered by those timed launches (a multi-frame sample launch or a
 * chunk_kernel launch covers several). */
LPCNET_EXPORT int lpcnet_batch_kernel_frames(LPCNetBatch *b, int which);

/* Debug / parity: per-sample trace of the pre-sampling logits (8 per sample,
 * nnet.c:186-211) and the sampled excitation of the LAST synthesize call.
 * logits [B][N][8], exc [B][N]. */
LPCNET_EXPORT int lpcnet_batch_set_trace(LPCNetBatch *b, int enable);
LPCNET_EXPORT int lpcnet_batch_get_trace(LPCNetBatch *b, float *logits, int *exc);
/* Diagnostics: per-phase s_memtime sums of the sample kernel, recorded for
 * the LAST launch when enabled: [workgroup][8 waves][16] u64 (phase B, wait,
 * phase C, wait, phase F, wait, loop total, samples, then F sub-phases:
 * GRU_B update, broadcast, tree levels 0-3, levels 4-7, output; the
 * pipelined kernel records [0] X->Y work, [1] wait, [2] Y->Z work, [3] wait,
 * [4] Z->X work, [5] wait per wave).  Returns #workgroups. */
LPCNET_EXPORT int lpcnet_batch_set_stamps(LPCNetBatch *b, int enable);
LPCNET_EXPORT int lpcnet_batch_get_stamps(LPCNetBatch *b, unsigned long long *out);
/* Frame-kernel phase stamps of the last launch: [B/4 workgroups][16]
 * (0 prologue, 1 conv1, 2 conv2, 3 dense1, 4 dense2, 5 projections,
 * 6 epilogue, 7 total), cycles. */
LPCNET_EXPORT int lpcnet_batch_get_frame_stamps(LPCNetBatch *b, unsigned long long *out);

/* Per-stream state snapshot: any pointer may be NULL. */
LPCNET_EXPORT int lpcnet_batch_get_state(LPCNetBatch *b, int stream, float *gru_a_cond /*1152*/, float *gru_b_cond /*48*/,
                                         float *lpc /*16*/, float *gru_a_state /*384*/, float *gru_b_state /*16*/,
                                         int *frame_count);

/* ---- tooling (host only, no GPU needed) -------------------------------- */
/* Deterministic synthetic default-size model in the reference blob format.
 * flags: bit0 = make some int8 pairs able to saturate maddubs; bit1 = GRU_A
 * block masks chosen as training_tf2/lpcnet.py:140-160 (Sparsify) does --
 * a global per-gate energy threshold -- over skewed row energies, so block
 * rows run far above the mean length, as in trained models; bit2 = append
 * synthetic 1.6 kb/s decoder codebooks (ceps_codebook1..3 [1024][17],
 * ceps_codebook_diff4 [4096][18]; the other arrays are unchanged).
 * Returns the blob size; writes it if buf != NULL and cap is large enough. */
LPCNET_EXPORT int lpcnet_mi355x_synthetic_model(unsigned seed, int variant, int flags, unsigned char *buf, int cap);
/* Synthetic feature frames (NB_TOTAL_FEATURES floats each) for stream `stream`. */
LPCNET_EXPORT void lpcnet_mi355x_synthetic_features(unsigned stream, int nframes, float *out);
/* lpc_from_cepstrum (freq.c:310-320) of n cepstra [n][18] -> lpc [n][16] on
 * GPU `device`, through the engine's lpc_kernel (diagnostics / parity: the
 * synthesis entry points run the same kernel per frame).  Returns 0 or -1. */
LPCNET_EXPORT int lpcnet_mi355x_device_lpc(int device, const float *cepstra, float *lpc, int n);
/* The rcpps table the device activations use by default (2048 entries:
 * the Intel build host's rcpps of the top 11 mantissa bits,
 * tests/golden/rcp_x86.bin). */
LPCNET_EXPORT const uint32_t *lpcnet_mi355x_rcp_table(void);
/* This host CPU's rcpps (_mm_rcp_ps, vec_avx.h:408,437) of every float in
 * [1, 2) as 4096 entries of the top 12 mantissa bits (entries == 4096).
 * Returns the number of mantissas / exponents the 12-bit, exponent-invariant
 * form does not reproduce (0: the table is exact), or -1. */
LPCNET_EXPORT int lpcnet_mi355x_host_rcp_table(uint32_t *tab, int entries);
/* Same-box parity: the device activations use rcpps table `tab` (4096
 * entries as lpcnet_mi355x_host_rcp_table returns; NULL restores the
 * default Intel table).  A table other than the default disables the
 * hardware-reciprocal shortcut (proven equal only to the Intel table), so
 * the batch runs the lockstep sample kernel and the per-frame frame kernel
 * (every activation through the table).  The environment variable
 * LPCNET_RCP=host selects this host's table at load time (drop-in API).
 * Returns 0, or -1 (no model loaded / device error). */
LPCNET_EXPORT int lpcnet_batch_set_rcp_table(LPCNetBatch *b, const uint32_t *tab);
/* Device numerics self-test (diagnostics, not the synthesis path): runs one
 * routine of the kernels' arithmetic (lpcnet_amd/csrc/device_math.h) on GPU
 * `device` elementwise over n 32-bit inputs: op 0 tanh8_approx, 1
 * sigmoid8_approx (vec_avx.h:393-440, rcpps from the table), 2 / 3 the
 * batched forms of 0 / 1 with the hardware rcpps form, 4 vector_ps_to_epi8 byte (vec_avx.h:321-336), 5 lin2ulaw
 * (common.h:47-58), 6 floor(.5 + x) (lpcnet.c:266), 7 _mm256_cvtps_epi32;
 * op 8: n kiss99 draws (kiss99.c:59-81) from the 4-word state in[0..3];
 * op 9: the band power of lpc_from_cepstrum, (float)(pow(10, x) *
 * compensation[i % 18]) (freq.c:318, pow10_dd.h); op 10 _mm256_rcp_ps of a
 * Pade denominator (vec_avx.h:408,437, hardware form); op 11 / 12
 * sigmoid8_approx of the int8 gates' inputs (|x| < 2^18, device_math.h
 * sigmoid_x86_fin_n), hardware / table rcpps.
 * Returns 0, or -1 on bad arguments / HIP failure. */
LPCNET_EXPORT int lpcnet_mi355x_device_numerics(int device, int op, const void *in, void *out, int n);
/* Validate a weight blob with every rule lpcnet_load_model applies
 * (parse_lpcnet_weights.c:36-113 record/idx rules, array sizes, LDS budget)
 * without a device.  Returns 0 or -1 (lpcnet_mi355x_last_error). */
LPCNET_EXPORT int lpcnet_mi355x_validate_model(const unsigned char *data, int len);
/* Number of visible HIP devices (0 on a machine without GPU). */
LPCNET_EXPORT int lpcnet_mi355x_device_count(void);
/* Host-only view of the GRU_A plans a blob (data, len) gets on a wide batch
 * (no device touched): out[0] = split model (0/1), out[1] = mfw_kernel's
 * split form available (0/1), out[2 + 2w], out[3 + 2w] = its z/r and h
 * 4-slot groups of table wave w (R waves 0..5, host waves 6..7),
 * out[18..20] = pieces per gate.  int out[24].  0 / -1. */
LPCNET_EXPORT int lpcnet_mi355x_wide_plan(const unsigned char *data, int len, int *out);
/* The drop-in handles (include/lpcnet.h) bound to the same model on the
 * same device share one device copy of it and one work batch; concurrent
 * lpcnet_synthesize calls on them coalesce into one launch.  Statistics of
 * the pool `st` belongs to: coalesced launches, handled requests, handles
 * bound.  -1 if st is not bound. */
LPCNET_EXPORT int lpcnet_mi355x_pool_stats(const LPCNetState *st, long *launches, long *requests, int *streams);
/* Placement of drop-in handles (lpcnet_init / lpcnet_create /
 * lpcnet_decoder_init take no device, lpcnet.c:184-219).  Default: every
 * handle on one device -- LOCAL_RANK mod the visible devices when LOCAL_RANK
 * is set (one process per GPU), device 0 otherwise -- resolved at the first
 * lpcnet_load_model, so creating handles never starts the HIP runtime.
 * Spreading is opt-in: over `devices[0..n)` here, or over env
 * LPCNET_DEVICES="0,1,..." / "all" (checked against the visible devices at
 * the first lpcnet_init: a bad list fails it), each new handle goes to the
 * placement with the fewest live handles (a device may appear twice: two
 * placements, two pools on one GPU).  Live handles keep their device;
 * handles initialised afterwards are placed over the new list; n = 0
 * restores the default.  LPCNET_DEVICE=d pins every new handle to device d
 * instead.  0 / -1. */
LPCNET_EXPORT int lpcnet_mi355x_set_placement(const int *devices, int n);
/* The device and placement index (-1: pinned by LPCNET_DEVICE) of handle st. */
LPCNET_EXPORT int lpcnet_mi355x_handle_placement(const LPCNetState *st, int *device, int *placement);
/* Milliseconds the pool of `st` has spent inside its coalesced launches
 * (host I/O, state moves and kernels of each launch; the rest of a caller's
 * wait is hand-off and thread wake-up).  -1 if st is not bound. */
LPCNET_EXPORT double lpcnet_mi355x_pool_run_ms(const LPCNetState *st);
/* ---- reference-internal entry points on a drop-in handle ----------------
 * The reference's PLC (lpcnet_plc.c:188-337) drives one LPCNetState through
 * these functions of lpcnet_private.h:126-132; they are exported here under
 * the same names and signatures so that code links against this library
 * unchanged, except for its LPCNetState struct copies (lpcnet_plc.c:223,230),
 * which become lpcnet_mi355x_state_save / _restore. */
LPCNET_EXPORT void lpcnet_synthesize_impl(LPCNetState *st, const float *features, short *output, int N, int preload);
LPCNET_EXPORT void lpcnet_synthesize_tail_impl(LPCNetState *st, short *output, int N, int preload);
LPCNET_EXPORT void run_frame_network_deferred(LPCNetState *st, const float *features);
LPCNET_EXPORT void run_frame_network_flush(LPCNetState *st);
LPCNET_EXPORT void lpcnet_reset_signal(LPCNetState *st);
/* A handle's whole synthesis state (device stream state + the deferred
 * feature buffer): buf holds lpcnet_mi355x_state_size() bytes.  Restore
 * refuses a buffer this engine cannot have produced.  0 / -1. */
#define LPCNET_MI355X_STATE_MAX 16384 /* >= lpcnet_mi355x_state_size() (stack buffers) */
LPCNET_EXPORT int lpcnet_mi355x_state_size(void);
LPCNET_EXPORT int lpcnet_mi355x_state_save(LPCNetState *st, void *buf);
LPCNET_EXPORT int lpcnet_mi355x_state_restore(LPCNetState *st, const void *buf);
/* Release what lpcnet_init bound to st without freeing st: for an
 * LPCNetState embedded in a caller's struct (as lpcnet_plc.c:63 / lpcnet.c:293
 * embed theirs) that the caller frees itself.  Memory freed without it is
 * detected as stale by the next lpcnet_init at that address. */
LPCNET_EXPORT void lpcnet_mi355x_deinit(LPCNetState *st);
/* Bind a model to a decoder (the reference binds its compiled-in model and
 * codebooks in lpcnet_decoder_init; this library has none).  -1 if the blob
 * is rejected or carries no codebooks. */
LPCNET_EXPORT int lpcnet_mi355x_decoder_load_model(LPCNetDecState *st, const unsigned char *data, int len);

/* Last error string of this thread. */
LPCNET_EXPORT const char *lpcnet_mi355x_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
