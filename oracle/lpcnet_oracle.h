/*
 * lpcnet_oracle.h -- CPU restatement of the reference LPCNet synthesis path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the shipped product (lpcnet_amd/,
 * liblpcnet_mi355x.so) may include, link or call this code; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as
 * the checker / the timed CPU baseline.
 *
 * The synthesis glue (lpcnet.c / nnet.c composition) is restated once here and
 * drives a pluggable table of arithmetic kernels:
 *   - oracle_port_kernels(): portable C emulation of the AVX2 numerics
 *     (rcpps through a 2048-entry table, u8 x s8 maddubs with int16
 *     saturation, ...).  Runs anywhere; this is what the GPU path is checked
 *     against on the MI355X box.
 *   - ref_kernels() in oracle/_ref/libref_kernels.so: the reference's OWN
 *     vec_avx.h / kiss99.c / common.h / freq.c+kiss_fft.c+lpcnet_tables.c,
 *     compiled from /root/reference/src (see oracle/Makefile).  Used in the
 *     build container to pin the port kernels and to generate tests/golden/.
 *
 * Parity status: kernel level pinned against the compiled reference kernels;
 * the layer composition (lpcnet.c, nnet.c) is restated because those two
 * files need the generated nnet_data.h, which the reference does not ship
 * (see DESIGN.md "Oracle").
 */
#ifndef LPCNET_ORACLE_H
#define LPCNET_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint32_t z, w, jsr, jcong;
} oracle_rng;

/* Arithmetic kernels the synthesis glue calls.  Signatures follow the
 * reference functions named in each comment. */
typedef struct {
  /* vec_avx.h:552-582 vec_tanh / vec_sigmoid (Pade + rcpps) */
  void (*vec_tanh)(float *y, const float *x, int n);
  void (*vec_sigmoid)(float *y, const float *x, int n);
  /* vec_avx.h:442-450 tanh_approx (scalar path used by sample_mdense) */
  float (*tanh1)(float x);
  /* vec_avx.h:618-643 sgemv_accum16 (sequential FMA per output row) */
  void (*sgemv16)(float *out, const float *w, int rows, int cols, int col_stride, const float *x);
  /* vec_avx.h:790-858 sparse_sgemv_accum8x4 (DOT_PROD, int8 weights) */
  void (*sparse8x4_i8)(float *out, const int8_t *w, int rows, int cols, const int *idx, const float *x);
  /* vec_avx.h:690-755 sgemv_accum8x4 (DOT_PROD, dense int8) */
  void (*dense8x4_i8)(float *out, const int8_t *w, int rows, int cols, const float *x);
  /* vec_avx.h:861-904 sparse_sgemv_accum8x4 (no DOT_PROD, fp32 weights) */
  void (*sparse8x4_f32)(float *out, const float *w, int rows, const int *idx, const float *x);
  /* common.h:37-58 */
  int (*lin2ulaw)(float x);
  float (*ulaw2lin)(float u);
  /* kiss99.c:32-81 */
  void (*rng_srand)(oracle_rng *r, const unsigned char *data, int n);
  uint32_t (*rng_rand)(oracle_rng *r);
  /* freq.c:310-320 lpc_from_cepstrum, freq.c:299-308 lpc_weighting */
  float (*lpc_from_cepstrum)(float *lpc, const float *cepstrum);
  void (*lpc_weighting)(float *lpc, float gamma);
} oracle_kernels;

const oracle_kernels *oracle_port_kernels(void);

/* The portable kernels need the 2048-entry rcpps table (tests/golden/rcp_x86.bin). */
void oracle_set_rcp_table(const uint32_t *tab2048);

/* Individual portable kernels (exported for unit tests). */
float oracle_rcp(float x);
float oracle_tanh(float x);
float oracle_sigmoid(float x);
void oracle_quantize_u8(unsigned char *x, const float *xf, int n);

#define ORACLE_INT8 0
#define ORACLE_FP32 1

typedef struct OracleState OracleState;

/* Binds a reference-format weight blob (nnet.h:54-61 WeightHead records).
 * variant: ORACLE_INT8 (default AVX2 DOT_PROD build) or ORACLE_FP32
 * (--disable-dot-product build).  Returns NULL when an array is missing or
 * has the wrong size (lpcnet_load_model returns -1 in that case). */
OracleState *oracle_create(const unsigned char *blob, int len, int variant, const oracle_kernels *k);
void oracle_destroy(OracleState *st);
void oracle_reset(OracleState *st);
/* lpcnet.c:273-277 lpcnet_synthesize_impl(st, features, output, N, preload) */
void oracle_synthesize(OracleState *st, const float *features, short *output, int N, int preload);

/* lpcnet.c:235-271 lpcnet_synthesize_tail_impl */
void oracle_synthesize_tail(OracleState *st, short *output, int N, int preload);
/* lpcnet.c:122-144 run_frame_network_deferred / _flush */
void oracle_frame_deferred(OracleState *st, const float *features);
void oracle_frame_flush(OracleState *st);
/* lpcnet.c:226-233 lpcnet_reset_signal */
void oracle_reset_signal(OracleState *st);
/* whole-state snapshot (the PLC's LPCNetState struct copies) */
int oracle_state_size(void);
void oracle_state_save(const OracleState *st, void *buf);
void oracle_state_restore(OracleState *st, const void *buf);
/* lpcnet_dec.c:81-156 decode_packet (features [4][36]) and lpcnet.c:310-319
 * lpcnet_decode (pcm [640]); -1 if the blob had no codebooks.  The decoder's
 * vq_mem starts at zero (lpcnet_decoder_init). */
int oracle_decode_packet(OracleState *st, const unsigned char *buf, float *features);
int oracle_decode(OracleState *st, const unsigned char *buf, short *pcm);

/* Model constants the reference compiles in from nnet_data.h
 * (dump_lpcnet.py:423-446): LPC_GAMMA, FEATURES_DELAY (0..4), END2END.
 * Defaults 1.0, 2, 0.  Returns -1 for an unsupported value. */
int oracle_set_constants(OracleState *st, float lpc_gamma, int features_delay, int end2end);

/* Optional per-sample trace (pointers may be NULL); each call to
 * oracle_synthesize writes up to N entries from index 0. */
void oracle_set_trace(OracleState *st, float *logits8, int *exc, uint32_t *rng_words2);
/* Copies of per-frame conditioning (after the last synthesize call). */
void oracle_get_frame(const OracleState *st, float *gru_a_cond /*1152*/, float *gru_b_cond /*48*/, float *lpc /*16*/);
int oracle_frame_count(const OracleState *st);
void oracle_get_state(const OracleState *st, float *gru_a_state /*384*/, float *gru_b_state /*16*/);

#ifdef __cplusplus
}
#endif
#endif
