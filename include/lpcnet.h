/*
 * lpcnet.h -- drop-in synthesis API of liblpcnet_mi355x.so.
 *
 * Each entry point replaces the symbol of the same name in the reference's
 * include/lpcnet.h (auliaadila/LPCNet, cited as <file>:<line> relative to the
 * reference root) with identical signature, argument meaning and error
 * behaviour.  Provided: the synthesis entry points
 * and the 1.6 kb/s decoder (lpcnet_decoder_* / lpcnet_decode, row f4, which
 * feeds the same synthesis).  The encoder and PLC prototypes of the
 * reference header are out of scope (the PLC's internal entry points are in
 * lpcnet_mi355x.h).
 *
 * Behavioural notes versus the reference:
 *  - The reference binds a compiled-in model in lpcnet_init unless built with
 *    USE_WEIGHTS_FILE (src/lpcnet.c:192-196).  This library has no compiled-in
 *    model: it always behaves like the USE_WEIGHTS_FILE build, so callers load a
 *    weight blob with lpcnet_load_model() (as src/lpcnet_demo.c:204-207 does).
 *  - LPCNetState is a fixed-size host handle; the per-stream synthesis state
 *    and the model live in MI355X device memory, bound lazily on first use.
 *  - Output is PCM-identical to the reference's x86 AVX2 (DOT_PROD) build for
 *    int8 blobs and to its --disable-dot-product build for fp32 blobs.
 */
#ifndef LPCNET_H_MI355X
#define LPCNET_H_MI355X

#ifndef LPCNET_EXPORT
#if defined(__GNUC__)
#define LPCNET_EXPORT __attribute__((visibility("default")))
#else
#define LPCNET_EXPORT
#endif
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define NB_FEATURES 20        /* include/lpcnet.h:45 */
#define NB_TOTAL_FEATURES 36  /* include/lpcnet.h:46 */
#define LPCNET_FRAME_SIZE (160) /* include/lpcnet.h:53 */
#define LPCNET_COMPRESSED_SIZE 8             /* include/lpcnet.h:49 */
#define LPCNET_PACKET_SAMPLES (4 * 160)      /* include/lpcnet.h:51 */

typedef struct LPCNetState LPCNetState;
typedef struct LPCNetDecState LPCNetDecState;

/* include/lpcnet.h:63-100 -- the 1.6 kb/s decoder.  lpcnet_decode decodes one
 * LPCNET_COMPRESSED_SIZE-byte packet into LPCNET_PACKET_SAMPLES samples
 * (src/lpcnet.c:310-319).  This library has no compiled-in model or
 * codebooks: bind a blob that carries them with
 * lpcnet_mi355x_decoder_load_model (include/lpcnet_mi355x.h) first;
 * lpcnet_decode returns -1 (and outputs silence) without one. */
LPCNET_EXPORT int lpcnet_decoder_get_size(void);
LPCNET_EXPORT int lpcnet_decoder_init(LPCNetDecState *st);
LPCNET_EXPORT LPCNetDecState *lpcnet_decoder_create(void);
LPCNET_EXPORT void lpcnet_decoder_destroy(LPCNetDecState *st);
LPCNET_EXPORT int lpcnet_decode(LPCNetDecState *st, const unsigned char *buf, short *pcm);

/* include/lpcnet.h:156-160 -- size of an LPCNetState (caller allocation). */
LPCNET_EXPORT int lpcnet_get_size(void);

/* include/lpcnet.h:162-169 -- placement-initialise st (>= lpcnet_get_size()
 * bytes).  Returns 0. */
LPCNET_EXPORT int lpcnet_init(LPCNetState *st);

/* include/lpcnet.h:171-174 -- allocate + initialise. */
LPCNET_EXPORT LPCNetState *lpcnet_create(void);

/* include/lpcnet.h:176-179 -- free a state from lpcnet_create (also releases
 * the device resources bound to it). */
LPCNET_EXPORT void lpcnet_destroy(LPCNetState *st);

/* src/lpcnet.c:174-182 lpcnet_reset (declared at include/lpcnet.h:78 area):
 * clear the dynamic synthesis state and reseed the RNG with "LPCNet". */
LPCNET_EXPORT void lpcnet_reset(LPCNetState *st);

/* include/lpcnet.h:181-188 -- synthesise N (<= 160) samples from one frame of
 * NB_FEATURES features. */
LPCNET_EXPORT void lpcnet_synthesize(LPCNetState *st, const float *features, short *output, int N);

/* include/lpcnet.h:214 -- bind a weight blob (src/write_lpcnet_weights.c
 * format).  Returns 0, or -1 if an array is missing or has the wrong size.
 * Unlike the reference the blob is copied to the device, so the caller may
 * free it afterwards. */
LPCNET_EXPORT int lpcnet_load_model(LPCNetState *st, const unsigned char *data, int len);

#ifdef __cplusplus
}
#endif
#endif
