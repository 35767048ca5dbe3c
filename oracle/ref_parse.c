/* oracle/ref_parse.c -- TEST INFRASTRUCTURE ONLY (never linked into the
 * product).  A driver of the reference's OWN weight-blob parser and layer
 * binders, /root/reference/src/parse_lpcnet_weights.c compiled unmodified in
 * place (oracle/Makefile), so that the engine's ingest rules can be checked
 * against the reference code itself rather than against a restatement.
 *
 *   _ref/ref_parse_int8  < blob   (DOT_PROD build: qweight = signed char)
 *   _ref/ref_parse_fp32  < blob   (-DDISABLE_DOT_PROD: qweight = float)
 *
 * Reads one blob from stdin, runs parse_weights (parse_lpcnet_weights.c:53-77)
 * and then the binder call list that dump_lpcnet.py generates for the
 * LPCNet model's init_lpcnet_model (training_tf2/dump_lpcnet.py:405-493 with
 * the per-layer lines :157-169 sparse_gru_init, :205-218 gru_init, :240-244
 * dense_init, :271-282 mdense_init, :308-318 conv1d_init, :329-333
 * embedding_init; layer sizes from lpcnet.py:312-427 / train_lpcnet.py
 * defaults).  The call list is restated here (the generated nnet_data.c that
 * holds it is absent); the parser and binders are the reference's.
 *
 * Exit status: 0 = accepted (every binder returned 0), 1 = a binder
 * rejected, 2 = parse_weights rejected.  Output: one line per bound array,
 * "<name> <offset into the blob> <bytes>", so a test can check which record a
 * binder took (first of a name, extra records ignored).
 *
 * The reference's parse_weights leaves the list terminator's size/data
 * uninitialised (:75 sets only .name), and find_array_entry returns that
 * terminator for a missing name (:79-82), so a missing array compares an
 * uninitialised size.  In a fresh process the list comes from untouched heap
 * (zeros): the behaviour the tests observe is "missing => rejected".  A
 * negative block count makes find_idx_check (:98-110) loop forever (nb = -1)
 * or walk off the array (nb < -1); the caller runs this driver under a
 * timeout. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "nnet.h"

/* defined in parse_lpcnet_weights.c:53, declared by no reference header */
int parse_weights(WeightArray **list, const unsigned char *data, int len);

/* the model struct the generated nnet_data.h declares (dump_lpcnet.py:405,504) */
typedef struct {
  EmbeddingLayer gru_a_embed_sig, gru_a_embed_pred, gru_a_embed_exc, embed_pitch, embed_sig;
  DenseLayer gru_a_dense_feature, gru_b_dense_feature, feature_dense1, feature_dense2;
  GRULayer gru_b;
  Conv1DLayer feature_conv1, feature_conv2;
  MDenseLayer dual_fc;
  SparseGRULayer sparse_gru_a;
} Model;

static const unsigned char *g_blob;

static void show(const char *name, const void *p, long bytes)
{
  printf("%s %ld %ld\n", name, (long)((const unsigned char *)p - g_blob), bytes);
}

int main(void)
{
  size_t cap = 1 << 20, len = 0;
  unsigned char *data = (unsigned char *)malloc(cap);
  for (;;) {
    size_t r = fread(data + len, 1, cap - len, stdin);
    len += r;
    if (len < cap) break;
    cap *= 2;
    data = (unsigned char *)realloc(data, cap);
  }
  g_blob = data;
  WeightArray *list = NULL;
  if (parse_weights(&list, data, (int)len) < 0) return 2;

  /* sizes: NA=384 GRU_A units, NB=16 GRU_B units, cond 128, embed 128,
   * pitch embed 64, 20 features + 64 = 84 conv1 inputs, kernel 3, 256
   * levels x 2 channels (train_lpcnet.py:82-101, lpcnet.py:312-427) */
  Model m;
  memset(&m, 0, sizeof(m));
  int bad = 0;
  /* dump_lpcnet.py:450-469: the folded embeddings, the two dense features, GRU_B */
  bad = bad || embedding_init(&m.gru_a_embed_sig, list, "gru_a_embed_sig_weights", 256, 1152);
  bad = bad || embedding_init(&m.gru_a_embed_pred, list, "gru_a_embed_pred_weights", 256, 1152);
  bad = bad || embedding_init(&m.gru_a_embed_exc, list, "gru_a_embed_exc_weights", 256, 1152);
  bad = bad || dense_init(&m.gru_a_dense_feature, list, "gru_a_dense_feature_bias", "gru_a_dense_feature_weights",
                          128, 1152, ACTIVATION_LINEAR);
  bad = bad || dense_init(&m.gru_b_dense_feature, list, "gru_b_dense_feature_bias", "gru_b_dense_feature_weights",
                          128, 48, ACTIVATION_LINEAR);
  bad = bad || gru_init(&m.gru_b, list, "gru_b_bias", "gru_b_subias", "gru_b_weights", "gru_b_weights_idx",
                        "gru_b_recurrent_weights", 384, 16, ACTIVATION_SIGMOID, 1);
  /* dump_lpcnet.py:471-474: model.layers in construction order (lpcnet.py:336-427) */
  bad = bad || conv1d_init(&m.feature_conv1, list, "feature_conv1_bias", "feature_conv1_weights", 84, 3, 128,
                           ACTIVATION_TANH);
  bad = bad || conv1d_init(&m.feature_conv2, list, "feature_conv2_bias", "feature_conv2_weights", 128, 3, 128,
                           ACTIVATION_TANH);
  bad = bad || embedding_init(&m.embed_pitch, list, "embed_pitch_weights", 256, 64);
  bad = bad || dense_init(&m.feature_dense1, list, "feature_dense1_bias", "feature_dense1_weights", 128, 128,
                          ACTIVATION_TANH);
  bad = bad || dense_init(&m.feature_dense2, list, "feature_dense2_bias", "feature_dense2_weights", 128, 128,
                          ACTIVATION_TANH);
  bad = bad || embedding_init(&m.embed_sig, list, "embed_sig_weights", 256, 128);
  bad = bad || mdense_init(&m.dual_fc, list, "dual_fc_bias", "dual_fc_weights", "dual_fc_factor", 16, 256, 2,
                           ACTIVATION_SIGMOID);
  /* dump_lpcnet.py:476 */
  bad = bad || sparse_gru_init(&m.sparse_gru_a, list, "sparse_gru_a_bias", "sparse_gru_a_subias",
                               "sparse_gru_a_recurrent_weights_diag", "sparse_gru_a_recurrent_weights",
                               "sparse_gru_a_recurrent_weights_idx", 384, ACTIVATION_TANH, 1);
  if (bad) {
    free(list);
    return 1;
  }
  const long q = (long)sizeof(qweight);
  show("gru_a_embed_sig_weights", m.gru_a_embed_sig.embedding_weights, 256L * 1152 * 4);
  show("gru_a_embed_pred_weights", m.gru_a_embed_pred.embedding_weights, 256L * 1152 * 4);
  show("gru_a_embed_exc_weights", m.gru_a_embed_exc.embedding_weights, 256L * 1152 * 4);
  show("gru_a_dense_feature_weights", m.gru_a_dense_feature.input_weights, 128L * 1152 * 4);
  show("gru_a_dense_feature_bias", m.gru_a_dense_feature.bias, 1152L * 4);
  show("gru_b_dense_feature_weights", m.gru_b_dense_feature.input_weights, 128L * 48 * 4);
  show("gru_b_dense_feature_bias", m.gru_b_dense_feature.bias, 48L * 4);
  show("gru_b_bias", m.gru_b.bias, 96L * 4);
  show("gru_b_subias", m.gru_b.subias, 96L * 4);
  show("gru_b_weights_idx", m.gru_b.input_weights_idx, 0);
  show("gru_b_weights", m.gru_b.input_weights, 0);
  show("gru_b_recurrent_weights", m.gru_b.recurrent_weights, 3L * 16 * 16 * q);
  show("feature_conv1_weights", m.feature_conv1.input_weights, 3L * 84 * 128 * 4);
  show("feature_conv1_bias", m.feature_conv1.bias, 128L * 4);
  show("feature_conv2_weights", m.feature_conv2.input_weights, 3L * 128 * 128 * 4);
  show("feature_conv2_bias", m.feature_conv2.bias, 128L * 4);
  show("embed_pitch_weights", m.embed_pitch.embedding_weights, 256L * 64 * 4);
  show("feature_dense1_weights", m.feature_dense1.input_weights, 128L * 128 * 4);
  show("feature_dense1_bias", m.feature_dense1.bias, 128L * 4);
  show("feature_dense2_weights", m.feature_dense2.input_weights, 128L * 128 * 4);
  show("feature_dense2_bias", m.feature_dense2.bias, 128L * 4);
  show("embed_sig_weights", m.embed_sig.embedding_weights, 256L * 128 * 4);
  show("dual_fc_bias", m.dual_fc.bias, 512L * 4);
  show("dual_fc_weights", m.dual_fc.input_weights, 16L * 512 * 4);
  show("dual_fc_factor", m.dual_fc.factor, 512L * 4);
  show("sparse_gru_a_bias", m.sparse_gru_a.bias, 6L * 384 * 4);
  show("sparse_gru_a_subias", m.sparse_gru_a.subias, 6L * 384 * 4);
  show("sparse_gru_a_recurrent_weights_diag", m.sparse_gru_a.diag_weights, 3L * 384 * 4);
  show("sparse_gru_a_recurrent_weights_idx", m.sparse_gru_a.idx, 0);
  show("sparse_gru_a_recurrent_weights", m.sparse_gru_a.recurrent_weights, 0);
  free(list);
  return 0;
}
