/*
 * model_gen.cpp -- deterministic synthetic LPCNet model + features.
 *
 * There is no network access for the reference's trained model
 * (download_model.sh:8), so benchmarks and parity tests run a synthetic model
 * of the default architecture (training_tf2/lpcnet.py:312-475: GRU_A 384,
 * GRU_B 16, cond 128, pitch embedding 64) written in the reference weight-blob
 * format (src/write_lpcnet_weights.c:47-67, nnet.h:54-61) with the array
 * names and layouts training_tf2/dump_lpcnet.py emits:
 *   - sparse GRU_A: 8(out)x4(in) blocks, idx = [nb, pos...] per 8-row block,
 *     int8 blocks row-major w[r*4+c] (dump_lpcnet.py:85-121), fp32 blocks
 *     w[c*8+r]; gate densities (.05,.05,.2) (train_lpcnet.py:159);
 *   - subias = bias - sum(q)/128 (dump_lpcnet.py:139-141, 190-192);
 *   - GRU_B recurrent int8 in (out_blk, in_blk, 8, 4) (dump_lpcnet.py:59-60);
 *   - dual_fc weights [256][2][16], bias/factor [2][256] (dump_lpcnet.py:264-266).
 * Values follow the SURVEY.md 8c recipe (pair clip |w0|+|w1| <= .992 on
 * adjacent inputs, shaped dual_fc bias) so PCM is well-conditioned.
 * The PRNG is kiss99 (kiss99.c), so the model is identical on every host.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "lpcnet_mi355x.h"

namespace {

struct Rng {
  uint32_t z, w, jsr, jcong;
  uint32_t next()
  {
    uint32_t znew = 36969 * (z & 0xFFFF) + (z >> 16);
    uint32_t wnew = 18000 * (w & 0xFFFF) + (w >> 16);
    uint32_t mwc = (znew << 16) + wnew;
    uint32_t shr3 = jsr ^ (jsr << 13);
    shr3 ^= shr3 >> 17;
    shr3 ^= shr3 << 5;
    uint32_t cong = 69069 * jcong + 1234567;
    z = znew; w = wnew; jsr = shr3; jcong = cong;
    return (mwc ^ cong) + shr3;
  }
  void seed(const char *tag, uint32_t s)
  {
    z = 362436069u ^ s; w = 521288629u ^ (s * 2654435761u); jsr = 123456789u ^ (s + 0x9e3779b9u); jcong = 380116160u;
    for (const char *p = tag; *p; p++) { jcong ^= (uint32_t)(unsigned char)*p; next(); }
    if (z == 0) z = 1;
    if (w == 0) w = 1;
    if (jsr == 0) jsr = 1;
    for (int i = 0; i < 16; i++) next();
  }
  float uni() { return (float)(next() >> 8) * (1.0f / 16777216.0f); }      /* [0,1) */
  float sym(float a) { return a * (2.f * uni() - 1.f); }                     /* U(-a,a) */
  float gauss() { float s = 0; for (int i = 0; i < 12; i++) s += uni(); return s - 6.f; }
};

constexpr int NA = 384, NB = 16, COND = 128, FIN = 84, EP = 64;

struct Blob {
  std::vector<unsigned char> data;
  void add(const char *name, const void *p, int size)
  {
    unsigned char h[64];
    memset(h, 0, sizeof(h));
    memcpy(h, "DNNw", 4);
    int version = 0, type = 0, block = (size + 63) / 64 * 64;
    memcpy(h + 4, &version, 4);
    memcpy(h + 8, &type, 4);
    memcpy(h + 12, &size, 4);
    memcpy(h + 16, &block, 4);
    strncpy((char *)h + 20, name, 43);
    data.insert(data.end(), h, h + 64);
    const unsigned char *b = (const unsigned char *)p;
    data.insert(data.end(), b, b + size);
    data.insert(data.end(), (size_t)(block - size), 0);
  }
  void addf(const char *name, const std::vector<float> &v) { add(name, v.data(), (int)(v.size() * 4)); }
  void addi(const char *name, const std::vector<int> &v) { add(name, v.data(), (int)(v.size() * 4)); }
};

std::vector<float> uvec(Rng &r, size_t n, float a)
{
  std::vector<float> v(n);
  for (auto &x : v) x = r.sym(a);
  return v;
}

int8_t q8(float w)
{
  float q = roundf(128.f * w);
  return (int8_t)(q > 127.f ? 127 : (q < -128.f ? -128 : q));
}

/* Block-sparse matrix [nout][nin] in 8x4 blocks.  mask[ob][ib]. */
struct Sparse {
  int nout, nin;
  std::vector<std::vector<int>> cols;             /* per 8-row block: input positions */
  std::vector<std::vector<std::vector<float>>> w; /* per block: 32 floats [r][c] */
};

/* Block mask of one gate as training_tf2/lpcnet.py:140-160 (Sparsify)
 * chooses it: the blocks whose energy reaches a GLOBAL per-gate threshold
 * (the (1 - density) quantile).  With skew, output rows (and input columns)
 * carry heterogeneous energy -- log-normal row / column scales -- so the
 * kept blocks pile up on the strong rows: block rows far above the mean
 * length, as a trained model's can be. */
std::vector<char> sparsify_mask(Rng &r, int rows, int cols, int want, float row_sigma, float col_sigma)
{
  std::vector<float> rs(rows), cs(cols), e((size_t)rows * cols);
  for (auto &v : rs) v = expf(row_sigma * r.gauss());
  for (auto &v : cs) v = expf(col_sigma * r.gauss());
  for (int i = 0; i < rows; i++)
    for (int j = 0; j < cols; j++) e[(size_t)i * cols + j] = rs[i] * cs[j] * (0.5f + r.uni());
  std::vector<float> sorted(e);
  std::sort(sorted.begin(), sorted.end());
  const float thresh = sorted[sorted.size() - (size_t)want];
  std::vector<char> mask(e.size(), 0);
  int have = 0;
  for (size_t k = 0; k < e.size(); k++)
    if (e[k] >= thresh && have < want) { mask[k] = 1; have++; }
  return mask;
}

Sparse make_sparse(Rng &r, int nout, int nin, const float density[3], float amp, bool saturate, float skew = 0.f)
{
  Sparse s;
  s.nout = nout;
  s.nin = nin;
  int nob = nout / 8, nib = nin / 4, gate_rows = nob / 3;
  s.cols.resize(nob);
  s.w.resize(nob);
  for (int g = 0; g < 3; g++) {
    /* choose exactly round(density * gate_rows * nib) blocks per gate */
    int total = gate_rows * nib;
    int want = (int)lrint(density[g] * total);
    std::vector<char> mask(total, 0);
    if (skew > 0.f) {
      mask = sparsify_mask(r, gate_rows, nib, want, skew, 0.5f * skew);
    } else {
      int have = 0;
      for (int i = 0; i < total && have < want; i++) {
        /* selection sampling: pick with probability (want-have)/(total-i) */
        uint32_t u = r.next() % (uint32_t)(total - i);
        if ((int)u < want - have) { mask[i] = 1; have++; }
      }
    }
    for (int ob = 0; ob < gate_rows; ob++)
      for (int ib = 0; ib < nib; ib++)
        if (mask[ob * nib + ib]) {
          int rb = g * gate_rows + ob;
          s.cols[rb].push_back(ib * 4);
          std::vector<float> blk(32);
          for (int rr = 0; rr < 8; rr++)
            for (int c = 0; c < 4; c += 2) {
              float a = r.sym(amp), b = r.sym(amp);
              float lim = 0.992f;
              if (saturate && (r.next() & 15) == 0) {
                /* large same-sign pair: |q0|+|q1| > 129 can saturate maddubs */
                float m = 0.8f + 0.19f * r.uni();
                a = m; b = m;
                if (r.next() & 1) { a = -m; b = -m; }
                lim = 2.f;
              }
              float sum = fabsf(a) + fabsf(b);
              if (sum > lim) { a *= lim / sum; b *= lim / sum; }
              blk[rr * 4 + c] = a;
              blk[rr * 4 + c + 1] = b;
            }
          s.w[rb].push_back(blk);
        }
  }
  return s;
}

void emit_sparse(Blob &blob, const Sparse &s, const std::string &wname, const std::string &idxname, int variant,
                 std::vector<double> *colsum /* per output: sum(q)/128 */)
{
  std::vector<int> idx;
  std::vector<int8_t> wq;
  std::vector<float> wf;
  if (colsum) colsum->assign(s.nout, 0.0);
  for (size_t rb = 0; rb < s.cols.size(); rb++) {
    idx.push_back((int)s.cols[rb].size());
    for (size_t k = 0; k < s.cols[rb].size(); k++) {
      idx.push_back(s.cols[rb][k]);
      const std::vector<float> &b = s.w[rb][k];
      for (int r = 0; r < 8; r++)
        for (int c = 0; c < 4; c++) {
          int8_t q = q8(b[r * 4 + c]);
          wq.push_back(q);
          if (colsum) (*colsum)[rb * 8 + r] += q * (1.0 / 128);
        }
      for (int c = 0; c < 4; c++)
        for (int r = 0; r < 8; r++) wf.push_back(b[r * 4 + c]);
    }
  }
  if (variant == LPCNET_VARIANT_INT8) blob.add(wname.c_str(), wq.data(), (int)wq.size());
  else blob.addf(wname.c_str(), wf);
  blob.addi(idxname.c_str(), idx);
}

}  // namespace

extern "C" LPCNET_EXPORT int lpcnet_mi355x_synthetic_model(unsigned seed, int variant, int flags, unsigned char *buf, int cap)
{
  Rng r;
  r.seed("lpcnet-mi355x-synthetic-model", seed);
  bool sat = (flags & 1) != 0;
  /* flags bit 1: GRU_A masks chosen like Sparsify with skewed row energy
   * (trained-model-like block rows: tens of blocks on the strongest rows) */
  const float skew = (flags & 2) ? 1.0f : 0.f;
  Blob blob;
  /* frame network (lpcnet.py:333-358) */
  blob.addf("embed_pitch_weights", uvec(r, 256 * EP, 0.5f));
  blob.addf("feature_conv1_weights", uvec(r, 3 * FIN * COND, sqrtf(3.f / (3 * FIN))));
  blob.addf("feature_conv1_bias", uvec(r, COND, 0.1f));
  blob.addf("feature_conv2_weights", uvec(r, 3 * COND * COND, sqrtf(3.f / (3 * COND))));
  blob.addf("feature_conv2_bias", uvec(r, COND, 0.1f));
  blob.addf("feature_dense1_weights", uvec(r, COND * COND, sqrtf(3.f / COND)));
  blob.addf("feature_dense1_bias", uvec(r, COND, 0.1f));
  blob.addf("feature_dense2_weights", uvec(r, COND * COND, sqrtf(3.f / COND)));
  blob.addf("feature_dense2_bias", uvec(r, COND, 0.1f));
  blob.addf("embed_sig_weights", uvec(r, 256 * 128, 1.0f)); /* bound by init, unused by synthesis */
  /* folded embeddings (dump_lpcnet.py:450-456) and conditioning projections */
  blob.addf("gru_a_embed_sig_weights", uvec(r, 256 * 3 * NA, 0.3f));
  blob.addf("gru_a_embed_pred_weights", uvec(r, 256 * 3 * NA, 0.3f));
  blob.addf("gru_a_embed_exc_weights", uvec(r, 256 * 3 * NA, 0.3f));
  blob.addf("gru_a_dense_feature_weights", uvec(r, COND * 3 * NA, 0.15f));
  blob.addf("gru_a_dense_feature_bias", uvec(r, 3 * NA, 0.1f));
  blob.addf("gru_b_dense_feature_weights", uvec(r, COND * 3 * NB, 0.15f));
  blob.addf("gru_b_dense_feature_bias", std::vector<float>(3 * NB, 0.f));
  /* GRU_B (dump_lpcnet.py:173-219) */
  {
    const float dens[3] = {1.f, 1.f, 1.f};
    Sparse sb = make_sparse(r, 3 * NB, NA, dens, 0.3f, sat);
    std::vector<double> colsum;
    emit_sparse(blob, sb, "gru_b_weights", "gru_b_weights_idx", variant, &colsum);
    std::vector<float> rec = uvec(r, NB * 3 * NB, 0.5f); /* [in 16][out 48] */
    std::vector<double> colsum2(3 * NB, 0.0);
    if (variant == LPCNET_VARIANT_INT8) {
      std::vector<int8_t> q;
      for (int ob = 0; ob < 3 * NB / 8; ob++)
        for (int ib = 0; ib < NB / 4; ib++)
          for (int rr = 0; rr < 8; rr++)
            for (int c = 0; c < 4; c++) q.push_back(q8(rec[(ib * 4 + c) * 3 * NB + ob * 8 + rr]));
      for (int i = 0; i < NB; i++)
        for (int o = 0; o < 3 * NB; o++) colsum2[o] += q8(rec[i * 3 * NB + o]) * (1.0 / 128);
      blob.add("gru_b_recurrent_weights", q.data(), (int)q.size());
    } else {
      blob.addf("gru_b_recurrent_weights", rec);
    }
    std::vector<float> bias = uvec(r, 6 * NB, 0.1f), subias(bias);
    for (int o = 0; o < 3 * NB; o++) {
      subias[o] = (float)(bias[o] - colsum[o]);
      subias[3 * NB + o] = (float)(bias[3 * NB + o] - colsum2[o]);
    }
    blob.addf("gru_b_bias", bias);
    blob.addf("gru_b_subias", subias);
  }
  /* dual_fc (mdense.py, dump_lpcnet.py:259-283) */
  {
    std::vector<float> w = uvec(r, 256 * 2 * NB, 0.1f), b(2 * 256), f(2 * 256);
    for (int c = 0; c < 2; c++)
      for (int i = 0; i < 256; i++) {
        int lvl = 0;
        while ((2 << lvl) <= i) lvl++;
        int bit = lvl >= 1 ? (i >> (lvl - 1)) & 1 : 0;
        b[c * 256 + i] = (bit ? -1.f : 1.f) + r.sym(0.2f);
        f[c * 256 + i] = 1.5f + r.sym(0.2f);
      }
    blob.addf("dual_fc_weights", w);
    blob.addf("dual_fc_bias", b);
    blob.addf("dual_fc_factor", f);
  }
  /* sparse GRU_A (dump_lpcnet.py:124-170) */
  {
    const float dens[3] = {0.05f, 0.05f, 0.2f};
    Sparse sa = make_sparse(r, 3 * NA, NA, dens, 0.6f, sat, skew);
    std::vector<double> colsum;
    blob.addf("sparse_gru_a_recurrent_weights_diag", uvec(r, 3 * NA, 0.5f));
    emit_sparse(blob, sa, "sparse_gru_a_recurrent_weights", "sparse_gru_a_recurrent_weights_idx", variant, &colsum);
    std::vector<float> bias = uvec(r, 6 * NA, 0.1f), subias(bias);
    for (int o = 0; o < 3 * NA; o++) subias[3 * NA + o] = (float)(bias[3 * NA + o] - colsum[o]);
    blob.addf("sparse_gru_a_bias", bias);
    blob.addf("sparse_gru_a_subias", subias);
  }
  /* flags bit 2: the 1.6 kb/s decoder's codebooks (lpcnet_private.h:109-112;
   * sizes from lpcnet_enc.c:109-119, 709), drawn from their own generator so
   * every other array is identical with or without them.  Scales follow the
   * synthetic features' cepstra (0.6/k on band k): stage 1 carries most of
   * it, stages 2 and 3 refine, the difference codebook is a residual. */
  if (flags & 4) {
    Rng c;
    c.seed("lpcnet-mi355x-synthetic-codebooks", seed);
    const float stage[3] = {1.f, 0.35f, 0.15f};
    const char *names[3] = {"ceps_codebook1", "ceps_codebook2", "ceps_codebook3"};
    for (int k = 0; k < 3; k++) {
      std::vector<float> cb((size_t)1024 * 17);
      for (int e = 0; e < 1024; e++)
        for (int i = 0; i < 17; i++) cb[(size_t)e * 17 + i] = stage[k] * (0.6f / (i + 1)) * c.gauss();
      blob.addf(names[k], cb);
    }
    std::vector<float> d((size_t)4096 * 18);
    for (int e = 0; e < 4096; e++)
      for (int i = 0; i < 18; i++) d[(size_t)e * 18 + i] = (i == 0 ? 0.5f : 0.25f / i) * c.gauss();
    blob.addf("ceps_codebook_diff4", d);
  }
  int size = (int)blob.data.size();
  if (buf && cap >= size) memcpy(buf, blob.data.data(), size);
  return size;
}

extern "C" LPCNET_EXPORT void lpcnet_mi355x_synthetic_features(unsigned stream, int nframes, float *out)
{
  Rng r;
  r.seed("lpcnet-mi355x-synthetic-features", stream);
  for (int f = 0; f < nframes; f++) {
    float *x = out + (size_t)f * NB_TOTAL_FEATURES;
    x[0] = 4.f * r.uni();
    for (int k = 1; k < 18; k++) x[k] = (0.6f / k) * r.gauss();
    x[18] = -1.3f + 2.8f * r.uni();
    x[19] = -0.5f + r.uni();
    for (int k = 20; k < NB_TOTAL_FEATURES; k++) x[k] = 0.f;
  }
}
