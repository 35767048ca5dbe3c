/*
 * engine.cpp -- host side of the MI355X LPCNet synthesis engine and the
 * C-ABI entry points declared in include/lpcnet.h and include/lpcnet_mi355x.h.
 *
 * Responsibilities
 *  - weight-blob ingest with the reference's validation rules
 *    (parse_lpcnet_weights.c:36-113, 115-221) and re-tiling of the
 *    block-sparse GRU weights into the sample kernel's LDS image;
 *  - per-stream device state (lpcnet_private.h:28-48) and reset semantics
 *    (lpcnet.c:174-182);
 *  - per-frame scheduling: lpc_kernel (lpc_from_cepstrum), frame_kernel and
 *    the sample kernel on the batch's HIP stream (the first two on a second
 *    stream, one frame ahead, for small batches).
 * Compile with -ffp-contract=off (the u-law / logit tables are computed here
 * with the reference's exact expressions).
 */
#include <hip/hip_runtime.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "lpcnet_engine.h"
#include "lpcnet_mi355x.h"

using namespace lpcnet_mi355x;

namespace {

thread_local std::string g_err;
void set_err(const std::string &e) { g_err = e; }

const uint32_t kRcpTable[2048] = {
#include "rcp_table_x86.inc"
};

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      set_err(std::string(#x) + ": " + hipGetErrorString(e_));                            \
      return -1;                                                                           \
    }                                                                                      \
  } while (0)

/* ---- host restatements of the scalar helpers used at init/reset -------- */

/* common.h:18-33 + 47-58 */
int host_lin2ulaw(float x)
{
  float scale = 255.f / 32768.f;
  int s = x >= 0 ? 1 : -1;
  x = fabsf(x);
  float y = 1 + scale * x;
  uint32_t bits;
  memcpy(&bits, &y, 4);
  int integer = (int)(bits >> 23) - 127;
  bits -= (uint32_t)integer << 23;
  float m;
  memcpy(&m, &bits, 4);
  float frac = m - 1.5f;
  frac = -0.41445418f + frac * (0.95909232f + frac * (-0.33951290f + frac * 0.16541097f));
  float l2 = 1 + integer + frac;
  float u = (s * (128 * (0.69315f * l2) / 5.5451774445f));
  u = 128 + u;
  if (u < 0) u = 0;
  if (u > 255) u = 255;
  return (int)floor(.5 + u);
}

/* common.h:37-45 */
float host_ulaw2lin(float u)
{
  float scale_1 = 32768.f / 255.f;
  u = u - 128.f;
  float s = u >= 0.f ? 1.f : -1.f;
  u = fabsf(u);
  return s * scale_1 * (exp(u / 128. * 5.5451774445f) - 1);
}

/* kiss99.c:32-81 */
struct Kiss {
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
  void srand(const unsigned char *d, int n)
  {
    int i;
    z = 362436069; w = 521288629; jsr = 123456789; jcong = 380116160;
    for (i = 3; i < n; i += 4) {
      z ^= d[i - 3]; w ^= d[i - 2]; jsr ^= d[i - 1]; jcong ^= d[i];
      next();
    }
    if (i - 3 < n) z ^= d[i - 3];
    if (i - 2 < n) w ^= d[i - 2];
    if (i - 1 < n) jsr ^= d[i - 1];
    if (z == 0 || z == 0x9068FFFF) z++;
    if (w == 0 || w == 0x464FFFFF) w++;
    if (jsr == 0) jsr++;
  }
};

/* ---- blob parsing (parse_lpcnet_weights.c:36-113) ---------------------- */
int check_constants(const ModelConst &mc)
{
  if (!std::isfinite(mc.lpc_gamma)) { set_err("LPC_GAMMA must be finite"); return -1; }
  if (mc.delay < 0 || mc.delay > MAX_FEATURES_DELAY) {
    set_err("FEATURES_DELAY must lie in [0, " + std::to_string(MAX_FEATURES_DELAY) + "]");
    return -1;
  }
  if (mc.end2end != 0 && mc.end2end != 1) { set_err("END2END must be 0 or 1"); return -1; }
  return 0;
}

struct Arr {
  std::string name;
  int size;
  const unsigned char *data;
};

bool parse_blob(std::vector<Arr> &out, const unsigned char *data, int len)
{
  while (len > 0) {
    if (len < 64) return false;
    int size, block;
    memcpy(&size, data + 12, 4);
    memcpy(&block, data + 16, 4);
    if (block < size || block > len - 64 || data[63] != 0 || size <= 0) return false;
    out.push_back(Arr{std::string((const char *)data + 20), size, data + 64});
    data += block + 64;
    len -= block + 64;
  }
  return true;
}

const Arr *find(const std::vector<Arr> &l, const char *name)
{
  for (const Arr &a : l)
    if (a.name == name) return &a;
  return nullptr;
}

const void *find_check(const std::vector<Arr> &l, const char *name, int size)
{
  const Arr *a = find(l, name);
  if (!a || a->size != size) {
    set_err(std::string("weight array missing or mis-sized: ") + name);
    return nullptr;
  }
  return a->data;
}

/* find_idx_check: per 8-row block [nb, pos...], pos 4-aligned and < nb_in-3 */
bool parse_idx(const std::vector<Arr> &l, const char *name, int nb_in, int nb_out, std::vector<std::vector<int>> &blocks)
{
  const Arr *a = find(l, name);
  if (!a) { set_err(std::string("missing ") + name); return false; }
  std::vector<int> idx(a->size / 4);
  memcpy(idx.data(), a->data, idx.size() * 4);
  size_t p = 0;
  int remain = (int)idx.size();
  blocks.clear();
  while (remain > 0) {
    int nb = idx[p++];
    if (nb < 0 || remain < nb + 1) { set_err(std::string("bad idx ") + name); return false; }
    std::vector<int> pos(nb);
    for (int k = 0; k < nb; k++) {
      pos[k] = idx[p++];
      if (pos[k] + 3 >= nb_in || (pos[k] & 3) || pos[k] < 0) { set_err(std::string("bad idx pos ") + name); return false; }
    }
    blocks.push_back(pos);
    nb_out -= 8;
    remain -= nb + 1;
  }
  if (nb_out != 0) { set_err(std::string("idx rows mismatch ") + name); return false; }
  return true;
}

int total_blocks(const std::vector<std::vector<int>> &b)
{
  int t = 0;
  for (auto &v : b) t += (int)v.size();
  return t;
}

/* ---- lpc_from_cepstrum tables (lpc_kernel.hip) ------------------------- */
/* The reference's constants, built as the reference builds them: the idct
 * matrix (freq.c:56-59 dct_table), the 320-point kiss FFT twiddles
 * (lpcnet_tables.c kfft, generated by dump_lpcnet_tables.c:88-95 as
 * (float)cos/sin of -2*pi*i/320 in double), kiss_fft's input permutation for
 * factors (4,4,4,5) applied outermost-5-first, and per spectrum bin the band
 * and (float)j/band_size interpolation fraction (freq.c:202-216). */
void build_lpc_tables(LpcTables &T)
{
  static const short eband[LPC_NBANDS] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28, 34, 40};
  static const float comp[LPC_NBANDS] = {0.8f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 0.666667f, 0.5f, 0.5f, 0.5f,
                                         0.333333f, 0.25f, 0.25f, 0.2f, 0.166667f, 0.173913f};
  memset(&T, 0, sizeof(T));
  const double pi = 3.14159265358979323846264338327;
  for (int i = 0; i < LPC_WIN; i++) {
    const double ph = (-2 * pi / LPC_WIN) * i;
    T.twr[i] = (float)cos(ph);
    T.twi[i] = (float)sin(ph);
  }
  /* per spectrum bin k < 160: band and (float)j/band_size (freq.c:206-213) */
  unsigned char band[160];
  float frac[160];
  for (int b = 0; b < LPC_NBANDS - 1; b++) {
    const int n = (eband[b + 1] - eband[b]) * 4;
    for (int j = 0; j < n; j++) {
      band[eband[b] * 4 + j] = (unsigned char)b;
      frac[eband[b] * 4 + j] = (float)j / n;
    }
  }
  /* input sample d0 + 5*d1 + 20*d2 + 80*d3 feeds FFT slot d0*64 + d1*16 + d2*4 + d3 */
  for (int d0 = 0; d0 < 5; d0++)
    for (int d1 = 0; d1 < 4; d1++)
      for (int d2 = 0; d2 < 4; d2++)
        for (int d3 = 0; d3 < 4; d3++) {
          const int i = d0 * 64 + d1 * 16 + d2 * 4 + d3, bin = d0 + 5 * d1 + 20 * d2 + 80 * d3;
          const int k = bin <= 160 ? bin : LPC_WIN - bin;
          LpcSlot &sl = T.slot[i];
          sl.band = k < 160 ? band[k] : (unsigned char)(LPC_NBANDS - 1);
          sl.frac = k < 160 ? frac[k] : 0.f;
          sl.conj = bin > 160 ? 1 : 0;
        }
  for (int i = 0; i < LPC_NBANDS; i++)
    for (int j = 0; j < LPC_NBANDS; j++) {
      float v = (float)cos((i + .5) * j * M_PI / LPC_NBANDS);
      if (j == 0) v = (float)(v * sqrt(.5));
      T.dct[i * LPC_NBANDS + j] = v;
    }
  for (int i = 0; i < LPC_NBANDS; i++) T.comp[i] = comp[i];
  T.sqrt_2_18 = sqrt(2. / LPC_NBANDS);
  T.scale = 1.f / 320.f;
}

}  // namespace

/* ---- launcher helpers (lpcnet_engine.h), keyed by the current device ---- */
namespace lpcnet_mi355x {

int ensure_dyn_lds(const void *kernel, int bytes)
{
  static std::mutex mu;
  static std::map<std::pair<const void *, int>, int> done; /* (kernel, device) -> bytes set */
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  std::lock_guard<std::mutex> lk(mu);
  int &have = done[{kernel, dev}];
  if (have >= bytes) return 0;
  if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess) return -1;
  have = bytes;
  return 0;
}

int current_device_cus()
{
  static std::mutex mu;
  static std::map<int, int> cus;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cus.find(dev);
  if (it != cus.end()) return it->second;
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  cus[dev] = n;
  return n;
}

}  // namespace lpcnet_mi355x

/* ------------------------------------------------------------------------ */
struct LPCNetBatch {
  int device = 0;
  int B = 0;
  int S = 1;
  hipStream_t stream = nullptr;
  /* model */
  bool have_model = false;
  int variant = 0;
  bool sat = false;
  bool reg = false;
  int kernel_mode = 0;   /* 0 auto, 1 lockstep sample_kernel, 4 matrix-core mf_kernel, 5 fp32 fp_kernel */
  ModelConst mc{1.0f, DEFAULT_FEATURES_DELAY, 0}; /* FEATURES_DELAY / LPC_GAMMA / END2END of the model */
  /* rcpps table of the device activations (RCP_ENTRIES, device form t + kRcpBias);
   * rcp_custom: not the default Intel table (lpcnet_batch_set_rcp_table) */
  bool rcp_custom = false;
  std::vector<uint32_t> rcp_dev;
  bool mf_ok = false;    /* model fits the matrix-core register tables */
  bool mf = false;       /* mf_kernel (mode 4) */
  bool mf2 = false;      /* large batches: mf2_kernel (two staggered 4-stream groups per workgroup) for
                            launches without preload / trace / stamps */
  int mfw_g = 3;         /* mfw_kernel's four-stream groups per workgroup (2 or 3) */
  bool mfw_forced = false; /* LPCNET_MFW=1: mfw_kernel for every launch, however narrow */
  int cus = 256;           /* compute units of the batch's device */
  bool mfw = false;      /* wider batches: mfw_kernel (two or three 4-stream groups, dedicated gather /
                            recurrent / sampler waves; split models in its split form) for the same
                            launches, models with the default rcpps */
  bool plan_wide = false; /* the register tables were planned for mfw_kernel (plan class 3) */
  L2Warm ck_warm{};       /* the chunk kernel's re-tiled weights (deferred LPC warms them) */
  std::vector<unsigned char> blob; /* the loaded model's blob: replanned when the kernel choice moves */
  double mf_ga_ops = 0;  /* int8 matrix-core ops per workgroup per sample: the GRU_A recurrent pass */
  double mf_gb_ops = 0;  /* the GRU_B tiles of both sampler waves */
  bool fp_ok = false;    /* fp32 model fits the fp_kernel tables */
  bool fp = false;       /* fp_kernel (mode 5) */
  int image_bytes = 0;
  LPCNetModelInfo info{};
  std::vector<void *> model_bufs;
  FrameArgs fa{};
  SampleArgs sa{};
  int lds_bytes = 0;
  /* streams */
  StreamState *d_state = nullptr;
  float *d_feat = nullptr;
  short *d_pcm = nullptr;
  float *d_lpc = nullptr;          /* [LPC_CHUNK][B][NLPC] lpc_from_cepstrum of queued frames */
  LpcTables *d_lpc_tab = nullptr;
  /* overlapped multi-frame path (few streams, free CUs): frame kernel f+1 on
   * fstream beside sample kernel f on stream, outputs double-buffered in
   * d_cond[f & 1] */
  hipStream_t fstream = nullptr;
  FrameCond *d_cond[2] = {nullptr, nullptr};
  hipEvent_t ev_frame[2] = {nullptr, nullptr}, ev_samp[2] = {nullptr, nullptr}, ev_start = nullptr;
  bool ev_samp_used[2] = {false, false};
  hipEvent_t ev_samp_cur[2] = {nullptr, nullptr}; /* the event slot c's reuse waits on */
  /* chunked multi-frame path (batches above OVERLAP_MAX_STREAMS): the frame
   * network of up to LPC_CHUNK frames in one chunk_kernel launch, outputs of
   * frame f in d_chunk[f][B] */
  FrameCond *d_chunk = nullptr;
  bool chunking = true;
  /* per-frame host-I/O path of large batches (synth_first): one frame's
   * chunk_kernel outputs [B], and pinned staging of the caller's features and
   * PCM (so both copies are asynchronous, behind one synchronisation) */
  float *h_io_feat = nullptr;
  short *h_io_pcm = nullptr;
  short *d_io_pcm = nullptr; /* h_io_pcm's device address (mapped) */
  float *d_io_feat = nullptr; /* h_io_feat's device address (mapped) */
  bool io_feat_vram = false;  /* h_io_feat is host-visible device memory (fine-grained VRAM, large BAR) */
  float *h_stg_feat = nullptr; /* pinned staging of the caller's own buffers */
  short *h_stg_pcm = nullptr;
  hipEvent_t ev_tick = nullptr; /* end of a host-I/O tick (spin-polled) */
  /* trace */
  bool trace = false;
  float *d_trace_logits = nullptr;
  int *d_trace_exc = nullptr;
  int trace_N = 0;
  /* device -> host status word (pinned, mapped): a kernel that aborts sets
   * STATUS_* bits; every synchronising entry point checks and clears it */
  int *h_status = nullptr;
  int *d_status = nullptr;
  int *d_ck_sync = nullptr; /* [ceil(B / 16)] arrival counters of the sliced one-frame chunk kernel */
  int spin_limit = FLAG_SPIN_LIMIT_DEFAULT;
  /* 1.6 kb/s decoder (decode_kernel.hip): the model's ceps codebooks (optional
   * blob records), packets and decoded features of up to DEC_MAX_PACKETS
   * packets per stream, the host-I/O path's 4-frame PCM */
  DecodeArgs da{};
  bool has_codebooks = false;
  unsigned char *d_packets = nullptr;
  float *d_dfeat = nullptr;
  short *d_dpcm = nullptr;
  /* diagnostics */
  unsigned long long *d_stamps = nullptr;
  /* timing */
  int timing = 0;        /* 0 off, 1 sample kernel, 2 sample + frame kernel */
  std::vector<hipEvent_t> ev_taken; /* events handed out since the last reset */
  std::vector<hipEvent_t> ev_pairs[2];
  std::vector<int> ev_frames[2];    /* frames covered by each pair */
  std::vector<hipEvent_t> ev_free;
  /* lower bound of every stream's frame_count (lpcnet.c:119) before the next
   * frame: the multi-frame sample launches start where no stream can still
   * be inside its first `delay` (FEATURES_DELAY) frames */
  int min_fc = 0;
  void frames_done(int n) { min_fc = min_fc >= 1000 ? min_fc : std::min(min_fc + n, 1000); }
  int set_device() { return hipSetDevice(device) == hipSuccess ? 0 : -1; }
};

namespace {

template <typename T>
T *dev_upload(LPCNetBatch *b, const void *src, size_t bytes)
{
  void *p = nullptr;
  if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
  if (bytes && hipMemcpy(p, src, bytes, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  b->model_bufs.push_back(p);
  return (T *)p;
}

void free_model(LPCNetBatch *b)
{
  for (void *p : b->model_bufs) (void)hipFree(p);
  b->model_bufs.clear();
  b->have_model = false;
  b->ck_warm = L2Warm{};
}

hipEvent_t get_event(LPCNetBatch *b)
{
  if (!b->ev_free.empty()) {
    hipEvent_t e = b->ev_free.back();
    b->ev_free.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

/* pair sums of an int8 8x4 block that could saturate maddubs (x in [0,255]) */
bool block_may_saturate(const int8_t *w)
{
  for (int r = 0; r < 8; r++)
    for (int c = 0; c < 4; c += 2) {
      int a = w[r * 4 + c], bb = w[r * 4 + c + 1];
      int pos = std::max(a, 0) + std::max(bb, 0), neg = std::max(-a, 0) + std::max(-bb, 0);
      if (255 * pos > 32767 || 255 * neg > 32768) return true;
    }
  return false;
}

int mfw_groups(int B, int cus)
{
  if (cus < 1 || B <= 4 * cus) return 0;
  const double c2 = (double)((B + 8 * cus - 1) / (8 * cus)) * 2;
  const double c3 = (double)((B + 12 * cus - 1) / (12 * cus)) * 3 * MFW_G3_PHASE;
  return c3 < c2 ? 3 : 2;
}

/* Per launch: a batch that runs mfw_kernel gives its launches of at most
 * one mf_kernel<4> round (nB <= 4 streams per CU: a drop-in pool's work
 * batch is sized for its widest launch, a partial step of a batch) to
 * mf_kernel, whose one-group sample is the shorter chain there. */
/* whether choose_kernel will run mfw_kernel on this batch, the model's own
 * limits (split plan, LDS) aside: the plan class of its register tables
 * follows the same predicate */
static bool mfw_planned(const LPCNetBatch *b, int cus)
{
  if ((b->kernel_mode != 0 && b->kernel_mode != 4) || b->rcp_custom) return false;
  const char *e2 = getenv("LPCNET_MF2");
  if (e2 && atoi(e2) == 0) return false;
  const char *ew = getenv("LPCNET_MFW");
  if (ew) return atoi(ew) != 0;
  return mfw_groups(b->B, cus) > 0;
}

static bool wide_for(const LPCNetBatch *b, int nB) { return b->mfw && (b->mfw_forced || nB > 4 * b->cus); }
static bool mf2_for(const LPCNetBatch *b, int nB) { return b->mf2 && (!b->mfw || wide_for(b, nB)); }

/* Sample-kernel choice (mode 0 = automatic):
 *   5  fp_kernel  -- fp32 models with a dense GRU_B within the FP_* limits
 *   4  mf_kernel  -- non-saturating int8 models within the MF_* limits
 *   1  sample_kernel (lockstep) -- every other model: saturating int8 models
 *      (int16 maddubs saturation emulated) and fp32 models with a sparse GRU_B.
 * A mode the model cannot run falls back to the lockstep kernel. */
void choose_kernel(LPCNetBatch *b)
{
  b->mf = false;
  b->mf2 = false;
  b->mfw = false;
  b->fp = false;
  b->info.mfma_ops_per_group_sample = 0;
  int mode = b->kernel_mode;
  if (mode == 0) mode = b->fp_ok ? 5 : (b->mf_ok ? 4 : 1);
  /* a custom rcpps table (another host's, same-box parity): the fast
   * kernels run their table-only forms (the hardware-reciprocal shortcut is
   * proven for the Intel table only) */
  b->sa.rcp_hw = b->fa.rcp_hw = b->rcp_custom ? 0 : 1;
  b->info.rcp_hw = b->sa.rcp_hw;
  if (mode == 5 && b->fp_ok && fp_lds_bytes() <= 160 * 1024) {
    b->fp = true;
    b->info.streams_per_workgroup = 1;
    b->info.lds_bytes = fp_lds_bytes();
    b->info.quad_path = 5;
    return;
  }
  if (mode == 4 && b->mf_ok && mf_lds_bytes(b->S, b->sa.mf_split) <= 160 * 1024) {
    b->mf = true;
    b->info.mfma_ops_per_group_sample = b->mf_ga_ops + b->mf_gb_ops;
    b->info.streams_per_workgroup = b->S;
    b->info.lds_bytes = mf_lds_bytes(b->S, b->sa.mf_split);
    b->info.quad_path = 4;
    /* two staggered 4-stream groups per workgroup from MF2_MIN_STREAMS on
     * (LPCNET_MF2=0 off, =1 at any batch size); above one mf_kernel<4>
     * round, mfw_kernel (two or three groups with dedicated roles) where the
     * model allows it (LPCNET_MFW=0/1 off / on wherever mf2 runs,
     * LPCNET_MFW_G=2/3 forces the group count) */
    b->cus = current_device_cus();
    const int gauto = mfw_groups(b->B, b->cus);
    /* split models: the wide kernel's own split form where its tables exist
     * (mfw_split_tables), two groups only (LDS) */
    const bool mfw_ok = (!b->sa.mf_split || b->sa.mfw_split) && b->sa.rcp_hw;
    const char *ew = getenv("LPCNET_MFW");
    const bool wantw = ew ? atoi(ew) != 0 : gauto > 0;
    b->mfw_forced = ew && atoi(ew) != 0;
    const char *e2 = getenv("LPCNET_MF2");
    const bool want2 = e2 ? atoi(e2) != 0 : b->B >= MF2_MIN_STREAMS || (wantw && mfw_ok);
    if (want2 && mf2_lds_bytes(4, b->sa.mf_split) <= 160 * 1024) {
      b->mf2 = true;
      b->info.mfma_ops_per_group_sample = 2 * (b->mf_ga_ops + b->mf_gb_ops);
      b->info.streams_per_workgroup = 8;
      b->info.lds_bytes = mf2_lds_bytes(4, b->sa.mf_split);
      b->info.quad_path = 6;
      const char *eg = getenv("LPCNET_MFW_G");
      b->mfw_g = b->sa.mf_split ? 2 : eg ? (atoi(eg) == 2 ? 2 : 3) : (gauto ? gauto : 2);
      if (wantw && mfw_ok && mfw_lds_bytes(b->mfw_g, b->sa.mf_split) <= 160 * 1024) {
        b->mfw = true;
        b->info.mfma_ops_per_group_sample = b->mfw_g * (b->mf_ga_ops + b->mf_gb_ops);
        b->info.streams_per_workgroup = 4 * b->mfw_g;
        b->info.lds_bytes = mfw_lds_bytes(b->mfw_g, b->sa.mf_split);
        b->info.quad_path = 7;
      }
    }
    return;
  }
  b->info.streams_per_workgroup = b->S;
  b->info.lds_bytes = b->lds_bytes;
  b->info.quad_path = b->reg ? 1 : 0;
}

/* Parse, validate and re-tile a weight blob; with upload, replace the
 * batch's model on its device.  Nothing in *b changes unless every check
 * passes (the SampleArgs are built locally and committed at the end), so a
 * failed reload leaves either the previous model intact or, after the old
 * buffers were freed, no model at all (have_model false). */
/* mf_kernel GRU_A layout helpers (host side, deterministic).
 *
 * Unit blocks (8 units = one block row of each gate) are dealt to the six
 * GRU_A waves.  A wave runs as many 4x4x4 MFMA slots per gate as its
 * longest block row has blocks (rounded up to 4), so the assignment
 * decides both the padding and the balance between the two waves sharing
 * each SIMD (w, w+4; waves 2 and 3 share theirs with the samplers). */
static int mf_wave_cost(const std::vector<std::vector<int>> &ga, const int *ub8)
{
  size_t mz = 0, mh = 0;
  for (int j = 0; j < 8; j++) {
    mz = std::max(mz, std::max(ga[ub8[j]].size(), ga[NA / 8 + ub8[j]].size()));
    mh = std::max(mh, ga[2 * (NA / 8) + ub8[j]].size());
  }
  return 8 * (int)((mz + 3) / 4) + 4 * (int)((mh + 3) / 4);
}

#ifndef MF_SAMPLER_SIMD_WEIGHT
#define MF_SAMPLER_SIMD_WEIGHT 27
#endif

/* per-SIMD load of six GRU_A wave costs: waves 0/4 and 1/5 pair up; 2 and 3
 * pair with a sampler (its priority chain takes most of their SIMD: measured
 * ~74 cycles per slot there against ~27 per slot of a wave pair) */
static thread_local int g_mf_simd_weight = MF_SAMPLER_SIMD_WEIGHT; /* set per layout (LPCNET_MF_SIMD_W: tuning hook) */

static int mf_simd_score(const int *c)
{
  return std::max(std::max(c[0] + c[4], c[1] + c[5]), (g_mf_simd_weight * std::max(c[2], c[3])) / 10);
}

/* extra[w]: a fixed per-wave cost on top of its own rows (split models: the
 * hosted pieces) */
static std::vector<int> mf_assign_unit_blocks(const std::vector<std::vector<int>> &ga, const int *extra = nullptr,
                                              int iters = 40000)
{
  constexpr int NUB = NA / 8;
  std::vector<int> perm(NUB);
  /* start: unit blocks by descending z/r length, dealt in order */
  for (int u = 0; u < NUB; u++) perm[u] = u;
  auto zr = [&](int u) { return std::max(ga[u].size(), ga[NUB + u].size()); };
  std::stable_sort(perm.begin(), perm.end(), [&](int a, int b) { return zr(a) > zr(b); });
  auto score = [&](const std::vector<int> &p, long &sum) {
    int c[SAMPLE_WAVES];
    sum = 0;
    for (int w = 0; w < SAMPLE_WAVES; w++) sum += (c[w] = mf_wave_cost(ga, &p[8 * w]) + (extra ? extra[w] : 0));
    return mf_simd_score(c);
  };
  long best_sum;
  int best = score(perm, best_sum);
  uint32_t rng = 12345u;
  for (int it = 0; it < iters; it++) {
    rng = rng * 1664525u + 1013904223u;
    const int a = (rng >> 8) % NUB;
    rng = rng * 1664525u + 1013904223u;
    const int b = (rng >> 8) % NUB;
    if (a / 8 == b / 8) continue;
    std::swap(perm[a], perm[b]);
    long sum;
    const int sc = score(perm, sum);
    if (sc < best || (sc == best && sum <= best_sum)) {
      best = sc;
      best_sum = sum;
    } else {
      std::swap(perm[a], perm[b]);
    }
  }
  return perm;
}

/* Slot order of the 4 block rows one 32-lane LDS group reads in the same
 * ds_read_b32 (rows4[k]: input offsets of row k's blocks).  Input quad c of
 * stream m sits at dword c + 104 m, bank (c + 8 m) mod 32: quads of
 * different c mod 8 never share a bank, equal quads broadcast.  Each row's
 * blocks are matched to slots (Kuhn augmenting paths) so that every slot's
 * quads are bank-disjoint; blocks that cannot be placed so take any free
 * slot.  Empty positions (zero weights) read a quad another row reads in
 * that slot.  Integer sums do not depend on the order. */
static void mf_bank_slots(const std::vector<int> *const rows4[4], int nslot, int slot_of[4][MF_HMAX], int cb_at[4][MF_HMAX])
{
  int owner[4][MF_HMAX];
  int cls[MF_HMAX][8];
  for (int t = 0; t < MF_HMAX; t++)
    for (int c = 0; c < 8; c++) cls[t][c] = -1;
  for (int k = 0; k < 4; k++)
    for (int t = 0; t < MF_HMAX; t++) owner[k][t] = -1;
  int order[4] = {0, 1, 2, 3};
  std::stable_sort(order, order + 4, [&](int a, int b) { return rows4[a]->size() > rows4[b]->size(); });
  for (int oi = 0; oi < 4; oi++) {
    const int k = order[oi];
    const std::vector<int> &row = *rows4[k];
    const int n = (int)row.size();
    auto ok = [&](int i, int t) {
      const int cb = row[i] / 4, c = cb & 7;
      return cls[t][c] < 0 || cls[t][c] == cb;
    };
    int match_slot[MF_HMAX];  /* slot -> item of this row */
    for (int t = 0; t < nslot; t++) match_slot[t] = -1;
    std::vector<int> item_slot(n, -1);
    for (int i = 0; i < n; i++) {
      bool seen[MF_HMAX] = {};
      std::function<bool(int)> aug = [&](int it) -> bool {
        for (int t = 0; t < nslot; t++) {
          if (seen[t] || !ok(it, t)) continue;
          seen[t] = true;
          if (match_slot[t] < 0 || aug(match_slot[t])) {
            match_slot[t] = it;
            item_slot[it] = t;
            return true;
          }
        }
        return false;
      };
      aug(i);
    }
    for (int i = 0; i < n; i++)
      if (item_slot[i] < 0)
        for (int t = 0; t < nslot; t++)
          if (match_slot[t] < 0) {
            match_slot[t] = i;
            item_slot[i] = t;
            break;
          }
    for (int i = 0; i < n; i++) {
      const int t = item_slot[i], cb = row[i] / 4;
      slot_of[k][i] = t;
      owner[k][t] = cb;
      if (cls[t][cb & 7] < 0) cls[t][cb & 7] = cb;
    }
  }
  for (int t = 0; t < nslot; t++) {
    int any = 0;
    for (int k = 0; k < 4; k++)
      if (owner[k][t] >= 0) { any = owner[k][t]; break; }
    for (int k = 0; k < 4; k++) cb_at[k][t] = owner[k][t] >= 0 ? owner[k][t] : any;
  }
}

/* mf_kernel work plan of the GRU_A recurrent product.
 *
 * Each GRU_A lane group (8 lanes) owns one unit block (8 units, one 8-row
 * block row per gate) and runs, per gate, `own` slots of its row's blocks.
 * A trained model's block rows can be far longer than the mean -- Sparsify
 * keeps blocks by a global per-gate energy threshold (training_tf2/
 * lpcnet.py:140-160) -- so a row longer than the own cap is split: its first
 * own[g] blocks stay with the owner, the rest go in pieces of at most
 * piece[g] blocks to other lane groups' hosted region (at most one piece per
 * lane group and gate), whose int32 partial sums the kernel adds into the
 * owner's accumulator through LDS.  Integer sums are exact in any order, so
 * the result is bit-identical to the unsplit product. */
struct MfPiece {
  int unit, t0, t1; /* blocks [t0, t1) of unit block `unit`'s row of the gate */
};
struct MfPlan {
  bool split = false;
  std::vector<int> perm;               /* lane group -> own unit block */
  int own[3] = {MF_ZMAX, MF_ZMAX, MF_HMAX};
  std::vector<MfPiece> pieces[3];
  std::vector<int> host[3];            /* lane group -> piece index (-1 none) */
  int nzr[SAMPLE_WAVES] = {}, nh[SAMPLE_WAVES] = {}, nfzr[SAMPLE_WAVES] = {}, nfh[SAMPLE_WAVES] = {};
};

/* hosted-piece merge cost of a wave, in MFMA slots: its partial sums'
 * LDS adds (per gate hosted) */
#ifndef MF_HOSTED_WEIGHT
#define MF_HOSTED_WEIGHT 14 /* tenths: cost of a hosted slot relative to an own one */
#endif
static thread_local int g_mf_hosted_f = MF_HOSTED_WEIGHT;
#ifndef MF_PIECE_WEIGHT
#define MF_PIECE_WEIGHT 10 /* tenths of a score unit per hosted piece (its LDS atomics) */
#endif
static thread_local int g_mf_piece_w = MF_PIECE_WEIGHT;
#ifndef MF_HOST_ADD_SLOTS
#define MF_HOST_ADD_SLOTS 4
#endif

/* One candidate split (own caps T, piece sizes F) laid out: own rows ->
 * lane groups balanced together with the hosted pieces (which waves host z/r
 * and h pieces: every subset that holds them and fits the registers, scored
 * by the per-SIMD load), pieces -> lane groups of the hosting waves.
 * Returns the score (-1: does not fit). */
static long mf_layout(const std::vector<std::vector<int>> &ga, MfPlan &P, const int T[3], const int F[3], int iters,
                      int simd_w = MF_SAMPLER_SIMD_WEIGHT)
{
  constexpr int NUB = NA / 8, NLG = SAMPLE_WAVES * 8;
  P.own[0] = T[0];
  P.own[1] = T[1];
  P.own[2] = T[2];
  for (int g = 0; g < 3; g++) {
    P.pieces[g].clear();
    for (int u = 0; u < NUB; u++) {
      const int K = (int)ga[g * NUB + u].size();
      if (K > T[g] && F[g] <= 0) return -1;
      for (int t0 = T[g]; t0 < K; t0 += F[g]) P.pieces[g].push_back(MfPiece{u, t0, std::min(K, t0 + F[g])});
    }
    if ((int)P.pieces[g].size() > NLG) return -1;
  }
  std::vector<std::vector<int>> own(ga.size());
  for (int g = 0; g < 3; g++)
    for (int u = 0; u < NUB; u++) {
      const std::vector<int> &v = ga[g * NUB + u];
      own[g * NUB + u].assign(v.begin(), v.begin() + std::min((int)v.size(), T[g]));
    }
  const int npz = (int)std::max(P.pieces[0].size(), P.pieces[1].size()), nph = (int)P.pieces[2].size();
  const int npieces = (int)(P.pieces[0].size() + P.pieces[1].size() + P.pieces[2].size());
  int extra[SAMPLE_WAVES] = {};
  int mz = 0, mh = 0; /* hosting waves (bit masks) */
  long best = -1;
  if (const char *v = getenv("LPCNET_MF_ITERS")) iters = atoi(v); /* tuning hooks */
  g_mf_simd_weight = getenv("LPCNET_MF_SIMD_W") ? atoi(getenv("LPCNET_MF_SIMD_W")) : simd_w;
  g_mf_hosted_f = getenv("LPCNET_MF_HOSTED_F") ? atoi(getenv("LPCNET_MF_HOSTED_F")) : MF_HOSTED_WEIGHT;
  g_mf_piece_w = getenv("LPCNET_MF_PIECE_W") ? atoi(getenv("LPCNET_MF_PIECE_W")) : MF_PIECE_WEIGHT;
  P.perm = mf_assign_unit_blocks(own, extra, iters);
  for (int round = 0; round < 2; round++) {
    int c[SAMPLE_WAVES], gz[SAMPLE_WAVES], gh[SAMPLE_WAVES];
    for (int w = 0; w < SAMPLE_WAVES; w++) {
      c[w] = mf_wave_cost(own, &P.perm[8 * w]);
      size_t az = 0, ah = 0;
      for (int j = 0; j < 8; j++) {
        const int ub = P.perm[8 * w + j];
        az = std::max(az, std::max(own[ub].size(), own[NUB + ub].size()));
        ah = std::max(ah, own[2 * NUB + ub].size());
      }
      gz[w] = (int)(az + 3) / 4;
      gh[w] = (int)(ah + 3) / 4;
    }
    best = -1;
    for (int sz = 0; sz < (1 << SAMPLE_WAVES); sz++) {
      if (8 * __builtin_popcount(sz) < npz || (npz == 0 && sz)) continue;
      for (int sh = 0; sh < (1 << SAMPLE_WAVES); sh++) {
        if (8 * __builtin_popcount(sh) < nph || (nph == 0 && sh)) continue;
        int cc[SAMPLE_WAVES];
        bool ok = true;
        long sum = 0;
        for (int w = 0; w < SAMPLE_WAVES && ok; w++) {
          cc[w] = c[w];
          if (sz >> w & 1) {
            ok &= 4 * gz[w] + F[0] <= MF_ZMAX;
            cc[w] += (g_mf_hosted_f * 2 * F[0]) / 10 + 2 * MF_HOST_ADD_SLOTS;
          }
          if (sh >> w & 1) {
            ok &= 4 * gh[w] + F[2] <= MF_HMAX;
            cc[w] += (g_mf_hosted_f * F[2]) / 10 + MF_HOST_ADD_SLOTS;
          }
          sum += cc[w];
        }
        if (!ok) continue;
        const long sc = ((long)mf_simd_score(cc) + (long)g_mf_piece_w * npieces / 10) * 4096 + sum;
        if (best < 0 || sc < best) {
          best = sc;
          mz = sz;
          mh = sh;
        }
      }
    }
    if (best < 0) return -1;
    if (round == 1) break;
    /* re-balance the own rows around the hosting waves' extra load */
    for (int w = 0; w < SAMPLE_WAVES; w++)
      extra[w] = (mz >> w & 1 ? (g_mf_hosted_f * 2 * F[0]) / 10 + 2 * MF_HOST_ADD_SLOTS : 0) +
                 (mh >> w & 1 ? (g_mf_hosted_f * F[2]) / 10 + MF_HOST_ADD_SLOTS : 0);
    P.perm = mf_assign_unit_blocks(own, extra, iters);
  }
  /* pieces -> lane groups of the hosting waves, spread over those waves
   * (lane group j of each hosting wave, then j + 1) */
  for (int g = 0; g < 3; g++) {
    const int m = g < 2 ? mz : mh;
    std::vector<int> lgs;
    for (int j = 0; j < 8; j++)
      for (int w = 0; w < SAMPLE_WAVES; w++)
        if (m >> w & 1) lgs.push_back(8 * w + j);
    P.host[g].assign(NLG, -1);
    for (int p = 0; p < (int)P.pieces[g].size(); p++) P.host[g][lgs[p]] = p;
  }
  for (int w = 0; w < SAMPLE_WAVES; w++) {
    int kz = 0, kh = 0, fz = 0, fh = 0;
    for (int j = 0; j < 8; j++) {
      const int lg = 8 * w + j, ub = P.perm[lg];
      kz = std::max(kz, (int)std::max(own[ub].size(), own[NUB + ub].size()));
      kh = std::max(kh, (int)own[2 * NUB + ub].size());
      for (int g = 0; g < 3; g++)
        if (P.host[g][lg] >= 0) {
          const MfPiece &pc = P.pieces[g][P.host[g][lg]];
          (g < 2 ? fz : fh) = std::max(g < 2 ? fz : fh, pc.t1 - pc.t0);
        }
    }
    P.nzr[w] = (kz + 3) / 4;
    P.nh[w] = (kh + 3) / 4;
    P.nfzr[w] = (fz + 3) / 4;
    P.nfh[w] = (fh + 3) / 4;
    if (4 * (P.nzr[w] + P.nfzr[w]) > MF_ZMAX || 4 * (P.nh[w] + P.nfh[w]) > MF_HMAX) return -1;
  }
  return best;
}

/* mfw_kernel's split form (trained Sparsify masks on the wide kernel): the
 * six R waves keep the unit blocks of `perm` (the batch's main plan, so the
 * E waves' lane-ordered tables stay valid) up to the full register caps
 * (16 z/r, 32 h blocks: the unsplit kernel's largest tables), and every
 * block beyond goes, in pieces of at most those caps, to the 16 lane groups
 * of two host waves (MFW_H_WAVES): one piece per host lane group and gate,
 * longest pieces first, dealt alternately to the two waves.  A host lane's
 * int32 partial sums reach its row's owner through LDS adds into a compact
 * part area: per gate, the unit blocks with pieces (at most 16) take part
 * rows 8 slot .. 8 slot + 7.  Exact int32 sums in any order: bit-identical
 * to the unsplit product.  Tables: [MFW_TAB_WAVES][MF_LANE_U32][64] as the
 * mf tables (host waves: their piece at slot 0 of each gate), frow
 * [3][SAMPLE_THREADS + 128]: an E thread's part row | 1 << 16 when its unit
 * has pieces (else MFW_NOROW), a host lane's target part row (else
 * MFW_NOROW).  False when a gate needs more than 16 pieces. */
struct MfwSplitTab {
  int nzr[MFW_TAB_WAVES] = {}, nh[MFW_TAB_WAVES] = {};
  std::vector<uint32_t> tab;
  std::vector<int> frow;
  std::vector<int> units; /* [SAMPLE_THREADS] own unit of each lane (perm below) */
};

static bool mfw_split_tables(const std::vector<std::vector<int>> &ga, const std::vector<int> &ga_first,
                             const int8_t *wa, MfwSplitTab &T)
{
  constexpr int NUB = NA / 8, NHL = 8 * MFW_H_WAVES, FS = SAMPLE_THREADS + 64 * MFW_H_WAVES;
  const int cap[3] = {MF_ZMAX, MF_ZMAX, MF_HMAX};
  std::vector<MfPiece> pcs[3];
  std::vector<int> host[3]; /* host lane group (0..15) -> piece index */
  std::vector<int> slot_of_ub[3];
  for (int g = 0; g < 3; g++) {
    for (int u = 0; u < NUB; u++) {
      const int K = (int)ga[g * NUB + u].size();
      for (int t0 = cap[g]; t0 < K; t0 += cap[g]) pcs[g].push_back(MfPiece{u, t0, std::min(K, t0 + cap[g])});
    }
    if ((int)pcs[g].size() > NHL) return false;
    std::stable_sort(pcs[g].begin(), pcs[g].end(), [](const MfPiece &a, const MfPiece &b) { return a.t1 - a.t0 > b.t1 - b.t0; });
    host[g].assign(NHL, -1);
    for (int k = 0; k < (int)pcs[g].size(); k++) host[g][(k % MFW_H_WAVES) * 8 + k / MFW_H_WAVES] = k;
    slot_of_ub[g].assign(NUB, -1);
    int ns = 0;
    for (const MfPiece &pc : pcs[g])
      if (slot_of_ub[g][pc.unit] < 0) slot_of_ub[g][pc.unit] = ns++;
    if (ns > 16) return false;
  }
  /* own unit blocks over the six R waves for the capped rows; the E waves'
   * lane order follows.  The R waves on SIMDs 2 / 3 share them with a
   * sampler, a host wave and an E wave, all at a higher issue priority:
   * their rows are weighted 6x (the unsplit kernel's 2.5x: skewed 8,192
   * streams 486 -> 494 M, 4x-10x alike, profiles/r06/split_simdw_8192.log) */
  std::vector<std::vector<int>> own(ga.size());
  for (int g = 0; g < 3; g++)
    for (int u = 0; u < NUB; u++) {
      const std::vector<int> &v = ga[g * NUB + u];
      own[g * NUB + u].assign(v.begin(), v.begin() + std::min((int)v.size(), cap[g]));
    }
  g_mf_simd_weight = getenv("LPCNET_MF_SIMD_W") ? atoi(getenv("LPCNET_MF_SIMD_W")) : 60;
  const std::vector<int> perm = mf_assign_unit_blocks(own, nullptr, 40000);
  T.units.assign(SAMPLE_THREADS, 0);
  for (int t = 0; t < SAMPLE_THREADS; t++) T.units[t] = 8 * perm[t / 8] + (t & 7);
  T.tab.assign((size_t)MFW_TAB_WAVES * MF_LANE_U32 * 64, 0);
  T.frow.assign((size_t)3 * FS, MFW_NOROW);
  for (int w = 0; w < MFW_TAB_WAVES; w++) {
    const bool hw = w >= SAMPLE_WAVES;
    /* this wave's rows per lane group and gate: (row block, first, end) */
    int rb[8][3], t0[8][3], t1[8][3];
    int kz = 1, kh = 1; /* at least one slot group (zero weights: exact) */
    for (int j = 0; j < 8; j++)
      for (int g = 0; g < 3; g++) {
        rb[j][g] = -1;
        t0[j][g] = t1[j][g] = 0;
        if (!hw) {
          const int u = perm[w * 8 + j];
          rb[j][g] = g * NUB + u;
          t1[j][g] = std::min((int)ga[rb[j][g]].size(), cap[g]);
        } else if (host[g][(w - SAMPLE_WAVES) * 8 + j] >= 0) {
          const MfPiece &pc = pcs[g][host[g][(w - SAMPLE_WAVES) * 8 + j]];
          rb[j][g] = g * NUB + pc.unit;
          t0[j][g] = pc.t0;
          t1[j][g] = pc.t1;
          for (int r = 0; r < 8; r++)
            T.frow[(size_t)g * FS + SAMPLE_THREADS + (w - SAMPLE_WAVES) * 64 + 8 * j + r] =
                8 * slot_of_ub[g][pc.unit] + r;
        }
        (g < 2 ? kz : kh) = std::max(g < 2 ? kz : kh, t1[j][g] - t0[j][g]);
      }
    T.nzr[w] = (kz + 3) / 4;
    T.nh[w] = (kh + 3) / 4;
    auto word = [&](int k, int l) -> uint32_t & { return T.tab[((size_t)w * MF_LANE_U32 + k) * 64 + l]; };
    for (int g = 0; g < 3; g++) {
      const int base = g == 0 ? 0 : (g == 1 ? MF_ZMAX : 2 * MF_ZMAX);
      const int nslot = 4 * (g < 2 ? T.nzr[w] : T.nh[w]);
      for (int half = 0; half < 2; half++) {
        std::vector<int> lists[4];
        for (int k = 0; k < 4; k++) {
          const int j = 4 * half + k;
          if (rb[j][g] >= 0) lists[k].assign(ga[rb[j][g]].begin() + t0[j][g], ga[rb[j][g]].begin() + t1[j][g]);
        }
        const std::vector<int> *rows4[4] = {&lists[0], &lists[1], &lists[2], &lists[3]};
        int slot_of[4][MF_HMAX], cb_at[4][MF_HMAX];
        mf_bank_slots(rows4, nslot, slot_of, cb_at);
        for (int k = 0; k < 4; k++) {
          const int j = 4 * half + k;
          for (int r = 0; r < 8; r++) {
            const int l = 8 * j + r;
            for (int t = 0; t < (int)lists[k].size(); t++)
              memcpy(&word(base + slot_of[k][t], l), wa + 32 * (ga_first[rb[j][g]] + t0[j][g] + t) + 4 * r, 4);
            for (int t = 0; t < nslot; t++) word(MF_GA + (base + t) / 4, l) |= (uint32_t)cb_at[k][t] << (8 * ((base + t) & 3));
          }
        }
      }
    }
  }
  /* the E threads' merge entries: thread t owns unit 8 perm[t / 8] + t % 8 */
  for (int g = 0; g < 3; g++)
    for (int t = 0; t < SAMPLE_THREADS; t++) {
      const int u = perm[t / 8], sl = slot_of_ub[g][u];
      if (sl >= 0) T.frow[(size_t)g * FS + t] = (8 * sl + (t % 8)) | 1 << 16;
    }
  return true;
}

/* cls: the kernel the plan serves.  1: mf_kernel at 4 streams per
 * workgroup (1024-2047 streams), whose Y -> X half is bound by the GRU_A
 * recurrent product of the waves sharing a SIMD with a sampler (~3x the
 * cycles per MFMA of a wave pair): those SIMDs weighted 3.3x and a longer
 * search (same box, 1024 streams: -0.6 to -1.1 % frame step).  2:
 * mf2_kernel (from 2048 streams), whose samplers idle half of each phase:
 * 2.0x (2048 streams -2.1 %, 8192 -0.7 %).  3: mfw_kernel (its R waves
 * on SIMDs 2/3 share them with a sampler and an E wave): 2.5x (8192 and
 * 24,576 streams -1.0 / -0.8 % against 2.0x; 1.0, 1.4, 1.7, 2.3, 2.8, 3.3x
 * measured, profiles/r05/simdw_ab*.log).  0: 2.7x, one and two streams per
 * workgroup.  Split plans: 3.3x on mf_kernel<4>, 2.7x otherwise. */
bool mf_plan(const std::vector<std::vector<int>> &ga, MfPlan &P, int cls = 0, int cls_split = -1)
{
  if (cls_split < 0) cls_split = cls;
  const bool S4 = cls == 1;
  const int w_unsplit = cls == 1 ? 33 : cls == 2 ? 20 : cls == 3 ? 25 : MF_SAMPLER_SIMD_WEIGHT;
  constexpr int NUB = NA / 8;
  int kmax[3] = {0, 0, 0};
  for (int g = 0; g < 3; g++)
    for (int u = 0; u < NUB; u++) kmax[g] = std::max(kmax[g], (int)ga[g * NUB + u].size());
  const bool force = getenv("LPCNET_MF_FORCE_SPLIT") != nullptr;
  if (std::max(kmax[0], kmax[1]) <= MF_ZMAX && kmax[2] <= MF_HMAX && !force) {
    P.split = false;
    const int T[3] = {MF_ZMAX, MF_ZMAX, MF_HMAX}, F[3] = {0, 0, 0};
    return mf_layout(ga, P, T, F, S4 ? 400000 : 40000, w_unsplit) >= 0;
  }
  /* split plans weight the sampler SIMDs 3.3x on mf_kernel (1-4 streams per
   * workgroup: measured best plans at 256 and 1024 streams) and 2.0x on
   * mf2_kernel (skewed model, 8192 / 2048 streams -3.3 / -1.2 % against
   * 2.7x; 1.5, 1.7, 2.2, 2.4, 3.3x measured, profiles/r05/simdw_skew*.log) */
  const int w_split = cls_split == 2 ? 20 : 33;
  /* split: every own cap / piece size pair, screened with a short
   * assignment search, the best re-laid-out in full (LPCNET_MF_FORCE_SPLIT:
   * split even a model that fits -- pieces required -- for tests) */
  P.split = true;
  long best = -1;
  int bt[3] = {0, 0, 0}, bf[3] = {0, 0, 0};
  if (const char *v = getenv("LPCNET_MF_CAPS")) {
    /* tuning hook: "Tz,Fz,Th,Fh" (own caps and piece sizes in blocks) */
    int c[4];
    if (sscanf(v, "%d,%d,%d,%d", &c[0], &c[1], &c[2], &c[3]) == 4) {
      const int T[3] = {c[0], c[0], c[2]}, F[3] = {c[1], c[1], c[3]};
      if (mf_layout(ga, P, T, F, 40000, w_split) >= 0) return true;
    }
  }
  for (int Tz = 4; Tz <= MF_ZMAX; Tz += 4)
    for (int Fz = 0; Tz + Fz <= MF_ZMAX; Fz += 4)
      for (int Th = 4; Th <= MF_HMAX; Th += 4)
        for (int Fh = 0; Th + Fh <= MF_HMAX; Fh += 4) {
          bool need = false, fits = true;
          for (int g = 0; g < 3; g++) {
            const int T = g < 2 ? Tz : Th, F = g < 2 ? Fz : Fh;
            for (int u = 0; u < NUB; u++) {
              const int K = (int)ga[g * NUB + u].size();
              need |= K > T;
              if (K > T && F == 0) fits = false;
            }
            /* a piece size with nothing to carry is padding */
            bool any = false;
            for (int u = 0; u < NUB; u++) any |= (int)ga[g * NUB + u].size() > T;
            if (F > 0 && !any && g != 0 && g != 1) fits = false;
          }
          if (Fz > 0) {
            bool any = false;
            for (int u = 0; u < NUB; u++) any |= std::max(ga[u].size(), ga[NUB + u].size()) > (size_t)Tz;
            if (!any) fits = false;
          }
          if (!fits || (force && !need)) continue;
          MfPlan C;
          const int T[3] = {Tz, Tz, Th}, F[3] = {Fz, Fz, Fh};
          const long sc = mf_layout(ga, C, T, F, 1500, w_split);
          if (sc < 0) continue;
          if (best < 0 || sc < best) {
            best = sc;
            bt[0] = bt[1] = Tz; bt[2] = Th;
            bf[0] = bf[1] = Fz; bf[2] = Fh;
          }
        }
  if (best < 0) return false; /* does not fit even split: the lockstep kernel runs it */
  return mf_layout(ga, P, bt, bf, 40000, w_split) >= 0;
}

/* The model constants of a blob (see load_model); -1 on a malformed record
 * or an unsupported value. */
int model_constants(const std::vector<Arr> &L, ModelConst &mc)
{
  if (const Arr *a = find(L, "LPC_GAMMA")) {
    if (a->size != 4) { set_err("LPC_GAMMA record must hold one float"); return -1; }
    memcpy(&mc.lpc_gamma, a->data, 4);
  }
  if (const Arr *a = find(L, "FEATURES_DELAY")) {
    if (a->size != 4) { set_err("FEATURES_DELAY record must hold one int"); return -1; }
    memcpy(&mc.delay, a->data, 4);
  }
  if (const Arr *a = find(L, "END2END")) {
    if (a->size != 4) { set_err("END2END record must hold one int"); return -1; }
    memcpy(&mc.end2end, a->data, 4);
  }
  if (const char *v = getenv("LPCNET_LPC_GAMMA")) mc.lpc_gamma = strtof(v, nullptr);
  if (const char *v = getenv("LPCNET_FEATURES_DELAY")) mc.delay = atoi(v);
  if (const char *v = getenv("LPCNET_END2END")) mc.end2end = atoi(v);
  return check_constants(mc);
}

int load_model(LPCNetBatch *b, const unsigned char *data, int len, bool upload = true)
{
  std::vector<Arr> L;
  if (!data || len <= 0 || !parse_blob(L, data, len)) {
    set_err("malformed weight blob");
    return -1;
  }
  std::vector<std::vector<int>> ga_blocks, gb_blocks;
  if (!parse_idx(L, "sparse_gru_a_recurrent_weights_idx", NA, GA_ROWS, ga_blocks)) return -1;
  if (!parse_idx(L, "gru_b_weights_idx", NA, GB_ROWS, gb_blocks)) return -1;
  const int nba = total_blocks(ga_blocks), nbb = total_blocks(gb_blocks);
  const Arr *gaw = find(L, "sparse_gru_a_recurrent_weights");
  if (!gaw) { set_err("missing sparse_gru_a_recurrent_weights"); return -1; }
  int variant;
  if (gaw->size == 32 * nba) variant = LPCNET_VARIANT_INT8;
  else if (gaw->size == 32 * nba * 4) variant = LPCNET_VARIANT_FP32;
  else { set_err("sparse_gru_a_recurrent_weights size matches neither int8 nor fp32"); return -1; }
  const int q = variant == LPCNET_VARIANT_FP32 ? 4 : 1;

#define F(var, name, cnt) const float *var = (const float *)find_check(L, name, (cnt)*4); if (!var) return -1
  F(conv1_w, "feature_conv1_weights", 3 * FIN * COND);
  F(conv1_b, "feature_conv1_bias", COND);
  F(conv2_w, "feature_conv2_weights", 3 * COND * COND);
  F(conv2_b, "feature_conv2_bias", COND);
  F(dense1_w, "feature_dense1_weights", COND * COND);
  F(dense1_b, "feature_dense1_bias", COND);
  F(dense2_w, "feature_dense2_weights", COND * COND);
  F(dense2_b, "feature_dense2_bias", COND);
  F(gadf_w, "gru_a_dense_feature_weights", COND * GA_ROWS);
  F(gadf_b, "gru_a_dense_feature_bias", GA_ROWS);
  F(gbdf_w, "gru_b_dense_feature_weights", COND * GB_ROWS);
  F(gbdf_b, "gru_b_dense_feature_bias", GB_ROWS);
  F(embed_pitch, "embed_pitch_weights", 256 * EP);
  F(embed_sig, "embed_sig_weights", 256 * 128);
  F(emb_sig, "gru_a_embed_sig_weights", 256 * GA_ROWS);
  F(emb_pred, "gru_a_embed_pred_weights", 256 * GA_ROWS);
  F(emb_exc, "gru_a_embed_exc_weights", 256 * GA_ROWS);
  F(ga_bias, "sparse_gru_a_bias", 6 * NA);
  F(ga_subias, "sparse_gru_a_subias", 6 * NA);
  F(ga_diag, "sparse_gru_a_recurrent_weights_diag", 3 * NA);
  F(gb_bias, "gru_b_bias", 6 * NB);
  F(gb_subias, "gru_b_subias", 6 * NB);
  F(fc_b, "dual_fc_bias", 512);
  F(fc_w, "dual_fc_weights", 256 * 32);
  F(fc_f, "dual_fc_factor", 512);
#undef F
  (void)embed_sig;
  /* model constants: optional side records named like the #defines
   * dump_lpcnet.py:423-446 writes into nnet_data.h (LPC_GAMMA float,
   * FEATURES_DELAY int, END2END int; the reference's parser ignores unknown
   * records), else the dump defaults; LPCNET_LPC_GAMMA /
   * LPCNET_FEATURES_DELAY / LPCNET_END2END override both (drop-in callers) */
  ModelConst mc{1.0f, DEFAULT_FEATURES_DELAY, 0};
  if (model_constants(L, mc)) return -1;
  /* the 1.6 kb/s decoder's codebooks (lpcnet_private.h:109-112, generated
   * ceps_codebooks.c in the reference; lpcnet_enc.c:109-119, 709 give their
   * sizes): optional records -- a blob without them (or with mis-sized ones,
   * which the reference's parser would never bind either) still synthesises,
   * only lpcnet_decode refuses it */
  const Arr *cb[4] = {find(L, "ceps_codebook1"), find(L, "ceps_codebook2"), find(L, "ceps_codebook3"),
                      find(L, "ceps_codebook_diff4")};
  bool cb_ok = true;
  for (int k = 0; k < 4; k++) cb_ok &= cb[k] && cb[k]->size == (k < 3 ? 1024 * (NBANDS - 1) : 4096 * NBANDS) * 4;
  const void *gbw = find_check(L, "gru_b_weights", 32 * nbb * q);

  const void *gbrec = find_check(L, "gru_b_recurrent_weights", 3 * NB * NB * q);
  if (!gbw || !gbrec) return -1;

  /* ---- derived host layouts ---- */
  const bool int8 = variant == LPCNET_VARIANT_INT8;
  bool sat = false;
  if (int8) {
    const int8_t *wa = (const int8_t *)gaw->data, *wb = (const int8_t *)gbw, *wr = (const int8_t *)gbrec;
    for (int k = 0; k < nba && !sat; k++) sat |= block_may_saturate(wa + 32 * k);
    for (int k = 0; k < nbb && !sat; k++) sat |= block_may_saturate(wb + 32 * k);
    for (int k = 0; k < 3 * NB * NB / 32 && !sat; k++) sat |= block_may_saturate(wr + 32 * k);
  }
  const float *abias = int8 ? ga_subias : ga_bias; /* USE_SU_BIAS only with DOT_PROD */
  const float *bbias = int8 ? gb_subias : gb_bias;
  std::vector<float> ga_par(6 * NA), gb_par(2 * GB_ROWS);
  std::vector<int> ga_wsum(3 * NA, 0), gb_wsum(2 * GB_ROWS, 0);
  for (int g = 0; g < 3; g++)
    for (int i = 0; i < NA; i++) {
      ga_par[g * NA + i] = abias[3 * NA + g * NA + i];
      ga_par[(3 + g) * NA + i] = ga_diag[g * NA + i];
    }
  for (int r = 0; r < GB_ROWS; r++) {
    gb_par[r] = bbias[r];
    gb_par[GB_ROWS + r] = bbias[GB_ROWS + r];
  }

  /* per-block offsets into the blob weights */
  std::vector<int> ga_first(ga_blocks.size() + 1, 0), gb_first(gb_blocks.size() + 1, 0);
  for (size_t r = 0; r < ga_blocks.size(); r++) ga_first[r + 1] = ga_first[r] + (int)ga_blocks[r].size();
  for (size_t r = 0; r < gb_blocks.size(); r++) gb_first[r + 1] = gb_first[r] + (int)gb_blocks[r].size();

  if (int8 && !sat) {
    const int8_t *wa = (const int8_t *)gaw->data, *wb = (const int8_t *)gbw, *wr = (const int8_t *)gbrec;
    for (int rb = 0; rb < GA_ROWS / 8; rb++)
      for (int k = ga_first[rb]; k < ga_first[rb + 1]; k++)
        for (int r = 0; r < 8; r++)
          for (int c = 0; c < 4; c++) ga_wsum[rb * 8 + r] += 128 * wa[32 * k + r * 4 + c];
    for (int rb = 0; rb < GB_ROWS / 8; rb++)
      for (int k = gb_first[rb]; k < gb_first[rb + 1]; k++)
        for (int r = 0; r < 8; r++)
          for (int c = 0; c < 4; c++) gb_wsum[rb * 8 + r] += 128 * wb[32 * k + r * 4 + c];
    for (int rb = 0; rb < GB_ROWS / 8; rb++)
      for (int cb = 0; cb < NB / 4; cb++)
        for (int r = 0; r < 8; r++)
          for (int c = 0; c < 4; c++) gb_wsum[GB_ROWS + rb * 8 + r] += 128 * wr[32 * (rb * (NB / 4) + cb) + r * 4 + c];
  }

  /* ---- LDS image ---- */
  std::vector<unsigned char> img(IMG_VAR, 0);
  /* device form: t + (127 << 23), see rcp_x86_fix; the default is the Intel
   * table (11 bits, each entry twice); a custom table stays across reloads,
   * LPCNET_RCP=host selects this host's at load time */
  std::vector<uint32_t> rcp_dev(RCP_ENTRIES);
  if (b->rcp_custom && (int)b->rcp_dev.size() == RCP_ENTRIES) {
    rcp_dev = b->rcp_dev;
  } else {
    for (int i = 0; i < RCP_ENTRIES; i++) rcp_dev[i] = kRcpTable[i >> (RCP_TABLE_BITS - 11)] + kRcpBias;
    if (const char *e = getenv("LPCNET_RCP"))
      if (!strcmp(e, "host")) {
        std::vector<uint32_t> h(RCP_ENTRIES);
        if (lpcnet_mi355x_host_rcp_table(h.data(), RCP_ENTRIES) != 0) {
          set_err("LPCNET_RCP=host: this host's rcpps is not a 12-bit exponent-invariant table");
          return -1;
        }
        for (int i = 0; i < RCP_ENTRIES; i++) rcp_dev[i] = h[i] + kRcpBias;
      }
  }
  memcpy(&img[IMG_RCP], rcp_dev.data(), RCP_ENTRIES * 4);
  for (int i = 0; i < 256; i++) {
    float u = host_ulaw2lin((float)i);
    memcpy(&img[IMG_ULAW + 4 * i], &u, 4);
    /* lpcnet.c:188-191 */
    float prob = .025f + .95f * i / 255.f;
    float lg = (float)-log((double)((1 - prob) / prob)); /* C double log, not logf */
    memcpy(&img[IMG_LOGIT + 4 * i], &lg, 4);
  }
  memcpy(&img[IMG_FCW], fc_w, 256 * 32 * 4);
  bool fc_fin = true;
  {
    /* dual-FC node sums (nnet.c:193-199) are bounded by |bias| + 2 sum|w|
     * for GRU_B states within [-2, 2]: far below 2^60 and finite, tanh8's
     * flush and NaN selects are dead (tanh_x86_fin_n) */
    bool fin = true;
    for (int c = 0; c < 2 && fin; c++)
      for (int i = 0; i < 256 && fin; i++) {
        double bd = fabs((double)fc_b[c * 256 + i]);
        for (int j = 0; j < 16; j++) bd += 2.0 * fabs((double)fc_w[i * 32 + c * 16 + j]);
        fin = std::isfinite(bd) && bd < 0x1p59;
      }
    const char *fe = getenv("LPCNET_FC_EXACT"); /* test hook: force the exact form */
    fc_fin = fin && !(fe && atoi(fe));
  }
  memcpy(&img[IMG_FCB], fc_b, 512 * 4);
  memcpy(&img[IMG_FCF], fc_f, 512 * 4);
  auto align16 = [&]() { img.resize((img.size() + 15) / 16 * 16, 0); };
  auto put = [&](const void *p, size_t n) -> size_t {
    align16();
    size_t off = img.size();
    img.resize(off + n);
    memcpy(&img[off], p, n);
    return off;
  };
  SampleArgs sa;
  memset(&sa, 0, sizeof(sa));
  sa.fc_fin = fc_fin ? 1 : 0;
  std::vector<float4> ga_wf, gb_wf_unused;
  if (int8) sa.gb_rec_off = (int)put(gbrec, 3 * NB * NB);
  /* blocks per lane for each (wave, gate) of the GRU_A layout */
  int gaK[SAMPLE_WAVES][3];
  bool reg = int8;
  for (int w = 0; w < SAMPLE_WAVES; w++)
    for (int g = 0; g < 3; g++) {
      int K = 0;
      for (int j = 0; j < 8; j++) K = std::max(K, (int)ga_blocks[g * (NA / 8) + w * 8 + j].size());
      gaK[w][g] = K;
      if (K > 96) reg = false;
    }
  for (int rb = 0; rb < GB_ROWS / 8; rb++)
    if ((int)gb_blocks[rb].size() > 8 * REG_GB) reg = false;
  if (getenv("LPCNET_NO_QUAD")) reg = false; /* A/B switch: per-slot LDS layout */
  if (reg) {
    /* quad layout: wave w, gate g, group gi of 4 slots, lane l = 8*(row block in wave) + row.
     * The z, r and h groups of one wave are contiguous (weights and column
     * words alike), so the kernel runs them as one software-pipelined stream. */
    for (int w = 0; w < SAMPLE_WAVES; w++) {
      int K4[3], G = 0;
      for (int g = 0; g < 3; g++) {
        K4[g] = (gaK[w][g] + 3) / 4;
        sa.ga_K4[w][g] = K4[g];
        G += K4[g];
      }
      std::vector<uint32_t> q((size_t)std::max(G, 1) * 64 * 4, 0), c((size_t)std::max(G, 1) * 8, 0);
      int g0 = 0;
      for (int g = 0; g < 3; g++) {
        for (int l = 0; l < 64; l++) {
          const int j = l >> 3, r = l & 7, rb = g * (NA / 8) + w * 8 + j;
          for (int k = 0; k < (int)ga_blocks[rb].size(); k++) {
            memcpy(&q[((size_t)(g0 + k / 4) * 64 + l) * 4 + (k & 3)], (const int8_t *)gaw->data + 32 * (ga_first[rb] + k) + 4 * r, 4);
            if (r == 0) c[(g0 + k / 4) * 8 + j] |= (uint32_t)(ga_blocks[rb][k] / 4) << (8 * (k & 3));
          }
        }
        g0 += K4[g];
      }
      const int qbase = (int)(put(q.data(), q.size() * 4) / 16);
      const int cbase = (int)(put(c.data(), c.size() * 4) / 4);
      for (int g = 0, acc = 0; g < 3; acc += K4[g], g++) {
        sa.ga_qoff[w][g] = qbase + acc * 64;
        sa.ga_coff[w][g] = cbase + acc * 8;
      }
    }
    for (int rb = 0; rb < GB_ROWS / 8; rb++) {
      std::vector<uint32_t> q((size_t)(REG_GB / 4) * 64 * 4, 0), c((size_t)(REG_GB / 4) * 8, 0);
      for (int l = 0; l < 64; l++) {
        const int r = l & 7, ks = l >> 3;
        for (int j = 0; j < REG_GB; j++) {
          const int k = ks + 8 * j;
          if (k >= (int)gb_blocks[rb].size()) continue;
          memcpy(&q[((size_t)(j / 4) * 64 + l) * 4 + (j & 3)], (const int8_t *)gbw + 32 * (gb_first[rb] + k) + 4 * r, 4);
          if (r == 0) c[(j / 4) * 8 + ks] |= (uint32_t)(gb_blocks[rb][k] / 4) << (8 * (j & 3));
        }
      }
      sa.gb_qoff[rb] = (int)(put(q.data(), q.size() * 4) / 16);
      sa.gb_coff[rb] = (int)(put(c.data(), c.size() * 4) / 4);
    }
  }
  /* GRU_B input blocks: [rb][k][row] (u32 int8 row quads | float4 fp32 rows) */
  for (int rb = 0; rb < GB_ROWS / 8; rb++) {
    int nb = (int)gb_blocks[rb].size();
    sa.gb_nb[rb] = nb;
    if (reg) continue;
    if (int8) {
      std::vector<uint32_t> w(nb * 8);
      for (int k = 0; k < nb; k++)
        for (int r = 0; r < 8; r++) memcpy(&w[k * 8 + r], (const int8_t *)gbw + 32 * (gb_first[rb] + k) + 4 * r, 4);
      sa.gb_woff[rb] = (int)(put(w.data(), w.size() * 4) / 4);
    } else {
      std::vector<float> w(nb * 8 * 4);
      const float *src = (const float *)gbw;
      for (int k = 0; k < nb; k++)
        for (int r = 0; r < 8; r++)
          for (int c = 0; c < 4; c++) w[(k * 8 + r) * 4 + c] = src[32 * (gb_first[rb] + k) + c * 8 + r];
      sa.gb_woff[rb] = (int)(put(w.data(), w.size() * 4) / 4);
    }
    std::vector<uint16_t> cbs(nb);
    for (int k = 0; k < nb; k++) cbs[k] = (uint16_t)(gb_blocks[rb][k] / 4);
    sa.gb_coff[rb] = (int)(put(cbs.data(), cbs.size() * 2) / 2);
  }
  /* GRU_A blocks (LDS / fp32 global path): per (wave, gate) chunk [k][64 lanes] */
  for (int w = 0; w < SAMPLE_WAVES && !reg; w++)
    for (int g = 0; g < 3; g++) {
      int K = gaK[w][g];
      sa.ga_K[w][g] = K;
      std::vector<uint16_t> cbs(K * 8, int8 ? 0 : 0xFFFF);
      std::vector<uint32_t> wq(int8 ? K * 64 : 0, 0);
      size_t fbase = ga_wf.size();
      if (!int8) ga_wf.resize(fbase + (size_t)K * 64, make_float4(0, 0, 0, 0));
      for (int j = 0; j < 8; j++) {
        int rb = g * (NA / 8) + w * 8 + j;
        for (int k = 0; k < (int)ga_blocks[rb].size(); k++) {
          cbs[k * 8 + j] = (uint16_t)(ga_blocks[rb][k] / 4);
          for (int r = 0; r < 8; r++) {
            int blk = ga_first[rb] + k;
            if (int8) {
              memcpy(&wq[k * 64 + j * 8 + r], (const int8_t *)gaw->data + 32 * blk + 4 * r, 4);
            } else {
              const float *src = (const float *)gaw->data + 32 * blk;
              ga_wf[fbase + k * 64 + j * 8 + r] = make_float4(src[0 * 8 + r], src[1 * 8 + r], src[2 * 8 + r], src[3 * 8 + r]);
            }
          }
        }
      }
      if (int8) sa.ga_woff[w][g] = (int)(put(wq.data(), wq.size() * 4) / 4);
      else sa.ga_woff[w][g] = (int)fbase;
      sa.ga_coff[w][g] = (int)(put(cbs.data(), cbs.size() * 2) / 2);
    }
  align16();

  /* ---- matrix-core tables (non-saturating int8 models, mf_kernel) ---- */
  std::vector<uint32_t> mft, mfgb;
  bool mf_ok = int8 && !sat && !getenv("LPCNET_NO_MFMA");
  /* the matrix-core GRU_B is a dense tile: a row block listing one block
   * position twice (find_idx_check accepts it, and sparse_sgemv_accum8x4
   * adds both blocks) has no dense form -- the lockstep kernel runs such a
   * model, block by block as the reference does */
  for (int rb = 0; rb < GB_ROWS / 8 && mf_ok; rb++) {
    std::vector<int> pos = gb_blocks[rb];
    std::sort(pos.begin(), pos.end());
    if (std::adjacent_find(pos.begin(), pos.end()) != pos.end()) mf_ok = false;
  }
  MfPlan plan;
  if (mf_ok) {
    /* the plan's SIMD weights follow the kernel the batch will run (see
     * mf_plan): the wide kernel above one mf_kernel<4> round unless turned
     * off */
    const bool wide = mfw_planned(b, current_device_cus());
    b->plan_wide = wide;
    const int cls = b->B >= MF2_MIN_STREAMS ? 2 : b->B >= 1024 ? 1 : 0;
    /* a split plan's own tables serve mf_kernel / mf2_kernel (class cls);
     * the wide kernel's split form gets tables of its own below
     * (mfw_split_tables) */
    mf_ok = mf_plan(ga_blocks, plan, wide ? 3 : cls, cls);
  }
  if (getenv("LPCNET_VERBOSE")) {
    fprintf(stderr, "lpcnet: mf_kernel plan: %s", !mf_ok ? "not applicable" : plan.split ? "split" : "unsplit");
    if (mf_ok) {
      fprintf(stderr, " own caps z/r %d h %d, pieces z %zu r %zu h %zu; groups per wave (own zr, hosted zr, own h, hosted h):",
              plan.own[0], plan.own[2], plan.pieces[0].size(), plan.pieces[1].size(), plan.pieces[2].size());
      for (int w = 0; w < SAMPLE_WAVES; w++) fprintf(stderr, " (%d %d %d %d)", plan.nzr[w], plan.nfzr[w], plan.nh[w], plan.nfh[w]);
      for (int g = 0; g < 3; g++) {
        std::vector<int> per(NA / 8, 0);
        for (const MfPiece &pc : plan.pieces[g]) per[pc.unit]++;
        fprintf(stderr, "%s max pieces per row %d", g ? "," : ";", per.empty() ? 0 : *std::max_element(per.begin(), per.end()));
      }
    }
    fprintf(stderr, "\n");
  }
  std::vector<int> mf_units, mf_frow;
  MfwSplitTab mfw_tabs;
  if (mf_ok) {
    const int8_t *wa = (const int8_t *)gaw->data, *wb = (const int8_t *)gbw, *wr = (const int8_t *)gbrec;
    /* GRU_A: lane l of wave w = row l%8 of unit block perm[8w + l/8] of each
     * gate (units 8 perm[.] .. +7); D row of that lane = that unit.  Its
     * own region holds the first own[g] blocks of that row block; a split
     * model's hosted region [own, own + hosted) the piece of another
     * (long) row block, whose partial sums go to that row's owner */
    const std::vector<int> &perm = plan.perm;
    mft.assign((size_t)SAMPLE_WAVES * MF_LANE_U32 * 64, 0);
    mf_units.assign((size_t)SAMPLE_WAVES * 64, 0);
    mf_frow.assign((size_t)3 * SAMPLE_WAVES * 64, NA); /* NA: no hosted piece (a dummy row) */
    sa.mf_split = plan.split ? 1 : 0;
    for (int w = 0; w < SAMPLE_WAVES; w++) {
      auto word = [&](int k, int l) -> uint32_t & { return mft[((size_t)w * MF_LANE_U32 + k) * 64 + l]; };
      sa.mf_nzr[w] = plan.nzr[w];
      sa.mf_nh[w] = plan.nh[w];
      sa.mf_nfzr[w] = plan.nfzr[w];
      sa.mf_nfh[w] = plan.nfh[w];
      for (int l = 0; l < 64; l++) mf_units[w * 64 + l] = 8 * perm[w * 8 + (l >> 3)] + (l & 7);
      for (int g = 0; g < 3; g++) {
        const int base = g == 0 ? 0 : (g == 1 ? MF_ZMAX : 2 * MF_ZMAX);
        const int nown = 4 * (g < 2 ? plan.nzr[w] : plan.nh[w]), nfor = 4 * (g < 2 ? plan.nfzr[w] : plan.nfh[w]);
        for (int region = 0; region < 2; region++) {
          const int nslot = region ? nfor : nown, off = region ? nown : 0;
          if (!nslot) continue;
          for (int half = 0; half < 2; half++) {
            /* the 4 block rows read by one 32-lane LDS group: slot order
             * chosen so their x words fall in distinct banks (mf_bank_slots) */
            std::vector<int> lists[4];
            int rbk[4], t0k[4];
            for (int k = 0; k < 4; k++) {
              const int lg = w * 8 + 4 * half + k;
              rbk[k] = -1;
              t0k[k] = 0;
              int t1 = 0;
              if (!region) {
                rbk[k] = g * (NA / 8) + perm[lg];
                t1 = std::min((int)ga_blocks[rbk[k]].size(), plan.own[g]);
              } else if (plan.host[g][lg] >= 0) {
                const MfPiece &pc = plan.pieces[g][plan.host[g][lg]];
                rbk[k] = g * (NA / 8) + pc.unit;
                t0k[k] = pc.t0;
                t1 = pc.t1;
                for (int r = 0; r < 8; r++) mf_frow[((size_t)g * SAMPLE_WAVES + w) * 64 + 8 * (4 * half + k) + r] = 8 * pc.unit + r;
              }
              if (rbk[k] >= 0) lists[k].assign(ga_blocks[rbk[k]].begin() + t0k[k], ga_blocks[rbk[k]].begin() + t1);
            }
            const std::vector<int> *rows4[4] = {&lists[0], &lists[1], &lists[2], &lists[3]};
            int slot_of[4][MF_HMAX], cb_at[4][MF_HMAX];
            mf_bank_slots(rows4, nslot, slot_of, cb_at);
            for (int k = 0; k < 4; k++) {
              const int j = 4 * half + k;
              for (int r = 0; r < 8; r++) {
                const int l = 8 * j + r;
                for (int t = 0; t < (int)lists[k].size(); t++)
                  memcpy(&word(base + off + slot_of[k][t], l), wa + 32 * (ga_first[rbk[k]] + t0k[k] + t) + 4 * r, 4);
                for (int t = 0; t < nslot; t++)
                  word(MF_GA + (base + off + t) / 4, l) |= (uint32_t)cb_at[k][t] << (8 * ((base + off + t) & 3));
              }
            }
          }
        }
      }
    }
    /* bit 16 of a lane's entry of gate g: its own row (unit mf_units[lane])
     * has hosted pieces there, whose sums it merges after barrier X */
    for (int g = 0; g < 3; g++) {
      std::vector<char> has(NA / 8, 0);
      for (const MfPiece &pc : plan.pieces[g]) has[pc.unit] = 1;
      for (int t = 0; t < SAMPLE_WAVES * 64; t++)
        if (has[mf_units[t] / 8]) mf_frow[(size_t)g * SAMPLE_WAVES * 64 + t] |= 1 << 16;
    }
    /* the wide kernel's split form (wide batches of split models) */
    sa.mfw_split = 0;
    if (plan.split && b->plan_wide && !getenv("LPCNET_NO_MFW_SPLIT") &&
        mfw_split_tables(ga_blocks, ga_first, wa, mfw_tabs)) {
      sa.mfw_split = 1;
      for (int w = 0; w < MFW_TAB_WAVES; w++) {
        sa.mfw_nzr[w] = mfw_tabs.nzr[w];
        sa.mfw_nh[w] = mfw_tabs.nh[w];
      }
    }
    /* GRU_B: dense A tiles, lane l = row 16g + l%16, k = 64kt + 16(l/16) + byte */
    std::vector<int8_t> dense((size_t)GB_ROWS * NA, 0), drec((size_t)GB_ROWS * NB, 0);
    for (int rb = 0; rb < GB_ROWS / 8; rb++)
      for (int t = 0; t < (int)gb_blocks[rb].size(); t++)
        for (int r = 0; r < 8; r++)
          for (int c = 0; c < 4; c++)
            dense[(size_t)(rb * 8 + r) * NA + gb_blocks[rb][t] + c] = wb[32 * (gb_first[rb] + t) + 4 * r + c];
    for (int rb = 0; rb < GB_ROWS / 8; rb++)
      for (int cb = 0; cb < NB / 4; cb++)
        for (int r = 0; r < 8; r++)
          for (int c = 0; c < 4; c++) drec[(rb * 8 + r) * NB + 4 * cb + c] = wr[32 * (rb * (NB / 4) + cb) + 4 * r + c];
    mfgb.assign((size_t)MF_GB_TILES * 64 * 4, 0);
    for (int g = 0; g < 3; g++)
      for (int l = 0; l < 64; l++) {
        const int row = 16 * g + (l & 15), k0 = 16 * (l >> 4);
        for (int kt = 0; kt < 6; kt++)
          memcpy((int8_t *)&mfgb[((size_t)(g * 6 + kt) * 64 + l) * 4], &dense[(size_t)row * NA + 64 * kt + k0], 16);
        if (k0 == 0) memcpy((int8_t *)&mfgb[((size_t)(18 + g) * 64 + l) * 4], &drec[row * NB], 16);
      }
  }

  /* ---- fp32 latency-kernel tables (fp_kernel, see FP_ZF) ---- */
  std::vector<float4> fpzr, fph, fpgb;
  std::vector<uint32_t> fpoff;
  int fp_nzr[SAMPLE_WAVES] = {}, fp_nh[SAMPLE_WAVES] = {};
  bool fp_ok = !int8 && !getenv("LPCNET_NO_FPK");
  for (int rb = 0; rb < GB_ROWS / 8 && fp_ok; rb++) {
    /* dense GRU_B only: blocks 0, 4, ..., NA-4 in order */
    if ((int)gb_blocks[rb].size() != NA / 4) fp_ok = false;
    for (int k = 0; k < (int)gb_blocks[rb].size() && fp_ok; k++)
      if (gb_blocks[rb][k] != 4 * k) fp_ok = false;
  }
  /* block rows longer than the register tables (trained masks, see
   * mf_plan): the long form streams every slot of the z/r and h chains */
  bool fp_long = false;
  for (int w = 0; w < SAMPLE_WAVES && fp_ok; w++)
    for (int j = 0; j < 8; j++) {
      if ((int)ga_blocks[w * 8 + j].size() > FP_ZF || (int)ga_blocks[NA / 8 + w * 8 + j].size() > FP_ZF ||
          (int)ga_blocks[2 * (NA / 8) + w * 8 + j].size() > FP_HF)
        fp_long = true;
    }
  if (getenv("LPCNET_FP_FORCE_LONG")) fp_long = true; /* tests: the long form on any model */
  std::vector<float4> fplzr, fplh;
  std::vector<uint32_t> fploff;
  if (fp_ok && fp_long) {
    const float *wa = (const float *)gaw->data;
    const float nz = -0.f;
    int KZ = 1, KH = 1;
    for (int rb = 0; rb < NA / 8; rb++) {
      KZ = std::max(KZ, (int)std::max(ga_blocks[rb].size(), ga_blocks[NA / 8 + rb].size()));
      KH = std::max(KH, (int)ga_blocks[2 * (NA / 8) + rb].size());
    }
    /* [wave][slot][64 lanes]: z/r weights as the packed pairs (2 float4), h
     * weights (float4); offsets: z quad | r quad << 8, then h quad */
    fplzr.assign((size_t)SAMPLE_WAVES * KZ * 64 * 2, make_float4(nz, nz, nz, nz));
    fplh.assign((size_t)SAMPLE_WAVES * KH * 64, make_float4(nz, nz, nz, nz));
    fploff.assign((size_t)SAMPLE_WAVES * (KZ + KH) * 64, (uint32_t)(NA / 4) * 0x0101u); /* the +0 quad */
    for (int w = 0; w < SAMPLE_WAVES; w++) {
      int kz = 0, kh = 0;
      for (int j = 0; j < 8; j++) {
        kz = std::max(kz, (int)std::max(ga_blocks[w * 8 + j].size(), ga_blocks[NA / 8 + w * 8 + j].size()));
        kh = std::max(kh, (int)ga_blocks[2 * (NA / 8) + w * 8 + j].size());
      }
      sa.fp_nzr[w] = kz;
      sa.fp_nh[w] = kh;
      for (int l = 0; l < 64; l++) {
        const int j = l >> 3, r = l & 7;
        for (int g = 0; g < 3; g++) {
          const int rb = g * (NA / 8) + w * 8 + j;
          for (int t = 0; t < (int)ga_blocks[rb].size(); t++) {
            const float *src = wa + 32 * (size_t)(ga_first[rb] + t);
            const float4 v = make_float4(src[0 * 8 + r], src[1 * 8 + r], src[2 * 8 + r], src[3 * 8 + r]);
            const uint32_t q = (uint32_t)(ga_blocks[rb][t] / 4);
            if (g < 2) {
              float4 &lo = fplzr[(((size_t)w * KZ + t) * 64 + l) * 2], &hi = fplzr[(((size_t)w * KZ + t) * 64 + l) * 2 + 1];
              (g == 0 ? lo.x : lo.y) = v.x;
              (g == 0 ? lo.z : lo.w) = v.y;
              (g == 0 ? hi.x : hi.y) = v.z;
              (g == 0 ? hi.z : hi.w) = v.w;
              uint32_t &o = fploff[((size_t)w * KZ + t) * 64 + l];
              o = (o & ~(0xFFu << (8 * g))) | (q << (8 * g));
            } else {
              fplh[((size_t)w * KH + t) * 64 + l] = v;
              fploff[(size_t)SAMPLE_WAVES * KZ * 64 + ((size_t)w * KH + t) * 64 + l] = q;
            }
          }
        }
      }
    }
    sa.fpl_kz = KZ;
    sa.fpl_kh = KH;
  }
  if (fp_ok && !fp_long) {
    const float *wa = (const float *)gaw->data;
    const float nz = -0.f;
    fpzr.assign((size_t)SAMPLE_WAVES * 2 * FP_ZF * 64, make_float4(nz, nz, nz, nz));
    fph.assign((size_t)SAMPLE_WAVES * FP_HF * 64, make_float4(nz, nz, nz, nz));
    fpoff.assign((size_t)SAMPLE_WAVES * FP_OFF_WORDS * 64, 0x60606060u); /* column quad NA/4 = 96: the +0 quad */
    for (int w = 0; w < SAMPLE_WAVES; w++) {
      int kz = 0, kh = 0;
      for (int j = 0; j < 8; j++) {
        kz = std::max(kz, (int)std::max(ga_blocks[w * 8 + j].size(), ga_blocks[NA / 8 + w * 8 + j].size()));
        kh = std::max(kh, (int)ga_blocks[2 * (NA / 8) + w * 8 + j].size());
      }
      fp_nzr[w] = kz;
      fp_nh[w] = kh;
      for (int l = 0; l < 64; l++) {
        const int j = l >> 3, r = l & 7;
        for (int g = 0; g < 3; g++) {
          const int rb = g * (NA / 8) + w * 8 + j;
          for (int t = 0; t < (int)ga_blocks[rb].size(); t++) {
            const float *src = wa + 32 * (size_t)(ga_first[rb] + t);
            const float4 v = make_float4(src[0 * 8 + r], src[1 * 8 + r], src[2 * 8 + r], src[3 * 8 + r]);
            if (g < 2) {
              /* packed (z, r) pairs: slot t = [z.x r.x z.y r.y] [z.z r.z z.w r.w] */
              float4 &lo = fpzr[((size_t)w * 2 * FP_ZF + t) * 64 + l], &hi = fpzr[((size_t)w * 2 * FP_ZF + FP_ZF + t) * 64 + l];
              (g == 0 ? lo.x : lo.y) = v.x;
              (g == 0 ? lo.z : lo.w) = v.y;
              (g == 0 ? hi.x : hi.y) = v.z;
              (g == 0 ? hi.z : hi.w) = v.w;
            } else {
              fph[((size_t)w * FP_HF + t) * 64 + l] = v;
            }
            const int slot = g * FP_ZF + t, word = slot / 4, sh = 8 * (slot & 3);
            uint32_t &o = fpoff[((size_t)w * FP_OFF_WORDS + word) * 64 + l];
            o = (o & ~(0xFFu << sh)) | ((uint32_t)(ga_blocks[rb][t] / 4) << sh);
          }
        }
      }
    }
    for (int w = 0; w < SAMPLE_WAVES; w++) {
      sa.fp_nzr[w] = fp_nzr[w];
      sa.fp_nh[w] = fp_nh[w];
    }
  }
  if (fp_ok) {
    /* dense GRU_B input weights, column quad major (both forms) */
    const float *wb = (const float *)gbw;
    fpgb.resize((size_t)(NA / 4) * GB_ROWS);
    for (int rb = 0; rb < GB_ROWS / 8; rb++)
      for (int k = 0; k < NA / 4; k++)
        for (int r = 0; r < 8; r++) {
          const float *src = wb + 32 * (size_t)(gb_first[rb] + k);
          fpgb[(size_t)k * GB_ROWS + rb * 8 + r] = make_float4(src[0 * 8 + r], src[1 * 8 + r], src[2 * 8 + r], src[3 * 8 + r]);
        }
  }
  sa.fp_long = fp_ok && fp_long ? 1 : 0;

  /* choose streams per workgroup and check the LDS budget of the lockstep
   * kernel: the whole image in LDS, or -- models with long block rows -- only
   * its fixed tables, the weight sections read from global memory */
  int S = b->B >= 1024 ? 4 : (b->B >= 512 ? 2 : 1);
  int image_lds = (int)img.size();
  int lds = sample_lds_bytes(S, variant, image_lds);
  while (lds > 160 * 1024 && S > 1) {
    S /= 2;
    lds = sample_lds_bytes(S, variant, image_lds);
  }
  if (lds > 160 * 1024) {
    image_lds = IMG_VAR;
    S = b->B >= 1024 ? 4 : (b->B >= 512 ? 2 : 1);
    lds = sample_lds_bytes(S, variant, image_lds);
    while (lds > 160 * 1024 && S > 1) {
      S /= 2;
      lds = sample_lds_bytes(S, variant, image_lds);
    }
  }
  if (lds > 160 * 1024) {
    set_err("model does not fit the 160 KiB LDS budget");
    return -1;
  }
  if (!upload) return 0;

  if (b->set_device()) { set_err("hipSetDevice failed"); return -1; }
  free_model(b);
  FrameArgs fa;
  memset(&fa, 0, sizeof(fa));
#define UP(dst, src, n) if (!(dst = dev_upload<std::remove_const<std::remove_pointer<decltype(dst)>::type>::type>(b, src, n))) { set_err("device upload failed"); free_model(b); return -1; }
  /* frame-network weights keep the blob's [in][out] layout, padded with
   * FRAME_PREFETCH zero input rows: frame_kernel reads that far ahead */
  auto padded = [](const float *w, int nin, int nout) {
    std::vector<float> v((size_t)(nin + FRAME_PREFETCH) * nout, 0.f);
    memcpy(v.data(), w, (size_t)nin * nout * 4);
    return v;
  };
  std::vector<float> c1p = padded(conv1_w, 3 * FIN, COND), c2p = padded(conv2_w, 3 * COND, COND);
  std::vector<float> d1p = padded(dense1_w, COND, COND), d2p = padded(dense2_w, COND, COND);
  UP(fa.conv1_w, c1p.data(), c1p.size() * 4);
  UP(fa.conv1_b, conv1_b, COND * 4);
  UP(fa.conv2_w, c2p.data(), c2p.size() * 4);
  UP(fa.conv2_b, conv2_b, COND * 4);
  UP(fa.dense1_w, d1p.data(), d1p.size() * 4);
  UP(fa.dense1_b, dense1_b, COND * 4);
  UP(fa.dense2_w, d2p.data(), d2p.size() * 4);
  UP(fa.dense2_b, dense2_b, COND * 4);
  UP(fa.gadf_w, gadf_w, COND * GA_ROWS * 4);
  UP(fa.gadf_b, gadf_b, GA_ROWS * 4);
  UP(fa.gbdf_w, gbdf_w, COND * GB_ROWS * 4);
  UP(fa.gbdf_b, gbdf_b, GB_ROWS * 4);
  {
    /* the two conditioning projections as one [COND][GA_ROWS + GB_ROWS] matrix */
    std::vector<float> pw((size_t)(COND + FRAME_PREFETCH) * (GA_ROWS + GB_ROWS), 0.f), pb(GA_ROWS + GB_ROWS);
    for (int j = 0; j < COND; j++) {
      memcpy(&pw[(size_t)j * (GA_ROWS + GB_ROWS)], gadf_w + (size_t)j * GA_ROWS, GA_ROWS * 4);
      memcpy(&pw[(size_t)j * (GA_ROWS + GB_ROWS) + GA_ROWS], gbdf_w + (size_t)j * GB_ROWS, GB_ROWS * 4);
    }
    memcpy(pb.data(), gadf_b, GA_ROWS * 4);
    memcpy(pb.data() + GA_ROWS, gbdf_b, GB_ROWS * 4);
    UP(fa.proj_w, pw.data(), pw.size() * 4);
    UP(fa.proj_b, pb.data(), pb.size() * 4);
  }
  {
    /* chunk_kernel's copies: each row tile's k steps as per-lane float4 quads
     * (one 1 KiB wave-instruction per 4 k steps instead of 256 B per step:
     * the kernel streams the weights from the Infinity Cache with 4x the
     * bytes in flight per CU) */
    auto tiled = [](const float *w, int nin, int nout) {
      const int ks = nin / 4, nq = (ks + 3) / 4, nrt = nout / 16;
      std::vector<float> t((size_t)nrt * (nq + CK_WPAD) * 64 * 4, 0.f);
      for (int rt = 0; rt < nrt; rt++)
        for (int q = 0; q < nq; q++)
          for (int l = 0; l < 64; l++)
            for (int j = 0; j < 4; j++) {
              const int k = 4 * (4 * q + j) + (l >> 4), row = 16 * rt + (l & 15);
              if (k < nin) t[(((size_t)rt * (nq + CK_WPAD) + q) * 64 + l) * 4 + j] = w[(size_t)k * nout + row];
            }
      return t;
    };
    std::vector<float> pwf((size_t)COND * (GA_ROWS + GB_ROWS));
    for (int j = 0; j < COND; j++) {
      memcpy(&pwf[(size_t)j * (GA_ROWS + GB_ROWS)], gadf_w + (size_t)j * GA_ROWS, GA_ROWS * 4);
      memcpy(&pwf[(size_t)j * (GA_ROWS + GB_ROWS) + GA_ROWS], gbdf_w + (size_t)j * GB_ROWS, GB_ROWS * 4);
    }
    std::vector<float> t1 = tiled(conv1_w, 3 * FIN, COND), t2 = tiled(conv2_w, 3 * COND, COND);
    std::vector<float> t3 = tiled(dense1_w, COND, COND), t4 = tiled(dense2_w, COND, COND);
    std::vector<float> t5 = tiled(pwf.data(), COND, GA_ROWS + GB_ROWS);
    /* conv1 .. dense2 once per projection slice of the one-frame kernel
     * (CK_SLICES_MAX copies): the slices of all 16-stream groups of an XCD
     * stream these rows in near lockstep, and one copy per slice spreads
     * their same-line L2 reads over four times the lines */
    auto rep = [](const std::vector<float> &t) {
      std::vector<float> r;
      r.reserve(t.size() * CK_SLICES_MAX);
      for (int k = 0; k < CK_SLICES_MAX; k++) r.insert(r.end(), t.begin(), t.end());
      return r;
    };
    const std::vector<float> r1 = rep(t1), r2 = rep(t2), r3 = rep(t3), r4 = rep(t4);
    UP(fa.ck_conv1, r1.data(), r1.size() * 4);
    UP(fa.ck_conv2, r2.data(), r2.size() * 4);
    UP(fa.ck_dense1, r3.data(), r3.size() * 4);
    UP(fa.ck_dense2, r4.data(), r4.size() * 4);
    fa.ck_rep[0] = (int)(t1.size() / 4);
    fa.ck_rep[1] = (int)(t2.size() / 4);
    fa.ck_rep[2] = (int)(t3.size() / 4);
    fa.ck_rep[3] = (int)(t4.size() / 4);
    UP(fa.ck_proj, t5.data(), t5.size() * 4);
    const float4 *wm[5] = {fa.ck_conv1, fa.ck_conv2, fa.ck_dense1, fa.ck_dense2, fa.ck_proj};
    const size_t wn[5] = {t1.size(), t2.size(), t3.size(), t4.size(), t5.size()};
    for (int t = 0; t < 5; t++) {
      b->ck_warm.m[t] = (const uint32_t *)wm[t];
      b->ck_warm.lines[t] = (int)(wn[t] * 4 / 128);
    }
  }
  UP(fa.embed_pitch, embed_pitch, 256 * EP * 4);
  UP(fa.rcp, rcp_dev.data(), RCP_ENTRIES * 4);
  UP(sa.emb_sig, emb_sig, 256 * GA_ROWS * 4);
  UP(sa.emb_pred, emb_pred, 256 * GA_ROWS * 4);
  UP(sa.emb_exc, emb_exc, 256 * GA_ROWS * 4);
  UP(sa.ga_par, ga_par.data(), ga_par.size() * 4);
  UP(sa.ga_wsum, ga_wsum.data(), ga_wsum.size() * 4);
  UP(sa.gb_par, gb_par.data(), gb_par.size() * 4);
  UP(sa.gb_wsum, gb_wsum.data(), gb_wsum.size() * 4);
  UP(sa.image, img.data(), img.size());
  if (mf_ok) {
    UP(sa.mf, mft.data(), mft.size() * 4);
    UP(sa.mf_unit, mf_units.data(), mf_units.size() * 4);
    UP(sa.mf_frow, mf_frow.data(), mf_frow.size() * 4);
    if (sa.mfw_split) {
      UP(sa.mfw_tab, mfw_tabs.tab.data(), mfw_tabs.tab.size() * 4);
      UP(sa.mfw_frow, mfw_tabs.frow.data(), mfw_tabs.frow.size() * 4);
      UP(sa.mfw_unit, mfw_tabs.units.data(), mfw_tabs.units.size() * 4);
    }
    {
      /* Range of the GRU_A gates' inputs for the elementwise fast path:
       * z/r: cvt_rne((bias + diag st + ((cond + Esig) + Epred) + Eexc) * 16256)
       * cannot leave int32 (x86: INT_MIN) while |that sum| < 2^31 / 16256, with
       * |st| <= 2 (restore-enforced); h: tanh's Pade denominator cannot overflow
       * nor go NaN while its input is finite and < 2^60.  The kernel checks a
       * workgroup's conditioning against these bounds once per launch. */
      double bz = 0, bh = 0, ez = 0, eh = 0;
      bool finite = true;
      for (int i = 0; i < NA; i++)
        for (int g = 0; g < 3; g++) {
          const double b = fabs((double)ga_par[g * NA + i]) + 2.0 * fabs((double)ga_par[(3 + g) * NA + i]);
          finite &= std::isfinite(b);
          (g < 2 ? bz : bh) = std::max(g < 2 ? bz : bh, b);
        }
      const float *tabs[3] = {emb_sig, emb_pred, emb_exc};
      for (int g = 0; g < 3; g++) {
        double e = 0;
        for (int t = 0; t < 3; t++) {
          double m = 0;
          for (int row = 0; row < 256; row++)
            for (int i = 0; i < NA; i++) {
              const float v = tabs[t][(size_t)row * GA_ROWS + g * NA + i];
              finite &= std::isfinite(v);
              m = std::max(m, (double)fabsf(v));
            }
          e += m;
        }
        (g < 2 ? ez : eh) = std::max(g < 2 ? ez : eh, e);
      }
      const double zr = 0.99 * (2147483648.0 / 16256.0) - bz - ez, hb = 1e17 - bh - eh;
      sa.mf_zr_bound = finite && zr > 0 ? (float)zr : -1.f;
      sa.mf_h_bound = finite && hb > 0 ? (float)hb : -1.f;
      /* test hooks: force the exact path everywhere, or lower the z/r bound
       * so that some workgroups take each path */
      if (getenv("LPCNET_MF_EXACT")) sa.mf_zr_bound = sa.mf_h_bound = -1.f;
      if (const char *v = getenv("LPCNET_MF_ZR_BOUND")) sa.mf_zr_bound = std::min(sa.mf_zr_bound, (float)atof(v));
      if (getenv("LPCNET_VERBOSE"))
        fprintf(stderr, "lpcnet: GRU_A range bounds: z/r %g (bias+diag %g, embeddings %g), h %g\n", sa.mf_zr_bound, bz, ez,
                sa.mf_h_bound);
    }
    {
      /* embedding tables with their columns in lane order (coalesced gathers) */
      std::vector<float> pt((size_t)256 * GA_ROWS);
      const float *src[3] = {emb_sig, emb_pred, emb_exc};
      for (int t = 0; t < 3; t++) {
        for (int row = 0; row < 256; row++)
          for (int g = 0; g < 3; g++)
            for (int p = 0; p < NA; p++) pt[(size_t)row * GA_ROWS + g * NA + p] = src[t][(size_t)row * GA_ROWS + g * NA + mf_units[p]];
        const float *d = nullptr;
        UP(d, pt.data(), pt.size() * 4);
        sa.mf_emb[t] = d;
        if (sa.mfw_split) {
          /* the same in the wide split form's lane order */
          for (int row = 0; row < 256; row++)
            for (int g = 0; g < 3; g++)
              for (int p = 0; p < NA; p++)
                pt[(size_t)row * GA_ROWS + g * NA + p] = src[t][(size_t)row * GA_ROWS + g * NA + mfw_tabs.units[p]];
          const float *dw = nullptr;
          UP(dw, pt.data(), pt.size() * 4);
          sa.mfw_emb[t] = dw;
        }
      }
    }
    UP(sa.mf_gb, mfgb.data(), mfgb.size() * 4);
  }
  if (fp_ok && !fp_long) {
    UP(sa.fp_zr, fpzr.data(), fpzr.size() * sizeof(float4));
    UP(sa.fp_h, fph.data(), fph.size() * sizeof(float4));
    UP(sa.fp_off, fpoff.data(), fpoff.size() * 4);
  }
  if (fp_ok && fp_long) {
    UP(sa.fpl_zr, fplzr.data(), fplzr.size() * sizeof(float4));
    UP(sa.fpl_h, fplh.data(), fplh.size() * sizeof(float4));
    UP(sa.fpl_off, fploff.data(), fploff.size() * 4);
  }
  if (fp_ok) UP(sa.fp_gb, fpgb.data(), fpgb.size() * sizeof(float4));
  if (!int8) {
    UP(sa.ga_wf, ga_wf.data(), ga_wf.size() * sizeof(float4));
    UP(sa.gb_recf, gbrec, 3 * NB * NB * 4);
  }
  DecodeArgs da{};
  if (cb_ok) {
    /* lpcnet_dec.c:118: float p = pow(2.f, main_pitch/21.)*PITCH_MIN_PERIOD, per 6-bit main_pitch */
    std::vector<float> pt(64);
    for (int m = 0; m < 64; m++) pt[m] = (float)(pow(2.0, m / 21.) * 32);
    UP(da.cb1, cb[0]->data, cb[0]->size);
    UP(da.cb2, cb[1]->data, cb[1]->size);
    UP(da.cb3, cb[2]->data, cb[2]->size);
    UP(da.cbd, cb[3]->data, cb[3]->size);
    UP(da.pitch, pt.data(), pt.size() * 4);
  }
#undef UP
  b->da = da;
  b->has_codebooks = cb_ok;
  sa.image_bytes = (int)img.size();
  sa.image_lds_bytes = image_lds;
  b->sa = sa;
  b->fa = fa;
  b->mc = mc;
  {
    std::vector<uint32_t> dflt(RCP_ENTRIES);
    for (int i = 0; i < RCP_ENTRIES; i++) dflt[i] = kRcpTable[i >> (RCP_TABLE_BITS - 11)] + kRcpBias;
    b->rcp_custom = rcp_dev != dflt;
    b->rcp_dev = rcp_dev;
  }
  b->variant = variant;
  b->sat = sat;
  b->reg = reg;
  b->mf_ok = mf_ok;
  b->fp_ok = fp_ok;
  b->image_bytes = (int)img.size();
  b->S = S;
  b->lds_bytes = lds;
  b->have_model = true;

  /* algorithmic work, recomputed from the loaded index */
  LPCNetModelInfo &in = b->info;
  in.variant = variant;
  in.gru_a_blocks = nba;
  in.gru_b_blocks = nbb;
  in.may_saturate = sat ? 1 : 0;
  in.quad_path = reg ? 1 : 0;
  double frame_w = (3.0 * FIN * COND + 3.0 * COND * COND + 2.0 * COND * COND + COND * GA_ROWS + COND * GB_ROWS) * 4 +
                   (2.0 * COND + 2 * COND + GA_ROWS + GB_ROWS) * 4 + EP * 4;
  double wbytes = int8 ? 1 : 4;
  in.bytes_shared_per_frame = frame_w;
  in.bytes_shared_per_sample = 32.0 * nba * wbytes + 4.0 * (nba + GA_ROWS / 8) /* idx */ + 6.0 * NA * 4 /* bias+diag */ +
                               32.0 * nbb * wbytes + 4.0 * (nbb + GB_ROWS / 8) + 3.0 * NB * NB * wbytes + 2.0 * GB_ROWS * 4;
  /* 3 gathered embedding rows, the 8 dual_fc nodes on the path (2
   * channels x (16 weights + bias + factor)), and the frame's conditioning +
   * features per sample, the output sample */
  in.bytes_per_stream_sample = 3.0 * GA_ROWS * 4 + 8 * 2 * (NB + 2) * 4 + (GA_ROWS + GB_ROWS + NF) * 4.0 / FRAME + 2;
  /* mf_kernel matrix-core work: per GRU_A wave 8 nzr + 4 nh 4x4x4 MFMAs of
   * 16 x 4x4x4 MACs; per sampler wave 21 16x16x64 MFMAs (2 sampler waves).
   */
  b->mf_ga_ops = b->mf_gb_ops = 0;
  if (mf_ok) {
    double n4 = 0;
    for (int w = 0; w < SAMPLE_WAVES; w++) n4 += 8.0 * (sa.mf_nzr[w] + sa.mf_nfzr[w]) + 4.0 * (sa.mf_nh[w] + sa.mf_nfh[w]);
    b->mf_ga_ops = 2.0 * n4 * 1024.0;
    b->mf_gb_ops = 2.0 * 2.0 * MF_GB_TILES * 16384.0;
  }
  in.long_rows = (mf_ok && sa.mf_split) || (fp_ok && sa.fp_long) ? 1 : 0;
  in.has_codebooks = cb_ok ? 1 : 0;
  in.lpc_gamma = mc.lpc_gamma;
  in.features_delay = mc.delay;
  in.end2end = mc.end2end;
  in.ops_per_sample = 2.0 * (32.0 * nba + 32.0 * nbb + 3 * NB * NB + 8 * 2 * NB + NLPC) +
                      2.0 * (3.0 * FIN * COND + 3.0 * COND * COND + 2.0 * COND * COND + COND * GA_ROWS + COND * GB_ROWS) / FRAME;
  choose_kernel(b); /* also sets mfma_ops_per_group_sample for the chosen kernel */
  return 0;
}

void host_reset_state(StreamState &s)
{
  memset(&s, 0, sizeof(s));
  s.last_exc = host_lin2ulaw(0.f);
  Kiss k;
  k.srand((const unsigned char *)"LPCNet", 6);
  s.rng[0] = k.z; s.rng[1] = k.w; s.rng[2] = k.jsr; s.rng[3] = k.jcong;
}

int ensure_trace(LPCNetBatch *b, int N)
{
  if (!b->trace) {
    b->sa.trace_logits = nullptr;
    b->sa.trace_exc = nullptr;
    return 0;
  }
  if (!b->d_trace_logits) {
    HIPCHK(hipMalloc(&b->d_trace_logits, (size_t)b->B * FRAME * 8 * 4));
    HIPCHK(hipMalloc(&b->d_trace_exc, (size_t)b->B * FRAME * 4));
  }
  b->sa.trace_logits = b->d_trace_logits;
  b->sa.trace_exc = b->d_trace_exc;
  b->trace_N = N;
  return 0;
}

/* ovl >= 0: overlapped form, frame f = ovl.  The frame kernel runs on
 * fstream, followed by a copy of its outputs into d_cond[f & 1] (which
 * sample kernel f-2 read: ev_samp); the sample kernel on stream waits only
 * for that copy (ev_frame) and reads the frame's outputs there, so frame
 * kernel f+1 runs beside sample kernel f.  The sample kernels read nothing
 * else the frame kernel writes.  Every fstream launch precedes a stream
 * launch that waits for it, so a sync of stream covers both. */
/* d_lpc_frame: this frame's lpc_from_cepstrum output ([B][NLPC]); with
 * run_lpc the LPC kernel computing it is launched first, otherwise it was
 * computed earlier on the same queue (lpcnet_batch_synthesize_frames
 * batches it over many frames). */
int launch_frame_step(LPCNetBatch *b, const float *d_features, float *d_lpc_frame, bool run_lpc, short *d_pcm, int N,
                      int preload = 0, int ovl = -1, int nB = -1, bool run_frame = true, bool keep_cond = false)
{
  /* run_frame false: the sample network only, on the conditioning already in
   * the stream states (lpcnet_synthesize_tail_impl, lpcnet.c:235-271);
   * keep_cond: the frame network of run_frame_network_flush (lpcnet.c:134-144) */
  /* nB: run the first nB streams of the batch only (the drop-in pool's work
   * batch); the overlapped form always runs all of them */
  if (nB < 0 || ovl >= 0) nB = b->B;
  const int c = ovl & 1;
  hipStream_t fs = ovl >= 0 ? b->fstream : b->stream;
  FrameArgs fa = b->fa;
  fa.st = b->d_state;
  fa.mc = b->mc;
  fa.nstreams = nB;
  fa.features = d_features;
  fa.lpc_new = d_lpc_frame;
  fa.keep_cond = keep_cond ? 1 : 0;
  SampleArgs sa = b->sa;
  sa.st = b->d_state;
  sa.delay = b->mc.delay;
  sa.nstreams = nB;
  sa.N = N;
  sa.pcm = d_pcm;
  sa.preload = std::max(0, std::min(preload, N));
  sa.stamps = b->d_stamps;
  sa.status = b->d_status;
  sa.spin_limit = b->spin_limit;
  fa.stamps = b->d_stamps ? b->d_stamps + (size_t)b->B * STAMP_WAVES * 16 : nullptr;
  if (ovl >= 0) {
    sa.cond = b->d_cond[c];
  }
  /* timing 1: events around the sample kernel only; 2: the frame kernel too
   * (one event between the two kernels serves both pairs) */
  hipEvent_t e[3] = {nullptr, nullptr, nullptr};
  if (b->timing >= 2) e[0] = get_event(b);
  if (b->timing >= 1) {
    e[1] = get_event(b);
    e[2] = get_event(b);
  }
  if (ovl >= 0 && b->ev_samp_used[c]) HIPCHK(hipStreamWaitEvent(fs, b->ev_samp_cur[c], 0));
  hipEvent_t ef = nullptr; /* end of the frame kernel, overlapped form with frame timing */
  if (e[0]) HIPCHK(hipEventRecord(e[0], fs));
  /* lpc_from_cepstrum of this frame's features: the frame kernel pushes it
   * into the two-frame LPC ring (lpcnet.c:110-112) */
  if (run_frame && run_lpc && !b->mc.end2end && launch_lpc(d_features, d_lpc_frame, nB, b->d_lpc_tab, fs)) {
    set_err("lpc kernel launch failed");
    return -1;
  }
  if (run_frame && launch_frame(fa, fs)) { set_err("frame kernel launch failed"); return -1; }
  if (ovl >= 0 && launch_cond_copy(b->d_state, b->d_cond[c], b->B, fs)) {
    set_err("copy launch failed");
    return -1;
  }
  if (ovl >= 0) {
    if (e[0]) {
      ef = get_event(b);
      HIPCHK(hipEventRecord(ef, fs));
    }
    /* an event, not a device flag: a sample kernel polling a flag set by
     * the other queue was faster by ~1 % but gave wrong output wherever the
     * two queues do not run concurrently (rocprofv3 --pmc serialises
     * dispatches: the poll timed out and read a stale slot) */
    HIPCHK(hipEventRecord(b->ev_frame[c], fs));
    HIPCHK(hipStreamWaitEvent(b->stream, b->ev_frame[c], 0));
  }
  if (e[1]) HIPCHK(hipEventRecord(e[1], b->stream));
  const int lrc = N <= 0 ? 0
                : b->fp    ? launch_fp(sa, b->stream)
                : wide_for(b, sa.nstreams) && !sa.preload && !sa.trace_logits && !sa.stamps ? launch_mfw(sa, b->mfw_g, b->stream)
                : mf2_for(b, sa.nstreams) && !sa.preload && !sa.trace_logits && !sa.stamps ? launch_mf2(sa, 4, b->stream)
                : b->mf    ? launch_mf(sa, b->S, mf_lds_bytes(b->S, b->sa.mf_split), b->stream)
                             : launch_sample(sa, b->S, b->variant, b->sat ? 1 : 0, b->reg ? 1 : 0, b->lds_bytes, b->stream);
  if (lrc) {
    set_err(std::string("sample kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
    return -1;
  }
  if (e[2]) HIPCHK(hipEventRecord(e[2], b->stream));
  if (ovl >= 0) {
    /* every event record is a queue packet (~5 us between two kernels at
     * batch 1): the timing event after the sample kernel serves as ev_samp */
    if (e[2]) {
      b->ev_samp_cur[c] = e[2]; /* recycled only by reset_timers, which clears the use */
    } else {
      HIPCHK(hipEventRecord(b->ev_samp[c], b->stream));
      b->ev_samp_cur[c] = b->ev_samp[c];
    }
    b->ev_samp_used[c] = true;
  }
  if (e[0]) {
    b->ev_pairs[1].push_back(e[0]);
    b->ev_pairs[1].push_back(ef ? ef : e[1]);
    b->ev_frames[1].push_back(1);
  }
  if (ef) b->ev_taken.push_back(ef);
  if (e[1]) {
    b->ev_pairs[0].push_back(e[1]);
    b->ev_pairs[0].push_back(e[2]);
    b->ev_frames[0].push_back(1);
  }
  if (run_frame) b->frames_done(1);
  for (hipEvent_t x : e)
    if (x) b->ev_taken.push_back(x);
  return 0;
}

/* Chunked form: the frame network of frames [0, n) of d_features has run
 * (chunk_kernel, outputs in d_chunk[f]); launch the sample kernel of frames
 * f .. f + nfr - 1 on b->stream, reading their conditioning from d_chunk[f..]
 * and writing d_pcm [nfr][B][N].  nfr > 1: matrix-core kernel only, every
 * stream past its first `delay` frames (SampleArgs::nframes). */
int launch_chunk_samples(LPCNetBatch *b, int f, short *d_pcm, int N, int nfr = 1)
{
  SampleArgs sa = b->sa;
  sa.st = b->d_state;
  sa.delay = b->mc.delay;
  sa.cond = b->d_chunk + (size_t)f * b->B;
  sa.nstreams = b->B;
  sa.N = N;
  sa.nframes = nfr;
  sa.pcm = d_pcm;
  sa.preload = 0;
  sa.stamps = b->d_stamps;
  sa.status = b->d_status;
  sa.spin_limit = b->spin_limit;
  hipEvent_t e1 = nullptr, e2 = nullptr;
  if (b->timing >= 1) {
    e1 = get_event(b);
    e2 = get_event(b);
    HIPCHK(hipEventRecord(e1, b->stream));
  }
  const int lrc = N <= 0                                  ? 0
                  : b->fp                                 ? launch_fp(sa, b->stream)
                  : wide_for(b, sa.nstreams) && !sa.trace_logits && !sa.stamps ? launch_mfw(sa, b->mfw_g, b->stream)
                  : mf2_for(b, sa.nstreams) && !sa.trace_logits && !sa.stamps ? launch_mf2(sa, 4, b->stream)
                                                          : launch_mf(sa, b->S, mf_lds_bytes(b->S, b->sa.mf_split), b->stream);
  if (lrc) {
    set_err(std::string("sample kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
    return -1;
  }
  if (e1) {
    HIPCHK(hipEventRecord(e2, b->stream));
    b->ev_pairs[0].push_back(e1);
    b->ev_pairs[0].push_back(e2);
    b->ev_frames[0].push_back(nfr);
    b->ev_taken.push_back(e1);
    b->ev_taken.push_back(e2);
  }
  return 0;
}

/* Chunked form: the frame network of n frames (features [n][B][NF], their
 * LPC already in d_lpc) in one launch on b->stream. */
int launch_chunk_frames(LPCNetBatch *b, const float *d_features, int n)
{
  FrameArgs fa = b->fa;
  fa.st = b->d_state;
  fa.mc = b->mc;
  fa.nstreams = b->B;
  fa.features = d_features;
  fa.lpc_new = b->d_lpc;
  fa.nframes = n;
  fa.cond = b->d_chunk;
  fa.stamps = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (b->timing >= 2) {
    e0 = get_event(b);
    e1 = get_event(b);
    HIPCHK(hipEventRecord(e0, b->stream));
  }
  if (launch_chunk(fa, b->stream)) {
    set_err("chunk kernel launch failed");
    return -1;
  }
  if (e0) {
    HIPCHK(hipEventRecord(e1, b->stream));
    b->ev_pairs[1].push_back(e0);
    b->ev_pairs[1].push_back(e1);
    b->ev_frames[1].push_back(n);
    b->ev_taken.push_back(e0);
    b->ev_taken.push_back(e1);
  }
  b->frames_done(n);
  return 0;
}

/* After a sync of b->stream: report (and clear) a device-side abort. */
int check_status(LPCNetBatch *b)
{
  const int st = __atomic_load_n(b->h_status, __ATOMIC_ACQUIRE);
  if (st == 0) return 0;
  __atomic_store_n(b->h_status, 0, __ATOMIC_RELEASE);
  if (st & STATUS_FLAG_TIMEOUT)
    set_err("device abort: an LDS flag wait in the sample kernel exceeded its spin limit; the PCM of this call is invalid");
  else if (st & STATUS_SLICE_TIMEOUT)
    set_err("device abort: a sliced one-frame chunk kernel waited too long for its sibling workgroups; the PCM of "
            "this call is invalid");
  else if (st & STATUS_ACTIVITY)
    set_err("device abort: a multi-frame sample launch saw a stream turn active mid-launch (frame_count bound out of "
            "date); the PCM of this call is invalid");
  else
    set_err("device abort: unknown status " + std::to_string(st));
  return -1;
}

}  // namespace

/* ======================================================================== */
/* batch API                                                                 */

extern "C" {

LPCNET_EXPORT const char *lpcnet_mi355x_last_error(void) { return g_err.c_str(); }

/* Host-only view of the GRU_A plans a blob gets on a wide batch (no
 * device): the main plan (mf_plan, wide class) and, for split models, the
 * wide kernel's split tables.  out[0] = split (0/1), out[1] = mfw split form
 * available (0/1), out[2..17] = the split form's z/r and h 4-slot groups per
 * table wave (R waves 0..5, host waves 6..7), out[18..20] = pieces per gate.
 * 0 / -1 (malformed blob or no int8 matrix-core plan). */
LPCNET_EXPORT int lpcnet_mi355x_wide_plan(const unsigned char *data, int len, int *out)
{
  std::vector<Arr> L;
  if (!data || len <= 0 || !out || !parse_blob(L, data, len)) return -1;
  std::vector<std::vector<int>> ga;
  if (!parse_idx(L, "sparse_gru_a_recurrent_weights_idx", NA, GA_ROWS, ga)) return -1;
  const Arr *gaw = find(L, "sparse_gru_a_recurrent_weights");
  if (!gaw || gaw->size != 32 * total_blocks(ga)) return -1;
  std::vector<int> first(ga.size() + 1, 0);
  for (size_t r = 0; r < ga.size(); r++) first[r + 1] = first[r] + (int)ga[r].size();
  MfPlan plan;
  if (!mf_plan(ga, plan, 3, 2)) return -1;
  MfwSplitTab T;
  const bool ok = plan.split && mfw_split_tables(ga, first, (const int8_t *)gaw->data, T);
  out[0] = plan.split ? 1 : 0;
  out[1] = ok ? 1 : 0;
  for (int w = 0; w < MFW_TAB_WAVES; w++) {
    out[2 + 2 * w] = T.nzr[w];
    out[3 + 2 * w] = T.nh[w];
  }
  for (int g = 0; g < 3; g++) {
    int n = 0;
    for (int u = 0; u < NA / 8; u++) {
      const int K = (int)ga[g * (NA / 8) + u].size(), c = g < 2 ? MF_ZMAX : MF_HMAX;
      if (K > c) n += (K - c + c - 1) / c;
    }
    out[18 + g] = n;
  }
  return 0;
}

LPCNET_EXPORT int lpcnet_mi355x_device_count(void)
{
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

LPCNET_EXPORT const uint32_t *lpcnet_mi355x_rcp_table(void) { return kRcpTable; }

LPCNET_EXPORT int lpcnet_mi355x_device_lpc(int device, const float *cepstra, float *lpc, int n)
{
  if (n < 0 || (n > 0 && (!cepstra || !lpc))) { set_err("bad arguments"); return -1; }
  if (n == 0) return 0;
  if (hipSetDevice(device) != hipSuccess) { set_err("hipSetDevice failed"); return -1; }
  LpcTables T;
  build_lpc_tables(T);
  float *dc = nullptr, *dl = nullptr;
  LpcTables *dt = nullptr;
  int rc = -1;
  if (hipMalloc(&dc, sizeof(float) * NF * (size_t)n) == hipSuccess && hipMalloc(&dl, sizeof(float) * NLPC * (size_t)n) == hipSuccess &&
      hipMalloc(&dt, sizeof(T)) == hipSuccess && hipMemcpy(dt, &T, sizeof(T), hipMemcpyHostToDevice) == hipSuccess) {
    /* cepstra arrive as [n][NLPC+2] (18 bands); the kernel reads [n][NF] */
    std::vector<float> f((size_t)NF * n, 0.f);
    for (int i = 0; i < n; i++) memcpy(&f[(size_t)i * NF], cepstra + (size_t)i * LPC_NBANDS, sizeof(float) * LPC_NBANDS);
    if (hipMemcpy(dc, f.data(), f.size() * 4, hipMemcpyHostToDevice) == hipSuccess && launch_lpc(dc, dl, n, dt, nullptr) == 0 &&
        hipMemcpy(lpc, dl, sizeof(float) * NLPC * (size_t)n, hipMemcpyDeviceToHost) == hipSuccess)
      rc = 0;
  }
  if (rc) set_err("device LPC failed");
  (void)hipFree(dc);
  (void)hipFree(dl);
  (void)hipFree(dt);
  return rc;
}

LPCNET_EXPORT LPCNetBatch *lpcnet_batch_create(int nb_streams, int device)
{
  if (nb_streams < 1) { set_err("nb_streams < 1"); return nullptr; }
  int ndev = lpcnet_mi355x_device_count();
  if (device < 0 || device >= ndev) { set_err("no such HIP device"); return nullptr; }
  LPCNetBatch *b = new LPCNetBatch();
  b->device = device;
  b->B = nb_streams;
  bool ok = b->set_device() == 0;
  ok = ok && hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) == hipSuccess;
  ok = ok && hipMalloc(&b->d_state, sizeof(StreamState) * (size_t)nb_streams) == hipSuccess;
  ok = ok && hipMalloc(&b->d_feat, sizeof(float) * NF * (size_t)nb_streams) == hipSuccess;
  ok = ok && hipMalloc(&b->d_pcm, sizeof(short) * FRAME * (size_t)nb_streams) == hipSuccess;
  ok = ok && hipHostMalloc(&b->h_status, 64, hipHostMallocMapped) == hipSuccess;
  ok = ok && hipHostGetDevicePointer((void **)&b->d_status, b->h_status, 0) == hipSuccess;
  if (ok) *b->h_status = 0;
  ok = ok && hipMalloc(&b->d_lpc, sizeof(float) * NLPC * (size_t)nb_streams * LPC_CHUNK) == hipSuccess;
  ok = ok && hipMalloc(&b->d_ck_sync, sizeof(int) * (size_t)((nb_streams + 15) / 16)) == hipSuccess;
  ok = ok && hipMemset(b->d_ck_sync, 0, sizeof(int) * (size_t)((nb_streams + 15) / 16)) == hipSuccess;
  ok = ok && hipMalloc(&b->d_lpc_tab, sizeof(LpcTables)) == hipSuccess;
  /* d_chunk (the chunked path's frame outputs, LPC_CHUNK x 4.9 KB per
   * stream) is allocated by the first call that takes that path */
  if (ok) {
    LpcTables T;
    build_lpc_tables(T);
    ok = hipMemcpy(b->d_lpc_tab, &T, sizeof(T), hipMemcpyHostToDevice) == hipSuccess;
  }
  if (ok && nb_streams <= OVERLAP_MAX_STREAMS) {
    ok = ok && hipStreamCreateWithFlags(&b->fstream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&b->ev_start, hipEventDisableTiming) == hipSuccess;
    for (int i = 0; i < 2 && ok; i++) {
      ok = ok && hipMalloc(&b->d_cond[i], sizeof(FrameCond) * (size_t)nb_streams) == hipSuccess;
      ok = ok && hipEventCreateWithFlags(&b->ev_frame[i], hipEventDisableTiming) == hipSuccess;
      ok = ok && hipEventCreateWithFlags(&b->ev_samp[i], hipEventDisableTiming) == hipSuccess;
    }
  }
  if (!ok) {
    set_err("device allocation failed");
    lpcnet_batch_destroy(b);
    return nullptr;
  }
  if (const char *km = getenv("LPCNET_KERNEL")) b->kernel_mode = atoi(km);
  lpcnet_batch_reset(b);
  return b;
}

LPCNET_EXPORT void lpcnet_batch_destroy(LPCNetBatch *b)
{
  if (!b) return;
  b->set_device();
  if (b->stream) (void)hipStreamSynchronize(b->stream);
  if (b->fstream) (void)hipStreamSynchronize(b->fstream);
  free_model(b);
  (void)hipFree(b->d_state);
  (void)hipFree(b->d_ck_sync);
  (void)hipFree(b->d_feat);
  (void)hipFree(b->d_pcm);
  (void)hipFree(b->d_trace_logits);
  (void)hipFree(b->d_trace_exc);
  (void)hipFree(b->d_stamps);
  (void)hipFree(b->d_lpc);
  (void)hipFree(b->d_lpc_tab);
  (void)hipFree(b->d_chunk);
  if (b->io_feat_vram) (void)hipFree(b->h_io_feat);
  else (void)hipHostFree(b->h_io_feat);
  (void)hipHostFree(b->h_io_pcm);
  (void)hipHostFree(b->h_stg_feat);
  (void)hipHostFree(b->h_stg_pcm);
  if (b->ev_tick) (void)hipEventDestroy(b->ev_tick);
  (void)hipFree(b->d_packets);
  (void)hipFree(b->d_dfeat);
  (void)hipFree(b->d_dpcm);
  for (int i = 0; i < 2; i++) {
    (void)hipFree(b->d_cond[i]);
    if (b->ev_frame[i]) (void)hipEventDestroy(b->ev_frame[i]);
    if (b->ev_samp[i]) (void)hipEventDestroy(b->ev_samp[i]);
  }
  if (b->h_status) (void)hipHostFree(b->h_status);
  if (b->ev_start) (void)hipEventDestroy(b->ev_start);
  if (b->fstream) (void)hipStreamDestroy(b->fstream);
  for (hipEvent_t e : b->ev_taken) (void)hipEventDestroy(e);
  for (hipEvent_t e : b->ev_free) (void)hipEventDestroy(e);
  if (b->stream) (void)hipStreamDestroy(b->stream);
  delete b;
}

LPCNET_EXPORT int lpcnet_batch_load_model(LPCNetBatch *b, const unsigned char *data, int len)
{
  if (!b) return -1;
  if (b->set_device()) return -1;
  (void)hipStreamSynchronize(b->stream);
  const int rc = load_model(b, data, len);
  if (rc == 0) b->blob.assign(data, data + len);
  return rc;
}

/* after a change of the kernel mode or the rcpps table: re-plan the register
 * tables when the wide kernel's plan class no longer matches the choice
 * (speed only; the stream states stay) */
static int replan_if_needed(LPCNetBatch *b)
{
  if (!b->have_model || !b->mf_ok || b->blob.empty() || mfw_planned(b, b->cus) == b->plan_wide) return 0;
  if (b->set_device()) return -1;
  (void)hipStreamSynchronize(b->stream);
  const std::vector<unsigned char> blob = b->blob;
  return load_model(b, blob.data(), (int)blob.size());
}

LPCNET_EXPORT int lpcnet_batch_set_kernel(LPCNetBatch *b, int mode)
{
  if (!b || !(mode == 0 || mode == 1 || mode == 4 || mode == 5)) {
    set_err("kernel mode must be 0 (auto), 1 (lockstep), 4 (mf_kernel) or 5 (fp_kernel)");
    return -1;
  }
  b->kernel_mode = mode;
  if (b->have_model) choose_kernel(b);
  return replan_if_needed(b);
}

LPCNET_EXPORT int lpcnet_batch_set_model_constants(LPCNetBatch *b, float lpc_gamma, int features_delay, int end2end)
{
  if (!b || !b->have_model) { set_err("no model loaded"); return -1; }
  const ModelConst mc{lpc_gamma, features_delay, end2end};
  if (check_constants(mc)) return -1;
  if (b->set_device()) return -1;
  (void)hipStreamSynchronize(b->stream); /* queued frames keep the constants they were enqueued with */
  b->mc = mc;
  b->info.lpc_gamma = mc.lpc_gamma;
  b->info.features_delay = mc.delay;
  b->info.end2end = mc.end2end;
  return 0;
}

LPCNET_EXPORT int lpcnet_batch_set_rcp_table(LPCNetBatch *b, const uint32_t *tab)
{
  if (!b || !b->have_model) { set_err("no model loaded"); return -1; }
  std::vector<uint32_t> dev(RCP_ENTRIES), dflt(RCP_ENTRIES);
  for (int i = 0; i < RCP_ENTRIES; i++) {
    dflt[i] = kRcpTable[i >> (RCP_TABLE_BITS - 11)] + kRcpBias;
    dev[i] = tab ? tab[i] + kRcpBias : dflt[i];
  }
  if (b->set_device()) return -1;
  HIPCHK(hipStreamSynchronize(b->stream));
  /* the LDS image's table section and the frame network's global copy */
  HIPCHK(hipMemcpy((unsigned char *)b->sa.image + IMG_RCP, dev.data(), RCP_ENTRIES * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy((void *)b->fa.rcp, dev.data(), RCP_ENTRIES * 4, hipMemcpyHostToDevice));
  b->rcp_dev = dev;
  b->rcp_custom = dev != dflt;
  choose_kernel(b);
  return replan_if_needed(b);
}

LPCNET_EXPORT int lpcnet_batch_model_info(const LPCNetBatch *b, LPCNetModelInfo *info)
{
  if (!b || !b->have_model || !info) return -1;
  *info = b->info;
  return 0;
}

LPCNET_EXPORT int lpcnet_batch_nb_streams(const LPCNetBatch *b) { return b ? b->B : 0; }

LPCNET_EXPORT int lpcnet_batch_reset_stream(LPCNetBatch *b, int stream)
{
  if (!b || stream < 0 || stream >= b->B) return -1;
  if (b->set_device()) return -1;
  StreamState s;
  host_reset_state(s);
  HIPCHK(hipMemcpyAsync(&b->d_state[stream], &s, sizeof(s), hipMemcpyHostToDevice, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  b->min_fc = std::min(b->min_fc, s.frame_count);
  return 0;
}

LPCNET_EXPORT void lpcnet_batch_reset(LPCNetBatch *b)
{
  if (!b || b->set_device()) return;
  std::vector<StreamState> v(b->B);
  host_reset_state(v[0]);
  for (int i = 1; i < b->B; i++) v[i] = v[0];
  (void)hipMemcpyAsync(b->d_state, v.data(), sizeof(StreamState) * v.size(), hipMemcpyHostToDevice, b->stream);
  (void)hipStreamSynchronize(b->stream);
  b->min_fc = v[0].frame_count;
}

/* Work a caller enqueues on b->stream after a step's kernels, before its one
 * synchronisation (the drop-in pool's state scatter). */
using PreSync = std::function<int()>;

/* One frame of a large batch in the chunked form (a live server's tick:
 * lpcnet_batch_synthesize once per 10 ms): lpc_kernel, chunk_kernel with
 * stream-only columns (weights fetched once per 16-32 streams instead of the
 * per-frame frame_kernel's once per 4: at 1024 streams ~44 -> ~20 us, at
 * 28 K streams 28 rounds of workgroups -> 2-4), then the sample kernel
 * reading the frame's conditioning, LPC and frame_count from the stream
 * state (no per-frame output copy: half the chunk kernel's stores).  Same
 * arithmetic as every other frame
 * path (the chunk kernel is bit-identical to the frame kernel). */
static bool single_frame_chunked(const LPCNetBatch *b, int nB, int N, int preload)
{
  return b->chunking && (b->mf || b->fp) && nB > OVERLAP_MAX_STREAMS && N > 0 && preload == 0 && !b->d_stamps &&
         !b->sa.trace_logits && !getenv("LPCNET_NO_CHUNK");
}

/* Deferred LPC (one-frame ticks of models with FEATURES_DELAY >= 1): a
 * frame synthesises with the LPC of frame f - FEATURES_DELAY (lpcnet.c:
 * 110-118), already in the stream's ring, so lpc_from_cepstrum of this
 * frame's features is off the tick's critical path: the chunk kernel reads
 * the ring's oldest slot only, and lpc_kernel pushes the new LPC into the
 * ring after the sample kernel, while the caller consumes the PCM and
 * refills its features (the tick's end is the sample kernel's).
 * LPCNET_LPC_EAGER=1 keeps the LPC before the chunk kernel. */
static bool lpc_deferred(const LPCNetBatch *b)
{
  const char *e = getenv("LPCNET_LPC_EAGER");
  return !b->mc.end2end && b->mc.delay >= 1 && !(e && atoi(e) != 0);
}

/* d_features: device memory, or the mapped host buffer (mapped = true: a
 * deferred LPC then reads the chunk kernel's copy in b->d_feat) */
static int launch_single_frame_chunked(LPCNetBatch *b, int nB, const float *d_features, short *d_pcm, int N,
                                       bool defer = false, bool mapped = false)
{
  if (!b->mc.end2end && !defer && launch_lpc(d_features, b->d_lpc, nB, b->d_lpc_tab, b->stream)) {
    set_err("lpc kernel launch failed");
    return -1;
  }
  FrameArgs fa = b->fa;
  fa.st = b->d_state;
  fa.mc = b->mc;
  fa.nstreams = nB;
  fa.features = d_features;
  fa.lpc_new = b->d_lpc;
  fa.nframes = 1;
  fa.cond = nullptr;
  fa.stamps = nullptr;
  fa.lpc_defer = defer ? 1 : 0;
  fa.lpc_feat = defer && mapped ? b->d_feat : nullptr;
  fa.ck_sync = b->d_ck_sync;
  fa.status = b->d_status;
  hipEvent_t e[3] = {nullptr, nullptr, nullptr};
  if (b->timing >= 2) e[0] = get_event(b);
  if (b->timing >= 1) {
    e[1] = get_event(b);
    e[2] = get_event(b);
  }
  if (e[0]) HIPCHK(hipEventRecord(e[0], b->stream));
  if (launch_chunk(fa, b->stream)) {
    set_err("chunk kernel launch failed");
    return -1;
  }
  b->frames_done(1);
  SampleArgs sa = b->sa;
  sa.st = b->d_state;
  sa.delay = b->mc.delay;
  sa.cond = nullptr;
  sa.nstreams = nB;
  sa.N = N;
  sa.nframes = 1;
  sa.pcm = d_pcm;
  sa.preload = 0;
  sa.stamps = nullptr;
  sa.status = b->d_status;
  sa.spin_limit = b->spin_limit;
  if (e[1]) HIPCHK(hipEventRecord(e[1], b->stream));
  const int lrc = b->fp ? launch_fp(sa, b->stream)
                  : wide_for(b, nB) ? launch_mfw(sa, b->mfw_g, b->stream)
                  : mf2_for(b, nB) ? launch_mf2(sa, 4, b->stream)
                           : launch_mf(sa, b->S, mf_lds_bytes(b->S, b->sa.mf_split), b->stream);
  if (lrc) {
    set_err(std::string("sample kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
    return -1;
  }
  if (e[2]) HIPCHK(hipEventRecord(e[2], b->stream));
  if (e[0]) {
    b->ev_pairs[1].push_back(e[0]);
    b->ev_pairs[1].push_back(e[1]);
    b->ev_frames[1].push_back(1);
  }
  if (e[1]) {
    b->ev_pairs[0].push_back(e[1]);
    b->ev_pairs[0].push_back(e[2]);
    b->ev_frames[0].push_back(1);
  }
  for (hipEvent_t x : e)
    if (x) b->ev_taken.push_back(x);
  return 0;
}

/* the batch's pinned host I/O buffers ([B][NF] features, [B][FRAME] PCM,
 * mapped: the kernels read and store them over PCIe) and the pinned staging
 * of callers' own buffers (cached, DMA) */
static int ensure_host_io(LPCNetBatch *b)
{
  if (!b->h_io_feat) {
    /* features: host-visible device memory where the device has a large BAR
     * (the host's stores cross PCIe as posted writes, the chunk and LPC
     * kernels then read local HBM: 80 KB at 1024 streams, the chunk kernel's
     * input phase ~24 K -> ~12 K cycles against reads of mapped host memory),
     * else mapped pinned host memory.  LPCNET_FEAT_VRAM=0: always the latter. */
    int large_bar = 0;
    (void)hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, b->device);
    const char *ev = getenv("LPCNET_FEAT_VRAM");
    if (large_bar && !(ev && atoi(ev) == 0) &&
        hipExtMallocWithFlags((void **)&b->h_io_feat, sizeof(float) * NF * (size_t)b->B, hipDeviceMallocFinegrained) ==
            hipSuccess) {
      b->io_feat_vram = true;
      b->d_io_feat = b->h_io_feat;
    } else {
      b->h_io_feat = nullptr;
      HIPCHK(hipHostMalloc(&b->h_io_feat, sizeof(float) * NF * (size_t)b->B, hipHostMallocMapped));
      HIPCHK(hipHostGetDevicePointer((void **)&b->d_io_feat, b->h_io_feat, 0));
    }
  }
  if (!b->h_io_pcm) {
    HIPCHK(hipHostMalloc(&b->h_io_pcm, sizeof(short) * FRAME * (size_t)b->B, hipHostMallocMapped));
    HIPCHK(hipHostGetDevicePointer((void **)&b->d_io_pcm, b->h_io_pcm, 0));
  }
  if (!b->h_stg_feat) HIPCHK(hipHostMalloc(&b->h_stg_feat, sizeof(float) * NF * (size_t)b->B, hipHostMallocDefault));
  if (!b->h_stg_pcm) HIPCHK(hipHostMalloc(&b->h_stg_pcm, sizeof(short) * FRAME * (size_t)b->B, hipHostMallocDefault));
  return 0;
}

/* the end of a synchronous call.  poll: the calling thread polls the
 * call's event (no sleep / wake-up between the last kernel and the thread's
 * next step), handing over to a blocking wait after TICK_SPIN_MS -- the
 * drop-in pool's combiner (64 C threads: 19-20 -> 27.5 M samples/s, 256:
 * 58-60 -> 69-84 M); otherwise hipStreamSynchronize, 2-3 % faster for one
 * caller driving a batch (tools/sync_ab.sh, profiles/r05/sync_ab.log).
 * LPCNET_SYNC_BLOCK=1 / LPCNET_SYNC_POLL=1 force one form everywhere. */
static int tick_sync(LPCNetBatch *b, bool poll, const std::function<int()> &after = std::function<int()>())
{
  if (getenv("LPCNET_SYNC_POLL")) poll = true;
  const bool block = !poll || getenv("LPCNET_SYNC_BLOCK");
  if (block && !after) {
    HIPCHK(hipStreamSynchronize(b->stream));
    return 0;
  }
  if (!b->ev_tick) HIPCHK(hipEventCreateWithFlags(&b->ev_tick, hipEventDisableTiming));
  HIPCHK(hipEventRecord(b->ev_tick, b->stream));
  /* work queued behind the tick's end (the deferred LPC): not waited for */
  if (after && after()) return -1;
  if (block) {
    HIPCHK(hipEventSynchronize(b->ev_tick));
    return 0;
  }
  static const int pause = getenv("LPCNET_SYNC_PAUSE") ? atoi(getenv("LPCNET_SYNC_PAUSE")) : TICK_POLL_PAUSE;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipEventQuery(b->ev_tick);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) HIPCHK(q);
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(TICK_SPIN_MS)) break;
    for (int k = 0; k < pause; k++) __builtin_ia32_pause(); /* fewer runtime queries */
  }
  HIPCHK(hipEventSynchronize(b->ev_tick));
  return 0;
}

/* sample kernels whose PCM write-out is wide (a frame's samples, or 16 of
 * them, per stream in consecutive lanes): mf_kernel at the end of the
 * launch, mfw_kernel every 16 samples, fp_kernel at the end.  mf2_kernel
 * stores every sample as it is drawn (2-byte stores: over PCIe, one
 * transaction each), so its PCM goes through device memory and one copy. */
static bool pcm_store_coalesced(const LPCNetBatch *b)
{
  return !getenv("LPCNET_NO_DIRECT_PCM") && (b->fp || b->mfw || (b->mf && !b->mf2));  /* mfw batches: mfw or mf_kernel */
}

/* one frame for the first nB streams of a batch, host I/O ([nB][NF] in,
 * [nB][N] out) */
static int synth_first(LPCNetBatch *b, int nB, const float *features, short *pcm, int N, int preload,
                       const PreSync &pre = PreSync(), bool staged = false)
{
  if (!b || !b->have_model) { set_err("no model loaded"); return -1; }
  if (N < 0 || N > FRAME || !features || (N > 0 && !pcm) || preload < 0) { set_err("bad arguments"); return -1; }
  if (b->set_device()) return -1;
  if (ensure_trace(b, N)) return -1;
  /* the caller's stores into the VRAM feature buffer are write-combined:
   * drained before any command of this call can read them */
  if (features == b->h_io_feat && b->io_feat_vram) __builtin_ia32_sfence();
  if (!staged && !pre && single_frame_chunked(b, nB, N, preload)) {
    /* the caller's buffers through pinned staging: both copies truly
     * asynchronous, one synchronisation per frame.  Features already in the
     * batch's own pinned buffer (lpcnet_batch_host_features) skip the host
     * copy; PCM into the batch's own pinned buffer (lpcnet_batch_host_pcm)
     * is stored there by the sample kernel itself when its write-out is
     * coalesced (no device-to-host copy, no host copy) */
    if (ensure_host_io(b)) return -1;
    /* the batch's own buffers (mapped): up to ZC_FEAT_MAX streams the LPC
     * and chunk kernels read the features straight from host memory (80 B
     * per stream over PCIe, no copy command and its start latency), larger
     * batches take one DMA copy; the caller's buffers: host copy into the
     * cached pinned staging, one DMA copy each way */
    const bool own_feat = features == b->h_io_feat, own_pcm = pcm == b->h_io_pcm;
    const bool zc_feat = own_feat && (nB <= ZC_FEAT_MAX || b->io_feat_vram) && !getenv("LPCNET_FEAT_DMA");
    if (!own_feat) memcpy(b->h_stg_feat, features, sizeof(float) * NF * nB);
    if (!zc_feat)
      HIPCHK(hipMemcpyAsync(b->d_feat, own_feat ? b->h_io_feat : b->h_stg_feat, sizeof(float) * NF * nB,
                            hipMemcpyHostToDevice, b->stream));
    const bool direct = own_pcm && pcm_store_coalesced(b);
    const bool defer = lpc_deferred(b);
    if (launch_single_frame_chunked(b, nB, zc_feat ? b->d_io_feat : b->d_feat, direct ? b->d_io_pcm : b->d_pcm, N,
                                    defer, zc_feat))
      return -1;
    if (!direct)
      HIPCHK(hipMemcpyAsync(own_pcm ? b->h_io_pcm : b->h_stg_pcm, b->d_pcm, sizeof(short) * N * nB,
                            hipMemcpyDeviceToHost, b->stream));
    auto lpc_after = [&]() -> int {
      /* LPCNET_CK_WARM=1 (A/B, measured: no gain at 1024 streams): it also
       * warms every XCD's L2 with the chunk kernel's weights for the next tick */
      const char *cw = getenv("LPCNET_CK_WARM");
      const bool warm = cw && atoi(cw) != 0 && b->ck_warm.m[0];
      if (launch_lpc(b->d_feat, nullptr, nB, b->d_lpc_tab, b->stream, b->d_state, b->mc.delay,
                     warm ? &b->ck_warm : nullptr)) {
        set_err("deferred lpc kernel launch failed");
        return -1;
      }
      return 0;
    };
    if (tick_sync(b, false, defer ? std::function<int()>(lpc_after) : std::function<int()>())) return -1;
    if (check_status(b)) return -1;
    if (!own_pcm) memcpy(pcm, b->h_stg_pcm, sizeof(short) * N * nB);
    return 0;
  }
  /* everything below is ordered after work already queued on b->stream
   * (staged: the caller has queued the features / preload copies already) */
  if (!staged) {
    HIPCHK(hipMemcpyAsync(b->d_feat, features, sizeof(float) * NF * nB, hipMemcpyHostToDevice, b->stream));
    if (preload > 0 && N > 0)
      HIPCHK(hipMemcpyAsync(b->d_pcm, pcm, sizeof(short) * N * nB, hipMemcpyHostToDevice, b->stream));
  }
  if (launch_frame_step(b, b->d_feat, b->d_lpc, true, b->d_pcm, N, preload, -1, nB)) return -1;
  if (pre && pre()) return -1;
  if (N > 0) HIPCHK(hipMemcpyAsync(pcm, b->d_pcm, sizeof(short) * N * nB, hipMemcpyDeviceToHost, b->stream));
  if (tick_sync(b, pre || staged)) return -1;
  return check_status(b);
}

LPCNET_EXPORT int lpcnet_batch_synthesize_impl(LPCNetBatch *b, const float *features, short *pcm, int N, int preload)
{
  return synth_first(b, b ? b->B : 0, features, pcm, N, preload);
}

LPCNET_EXPORT int lpcnet_batch_synthesize(LPCNetBatch *b, const float *features, short *pcm, int N)
{
  return lpcnet_batch_synthesize_impl(b, features, pcm, N, 0);
}

LPCNET_EXPORT float *lpcnet_batch_host_features(LPCNetBatch *b)
{
  if (!b || b->set_device() || ensure_host_io(b)) return nullptr;
  return b->h_io_feat;
}

LPCNET_EXPORT short *lpcnet_batch_host_pcm(LPCNetBatch *b)
{
  if (!b || b->set_device() || ensure_host_io(b)) return nullptr;
  return b->h_io_pcm;
}

static int ensure_decode_bufs(LPCNetBatch *b, bool host_io)
{
  if (!b->d_packets) HIPCHK(hipMalloc(&b->d_packets, (size_t)DEC_MAX_PACKETS * b->B * 8));
  if (!b->d_dfeat) HIPCHK(hipMalloc(&b->d_dfeat, sizeof(float) * NF * 4 * DEC_MAX_PACKETS * (size_t)b->B));
  if (host_io && !b->d_dpcm) HIPCHK(hipMalloc(&b->d_dpcm, sizeof(short) * 4 * FRAME * (size_t)b->B));
  return 0;
}

static int decode_ready(LPCNetBatch *b)
{
  if (!b || !b->have_model) { set_err("no model loaded"); return -1; }
  if (!b->has_codebooks) {
    set_err("lpcnet_decode: the model blob carries no ceps_codebook1/2/3 / ceps_codebook_diff4 records "
            "(1024x17, 1024x17, 1024x17, 4096x18 floats)");
    return -1;
  }
  return b->set_device();
}

/* lpcnet_decode (lpcnet.c:310-319) on the first nB streams, host I/O:
 * packets [nB][8] -> pcm [nB][4 * FRAME] */
static int decode_first(LPCNetBatch *b, int nB, const unsigned char *packets, short *pcm, const PreSync &pre = PreSync())
{
  if (decode_ready(b)) return -1;
  if (!packets || !pcm) { set_err("bad arguments"); return -1; }
  if (ensure_trace(b, FRAME) || ensure_decode_bufs(b, true)) return -1;
  HIPCHK(hipMemcpyAsync(b->d_packets, packets, (size_t)nB * 8, hipMemcpyHostToDevice, b->stream));
  DecodeArgs da = b->da;
  da.packets = b->d_packets;
  da.npackets = 1;
  da.nstreams = nB;
  da.st = b->d_state;
  da.features = b->d_dfeat;
  if (launch_decode(da, b->stream)) { set_err("decode kernel launch failed"); return -1; }
  /* for (k=0;k<4;k++) lpcnet_synthesize(&st->lpcnet_state, features[k], &pcm[k*FRAME_SIZE], FRAME_SIZE) */
  for (int f = 0; f < 4; f++)
    if (launch_frame_step(b, b->d_dfeat + (size_t)f * nB * NF, b->d_lpc, true, b->d_dpcm + (size_t)f * nB * FRAME, FRAME, 0,
                          -1, nB))
      return -1;
  if (pre && pre()) return -1;
  std::vector<short> tmp((size_t)4 * nB * FRAME);
  HIPCHK(hipMemcpyAsync(tmp.data(), b->d_dpcm, sizeof(short) * tmp.size(), hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  if (check_status(b)) return -1;
  for (int k = 0; k < nB; k++)
    for (int f = 0; f < 4; f++)
      memcpy(pcm + ((size_t)k * 4 + f) * FRAME, &tmp[((size_t)f * nB + k) * FRAME], sizeof(short) * FRAME);
  return 0;
}

LPCNET_EXPORT int lpcnet_batch_decode(LPCNetBatch *b, const unsigned char *packets, short *pcm)
{
  return decode_first(b, b ? b->B : 0, packets, pcm);
}

LPCNET_EXPORT int lpcnet_batch_decode_frames(LPCNetBatch *b, const unsigned char *d_packets, short *d_pcm, int npackets)
{
  if (decode_ready(b)) return -1;
  if (!d_packets || !d_pcm || npackets < 0) { set_err("bad arguments"); return -1; }
  if (ensure_decode_bufs(b, false)) return -1;
  for (int p0 = 0; p0 < npackets; p0 += DEC_MAX_PACKETS) {
    const int np = std::min(DEC_MAX_PACKETS, npackets - p0);
    DecodeArgs da = b->da;
    da.packets = d_packets + (size_t)p0 * b->B * 8;
    da.npackets = np;
    da.nstreams = b->B;
    da.st = b->d_state;
    da.features = b->d_dfeat;
    /* queued behind every kernel that still reads d_dfeat (the previous
     * group's frame kernels precede the sample kernels on b->stream) */
    if (launch_decode(da, b->stream)) { set_err("decode kernel launch failed"); return -1; }
    if (lpcnet_batch_synthesize_frames(b, nullptr, b->d_dfeat, d_pcm + (size_t)4 * p0 * b->B * FRAME, 4 * np, FRAME))
      return -1;
  }
  return 0;
}

/* lpcnet_synthesize_tail_impl on the first nB streams: the sample network on
 * the conditioning and LPC already in the stream states, no frame network */
static int tail_first(LPCNetBatch *b, int nB, short *pcm, int N, int preload, const PreSync &pre = PreSync())
{
  if (!b || !b->have_model) { set_err("no model loaded"); return -1; }
  if (N < 0 || N > FRAME || (N > 0 && !pcm) || preload < 0) { set_err("bad arguments"); return -1; }
  if (N == 0) return 0;
  if (b->set_device()) return -1;
  if (ensure_trace(b, N)) return -1;
  if (preload > 0) HIPCHK(hipMemcpyAsync(b->d_pcm, pcm, sizeof(short) * N * nB, hipMemcpyHostToDevice, b->stream));
  if (launch_frame_step(b, nullptr, nullptr, false, b->d_pcm, N, preload, -1, nB, false, false)) return -1;
  if (pre && pre()) return -1;
  HIPCHK(hipMemcpyAsync(pcm, b->d_pcm, sizeof(short) * N * nB, hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  return check_status(b);
}

/* run_frame_network on the first nB streams (features [nB][NF]); keep_cond:
 * into the caller's locals as run_frame_network_flush does (lpcnet.c:134-144),
 * otherwise into the state's conditioning (lpcnet.c:275) */
static int frame_first(LPCNetBatch *b, int nB, const float *features, bool keep_cond, const PreSync &pre = PreSync())
{
  if (!b || !b->have_model) { set_err("no model loaded"); return -1; }
  if (!features) { set_err("bad arguments"); return -1; }
  if (b->set_device()) return -1;
  HIPCHK(hipMemcpyAsync(b->d_feat, features, sizeof(float) * NF * nB, hipMemcpyHostToDevice, b->stream));
  if (launch_frame_step(b, b->d_feat, b->d_lpc, true, nullptr, 0, 0, -1, nB, true, keep_cond)) return -1;
  if (pre && pre()) return -1;
  HIPCHK(hipStreamSynchronize(b->stream));
  return check_status(b);
}

LPCNET_EXPORT int lpcnet_batch_synthesize_tail_impl(LPCNetBatch *b, short *pcm, int N, int preload)
{
  return tail_first(b, b ? b->B : 0, pcm, N, preload);
}

LPCNET_EXPORT int lpcnet_batch_run_frame_network(LPCNetBatch *b, const float *features, int update_conditions)
{
  return frame_first(b, b ? b->B : 0, features, update_conditions == 0);
}

/* lpcnet.c:226-233 lpcnet_reset_signal on one stream */
static void reset_signal(StreamState &s)
{
  s.deemph_mem = 0;
  s.last_exc = host_lin2ulaw(0.f);
  memset(s.last_sig, 0, sizeof(s.last_sig));
  memset(s.gru_a_state, 0, sizeof(s.gru_a_state));
  memset(s.gru_b_state, 0, sizeof(s.gru_b_state));
}

LPCNET_EXPORT int lpcnet_batch_reset_signal(LPCNetBatch *b, int stream)
{
  if (!b || stream < 0 || stream >= b->B) { set_err("bad arguments"); return -1; }
  if (b->set_device()) return -1;
  StreamState s;
  HIPCHK(hipStreamSynchronize(b->stream));
  HIPCHK(hipMemcpy(&s, &b->d_state[stream], sizeof(s), hipMemcpyDeviceToHost));
  reset_signal(s);
  HIPCHK(hipMemcpy(&b->d_state[stream], &s, sizeof(s), hipMemcpyHostToDevice));
  return 0;
}

LPCNET_EXPORT int lpcnet_batch_state_size(void) { return (int)sizeof(StreamState); }

LPCNET_EXPORT int lpcnet_batch_save_state(LPCNetBatch *b, int stream, void *buf)
{
  if (!b || stream < 0 || stream >= b->B || !buf || b->set_device()) return -1;
  HIPCHK(hipStreamSynchronize(b->stream));
  HIPCHK(hipMemcpy(buf, &b->d_state[stream], sizeof(StreamState), hipMemcpyDeviceToHost));
  return 0;
}

/* A snapshot is restored only if it is one this engine can have produced. */
static bool snapshot_ok(const void *buf)
{
  /* GRU states are convex combinations of earlier states and tanh outputs:
   * |x| <= 1 (+ rounding) or NaN for every state the recurrence produces.
   * The int8 kernels' state quantiser relies on |x| < 2^24 (quant_s8_state),
   * so a snapshot outside that range is not one of ours: refuse it. */
  StreamState tmp;
  memcpy(&tmp, buf, sizeof(tmp));
  auto bad = [](const float *v, int n) {
    for (int k = 0; k < n; k++)
      if (v[k] > 2.f || v[k] < -2.f) return true;
    return false;
  };
  if (bad(tmp.gru_a_state, NA) || bad(tmp.gru_b_state, NB)) {
    set_err("snapshot GRU state outside [-2, 2]: not a state this engine produced");
    return false;
  }
  /* last_exc indexes the 256-row embedding tables (lpcnet.c:264: an
   * excitation is a u-law byte) */
  if (tmp.last_exc < 0 || tmp.last_exc > 255) {
    set_err("snapshot last_exc outside [0, 255]: not a state this engine produced");
    return false;
  }
  return true;
}

LPCNET_EXPORT int lpcnet_batch_restore_state(LPCNetBatch *b, int stream, const void *buf)
{
  if (!b || stream < 0 || stream >= b->B || !buf || b->set_device()) return -1;
  if (!snapshot_ok(buf)) return -1;
  HIPCHK(hipStreamSynchronize(b->stream));
  HIPCHK(hipMemcpy(&b->d_state[stream], buf, sizeof(StreamState), hipMemcpyHostToDevice));
  int fc;
  memcpy(&fc, (const unsigned char *)buf + offsetof(StreamState, frame_count), sizeof(fc));
  b->min_fc = std::min(b->min_fc, fc);
  return 0;
}

LPCNET_EXPORT int lpcnet_batch_synthesize_frames(LPCNetBatch *b, const float *h_features, const float *d_features,
                                                 short *d_pcm, int nframes, int N)
{
  (void)h_features; /* kept for ABI compatibility: lpc_from_cepstrum now runs on the device */
  if (!b || !b->have_model) { set_err("no model loaded"); return -1; }
  if (N < 0 || N > FRAME || nframes < 0 || !d_features || !d_pcm) { set_err("bad arguments"); return -1; }
  if (b->set_device()) return -1;
  if (ensure_trace(b, N)) return -1;
  const size_t fstride = (size_t)b->B * NF;
  if (nframes == 0) return 0;
  /* multi-frame matrix-core sample launches (SampleArgs::nframes): one
   * launch per chunk instead of one per frame (each costs a ~10 us dispatch
   * gap plus its prologue), behind the chunked frame network */
  const bool mfm = b->mf && b->chunking && !b->sa.trace_logits && N > 0 &&
                   nframes >= CHUNK_MIN_FRAMES && !getenv("LPCNET_NO_MULTIFRAME");
  /* otherwise overlapped frame kernels: matrix-core and fp32 latency kernels
   * (the only ones reading the frame outputs through FrameCond), when CUs
   * are free */
  const bool ovl = !mfm && b->fstream && (b->mf || b->fp) && nframes >= 2 && !b->d_stamps && !getenv("LPCNET_NO_OVERLAP");
  if (ovl) {
    /* the first frame kernel follows everything already on stream */
    HIPCHK(hipEventRecord(b->ev_start, b->stream));
    HIPCHK(hipStreamWaitEvent(b->fstream, b->ev_start, 0));
  }
  /* chunked frame network: batches too large for the overlapped path (the
   * sample kernels fill the GPU), matrix-core and fp32 sample kernels (the
   * ones reading FrameCond) */
  const bool chunked = mfm || (!ovl && b->chunking && (b->mf || b->fp) && b->B > OVERLAP_MAX_STREAMS && !b->d_stamps &&
                               !getenv("LPCNET_NO_CHUNK"));
  if (chunked && !b->d_chunk) {
    /* frame-network outputs of a chunk of frames (chunk_kernel -> sample
     * launches): sizeof(FrameCond) = 4.9 KB x LPC_CHUNK per stream (160 MB
     * at 1024 streams), only for batches that take this path */
    if (hipMalloc(&b->d_chunk, sizeof(FrameCond) * (size_t)LPC_CHUNK * b->B) != hipSuccess) {
      b->d_chunk = nullptr;
      set_err("device allocation of the chunked frame-network buffer failed");
      return -1;
    }
  }
  hipStream_t fs = ovl ? b->fstream : b->stream;
  for (int c0 = 0; c0 < nframes; c0 += LPC_CHUNK) {
    /* lpc_from_cepstrum depends only on the features: one launch for up to
     * LPC_CHUNK frames x B streams fills the GPU (a per-frame launch of B
     * one-wave streams is latency-bound); queued on the frame kernels' queue,
     * after the frame kernels of the previous chunk that read d_lpc */
    const int n = std::min(LPC_CHUNK, nframes - c0);
    if (!b->mc.end2end && launch_lpc(d_features + c0 * fstride, b->d_lpc, n * b->B, b->d_lpc_tab, fs)) {
      set_err("lpc kernel launch failed");
      return -1;
    }
    if (chunked && n >= CHUNK_MIN_FRAMES) {
      const int fc0 = b->min_fc;
      if (launch_chunk_frames(b, d_features + c0 * fstride, n)) return -1;
      /* frames in which a stream may still turn active: one launch each */
      const int k = mfm ? std::min(n, std::max(0, b->mc.delay - fc0)) : n;
      for (int f = c0; f < c0 + k; f++)
        if (launch_chunk_samples(b, f - c0, d_pcm + (size_t)f * b->B * N, N)) return -1;
      if (k < n && launch_chunk_samples(b, k, d_pcm + (size_t)(c0 + k) * b->B * N, N, n - k)) return -1;
      continue;
    }
    for (int f = c0; f < c0 + n; f++)
      if (launch_frame_step(b, d_features + f * fstride, b->d_lpc + (size_t)(f - c0) * b->B * NLPC, false,
                            d_pcm + (size_t)f * b->B * N, N, 0, ovl ? f : -1))
        return -1;
  }
  return 0;
}

LPCNET_EXPORT int lpcnet_batch_sync(LPCNetBatch *b)
{
  if (!b || b->set_device()) return -1;
  HIPCHK(hipStreamSynchronize(b->stream));
  return check_status(b);
}

LPCNET_EXPORT int lpcnet_batch_set_frame_chunking(LPCNetBatch *b, int enable)
{
  if (!b) return -1;
  b->chunking = enable != 0;
  return 0;
}

LPCNET_EXPORT int lpcnet_batch_set_spin_limit(LPCNetBatch *b, int polls)
{
  if (!b || polls < 0) return -1;
  /* clamped: the kernels' poll counter must be able to exceed the limit */
  b->spin_limit = polls == 0 ? FLAG_SPIN_LIMIT_DEFAULT : std::min(polls, FLAG_SPIN_LIMIT_MAX);
  return 0;
}

LPCNET_EXPORT void *lpcnet_batch_device_alloc(LPCNetBatch *b, size_t bytes)
{
  if (!b || b->set_device()) return nullptr;
  void *p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) { set_err("hipMalloc failed"); return nullptr; }
  return p;
}

LPCNET_EXPORT int lpcnet_batch_device_free(LPCNetBatch *b, void *p)
{
  if (!b || b->set_device()) return -1;
  HIPCHK(hipFree(p));
  return 0;
}

LPCNET_EXPORT int lpcnet_batch_memcpy_h2d(LPCNetBatch *b, void *dst, const void *src, size_t bytes)
{
  if (!b || b->set_device()) return -1;
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  return 0;
}

LPCNET_EXPORT int lpcnet_batch_memcpy_d2h(LPCNetBatch *b, void *dst, const void *src, size_t bytes)
{
  if (!b || b->set_device()) return -1;
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, b->stream));
  HIPCHK(hipStreamSynchronize(b->stream));
  return 0;
}

LPCNET_EXPORT void lpcnet_batch_reset_timers(LPCNetBatch *b, int enable)
{
  if (!b) return;
  b->set_device();
  (void)hipStreamSynchronize(b->stream);
  for (int k = 0; k < 2; k++) {
    b->ev_pairs[k].clear();
    b->ev_frames[k].clear();
  }
  /* stream is idle (and fstream with it): no slot reuse needs a wait */
  b->ev_samp_used[0] = b->ev_samp_used[1] = false;
  for (hipEvent_t e : b->ev_taken) b->ev_free.push_back(e);
  b->ev_taken.clear();
  b->timing = enable < 0 ? 0 : (enable > 2 ? 2 : enable);
}

LPCNET_EXPORT double lpcnet_batch_kernel_ms(LPCNetBatch *b, int which, int *launches)
{
  if (!b || which < 0 || which > 1) return -1;
  b->set_device();
  (void)hipStreamSynchronize(b->stream);
  double tot = 0;
  const std::vector<hipEvent_t> &v = b->ev_pairs[which];
  for (size_t i = 0; i + 1 < v.size(); i += 2) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, v[i], v[i + 1]) == hipSuccess) tot += ms;
  }
  if (launches) *launches = (int)(v.size() / 2);
  return tot;
}

LPCNET_EXPORT int lpcnet_batch_kernel_frames(LPCNetBatch *b, int which)
{
  if (!b || which < 0 || which > 1) return -1;
  int n = 0;
  for (int k : b->ev_frames[which]) n += k;
  return n;
}

static int stamp_groups(const LPCNetBatch *b)
{
  const int spw = std::max(1, b->info.streams_per_workgroup);
  return (b->B + spw - 1) / spw;
}

LPCNET_EXPORT int lpcnet_batch_set_stamps(LPCNetBatch *b, int enable)
{
  if (!b || b->set_device()) return -1;
  (void)hipStreamSynchronize(b->stream);
  if (b->d_stamps) (void)hipFree(b->d_stamps);
  b->d_stamps = nullptr;
  if (enable) {
    /* sample kernel [groups][STAMP_WAVES][16] (enough for any S), then the
     * frame kernel [B / FRAME_STREAMS][16] */
    size_t n = (size_t)b->B * STAMP_WAVES * 16 + (size_t)(frame_groups(b->B) + 1) * 16;
    HIPCHK(hipMalloc(&b->d_stamps, n * 8));
    HIPCHK(hipMemset(b->d_stamps, 0, n * 8));
  }
  return 0;
}

LPCNET_EXPORT int lpcnet_batch_get_stamps(LPCNetBatch *b, unsigned long long *out)
{
  if (!b || !b->d_stamps || !b->have_model || b->set_device()) return -1;
  HIPCHK(hipStreamSynchronize(b->stream));
  int g = stamp_groups(b);
  HIPCHK(hipMemcpy(out, b->d_stamps, (size_t)g * STAMP_WAVES * 16 * 8, hipMemcpyDeviceToHost));
  return g;
}

LPCNET_EXPORT int lpcnet_batch_get_frame_stamps(LPCNetBatch *b, unsigned long long *out)
{
  if (!b || !b->d_stamps || !b->have_model || b->set_device()) return -1;
  HIPCHK(hipStreamSynchronize(b->stream));
  const int g = frame_groups(b->B);
  HIPCHK(hipMemcpy(out, b->d_stamps + (size_t)b->B * STAMP_WAVES * 16, (size_t)g * 16 * 8, hipMemcpyDeviceToHost));
  return g;
}

LPCNET_EXPORT int lpcnet_batch_set_trace(LPCNetBatch *b, int enable)
{
  if (!b) return -1;
  b->trace = enable != 0;
  return 0;
}

LPCNET_EXPORT int lpcnet_batch_get_trace(LPCNetBatch *b, float *logits, int *exc)
{
  if (!b || !b->trace || !b->d_trace_logits || b->set_device()) return -1;
  HIPCHK(hipStreamSynchronize(b->stream));
  int N = b->trace_N;
  if (logits) HIPCHK(hipMemcpy(logits, b->d_trace_logits, sizeof(float) * 8 * N * b->B, hipMemcpyDeviceToHost));
  if (exc) HIPCHK(hipMemcpy(exc, b->d_trace_exc, sizeof(int) * N * b->B, hipMemcpyDeviceToHost));
  return 0;
}

LPCNET_EXPORT int lpcnet_batch_get_state(LPCNetBatch *b, int stream, float *gru_a_cond, float *gru_b_cond, float *lpc,
                                         float *gru_a_state, float *gru_b_state, int *frame_count)
{
  if (!b || stream < 0 || stream >= b->B || b->set_device()) return -1;
  StreamState s;
  HIPCHK(hipStreamSynchronize(b->stream));
  HIPCHK(hipMemcpy(&s, &b->d_state[stream], sizeof(s), hipMemcpyDeviceToHost));
  if (gru_a_cond) memcpy(gru_a_cond, s.gru_a_cond, sizeof(s.gru_a_cond));
  if (gru_b_cond) memcpy(gru_b_cond, s.gru_b_cond, sizeof(s.gru_b_cond));
  if (lpc) memcpy(lpc, s.lpc, sizeof(s.lpc));
  if (gru_a_state) memcpy(gru_a_state, s.gru_a_state, sizeof(s.gru_a_state));
  if (gru_b_state) memcpy(gru_b_state, s.gru_b_state, sizeof(s.gru_b_state));
  if (frame_count) *frame_count = s.frame_count;
  return 0;
}

/* ======================================================================== */
/* drop-in single-stream API (include/lpcnet.h)                              */

/* The drop-in handles share the GPU.  Every LPCNetState bound to the same
 * model (blob bytes, resolved model constants) on the same device is a slot
 * of one StatePool: one device copy of the model, the slots' stream states
 * in one device array, and one work batch.  Concurrent calls on different
 * handles coalesce into one launch (flat combining: the first caller to find
 * the pool idle runs every request pending at that moment that has the same
 * shape -- the slots' states are gathered into the work batch, one step
 * runs, the states are scattered back), so K reference-style callers on K
 * threads get batch-K launches instead of K batch-1 engines.  Each handle's
 * results are those of its own stream alone (streams of a batch are
 * independent), i.e. the reference's. */
struct StatePool {
  /* what a request runs on its slot */
  enum Kind {
    SYNTH = 0, /* lpcnet_synthesize_impl (lpcnet.c:273-277): frame + N samples, `preload` teacher-forced */
    TAIL = 1,  /* lpcnet_synthesize_tail_impl (lpcnet.c:235-271): samples only */
    FLUSH = 2, /* run_frame_network_flush (lpcnet.c:134-144): nfr frames, conditioning discarded */
    DECODE = 3 /* lpcnet_decode (lpcnet.c:310-319): one 8-byte packet -> 4 frames */
  };
  struct Req {
    int slot;
    int kind;
    const float *feat;           /* SYNTH [NF], FLUSH [nfr][NF] */
    const unsigned char *packet; /* DECODE [8] */
    short *out;                  /* SYNTH / TAIL [N] (the first `preload` are input), DECODE [4 * FRAME] */
    int N, preload, nfr;
    int rc = 0;
    std::string err;
    Req *next = nullptr;          /* the pool's inbox (a lock-free stack) */
    /* REQ_WAITING -> REQ_DONE (rc / err set) or REQ_COMBINE (the caller now
     * holds the pool): the caller sleeps on this word (futex), the notifier
     * stores it last */
    std::atomic<uint32_t> state{0};
    bool same_shape(const Req &o) const { return kind == o.kind && N == o.N && preload == o.preload && nfr == o.nfr; }
  };
  /* the work batch (its HIP stream) and its staging, driven by the combiner */
  struct Lane {
    LPCNetBatch *work = nullptr; /* work->B >= the largest coalesced call */
    int *d_map = nullptr;        /* [map_cap] work-batch stream -> slot */
    int map_cap = 0;
    /* pinned host staging of a launch ([map_cap] entries each), so the
     * copies are truly asynchronous: slot map, features, PCM */
    int *h_map = nullptr;
    float *h_feat = nullptr;
    short *h_pcm = nullptr;
  };
  uint64_t key = 0;
  int device = 0;
  int place = 0; /* placement index (g_pools key) */
  std::vector<unsigned char> blob;
  bool has_codebooks = false;
  Lane lane;
  StreamState *d_slots = nullptr;
  int cap = 0;
  std::vector<int> free_slots;
  int refs = 0; /* handles bound + transient acquisitions; changed under g_pools_mu only */
  std::mutex mu; /* slot bookkeeping (taken with the pool idle: PoolIdle) */
  /* Submission is lock-free: a request is pushed on `inbox` and its caller
   * either takes `busy` (0 -> 1) and combines, or sleeps on its request until
   * a combiner completes it or hands it the pool.  The combiner alone drains
   * the inbox, runs the launch and updates expect_n. */
  std::atomic<StatePool::Req *> inbox{nullptr};
  std::atomic<uint32_t> busy{0};       /* 1: a combiner or a slot I/O holds the pool */
  std::atomic<int> io_waiting{0};      /* slot I/O callers waiting: no new combiner takes the pool */
  std::atomic<uint32_t> arrivals{0};   /* requests pushed and not drained yet */
  std::atomic<uint32_t> win_target{0}; /* a combiner waits for this many arrivals (0: none waits) */
  int expect_n = 0;                    /* requests of the previous launch (combiner-owned) */
  /* broadcast wake-ups (LPCNET_POOL_BROADCAST): waiters sleep on wake_seq,
   * the combiner marks its completed requests and wakes them all at once */
  bool broadcast = false;
  std::atomic<uint32_t> wake_seq{0};
  int window_us = 0;                   /* LPCNET_POOL_WINDOW_US */
  /* statistics (tests / diagnostics) */
  std::atomic<long> launches{0}, requests{0};
  std::atomic<long long> run_ns{0}; /* time inside pool_run (the launches themselves) */
};

static std::mutex g_pools_mu;
/* (model key, placement) -> pool: one pool per model per placement, so
 * handles spread over devices (and, for tests, over several placements of
 * one device) never share a launch across placements */
static std::map<std::pair<uint64_t, int>, StatePool *> g_pools;

/* Gather window of a combiner: before its launch it waits up to this long
 * (plus 2 us per caller expected) until as many requests have arrived as the
 * previous launch carried (a thread calling lpcnet_synthesize in a loop is
 * back within microseconds), so K looping callers keep launching together
 * instead of settling into half-size launches that alternate.  Callers that
 * stopped cost one window once: the next launch expects only those that
 * came. */
#ifndef POOL_WINDOW_US_DEFAULT
#define POOL_WINDOW_US_DEFAULT 200
#endif


static uint64_t pool_key(const unsigned char *data, int len)
{
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](const void *p, size_t n) {
    for (size_t k = 0; k < n; k++) h = (h ^ ((const unsigned char *)p)[k]) * 1099511628211ull;
  };
  mix(data, (size_t)len);
  mix(&len, sizeof(len));
  /* load-time overrides change the model bound to the same bytes */
  for (const char *e : {"LPCNET_LPC_GAMMA", "LPCNET_FEATURES_DELAY", "LPCNET_END2END", "LPCNET_KERNEL", "LPCNET_RCP"}) {
    const char *v = getenv(e);
    mix(e, strlen(e));
    if (v) mix(v, strlen(v));
  }
  return h;
}

/* the pool of (blob, placement), created with its model on first use; refs+1 */
static StatePool *pool_acquire(const unsigned char *data, int len, int device, int place)
{
  if (!data || len <= 0) { set_err("lpcnet_load_model: empty blob"); return nullptr; }
  const uint64_t key = pool_key(data, len);
  std::lock_guard<std::mutex> lk(g_pools_mu);
  auto it = g_pools.find({key, place});
  if (it != g_pools.end() && it->second->blob.size() == (size_t)len && !memcmp(it->second->blob.data(), data, len)) {
    it->second->refs++;
    return it->second;
  }
  if (it != g_pools.end()) {
    /* a different blob with the same 64-bit key: refuse rather than mix models */
    set_err("lpcnet_load_model: model pool key collision between two different blobs");
    return nullptr;
  }
  LPCNetBatch *w = lpcnet_batch_create(1, device);
  if (!w) return nullptr;
  if (lpcnet_batch_load_model(w, data, len)) {
    const std::string e = g_err;
    lpcnet_batch_destroy(w);
    set_err(e);
    return nullptr;
  }
  StatePool *p = new StatePool();
  p->key = key;
  p->device = device;
  p->place = place;
  p->blob.assign(data, data + len);
  p->has_codebooks = w->has_codebooks;
  p->lane.work = w;
  p->refs = 1;
  if (const char *v = getenv("LPCNET_POOL_BROADCAST")) p->broadcast = atoi(v) != 0;
  if (const char *v = getenv("LPCNET_POOL_WINDOW_US")) p->window_us = std::max(0, atoi(v));
  else p->window_us = POOL_WINDOW_US_DEFAULT;
  g_pools[{key, place}] = p;
  return p;
}

/* Per-request wake-up: the caller sleeps on its request's state word, the
 * notifier stores the word (release) and wakes that one thread -- one
 * syscall, no lock the woken thread has to take.  The caller may return as
 * soon as it sees the store, so the wake can land on a word whose frame is
 * gone: a futex wake on a stale address wakes at most a waiter that rechecks
 * its own condition, or fails with EFAULT, both harmless. */
enum : uint32_t { REQ_WAITING = 0, REQ_DONE = 1, REQ_COMBINE = 2 };

static void futex_wake(std::atomic<uint32_t> *w, int n)
{
  syscall(SYS_futex, (uint32_t *)w, FUTEX_WAKE_PRIVATE, n, nullptr, nullptr, 0);
}

/* sleep while *w == v, at most `ns` nanoseconds (0: no limit) */
static void futex_wait(std::atomic<uint32_t> *w, uint32_t v, long long ns = 0)
{
  struct timespec ts;
  if (ns > 0) {
    ts.tv_sec = (time_t)(ns / 1000000000);
    ts.tv_nsec = (long)(ns % 1000000000);
  }
  syscall(SYS_futex, (uint32_t *)w, FUTEX_WAIT_PRIVATE, v, ns > 0 ? &ts : nullptr, nullptr, 0);
}

static void req_post(StatePool *p, StatePool::Req *q, uint32_t v)
{
  std::atomic<uint32_t> *w = &q->state;
  w->store(v, std::memory_order_release);
  if (p->broadcast) {
    p->wake_seq.fetch_add(1, std::memory_order_release);
    futex_wake(&p->wake_seq, INT32_MAX);
  } else {
    futex_wake(w, 1);
  }
}

/* r's state once it leaves `from` */
static uint32_t req_wait(StatePool *p, StatePool::Req &r, uint32_t from = REQ_WAITING)
{
  uint32_t v;
  if (p->broadcast) {
    for (;;) {
      const uint32_t seq = p->wake_seq.load(std::memory_order_acquire);
      if ((v = r.state.load(std::memory_order_acquire)) != from) return v;
      futex_wait(&p->wake_seq, seq);
    }
  }
  while ((v = r.state.load(std::memory_order_acquire)) == from) futex_wait(&r.state, from);
  return v;
}

static void inbox_push(StatePool *p, StatePool::Req *q)
{
  StatePool::Req *h = p->inbox.load(std::memory_order_relaxed);
  do q->next = h;
  /* seq_cst: pairs with pool_let_go's busy = 0 / inbox re-load (a
   * store-then-load hand-off on both sides; release alone would let the
   * let-go miss this push while our busy CAS still sees it held) */
  while (!p->inbox.compare_exchange_weak(h, q, std::memory_order_seq_cst, std::memory_order_relaxed));
}

/* The holder of `busy` lets go: to the slot I/O callers waiting, else to the
 * caller of the newest inbox request (REQ_COMBINE: `busy` stays held on its
 * behalf; no one else drains the inbox meanwhile), else to no one -- with a
 * recheck, since a request pushed just before the release found the pool
 * busy and sleeps. */
static void pool_let_go(StatePool *p)
{
  for (;;) {
    if (p->io_waiting.load(std::memory_order_acquire) > 0) {
      p->busy.store(0, std::memory_order_release);
      futex_wake(&p->busy, INT32_MAX);
      return;
    }
    StatePool::Req *h = p->inbox.load(std::memory_order_acquire);
    if (h) {
      req_post(p, h, REQ_COMBINE);
      return;
    }
    p->busy.store(0, std::memory_order_seq_cst);
    if (!p->inbox.load(std::memory_order_seq_cst)) return;
    uint32_t b = 0;
    if (!p->busy.compare_exchange_strong(b, 1, std::memory_order_seq_cst)) return; /* another caller took it */
  }
}

/* Slot I/O on an idle pool (lock held for the slot bookkeeping): takes
 * `busy` -- meanwhile no new combiner takes the pool, so a stream of
 * synthesis calls cannot starve it -- and on scope exit lets go (to any
 * requests that arrived meanwhile).  No combiner takes p->mu, so holding it
 * while waiting cannot deadlock. */
struct PoolIdle {
  StatePool *p;
  PoolIdle(StatePool *p_, std::unique_lock<std::mutex> &) : p(p_)
  {
    p->io_waiting.fetch_add(1, std::memory_order_seq_cst);
    for (;;) {
      uint32_t b = 0;
      if (p->busy.compare_exchange_strong(b, 1, std::memory_order_seq_cst)) break;
      futex_wait(&p->busy, 1, 1000000); /* woken by the combiner's let-go; re-polled every ms */
    }
    p->io_waiting.fetch_sub(1, std::memory_order_seq_cst);
  }
  ~PoolIdle() { pool_let_go(p); }
};

/* give back `slot` (if >= 0) and one reference; the last reference frees
 * the pool.  refs changes under g_pools_mu only, the lock pool_acquire holds
 * while it looks the pool up, so an acquisition and the last release can
 * never both succeed. */
static void pool_release(StatePool *p, int slot)
{
  if (slot >= 0) {
    std::unique_lock<std::mutex> lk(p->mu);
    PoolIdle idle(p, lk);
    p->free_slots.push_back(slot);
  }
  {
    std::lock_guard<std::mutex> lk(g_pools_mu);
    if (--p->refs > 0) return;
    g_pools.erase({p->key, p->place});
  }
  /* unreachable now: no handle holds it and the map no longer lists it */
  if (hipSetDevice(p->device) == hipSuccess) {
    (void)hipFree(p->d_slots);
    (void)hipFree(p->lane.d_map);
    (void)hipHostFree(p->lane.h_map);
    (void)hipHostFree(p->lane.h_feat);
    (void)hipHostFree(p->lane.h_pcm);
  }
  if (p->lane.work) lpcnet_batch_destroy(p->lane.work);
  delete p;
}

/* a free slot holding `init` (a reset state when null); -1 on failure */
static int pool_alloc_slot(StatePool *p, const StreamState *init)
{
  std::unique_lock<std::mutex> lk(p->mu);
  PoolIdle idle(p, lk);
  if (hipSetDevice(p->device) != hipSuccess) { set_err("hipSetDevice failed"); return -1; }
  if (p->free_slots.empty()) {
    const int ncap = std::max(4, 2 * p->cap);
    StreamState *d = nullptr;
    if (hipMalloc(&d, sizeof(StreamState) * (size_t)ncap) != hipSuccess) { set_err("device allocation failed"); return -1; }
    if (p->cap && hipMemcpy(d, p->d_slots, sizeof(StreamState) * (size_t)p->cap, hipMemcpyDeviceToDevice) != hipSuccess) {
      (void)hipFree(d);
      set_err("device copy failed");
      return -1;
    }
    (void)hipFree(p->d_slots);
    p->d_slots = d;
    for (int k = ncap - 1; k >= p->cap; k--) p->free_slots.push_back(k);
    p->cap = ncap;
  }
  const int slot = p->free_slots.back();
  StreamState s;
  if (init) s = *init;
  else host_reset_state(s);
  if (hipMemcpy(&p->d_slots[slot], &s, sizeof(s), hipMemcpyHostToDevice) != hipSuccess) { set_err("device copy failed"); return -1; }
  p->free_slots.pop_back();
  return slot;
}

static int pool_slot_io(StatePool *p, int slot, StreamState *get, const StreamState *put)
{
  std::unique_lock<std::mutex> lk(p->mu);
  PoolIdle idle(p, lk);
  if (hipSetDevice(p->device) != hipSuccess) { set_err("hipSetDevice failed"); return -1; }
  if (get && hipMemcpy(get, &p->d_slots[slot], sizeof(*get), hipMemcpyDeviceToHost) != hipSuccess) {
    set_err("device copy failed");
    return -1;
  }
  if (put && hipMemcpy(&p->d_slots[slot], put, sizeof(*put), hipMemcpyHostToDevice) != hipSuccess) {
    set_err("device copy failed");
    return -1;
  }
  return 0;
}

/* one coalesced step for requests rq (all of the same shape); the combiner
 * alone touches L */
static int pool_run(StatePool *p, StatePool::Lane &L, const std::vector<StatePool::Req *> &rq)
{
  const int n = (int)rq.size();
  const StatePool::Req &r0 = *rq[0];
  const int N = r0.N;
  if (!L.work || L.work->B < n) {
    int nb = 1;
    while (nb < n) nb *= 2;
    LPCNetBatch *w = lpcnet_batch_create(nb, p->device);
    if (!w) return -1;
    if (lpcnet_batch_load_model(w, p->blob.data(), (int)p->blob.size())) {
      lpcnet_batch_destroy(w);
      return -1;
    }
    if (L.work) lpcnet_batch_destroy(L.work);
    L.work = w;
  }
  LPCNetBatch *w = L.work;
  if (w->set_device()) return -1;
  if (L.map_cap < n) {
    (void)hipFree(L.d_map);
    (void)hipHostFree(L.h_map);
    (void)hipHostFree(L.h_feat);
    (void)hipHostFree(L.h_pcm);
    L.d_map = nullptr;
    L.h_map = nullptr;
    L.h_feat = nullptr;
    L.h_pcm = nullptr;
    L.map_cap = 0;
    HIPCHK(hipMalloc(&L.d_map, sizeof(int) * (size_t)w->B));
    HIPCHK(hipHostMalloc(&L.h_map, sizeof(int) * (size_t)w->B, hipHostMallocDefault));
    HIPCHK(hipHostMalloc(&L.h_feat, sizeof(float) * NF * (size_t)w->B, hipHostMallocDefault));
    HIPCHK(hipHostMalloc(&L.h_pcm, sizeof(short) * 4 * FRAME * (size_t)w->B, hipHostMallocDefault));
    L.map_cap = w->B;
  }
  float *feat = L.h_feat;
  short *pcm = L.h_pcm;
  const int nout = r0.kind == StatePool::DECODE ? 4 * FRAME : N;
  /* a synthesis step's inputs go first, so the copy engine's work precedes
   * every kernel of the launch (one copy -> kernel hand-over instead of two) */
  const bool staged = r0.kind == StatePool::SYNTH;
  if (staged) {
    for (int k = 0; k < n; k++) {
      memcpy(&feat[(size_t)k * NF], rq[k]->feat, sizeof(float) * NF);
      if (r0.preload > 0) memcpy(&pcm[(size_t)k * N], rq[k]->out, sizeof(short) * std::min(r0.preload, N));
    }
    HIPCHK(hipMemcpyAsync(w->d_feat, feat, sizeof(float) * NF * n, hipMemcpyHostToDevice, w->stream));
    if (r0.preload > 0 && N > 0)
      HIPCHK(hipMemcpyAsync(w->d_pcm, pcm, sizeof(short) * N * n, hipMemcpyHostToDevice, w->stream));
  }
  for (int k = 0; k < n; k++) L.h_map[k] = rq[k]->slot;
  HIPCHK(hipMemcpyAsync(L.d_map, L.h_map, sizeof(int) * n, hipMemcpyHostToDevice, w->stream));
  if (launch_state_copy(w->d_state, p->d_slots, nullptr, L.d_map, n, w->stream)) { set_err("state gather failed"); return -1; }
  /* every stream of the work batch is this call's: the multi-frame bound is its min */
  w->min_fc = 0;
  /* the states go back to their slots right behind the step's kernels, before
   * its one synchronisation */
  const PreSync scatter = [&]() -> int {
    if (launch_state_copy(p->d_slots, w->d_state, L.d_map, nullptr, n, w->stream)) {
      set_err("state scatter failed");
      return -1;
    }
    return 0;
  };
  int rc = 0;
  switch (r0.kind) {
  case StatePool::SYNTH:
  case StatePool::TAIL:
    if (!staged)
      for (int k = 0; k < n; k++) {
        if (r0.kind == StatePool::SYNTH) memcpy(&feat[(size_t)k * NF], rq[k]->feat, sizeof(float) * NF);
        if (r0.preload > 0) memcpy(&pcm[(size_t)k * N], rq[k]->out, sizeof(short) * std::min(r0.preload, N));
      }
    rc = r0.kind == StatePool::SYNTH ? synth_first(w, n, feat, pcm, N, r0.preload, scatter, staged)
                                     : tail_first(w, n, pcm, N, r0.preload, scatter);
    break;
  case StatePool::FLUSH:
    for (int j = 0; j < r0.nfr && rc == 0; j++) {
      for (int k = 0; k < n; k++) memcpy(&feat[(size_t)k * NF], rq[k]->feat + (size_t)j * NF, sizeof(float) * NF);
      rc = frame_first(w, n, feat, true, j + 1 == r0.nfr ? scatter : PreSync());
    }
    break;
  case StatePool::DECODE: {
    std::vector<unsigned char> pk((size_t)n * 8);
    for (int k = 0; k < n; k++) memcpy(&pk[(size_t)k * 8], rq[k]->packet, 8);
    rc = decode_first(w, n, pk.data(), pcm, scatter);
    break;
  }
  default:
    set_err("bad request");
    rc = -1;
  }
  if (rc == 0)
    for (int k = 0; k < n; k++)
      if (nout > 0 && r0.kind != StatePool::FLUSH) memcpy(rq[k]->out, &pcm[(size_t)k * nout], sizeof(short) * nout);
  return rc;
}

/* Flat combining with a hand-off, lock-free on the submission side: the
 * caller pushes its request and either takes the idle pool or sleeps on its
 * request.  The combiner waits (the gather window) until as many requests
 * have arrived as the previous launch carried, drains the inbox, runs every
 * request of the oldest one's shape, wakes exactly the callers it completed,
 * and lets the pool go -- to the newest pending request's caller if any (the
 * GPU idles until it launches).  No mutex on this path: with hundreds of C
 * threads, waking callers that then queue on one lock costs more than the
 * launch. */
static int pool_combine(StatePool *p, StatePool::Req &r)
{
  while (r.state.load(std::memory_order_acquire) != REQ_DONE) {
    const int expect = p->expect_n;
    if (p->window_us > 0 && expect > 1 && (int)p->arrivals.load(std::memory_order_acquire) < expect) {
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(p->window_us + 2 * expect);
      p->win_target.store((uint32_t)expect, std::memory_order_seq_cst);
      for (;;) {
        const uint32_t a = p->arrivals.load(std::memory_order_seq_cst);
        if ((int)a >= expect) break;
        const long long left = std::chrono::duration_cast<std::chrono::nanoseconds>(until - std::chrono::steady_clock::now()).count();
        if (left <= 0) break;
        futex_wait(&p->arrivals, a, left);
      }
      p->win_target.store(0, std::memory_order_relaxed);
    }
    /* drain: the stack reversed is arrival order */
    StatePool::Req *h = p->inbox.exchange(nullptr, std::memory_order_acquire);
    std::vector<StatePool::Req *> all;
    for (; h; h = h->next) all.push_back(h);
    if (all.empty()) {
      /* r ran in the launch of the combiner that let the pool go to us: it
       * still posts r's completion, so r's frame must outlive that store */
      /* r's state is read once: the other combiner may post REQ_DONE at any
       * moment, and waiting "while state == DONE" would never end */
      const uint32_t s = r.state.load(std::memory_order_acquire);
      pool_let_go(p);
      if (s != REQ_DONE) req_wait(p, r, s);
      if (r.rc) set_err(r.err);
      return r.rc;
    }
    std::reverse(all.begin(), all.end());
    p->arrivals.fetch_sub((uint32_t)all.size(), std::memory_order_acq_rel);
    std::vector<StatePool::Req *> mine, rest;
    for (StatePool::Req *q : all) (q->same_shape(*all[0]) ? mine : rest).push_back(q);
    /* oldest first onto the stack: the next drain's reversal gives arrival
     * order again */
    for (auto it = rest.begin(); it != rest.end(); ++it) {
      inbox_push(p, *it);
      p->arrivals.fetch_add(1, std::memory_order_acq_rel);
    }
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = pool_run(p, p->lane, mine);
    const std::string e = rc ? g_err : std::string();
    p->run_ns.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
    p->launches.fetch_add(1);
    p->requests.fetch_add((long)mine.size());
    p->expect_n = (int)mine.size();
    bool self = false;
    for (StatePool::Req *q : mine) {
      q->rc = rc;
      q->err = e;
      if (q == &r) self = true;
    }
    if (self) r.state.store(REQ_DONE, std::memory_order_release);
    /* the next launch first (the GPU idles until it starts), then the
     * wake-ups: one futex call per completed caller */
    auto post_all = [&]() {
      if (p->broadcast) {
        bool any = false;
        for (StatePool::Req *q : mine)
          if (q != &r) {
            q->state.store(REQ_DONE, std::memory_order_release);
            any = true;
          }
        if (any) {
          p->wake_seq.fetch_add(1, std::memory_order_release);
          futex_wake(&p->wake_seq, INT32_MAX);
        }
      } else {
        for (StatePool::Req *q : mine)
          if (q != &r) req_post(p, q, REQ_DONE);
      }
    };
    if (self) {
      pool_let_go(p);
      post_all();
      if (r.rc) set_err(r.err);
      return r.rc;
    }
    post_all();
  }
  pool_let_go(p);
  if (r.rc) set_err(r.err);
  return r.rc;
}

static int pool_submit(StatePool *p, StatePool::Req &r)
{
  inbox_push(p, &r);
  const uint32_t a = p->arrivals.fetch_add(1, std::memory_order_seq_cst) + 1;
  const uint32_t t = p->win_target.load(std::memory_order_seq_cst);
  if (t && a >= t) futex_wake(&p->arrivals, 1);
  if (p->io_waiting.load(std::memory_order_seq_cst) == 0) {
    uint32_t b = 0;
    if (p->busy.compare_exchange_strong(b, 1, std::memory_order_seq_cst)) return pool_combine(p, r);
  }
  if (req_wait(p, r) == REQ_DONE) {
    if (r.rc) set_err(r.err);
    return r.rc;
  }
  return pool_combine(p, r); /* REQ_COMBINE: the pool was handed over */
}

/* ---- handles -------------------------------------------------------------
 * An LPCNetState is caller memory (lpcnet_get_size + malloc, calloc through
 * lpcnet_create, or embedded in a larger struct as the reference's decoder
 * and PLC states embed theirs).  It holds a magic word and a 64-bit token;
 * everything else -- device, bound pool and slot, the deferred feature
 * buffer -- lives in a Handle found through the registry, so nothing read
 * from caller memory is ever dereferenced.  A registry entry whose token
 * does not match the memory at its address is stale (the memory was freed
 * without lpcnet_destroy / lpcnet_mi355x_deinit and reused): lpcnet_init
 * there drops it, releasing its slot, and starts a fresh handle. */
struct LPCNetState {
  uint32_t magic;
  uint32_t reserved;
  uint64_t token;
};
static const uint32_t kMagic = 0x4c50434eu; /* "LPCN" */

constexpr int MAX_FEATURE_BUFFER = 4; /* lpcnet_private.h:26 MAX_FEATURE_BUFFER_SIZE */

struct Handle {
  uint64_t token = 0;
  int device = 0;
  int place = 0;     /* placement index: auto placements 0.., LPCNET_DEVICE pins kPinned + device */
  unsigned place_gen = 0; /* generation of the placement list it was counted in */
  StatePool *pool = nullptr; /* bound model (nullptr: none) */
  int slot = -1;
  /* run_frame_network_deferred's buffer (lpcnet_private.h:37-38, lpcnet.c:122-132) */
  int fbuf_fill = 0;
  float fbuf[MAX_FEATURE_BUFFER][NF] = {};
};

/* A handle's complete synthesis state: lpcnet_mi355x_state_save/restore, the
 * replacement of the LPCNetState struct copies of lpcnet_plc.c:223,230. */
struct HandleSnapshot {
  StreamState s;
  int fbuf_fill;
  float fbuf[MAX_FEATURE_BUFFER][NF];
};

static_assert(sizeof(HandleSnapshot) <= LPCNET_MI355X_STATE_MAX, "LPCNET_MI355X_STATE_MAX too small");

/* the registry, sharded by address: every lpcnet_synthesize looks its
 * handle up, and one lock would serialise hundreds of calling threads */
struct LiveShard {
  std::mutex mu;
  std::unordered_map<const LPCNetState *, Handle *> map;
};
static LiveShard g_live[64];
static LiveShard &live_shard(const LPCNetState *st)
{
  const uint64_t a = (uint64_t)(uintptr_t)st;
  return g_live[((a >> 4) ^ (a >> 10) ^ (a >> 16)) & 63];
}

static uint64_t new_token()
{
  static std::atomic<uint64_t> ctr{0};
  static const uint64_t salt = (uint64_t)(uintptr_t)&ctr ^ ((uint64_t)time(nullptr) << 20);
  uint64_t z = (ctr.fetch_add(1) + 1) * 0x9E3779B97F4A7C15ull ^ salt; /* splitmix64 */
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z ? z : 1;
}

/* the live handle at st, or nullptr */
static Handle *live_handle(const LPCNetState *st)
{
  if (!st) return nullptr;
  LiveShard &sh = live_shard(st);
  std::lock_guard<std::mutex> lk(sh.mu);
  auto it = sh.map.find(st);
  if (it == sh.map.end() || st->magic != kMagic || st->token != it->second->token) return nullptr;
  return it->second;
}

/* ---- placement of drop-in handles over the visible GPUs ------------------
 * The reference's lpcnet_init/lpcnet_create take no device (lpcnet.c:184-219),
 * so placement is library policy.  By default every handle goes to one
 * device: LOCAL_RANK mod the device count in a one-process-per-GPU job
 * (torchrun ranks), device 0 otherwise -- resolved when a model is first
 * bound, so lpcnet_init/lpcnet_create never start the HIP runtime.
 * Spreading is opt-in: LPCNET_DEVICES="0,1,..." (or "all") or
 * lpcnet_mi355x_set_placement() name a list of placements, and each new
 * handle goes to the placement with the fewest live handles (one slot each
 * once a model is bound).  A list may name a device twice: two placements,
 * two pools, one GPU (the tests use this to exercise placement on a one-GPU
 * box).  LPCNET_DEVICE=d pins every new handle to device d. */
constexpr int kMaxPlace = 64;
constexpr int kPinned = 1 << 20;
constexpr int kDevDefault = -1; /* placement device resolved at the first model bind */
static std::mutex g_place_mu;
static std::vector<int> g_place_dev; /* placement -> device (empty: not set up yet) */
static int g_place_load[kMaxPlace];  /* live handles per placement (of generation g_place_gen) */
static unsigned g_place_gen = 1;     /* bumped by lpcnet_mi355x_set_placement */

static bool parse_device_list(const char *v, std::vector<int> &out)
{
  out.clear();
  while (v && *v) {
    char *end = nullptr;
    const long d = strtol(v, &end, 10);
    if (end == v || d < 0 || d > 1023) return false;
    out.push_back((int)d);
    v = end;
    while (*v == ',' || *v == ' ') v++;
  }
  return !out.empty() && out.size() <= (size_t)kMaxPlace;
}

/* the device of the default placement (starts the HIP runtime only under
 * LOCAL_RANK, to take the rank's device modulo the visible count) */
static int default_device()
{
  const char *lr = getenv("LOCAL_RANK");
  if (!lr || !*lr) return 0;
  const int r = atoi(lr), n = lpcnet_mi355x_device_count();
  return n > 0 && r > 0 ? r % n : 0;
}

/* the placement of a new handle (g_place_mu held); -1 (error set) when
 * LPCNET_DEVICES is malformed or names a device that is not visible */
static int place_new_handle(Handle *h)
{
  h->place_gen = g_place_gen;
  if (const char *d = getenv("LPCNET_DEVICE")) {
    h->device = atoi(d);
    h->place = kPinned + h->device;
    return 0;
  }
  if (g_place_dev.empty()) {
    const char *env = getenv("LPCNET_DEVICES");
    if (env && *env) {
      /* opt-in spreading: the list is checked against the visible devices
       * here, as lpcnet_mi355x_set_placement checks its own */
      std::vector<int> list;
      const int ndev = lpcnet_mi355x_device_count();
      if (strcmp(env, "all") == 0) {
        for (int k = 0; k < std::min(std::max(ndev, 1), kMaxPlace); k++) list.push_back(k);
      } else if (!parse_device_list(env, list)) {
        set_err("LPCNET_DEVICES: expected \"all\" or a comma-separated list of at most 64 device indices");
        return -1;
      }
      for (int d : list)
        if (d >= std::max(ndev, 1)) {
          set_err("LPCNET_DEVICES: device index outside the visible devices");
          return -1;
        }
      g_place_dev = list;
    } else {
      g_place_dev.assign(1, kDevDefault);
    }
  }
  int best = 0;
  for (int k = 1; k < (int)g_place_dev.size(); k++)
    if (g_place_load[k] < g_place_load[best]) best = k;
  g_place_load[best]++;
  h->place = best;
  h->device = g_place_dev[best];
  return 0;
}

static void unplace_handle(const Handle *h)
{
  std::lock_guard<std::mutex> lk(g_place_mu);
  if (h->place_gen == g_place_gen && h->place >= 0 && h->place < kMaxPlace && g_place_load[h->place] > 0)
    g_place_load[h->place]--;
}

static void handle_free(Handle *h)
{
  if (h->pool) pool_release(h->pool, h->slot);
  unplace_handle(h);
  delete h;
}

LPCNET_EXPORT int lpcnet_mi355x_set_placement(const int *devices, int n)
{
  if (n < 0 || n > kMaxPlace || (n > 0 && !devices)) { set_err("lpcnet_mi355x_set_placement: 0..64 devices"); return -1; }
  const int ndev = lpcnet_mi355x_device_count();
  for (int k = 0; k < n; k++)
    if (devices[k] < 0 || (ndev > 0 && devices[k] >= ndev)) {
      set_err("lpcnet_mi355x_set_placement: device index outside the visible devices");
      return -1;
    }
  /* live handles keep their device and pool; only handles initialised from
   * now on are counted against (and placed over) the new list */
  std::lock_guard<std::mutex> lk(g_place_mu);
  for (int k = 0; k < kMaxPlace; k++) g_place_load[k] = 0;
  g_place_gen++;
  g_place_dev.assign(devices, devices + n); /* n = 0: back to the default */
  return 0;
}

/* unregister st (if live) and release its device resources */
static void handle_deinit(LPCNetState *st)
{
  Handle *h = nullptr;
  {
    LiveShard &sh = live_shard(st);
    std::lock_guard<std::mutex> lk(sh.mu);
    auto it = sh.map.find(st);
    if (it != sh.map.end() && st->magic == kMagic && st->token == it->second->token) {
      h = it->second;
      sh.map.erase(it);
    }
  }
  if (h) handle_free(h);
  /* a later malloc may hand this block out again: leave nothing that looks live */
  st->magic = 0;
  st->token = 0;
}

LPCNET_EXPORT int lpcnet_get_size(void) { return (int)sizeof(LPCNetState); }

LPCNET_EXPORT int lpcnet_init(LPCNetState *st)
{
  if (!st) return -1;
  Handle *stale = nullptr, *live = nullptr;
  bool failed = false;
  {
    LiveShard &sh = live_shard(st);
    std::lock_guard<std::mutex> lk(sh.mu);
    auto it = sh.map.find(st);
    if (it != sh.map.end()) {
      if (st->magic == kMagic && st->token == it->second->token) {
        live = it->second;
      } else {
        stale = it->second;
        sh.map.erase(it);
      }
    }
    if (!live) {
      Handle *h = new Handle();
      h->token = new_token();
      int prc;
      {
        std::lock_guard<std::mutex> plk(g_place_mu);
        prc = place_new_handle(h);
      }
      if (prc) {
        delete h;
        st->magic = 0;
        st->token = 0;
        failed = true;
      } else {
        sh.map[st] = h;
        st->magic = kMagic;
        st->reserved = 0;
        st->token = h->token;
      }
    }
  }
  if (stale) handle_free(stale);
  if (failed) return -1;
  if (live) {
    /* src/lpcnet.c:184-200 ends with lpcnet_reset(): re-initialising a live
     * handle resets its stream and keeps its device binding and model */
    live->fbuf_fill = 0;
    if (live->pool) {
      StreamState s;
      host_reset_state(s);
      if (pool_slot_io(live->pool, live->slot, nullptr, &s)) return -1;
    }
  }
  return 0;
}

LPCNET_EXPORT LPCNetState *lpcnet_create(void)
{
  LPCNetState *st = (LPCNetState *)calloc(1, sizeof(LPCNetState));
  if (st && lpcnet_init(st) != 0) {
    free(st);
    return nullptr;
  }
  return st;
}

LPCNET_EXPORT void lpcnet_destroy(LPCNetState *st)
{
  if (!st) return;
  handle_deinit(st);
  free(st);
}

LPCNET_EXPORT void lpcnet_mi355x_deinit(LPCNetState *st)
{
  if (st) handle_deinit(st);
}

LPCNET_EXPORT void lpcnet_reset(LPCNetState *st)
{
  Handle *h = live_handle(st);
  if (!h) return;
  h->fbuf_fill = 0; /* lpcnet.c:177-179 clears from LPCNET_RESET_START, the feature buffer included */
  if (!h->pool) return;
  StreamState s;
  host_reset_state(s);
  pool_slot_io(h->pool, h->slot, nullptr, &s);
}

LPCNET_EXPORT int lpcnet_load_model(LPCNetState *st, const unsigned char *data, int len)
{
  Handle *h = live_handle(st);
  if (!h) { set_err("lpcnet_load_model: not an initialised LPCNetState"); return -1; }
  if (h->device == kDevDefault) h->device = default_device();
  /* pools per (model, placement, device): a placement index of a later
   * list may name another device */
  StatePool *p = pool_acquire(data, len, h->device, h->place >= kPinned ? h->place : h->place * 1024 + h->device);
  if (!p) return -1;
  if (p == h->pool) {
    pool_release(p, -1); /* same model: keep the binding */
    return 0;
  }
  /* the model changes, the stream state stays (lpcnet.c:202-210 only binds arrays) */
  StreamState s;
  bool have = h->pool && pool_slot_io(h->pool, h->slot, &s, nullptr) == 0;
  const int slot = pool_alloc_slot(p, have ? &s : nullptr);
  if (slot < 0) {
    pool_release(p, -1);
    return -1;
  }
  if (h->pool) pool_release(h->pool, h->slot);
  h->pool = p;
  h->slot = slot;
  return 0;
}

/* run one request on st's slot; the void entry points report failure as the
 * reference cannot: silence out, lpcnet_mi355x_last_error(), one stderr line */
static int handle_run(LPCNetState *st, StatePool::Req &r, const char *what)
{
  Handle *h = live_handle(st);
  int rc;
  if (!h || !h->pool) {
    set_err(std::string(what) +
            ": no model bound (call lpcnet_load_model first; liblpcnet_mi355x has no compiled-in model)");
    rc = -1;
  } else {
    r.slot = h->slot;
    rc = pool_submit(h->pool, r);
  }
  if (rc != 0) {
    static std::atomic<bool> warned{false};
    const int nout = r.kind == StatePool::DECODE ? 4 * FRAME : r.N;
    if (r.out && nout > 0 && r.kind != StatePool::FLUSH) memset(r.out, 0, sizeof(short) * nout);
    if (!warned.exchange(true)) fprintf(stderr, "liblpcnet_mi355x: %s\n", g_err.c_str());
  }
  return rc;
}

static bool req_args_ok(const float *features, const short *output, int N, int preload, bool need_features)
{
  if (N < 0 || N > FRAME || (need_features && !features) || (N > 0 && !output) || preload < 0) {
    set_err("bad arguments");
    return false;
  }
  return true;
}

LPCNET_EXPORT void lpcnet_synthesize_impl(LPCNetState *st, const float *features, short *output, int N, int preload)
{
  if (!req_args_ok(features, output, N, preload, true)) return;
  StatePool::Req r{-1, StatePool::SYNTH, features, nullptr, output, N, std::min(preload, N), 0, 0, std::string()};
  handle_run(st, r, "lpcnet_synthesize_impl");
}

LPCNET_EXPORT void lpcnet_synthesize(LPCNetState *st, const float *features, short *output, int N)
{
  if (!req_args_ok(features, output, N, 0, true)) {
    if (output && N > 0 && N <= FRAME) memset(output, 0, sizeof(short) * N);
    return;
  }
  StatePool::Req r{-1, StatePool::SYNTH, features, nullptr, output, N, 0, 0, 0, std::string()};
  handle_run(st, r, "lpcnet_synthesize");
}

LPCNET_EXPORT void lpcnet_synthesize_tail_impl(LPCNetState *st, short *output, int N, int preload)
{
  if (!req_args_ok(nullptr, output, N, preload, false) || N == 0) return;
  StatePool::Req r{-1, StatePool::TAIL, nullptr, nullptr, output, N, std::min(preload, N), 0, 0, std::string()};
  handle_run(st, r, "lpcnet_synthesize_tail_impl");
}

/* lpcnet.c:122-132: keep the last kernel_size(conv1) + kernel_size(conv2) - 2
 * frames (4 for the 3-tap convolutions of every LPCNet model) */
LPCNET_EXPORT void run_frame_network_deferred(LPCNetState *st, const float *features)
{
  Handle *h = live_handle(st);
  if (!h || !features) return;
  if (h->fbuf_fill == MAX_FEATURE_BUFFER)
    memmove(h->fbuf[0], h->fbuf[1], sizeof(float) * NF * (MAX_FEATURE_BUFFER - 1));
  else
    h->fbuf_fill++;
  memcpy(h->fbuf[h->fbuf_fill - 1], features, sizeof(float) * NF);
}

/* lpcnet.c:134-144: the frame network of every buffered frame, outputs into
 * locals (the state's conditioning and LPC stay), then an empty buffer */
LPCNET_EXPORT void run_frame_network_flush(LPCNetState *st)
{
  Handle *h = live_handle(st);
  if (!h || h->fbuf_fill == 0) return;
  float f[MAX_FEATURE_BUFFER][NF];
  memcpy(f, h->fbuf, sizeof(f));
  StatePool::Req r{-1, StatePool::FLUSH, &f[0][0], nullptr, nullptr, 0, 0, h->fbuf_fill, 0, std::string()};
  h->fbuf_fill = 0;
  handle_run(st, r, "run_frame_network_flush");
}

/* lpcnet.c:226-233 */
LPCNET_EXPORT void lpcnet_reset_signal(LPCNetState *st)
{
  Handle *h = live_handle(st);
  if (!h || !h->pool) return;
  StreamState s;
  if (pool_slot_io(h->pool, h->slot, &s, nullptr)) return;
  reset_signal(s);
  pool_slot_io(h->pool, h->slot, nullptr, &s);
}

LPCNET_EXPORT int lpcnet_mi355x_handle_placement(const LPCNetState *st, int *device, int *placement)
{
  Handle *h = live_handle(st);
  if (!h) { set_err("not an initialised LPCNetState"); return -1; }
  /* before the first model bind the default placement's device is the one
   * lpcnet_load_model will take */
  if (device) *device = h->device == kDevDefault ? default_device() : h->device;
  if (placement) *placement = h->place >= kPinned ? -1 : h->place;
  return 0;
}

LPCNET_EXPORT int lpcnet_mi355x_state_size(void) { return (int)sizeof(HandleSnapshot); }

LPCNET_EXPORT int lpcnet_mi355x_state_save(LPCNetState *st, void *buf)
{
  Handle *h = live_handle(st);
  if (!h || !h->pool || !buf) { set_err("lpcnet_mi355x_state_save: no model bound or no buffer"); return -1; }
  HandleSnapshot snap;
  memset(&snap, 0, sizeof(snap));
  if (pool_slot_io(h->pool, h->slot, &snap.s, nullptr)) return -1;
  snap.fbuf_fill = h->fbuf_fill;
  memcpy(snap.fbuf, h->fbuf, sizeof(snap.fbuf));
  memcpy(buf, &snap, sizeof(snap));
  return 0;
}

LPCNET_EXPORT int lpcnet_mi355x_state_restore(LPCNetState *st, const void *buf)
{
  Handle *h = live_handle(st);
  if (!h || !h->pool || !buf) { set_err("lpcnet_mi355x_state_restore: no model bound or no buffer"); return -1; }
  HandleSnapshot snap;
  memcpy(&snap, buf, sizeof(snap));
  if (!snapshot_ok(&snap.s)) return -1;
  if (snap.fbuf_fill < 0 || snap.fbuf_fill > MAX_FEATURE_BUFFER) {
    set_err("snapshot feature buffer fill outside [0, 4]: not a state this engine produced");
    return -1;
  }
  if (pool_slot_io(h->pool, h->slot, nullptr, &snap.s)) return -1;
  h->fbuf_fill = snap.fbuf_fill;
  memcpy(h->fbuf, snap.fbuf, sizeof(h->fbuf));
  return 0;
}

LPCNET_EXPORT double lpcnet_mi355x_pool_run_ms(const LPCNetState *st)
{
  Handle *h = live_handle(st);
  if (!h || !h->pool) return -1.0;
  std::lock_guard<std::mutex> lk(h->pool->mu);
  return h->pool->run_ns.load() * 1e-6;
}

LPCNET_EXPORT int lpcnet_mi355x_pool_stats(const LPCNetState *st, long *launches, long *requests, int *streams)
{
  Handle *h = live_handle(st);
  if (!h || !h->pool) return -1;
  StatePool *p = h->pool;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    if (launches) *launches = p->launches.load();
    if (requests) *requests = p->requests.load();
  }
  if (streams) {
    std::lock_guard<std::mutex> lk(g_pools_mu);
    *streams = p->refs;
  }
  return 0;
}

/* ---- 1.6 kb/s decoder (include/lpcnet.h:63-100 of the reference) --------
 * LPCNetDecState embeds an LPCNetState as the reference's does
 * (lpcnet_private.h:50-53); vq_mem lives with the stream's device state. */
struct LPCNetDecState {
  LPCNetState lpcnet_state;
};

LPCNET_EXPORT int lpcnet_decoder_get_size(void) { return (int)sizeof(LPCNetDecState); }

/* lpcnet.c:290-295: memset + lpcnet_init.  A never-initialised (or stale)
 * decoder is zeroed and gets a fresh handle; a live one is re-initialised in
 * place (stream reset, model kept), as below */
LPCNET_EXPORT int lpcnet_decoder_init(LPCNetDecState *st)
{
  if (!st) return -1;
  /* re-initialising a live decoder resets its stream (vq_mem included:
   * host_reset_state) and keeps its model, as lpcnet_init does for a live
   * LPCNetState; only a never-initialised (or stale) one starts from zero */
  if (live_handle(&st->lpcnet_state)) return lpcnet_init(&st->lpcnet_state);
  memset(st, 0, sizeof(*st));
  return lpcnet_init(&st->lpcnet_state);
}

LPCNET_EXPORT LPCNetDecState *lpcnet_decoder_create(void)
{
  LPCNetDecState *st = (LPCNetDecState *)malloc(sizeof(LPCNetDecState));
  if (st && lpcnet_decoder_init(st) != 0) {
    free(st);
    return nullptr;
  }
  return st;
}

LPCNET_EXPORT void lpcnet_decoder_destroy(LPCNetDecState *st)
{
  if (!st) return;
  handle_deinit(&st->lpcnet_state);
  free(st);
}

LPCNET_EXPORT int lpcnet_mi355x_decoder_load_model(LPCNetDecState *st, const unsigned char *data, int len)
{
  if (!st) return -1;
  if (lpcnet_load_model(&st->lpcnet_state, data, len)) return -1;
  Handle *h = live_handle(&st->lpcnet_state);
  if (!h || !h->pool || !h->pool->has_codebooks) {
    set_err("lpcnet_decode needs the ceps_codebook1/2/3 / ceps_codebook_diff4 records in the blob");
    return -1;
  }
  return 0;
}

/* lpcnet.c:310-319: decode_packet, then lpcnet_synthesize of the 4 frames */
LPCNET_EXPORT int lpcnet_decode(LPCNetDecState *st, const unsigned char *buf, short *pcm)
{
  if (!st || !buf || !pcm) { set_err("bad arguments"); return -1; }
  StatePool::Req r{-1, StatePool::DECODE, nullptr, buf, pcm, 4 * FRAME, 0, 0, 0, std::string()};
  return handle_run(&st->lpcnet_state, r, "lpcnet_decode") ? -1 : 0;
}

/* Host-only check of a weight blob against every rule lpcnet_load_model
 * applies (no device needed). */
LPCNET_EXPORT int lpcnet_mi355x_validate_model(const unsigned char *data, int len)
{
  LPCNetBatch tmp;
  /* diagnostics: the batch size whose kernel plan to build (LPCNET_VERBOSE prints it) */
  const char *v = getenv("LPCNET_VALIDATE_STREAMS");
  tmp.B = v ? std::max(1, atoi(v)) : 1;
  return load_model(&tmp, data, len, false);
}

}  // extern "C"
