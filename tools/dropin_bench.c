/*
 * dropin_bench.c -- aggregate throughput of the drop-in API from C threads.
 *
 *   dropin_bench <threads> <frames> [pool]
 *   dropin_bench <threads> <frames> rt [burst|spread]
 *   dropin_bench <streams> <frames> live
 *
 * T pthreads, one LPCNetState each (include/lpcnet.h: lpcnet_create,
 * lpcnet_load_model, lpcnet_synthesize -- the reference's own calling
 * pattern, src/lpcnet.c:213-219, 279-281), all synthesising F frames at
 * once; the library's shared pool coalesces their calls into batched
 * launches.  Beside it, the same T streams through one LPCNetBatch with host
 * I/O frame by frame (lpcnet_batch_synthesize) and device-resident
 * (lpcnet_batch_synthesize_frames).  One JSON object on stdout.  The C
 * driver separates the pool's own cost from a Python caller's turnaround.
 * With "pool" only the drop-in part runs (for a kernel trace of it alone).
 *
 * "rt": real-time pacing, the way lpcnet_demo.c:208-219 drives one stream
 * per 10 ms of audio: each thread calls lpcnet_synthesize once per 10 ms
 * tick (absolute deadlines, CLOCK_MONOTONIC), "burst" with every thread on
 * the same tick phase, "spread" (default) with the T phases spaced evenly
 * over the 10 ms; per call the latency (call start to return) and whether
 * it returned after its tick's end (a missed deadline: the stream's next
 * frame is late).  One JSON object: latency p50 / p99 / max, misses,
 * coalesced launches.
 *
 * "live": the batch API's live tick from C (no Python in the loop): one
 * LPCNetBatch of <streams>, each frame's features copied into the batch's
 * own feature buffer (lpcnet_batch_host_features), lpcnet_batch_synthesize
 * into its own PCM buffer; per-tick wall time mean / p50 / p99.
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "lpcnet_mi355x.h"

static int T, F;
static unsigned char *blob;
static int blob_len;
static float *feats; /* [T][F][NB_TOTAL_FEATURES] */
static LPCNetState **nets;
static pthread_barrier_t go;

static double now(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* rt mode */
static double rt_t0;      /* first tick (CLOCK_MONOTONIC seconds) */
static int rt_spread = 1; /* phases spread over the tick */
static float *rt_lat;     /* [T][F] call latency, ms */
static int *rt_miss;      /* [T] calls that returned after their tick's end */
#define TICK_S 0.010

static void sleep_until(double t)
{
  struct timespec ts;
  ts.tv_sec = (time_t)t;
  ts.tv_nsec = (long)((t - (double)ts.tv_sec) * 1e9);
  while (clock_nanosleep(CLOCK_MONOTONIC, TIMER_ABSTIME, &ts, NULL) != 0) {
  }
}

static void *run_rt(void *arg)
{
  const int t = (int)(size_t)arg;
  short pcm[LPCNET_FRAME_SIZE];
  const double phase = rt_spread ? TICK_S * t / T : 0.0;
  pthread_barrier_wait(&go);
  for (int f = 0; f < F; f++) {
    const double tick = rt_t0 + phase + TICK_S * f;
    sleep_until(tick);
    const double a = now();
    lpcnet_synthesize(nets[t], &feats[((size_t)t * F + f) * NB_TOTAL_FEATURES], pcm, LPCNET_FRAME_SIZE);
    const double e = now();
    rt_lat[(size_t)t * F + f] = (float)((e - a) * 1e3);
    if (e > tick + TICK_S) rt_miss[t]++;
  }
  return NULL;
}

static int cmpf(const void *x, const void *y)
{
  const float a = *(const float *)x, b = *(const float *)y;
  return (a > b) - (a < b);
}

static int live_ticks(int B, int nf)
{
  const int len = lpcnet_mi355x_synthetic_model(1, LPCNET_VARIANT_INT8, 0, NULL, 0);
  unsigned char *m = malloc(len);
  lpcnet_mi355x_synthetic_model(1, LPCNET_VARIANT_INT8, 0, m, len);
  LPCNetBatch *b = lpcnet_batch_create(B, 0);
  if (!b || lpcnet_batch_load_model(b, m, len)) {
    fprintf(stderr, "batch failed: %s\n", lpcnet_mi355x_last_error());
    return 1;
  }
  const int ND = 16; /* distinct feature frames, cycled */
  float *all = malloc(sizeof(float) * (size_t)ND * B * NB_FEATURES);
  float *tmp = malloc(sizeof(float) * (size_t)ND * NB_TOTAL_FEATURES);
  for (int s = 0; s < B; s++) {
    lpcnet_mi355x_synthetic_features(s, ND, tmp);
    for (int f = 0; f < ND; f++)
      memcpy(&all[((size_t)f * B + s) * NB_FEATURES], &tmp[(size_t)f * NB_TOTAL_FEATURES], sizeof(float) * NB_FEATURES);
  }
  float *hf = lpcnet_batch_host_features(b);
  short *hp = lpcnet_batch_host_pcm(b);
  const int warm = 20;
  float *lat = malloc(sizeof(float) * nf);
  long sum = 0;
  for (int f = 0; f < warm + nf; f++) {
    const double a = now();
    memcpy(hf, &all[(size_t)(f % ND) * B * NB_FEATURES], sizeof(float) * (size_t)B * NB_FEATURES);
    if (lpcnet_batch_synthesize(b, hf, hp, LPCNET_FRAME_SIZE)) {
      fprintf(stderr, "synthesize failed: %s\n", lpcnet_mi355x_last_error());
      return 1;
    }
    const double e = now();
    if (f >= warm) lat[f - warm] = (float)((e - a) * 1e3);
    sum += hp[0];
  }
  double mean = 0;
  for (int f = 0; f < nf; f++) mean += lat[f];
  mean /= nf;
  qsort(lat, nf, sizeof(float), cmpf);
  printf("{\"streams\": %d, \"ticks\": %d, \"ms_per_tick_mean\": %.5f, \"ms_per_tick_p50\": %.5f, "
         "\"ms_per_tick_p99\": %.5f, \"samples_per_s\": %.1f, \"check\": %ld}\n",
         B, nf, mean, lat[nf / 2], lat[(int)(0.99 * (nf - 1))], B * 160.0 / (mean * 1e-3), sum);
  lpcnet_batch_destroy(b);
  return 0;
}

static void *run(void *arg)
{
  const int t = (int)(size_t)arg;
  short pcm[LPCNET_FRAME_SIZE];
  pthread_barrier_wait(&go);
  for (int f = 0; f < F; f++)
    lpcnet_synthesize(nets[t], &feats[((size_t)t * F + f) * NB_TOTAL_FEATURES], pcm, LPCNET_FRAME_SIZE);
  return NULL;
}

int main(int argc, char **argv)
{
  if (argc < 3) {
    fprintf(stderr, "usage: %s <threads> <frames> [pool]\n", argv[0]);
    return 2;
  }
  T = atoi(argv[1]);
  F = atoi(argv[2]);
  if (T < 1 || F < 1) return 2;
  if (argc > 3 && !strcmp(argv[3], "live")) return live_ticks(T, F);
  blob_len = lpcnet_mi355x_synthetic_model(1, LPCNET_VARIANT_INT8, 0, NULL, 0);
  blob = malloc(blob_len);
  lpcnet_mi355x_synthetic_model(1, LPCNET_VARIANT_INT8, 0, blob, blob_len);
  feats = malloc(sizeof(float) * T * F * NB_TOTAL_FEATURES);
  for (int t = 0; t < T; t++) lpcnet_mi355x_synthetic_features(t, F, &feats[(size_t)t * F * NB_TOTAL_FEATURES]);

  /* drop-in handles, one per thread; one warm call each (pool, work batch) */
  nets = malloc(sizeof(*nets) * T);
  short warm[LPCNET_FRAME_SIZE];
  for (int t = 0; t < T; t++) {
    nets[t] = lpcnet_create();
    if (!nets[t] || lpcnet_load_model(nets[t], blob, blob_len)) {
      fprintf(stderr, "load failed: %s\n", lpcnet_mi355x_last_error());
      return 1;
    }
  }
  pthread_t *th = malloc(sizeof(*th) * T);
  /* warm-up round: every thread one frame at once (sizes the work batch) */
  {
    int saveF = F;
    F = 1;
    pthread_barrier_init(&go, NULL, T + 1);
    for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, run, (void *)(size_t)t);
    pthread_barrier_wait(&go);
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    pthread_barrier_destroy(&go);
    F = saveF;
    for (int t = 0; t < T; t++) lpcnet_reset(nets[t]);
  }
  (void)warm;
  if (argc > 3 && !strcmp(argv[3], "rt")) {
    rt_spread = !(argc > 4 && !strcmp(argv[4], "burst"));
    rt_lat = calloc((size_t)T * F, sizeof(float));
    rt_miss = calloc(T, sizeof(int));
    long a0 = 0, q0 = 0;
    int nsb = 0;
    lpcnet_mi355x_pool_stats(nets[0], &a0, &q0, &nsb);
    pthread_barrier_init(&go, NULL, T + 1);
    rt_t0 = now() + 0.05 + 0.001 * T / 64.0; /* every thread started and asleep before the first tick */
    for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, run_rt, (void *)(size_t)t);
    pthread_barrier_wait(&go);
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    long a1 = 0, q1 = 0;
    lpcnet_mi355x_pool_stats(nets[0], &a1, &q1, &nsb);
    long misses = 0;
    for (int t = 0; t < T; t++) misses += rt_miss[t];
    const size_t n = (size_t)T * F;
    qsort(rt_lat, n, sizeof(float), cmpf);
    printf("{\"threads\": %d, \"frames\": %d, \"mode\": \"%s\", \"latency_ms_p50\": %.4f, \"latency_ms_p99\": %.4f, "
           "\"latency_ms_max\": %.4f, \"deadline_misses\": %ld, \"calls\": %zu, \"launches\": %ld, "
           "\"mean_coalesced_streams\": %.2f, \"realtime_p99\": %s}\n",
           T, F, rt_spread ? "spread" : "burst", rt_lat[n / 2], rt_lat[(size_t)(0.99 * (n - 1))], rt_lat[n - 1], misses, n,
           a1 - a0, (double)(q1 - q0) / (a1 - a0 > 0 ? a1 - a0 : 1), rt_lat[(size_t)(0.99 * (n - 1))] <= 10.0 ? "true" : "false");
    for (int t = 0; t < T; t++) lpcnet_destroy(nets[t]);
    return 0;
  }
  long la0 = 0, rq0 = 0;
  int ns = 0;
  lpcnet_mi355x_pool_stats(nets[0], &la0, &rq0, &ns);
  const double run0 = lpcnet_mi355x_pool_run_ms(nets[0]);
  pthread_barrier_init(&go, NULL, T + 1);
  for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, run, (void *)(size_t)t);
  pthread_barrier_wait(&go);
  const double t0 = now();
  for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
  const double dt_pool = now() - t0;
  long la = 0, rq = 0;
  lpcnet_mi355x_pool_stats(nets[0], &la, &rq, &ns);
  const double run_ms = lpcnet_mi355x_pool_run_ms(nets[0]) - run0;
  la -= la0;
  rq -= rq0;
  for (int t = 0; t < T; t++) lpcnet_destroy(nets[t]);
  const double samples = (double)T * F * LPCNET_FRAME_SIZE;
  if (argc > 3 && !strcmp(argv[3], "pool")) {
    printf("{\"threads\": %d, \"frames\": %d, \"dropin_c_threads\": {\"samples_per_s\": %.1f, \"launches\": %ld, "
           "\"requests\": %ld, \"ms_per_launch\": %.4f, \"launch_run_ms\": %.4f}}\n",
           T, F, samples / dt_pool, la, rq, 1e3 * dt_pool / (la > 0 ? la : 1), run_ms / (la > 0 ? la : 1));
    return 0;
  }

  /* the same streams through one batch: host I/O frame by frame */
  LPCNetBatch *b = lpcnet_batch_create(T, 0);
  if (!b || lpcnet_batch_load_model(b, blob, blob_len)) {
    fprintf(stderr, "batch failed: %s\n", lpcnet_mi355x_last_error());
    return 1;
  }
  float *ff = malloc(sizeof(float) * (size_t)F * T * NB_FEATURES); /* [F][T][20] */
  for (int f = 0; f < F; f++)
    for (int t = 0; t < T; t++)
      memcpy(&ff[((size_t)f * T + t) * NB_FEATURES], &feats[((size_t)t * F + f) * NB_TOTAL_FEATURES], sizeof(float) * NB_FEATURES);
  short *pcm = malloc(sizeof(short) * (size_t)T * LPCNET_FRAME_SIZE * F);
  lpcnet_batch_synthesize(b, ff, pcm, LPCNET_FRAME_SIZE);
  lpcnet_batch_reset(b);
  double t1 = now();
  for (int f = 0; f < F; f++) lpcnet_batch_synthesize(b, &ff[(size_t)f * T * NB_FEATURES], pcm, LPCNET_FRAME_SIZE);
  const double dt_host = now() - t1;
  /* device-resident, all frames enqueued at once */
  float *d_f = lpcnet_batch_device_alloc(b, sizeof(float) * (size_t)F * T * NB_FEATURES);
  short *d_p = lpcnet_batch_device_alloc(b, sizeof(short) * (size_t)F * T * LPCNET_FRAME_SIZE);
  lpcnet_batch_memcpy_h2d(b, d_f, ff, sizeof(float) * (size_t)F * T * NB_FEATURES);
  lpcnet_batch_reset(b);
  lpcnet_batch_sync(b);
  t1 = now();
  lpcnet_batch_synthesize_frames(b, NULL, d_f, d_p, F, LPCNET_FRAME_SIZE);
  lpcnet_batch_sync(b);
  const double dt_dev = now() - t1;
  lpcnet_batch_device_free(b, d_f);
  lpcnet_batch_device_free(b, d_p);
  lpcnet_batch_destroy(b);

  printf("{\"threads\": %d, \"frames\": %d, \"dropin_c_threads\": {\"samples_per_s\": %.1f, \"launches\": %ld, "
         "\"requests\": %ld, \"mean_coalesced_streams\": %.2f, \"ms_per_launch\": %.4f, \"launch_run_ms\": %.4f}, "
         "\"batch_host_io\": {\"samples_per_s\": %.1f, \"ms_per_frame\": %.4f}, "
         "\"batch_device\": {\"samples_per_s\": %.1f, \"ms_per_frame\": %.4f}}\n",
         T, F, samples / dt_pool, la, rq, (double)rq / (la > 0 ? la : 1), 1e3 * dt_pool / (la > 0 ? la : 1),
         run_ms / (la > 0 ? la : 1),
         samples / dt_host, 1e3 * dt_host / F, samples / dt_dev, 1e3 * dt_dev / F);
  return 0;
}
