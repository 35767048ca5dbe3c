/* Exhaustive check of the band-power step of lpc_from_cepstrum
 * (freq.c:318, TEST INFRASTRUCTURE ONLY):
 *
 *     (float)(pow(10.0, (double)E) * (double)comp)          glibc, the reference
 *  == (float)(pow10_dd((double)E) * (double)comp)           lpcnet_amd/csrc/pow10_dd.h
 *
 * for EVERY 32-bit float pattern E (NaN payloads and infinities included) and
 * each distinct compensation factor of freq.c:50-53.  pow10_dd is what the GPU
 * LPC kernel evaluates (IEEE double ops and fma only, so the device computes
 * the same bits as this host build; tests/test_lpc.py also compares device
 * and host on sampled inputs).
 *
 * Build: gcc -O2 -ffp-contract=off -pthread pow10_exhaustive.c -lm
 * Run:   ./a.out [threads] [stride]   (stride > 1 samples every stride-th
 *        pattern plus both ends; 1 = all 2^32).  Exit status 0 = identical.
 * Prints one line per mismatch (at most 64) and a summary.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../lpcnet_amd/csrc/pow10_dd.h"

static const float kComp[] = {0.8f, 1.f, 0.666667f, 0.5f, 0.333333f, 0.25f, 0.2f, 0.166667f, 0.173913f};
#define NCOMP ((int)(sizeof(kComp) / sizeof(kComp[0])))

static uint64_t g_stride = 1;
static int g_threads = 8;
static unsigned long long g_bad[64], g_checked[64];
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;
static int g_printed = 0;

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static void *work(void *arg)
{
  const int t = (int)(intptr_t)arg;
  const uint64_t total = 1ull << 32;
  unsigned long long bad = 0, checked = 0;
  for (uint64_t i = (uint64_t)t * g_stride; i < total; i += (uint64_t)g_threads * g_stride) {
    const float E = f_of((uint32_t)i);
    const double pr = pow(10.0, (double)E), pm = pow10_dd((double)E);
    for (int c = 0; c < NCOMP; c++) {
      const float a = (float)(pr * (double)kComp[c]), b = (float)(pm * (double)kComp[c]);
      checked++;
      if (u_of(a) != u_of(b)) {
        bad++;
        pthread_mutex_lock(&g_lock);
        if (g_printed++ < 64)
          printf("mismatch E=%a (0x%08x) comp=%a: glibc %a (0x%08x) dd %a (0x%08x)  [pow %a vs %a]\n", E, (uint32_t)i,
                 kComp[c], a, u_of(a), b, u_of(b), pr, pm);
        pthread_mutex_unlock(&g_lock);
      }
    }
  }
  g_bad[t] = bad;
  g_checked[t] = checked;
  return NULL;
}

int main(int argc, char **argv)
{
  if (argc > 1) g_threads = atoi(argv[1]);
  if (argc > 2) g_stride = strtoull(argv[2], NULL, 10);
  if (g_threads < 1 || g_threads > 64 || g_stride < 1) return 2;
  pthread_t th[64];
  for (int t = 0; t < g_threads; t++) pthread_create(&th[t], NULL, work, (void *)(intptr_t)t);
  unsigned long long bad = 0, checked = 0;
  for (int t = 0; t < g_threads; t++) {
    pthread_join(th[t], NULL);
    bad += g_bad[t];
    checked += g_checked[t];
  }
  /* edges a sampled run might skip */
  const float edge[] = {0.f, -0.f, INFINITY, -INFINITY, 38.531839f, 38.5318413f, -44.8f, -45.8f, -46.f, 1e-30f, -1e-30f};
  for (unsigned k = 0; k < sizeof(edge) / sizeof(edge[0]); k++)
    for (int c = 0; c < NCOMP; c++) {
      const float a = (float)(pow(10.0, (double)edge[k]) * (double)kComp[c]);
      const float b = (float)(pow10_dd((double)edge[k]) * (double)kComp[c]);
      checked++;
      if (u_of(a) != u_of(b)) {
        bad++;
        printf("edge mismatch E=%a comp=%a\n", edge[k], kComp[c]);
      }
    }
  printf("pow10_dd vs glibc pow: %llu float results checked (%d compensation factors, stride %llu), %llu mismatches\n",
         checked, NCOMP, (unsigned long long)g_stride, bad);
  return bad ? 1 : 0;
}
