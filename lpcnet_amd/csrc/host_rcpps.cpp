/*
 * host_rcpps.cpp -- this host CPU's _mm_rcp_ps (the instruction behind the
 * reference's Pade activations, vec_avx.h:408,437) in the engine's device
 * table format.  Host-only C++ (built with the system compiler, not hipcc).
 *
 * The reference's output depends on the CPU it runs on: an Intel host's
 * rcpps is a function of the top 11 mantissa bits, the GPU box's AMD EPYC
 * 9575F's of the top 12 (profiles/r03/box_rcpps.json); both are invariant
 * under the exponent over the Pade denominators' range.  The engine's
 * default table is the committed Intel one (tests/golden/rcp_x86.bin);
 * lpcnet_batch_set_rcp_table with this host's table reproduces the
 * reference running on THIS host ("same-box parity").
 */
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include "lpcnet_mi355x.h"

extern "C" LPCNET_EXPORT int lpcnet_mi355x_host_rcp_table(uint32_t *tab, int entries)
{
  if (!tab || entries != 4096) return -1;
  int bad = 0;
  /* every float in [1, 2): entry m >> 11 must be the same for the 2^11
   * mantissas sharing the top 12 bits */
  for (uint32_t m = 0; m < (1u << 23); m += 4) {
    uint32_t u[4] = {0x3f800000u | m, 0x3f800000u | (m + 1), 0x3f800000u | (m + 2), 0x3f800000u | (m + 3)};
    float f[4];
    memcpy(f, u, 16);
    const __m128 r = _mm_rcp_ps(_mm_loadu_ps(f));
    uint32_t o[4];
    _mm_storeu_si128((__m128i *)o, _mm_castps_si128(r));
    for (int k = 0; k < 4; k++) {
      const uint32_t mm = m + k;
      if ((mm & 0x7FF) == 0) tab[mm >> 11] = o[k];
      else if (tab[mm >> 11] != o[k]) bad++;
    }
  }
  /* exponent invariance over the Pade denominators' binades [2^9, 2^64) */
  for (int e = 9; e < 64; e += 3)
    for (int i = 0; i < 4096; i += 7) {
      const uint32_t ux = ((uint32_t)(127 + e) << 23) | ((uint32_t)i << 11) | 0x3FF;
      float x;
      memcpy(&x, &ux, 4);
      const float r = _mm_cvtss_f32(_mm_rcp_ss(_mm_set_ss(x)));
      uint32_t ur;
      memcpy(&ur, &r, 4);
      if (ur != tab[i] - ((uint32_t)e << 23)) bad++;
    }
  return bad;
}
