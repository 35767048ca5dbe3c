/* Exhaustive proofs of the float identities the HIP kernels use in place of
 * slower operations of the reference (TEST INFRASTRUCTURE ONLY):
 *  (1) lin2ulaw's float division by log(256) (common.h:47-58):
 *      RN(v / c) == fma(fma(-q0, c, v), rc, q0), q0 = RN(v*rc), rc = RN(1/c),
 *      for every float v in [2^-10, 2^15) -- lin2ulaw's numerator
 *      128*(0.69315*l2) lies in [0.0395, 11500] (y >= 1 gives l2 >= 4.4e-4);
 *  (2) (int)floor(.5 + (double)u) == k + (u - k >= .5f), k = (int)u, for
 *      every float u in [0, 255] (the u-law index, common.h:57);
 *  (3) (int)floor(.5 + (double)o) == (int)floorf(o) + (o - floorf(o) >= .5f)
 *      for every float o in [-32767, 32767] (the output sample, lpcnet.c:268).
 *  (4) the rcpps emulation of the Pade denominators of tanh8_approx /
 *      sigmoid8_approx (vec_avx.h:393-440), den = fma(fma(D2,X2,D1),X2,D0) with
 *      positive D's and X2 = X*X, i.e. den in [952.72, +inf] or NaN:
 *      ldexp(table[m], 127 - e) flushed to +0 below 2^-126 equals the
 *      general emulation (sign | table mantissa | rebiased exponent, 0 for
 *      denormal results, 0 for +inf) for every such finite or infinite den
 *      (argv[1] = the 2048-entry table, tests/golden/rcp_x86.bin);
 *  (5) the integer form of (4) the kernels use: q = (table[m] + (127 << 23))
 *      - (bits(den) & 0x7f800000) as int32, +0 when q < 2^23, for the same
 *      den range.
 * Build: gcc -O2 -ffp-contract=off exact_identities.c -lm; exit status 0 = all hold. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char **argv)
{
  unsigned long long bad = 0;
  const float c = 5.5451774445f, rc = 1.0f / c;
  for (uint32_t u = u_of(0x1p-10f); u < u_of(32768.f); u++) {
    const float v = f_of(u), ref = v / c, q0 = v * rc, q1 = fmaf(fmaf(-q0, c, v), rc, q0);
    if (u_of(ref) != u_of(q1)) bad++;
  }
  printf("division: %llu mismatches\n", bad);
  unsigned long long bad2 = 0;
  for (uint32_t u = 0; u <= u_of(255.f); u++) {
    const float x = f_of(u);
    const int ref = (int)floor(.5 + (double)x);
    const int k = (int)x;
    if (ref != k + (x - (float)k >= .5f)) bad2++;
  }
  printf("round u: %llu mismatches\n", bad2);
  unsigned long long bad3 = 0;
  for (int sgn = 0; sgn < 2; sgn++)
    for (uint32_t u = 0; u <= u_of(32767.f); u++) {
      const float x = sgn ? -f_of(u) : f_of(u);
      const int ref = (int)floor(.5 + (double)x);
      const float k = floorf(x);
      if (ref != (int)k + (x - k >= .5f)) bad3++;
    }
  printf("round o: %llu mismatches\n", bad3);
  unsigned long long bad4 = 0;
  if (argc > 1) {
    static uint32_t tab[2048];
    FILE *f = fopen(argv[1], "rb");
    if (!f || fread(tab, 4, 2048, f) != 2048) { printf("cannot read table\n"); return 2; }
    fclose(f);
    for (uint32_t u = u_of(952.72f); u <= 0x7f800000u; u++) {
      const uint32_t t = tab[(u >> 12) & 0x7ff];
      /* general form (kernels.hip rcp_x86 before specialisation) */
      const uint32_t sign = u & 0x80000000u;
      const int e = (int)((u >> 23) & 0xff);
      const int te = (int)((t >> 23) & 0xff) + 127 - e;
      uint32_t r = sign | (t & 0x007fffffu) | ((uint32_t)te << 23);
      r = te < 1 ? sign : r;
      const uint32_t spec = (u & 0x7fffffu) ? (u | 0x00400000u) : sign;
      r = e == 255 ? spec : r;
      /* specialised form */
      float q = ldexpf(f_of(t), 127 - e);
      q = q < 0x1p-126f ? 0.f : q;
      if (r != u_of(q)) bad4++;
      /* integer form */
      const int32_t qi = (int32_t)((t + (127u << 23)) - (u & 0x7f800000u));
      const uint32_t r5 = qi < 0x00800000 ? 0u : (uint32_t)qi;
      if (r5 != u_of(q)) bad4++;
    }
    printf("rcp pade (ldexp and integer forms): %llu mismatches\n", bad4);
  }
  return (bad || bad2 || bad3 || bad4) ? 1 : 0;
}
