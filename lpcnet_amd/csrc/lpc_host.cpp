/*
 * lpc_host.cpp -- per-frame LPC from cepstrum on the host.
 *
 * Restates freq.c:310-320 lpc_from_cepstrum (idct freq.c:230-240, band gain
 * interpolation :202-216, inverse_transform :256-273, lpc_from_bands :275-297,
 * lpcn_lpc :86-127) with Opus' 320-point kiss FFT (kiss_fft.c:101-305,
 * 518-586; factors 5x4x4x4, tables as kiss_fft.c:315-421 and
 * dump_lpcnet_tables.c:88-95 generate them).  Bit-exact with the reference
 * on the same libm (pow/cos/sin are only used to build tables and for the 18
 * band powers), which is why this step stays on the host in round 1: a device
 * pow() is not guaranteed to round like glibc's.  Must be compiled with
 * -ffp-contract=off.
 */
#include <math.h>
#include <string.h>

#include "lpcnet_engine.h"

namespace lpcnet_mi355x {

namespace {

constexpr int NBANDS = 18, WIN = 320, FREQ = 161;
constexpr short kEband[NBANDS] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28, 34, 40};
constexpr float kComp[NBANDS] = {0.8f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 0.666667f, 0.5f, 0.5f, 0.5f,
                                 0.333333f, 0.25f, 0.25f, 0.2f, 0.166667f, 0.173913f};

struct C { float r, i; };

struct Tables {
  C tw[WIN];
  short perm[WIN];
  float dct[NBANDS * NBANDS];
  Tables()
  {
    const double pi = 3.14159265358979323846264338327;
    for (int i = 0; i < WIN; i++) {
      double ph = (-2 * pi / WIN) * i;
      tw[i].r = (float)cos(ph);
      tw[i].i = (float)sin(ph);
    }
    /* digit reversal for radices (5,4,4,4) outermost first: input sample
     * d0 + 5*d1 + 20*d2 + 80*d3 feeds FFT slot d0*64 + d1*16 + d2*4 + d3. */
    for (int d0 = 0; d0 < 5; d0++)
      for (int d1 = 0; d1 < 4; d1++)
        for (int d2 = 0; d2 < 4; d2++)
          for (int d3 = 0; d3 < 4; d3++) perm[d0 * 64 + d1 * 16 + d2 * 4 + d3] = (short)(d0 + 5 * d1 + 20 * d2 + 80 * d3);
    for (int i = 0; i < NBANDS; i++)
      for (int j = 0; j < NBANDS; j++) {
        float v = (float)cos((i + .5) * j * M_PI / NBANDS);
        if (j == 0) v = (float)(v * sqrt(.5));
        dct[i * NBANDS + j] = v;
      }
  }
};

const Tables &tables()
{
  static const Tables t;
  return t;
}

inline C cmul(C a, C b) { return C{a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
inline C cadd(C a, C b) { return C{a.r + b.r, a.i + b.i}; }
inline C csub(C a, C b) { return C{a.r - b.r, a.i - b.i}; }

/* radix-4 stage: `groups` groups spaced `span` apart, butterflies of length m */
void radix4(C *f, const C *tw, int tstride, int m, int groups, int span)
{
  if (m == 1) {
    for (int g = 0; g < groups; g++, f += 4) {
      C s0 = csub(f[0], f[2]);
      f[0] = cadd(f[0], f[2]);
      C s1 = cadd(f[1], f[3]);
      f[2] = csub(f[0], s1);
      f[0] = cadd(f[0], s1);
      s1 = csub(f[1], f[3]);
      f[1] = C{s0.r + s1.i, s0.i - s1.r};
      f[3] = C{s0.r - s1.i, s0.i + s1.r};
    }
    return;
  }
  for (int g = 0; g < groups; g++) {
    C *p = f + g * span;
    for (int j = 0; j < m; j++, p++) {
      C a = cmul(p[m], tw[j * tstride]);
      C b = cmul(p[2 * m], tw[2 * j * tstride]);
      C c = cmul(p[3 * m], tw[3 * j * tstride]);
      C d = csub(p[0], b);
      p[0] = cadd(p[0], b);
      C e = cadd(a, c), h = csub(a, c);
      p[2 * m] = csub(p[0], e);
      p[0] = cadd(p[0], e);
      p[m] = C{d.r + h.i, d.i - h.r};
      p[3 * m] = C{d.r - h.i, d.i + h.r};
    }
  }
}

/* final radix-5 stage over m=64 */
void radix5(C *f, const C *tw)
{
  const int m = 64;
  C ya = tw[m], yb = tw[2 * m];
  for (int u = 0; u < m; u++) {
    C *q0 = f + u, *q1 = q0 + m, *q2 = q0 + 2 * m, *q3 = q0 + 3 * m, *q4 = q0 + 4 * m;
    C s0 = *q0;
    C s1 = cmul(*q1, tw[u]), s2 = cmul(*q2, tw[2 * u]), s3 = cmul(*q3, tw[3 * u]), s4 = cmul(*q4, tw[4 * u]);
    C s7 = cadd(s1, s4), s10 = csub(s1, s4), s8 = cadd(s2, s3), s9 = csub(s2, s3);
    q0->r = q0->r + (s7.r + s8.r);
    q0->i = q0->i + (s7.i + s8.i);
    C s5{s0.r + ((s7.r * ya.r) + (s8.r * yb.r)), s0.i + ((s7.i * ya.r) + (s8.i * yb.r))};
    C s6{(s10.i * ya.i) + (s9.i * yb.i), -((s10.r * ya.i) + (s9.r * yb.i))};
    *q1 = csub(s5, s6);
    *q4 = cadd(s5, s6);
    C s11{s0.r + ((s7.r * yb.r) + (s8.r * ya.r)), s0.i + ((s7.i * yb.r) + (s8.i * ya.r))};
    C s12{(s9.i * ya.i) - (s10.i * yb.i), (s10.r * yb.i) - (s9.r * ya.i)};
    *q2 = cadd(s11, s12);
    *q3 = csub(s11, s12);
  }
}

}  // namespace

float lpc_from_cepstrum_host(float *lpc, const float *ceps)
{
  const Tables &T = tables();
  float t[NBANDS], E[NBANDS];
  memcpy(t, ceps, sizeof(t));
  t[0] += 4;
  for (int i = 0; i < NBANDS; i++) {
    float acc = 0;
    for (int j = 0; j < NBANDS; j++) acc += t[j] * T.dct[i * NBANDS + j];
    E[i] = acc * sqrt(2. / NBANDS);
  }
  /* C semantics of freq.c:318: pow(10.f, Ex) promotes to double (not the C++ float overload) */
  for (int i = 0; i < NBANDS; i++) E[i] = (float)(pow(10.0, (double)E[i]) * (double)kComp[i]);

  /* Hermitian spectrum of the interpolated band energies */
  C x[WIN];
  for (int b = 0; b < NBANDS - 1; b++) {
    int n = (kEband[b + 1] - kEband[b]) * 4;
    for (int j = 0; j < n; j++) {
      float frac = (float)j / n;
      x[kEband[b] * 4 + j] = C{(1 - frac) * E[b] + frac * E[b + 1], 0.f};
    }
  }
  x[FREQ - 1] = C{0.f, 0.f};
  for (int i = FREQ; i < WIN; i++) x[i] = C{x[WIN - i].r, -x[WIN - i].i};

  /* forward FFT with 1/320 scaling, digit-reversed input order */
  C y[WIN];
  const float scale = 1.f / 320.f;
  for (int i = 0; i < WIN; i++) y[i] = C{scale * x[T.perm[i]].r, scale * x[T.perm[i]].i};
  radix4(y, T.tw, 80, 1, 80, 4);
  radix4(y, T.tw, 20, 4, 20, 16);
  radix4(y, T.tw, 5, 16, 5, 64);
  radix5(y, T.tw);

  float ac[17];
  ac[0] = WIN * y[0].r;
  for (int i = 1; i < 17; i++) ac[i] = WIN * y[WIN - i].r;
  ac[0] += ac[0] * 1e-4 + 320 / 12 / 38.;
  for (int i = 1; i < 17; i++) ac[i] *= (1 - 6e-5 * i * i);

  /* Levinson-Durbin (float build of lpcn_lpc) */
  float err = ac[0];
  for (int i = 0; i < 16; i++) lpc[i] = 0;
  if (ac[0] != 0) {
    for (int i = 0; i < 16; i++) {
      float rr = 0;
      for (int j = 0; j < i; j++) rr += lpc[j] * ac[i - j];
      rr += ac[i + 1];
      float r = -rr / err;
      lpc[i] = r;
      for (int j = 0; j < (i + 1) >> 1; j++) {
        float a = lpc[j], b = lpc[i - 1 - j];
        lpc[j] = a + r * b;
        lpc[i - 1 - j] = b + r * a;
      }
      err = err - (r * r) * err;
      if (err < .001f * ac[0]) break;
    }
  }
  return err;
}

}  // namespace lpcnet_mi355x
