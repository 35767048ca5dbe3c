// Probe: is rcpps (x86 table, tests/golden/rcp_x86.bin) of a Pade denominator
// equal to 12-bit rounding of the hardware reciprocal of the denominator's
// interval midpoint?  For every 11-bit mantissa prefix i and exponents
// spanning the denominators' range [952.72, 2^126): compares
//   A (table): rcp_x86_fix(den, tab[i])
//   B: round12(v_rcp_f32(den & ~0xFFF | 0x800))
//   C: as B with the rounding increment 0x3FF (ties and the one prefix the
//      hardware rounds up across the midpoint go down)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void probe(const uint32_t *tab, int *bad, uint32_t *first)
{
  /* combo c: midpoint bits OR-ed in = 0x7FC + (c / 3), rounding increment 0x3FF + (c % 3) */
  const int i = blockIdx.x * blockDim.x + threadIdx.x; // 11-bit prefix
  if (i >= 2048) return;
  for (int c = 0; c < 24; c++) {
    const uint32_t orc = 0x7FCu + (uint32_t)(c / 3), inc = 0x3FFu + (uint32_t)(c % 3);
    int nb = 0;
    for (int e = 136; e < 253; e++) {
      const uint32_t bits = ((uint32_t)e << 23) | ((uint32_t)i << 12) | 0x5A5u;
      const int q = (int)(tab[i] - (bits & 0x7f800000u));
      const uint32_t a = q < 0x00800000 ? 0u : (uint32_t)q;
      const float mid = __uint_as_float((bits & 0xFFFFF000u) | orc);
      const float r = __builtin_amdgcn_rcpf(mid);
      const uint32_t b = (__float_as_uint(r) + inc) & 0xFFFFF800u;
      nb += a != b;
    }
    bad[c * 2048 + i] = nb;
  }
  (void)first;
}

int main()
{
  std::vector<uint32_t> t(2048);
  FILE *f = fopen("tests/golden/rcp_x86.bin", "rb");
  if (!f || fread(t.data(), 4, 2048, f) != 2048) { printf("no table\n"); return 1; }
  fclose(f);
  for (auto &v : t) v += 127u << 23;              // device form: t + (127 << 23)
  uint32_t *dt, *dfirst; int *dbad;
  (void)hipMalloc(&dt, 8192); (void)hipMalloc(&dbad, 2048 * 8); (void)hipMalloc(&dfirst, 2048 * 8);
  (void)hipMemcpy(dt, t.data(), 8192, hipMemcpyHostToDevice);
  (void)hipMemset(dfirst, 0, 2048 * 8);
  (void)hipFree(dbad); (void)hipMalloc(&dbad, 24 * 2048 * 4);
  hipLaunchKernelGGL(probe, dim3(32), dim3(64), 0, 0, dt, dbad, dfirst);
  std::vector<int> bad(24 * 2048);
  (void)hipMemcpy(bad.data(), dbad, bad.size() * 4, hipMemcpyDeviceToHost);
  for (int c = 0; c < 24; c++) {
    int tot = 0, np = 0, p0 = -1;
    for (int i = 0; i < 2048; i++) if (bad[c * 2048 + i]) { tot += bad[c * 2048 + i]; np++; if (p0 < 0) p0 = i; }
    printf("or 0x%03x inc 0x%03x: %d mismatches over %d prefixes (first %d)\n", 0x7FC + c / 3, 0x3FF + c % 3, tot, np, p0);
  }
  return 0;
}
