/*
 * l2_warm.h -- batch-1 L2 warm-up of the GRU_A embedding tables.
 *
 * The L2 keeps nothing across kernel launches (profiles/r01: the batch-1
 * sample kernel hit L2 on 50 % of its requests, all within-launch reuse),
 * so with one stream every first touch of an embedding row is an Infinity
 * Cache round trip on the per-sample critical path.  One-workgroup launches
 * land on XCD 0, and a launch's workgroup b on XCD b % 8
 * (tools/probes/xcc_probe.hip), so the batch-1 launch carries extra
 * workgroups 8, 16, .., 8P that read the three 1.2 MB tables into XCD 0's
 * L2 while workgroup 0 runs the stream; the other extra workgroups exit at
 * once.  Placement only changes speed: the warmers read, never write.
 */
#ifndef LPCNET_L2_WARM_H
#define LPCNET_L2_WARM_H

#include <hip/hip_runtime.h>

#include "lpcnet_engine.h"

namespace lpcnet_mi355x {

constexpr int WARM_SLICES = 8;

/* grid of a launch whose first `groups` workgroups do the work */
inline int warm_grid(int groups, int nstreams) { return nstreams == 1 ? groups + 8 * WARM_SLICES : groups; }

/* true: this workgroup is a warmer (or idle) and has done its part */
__device__ __forceinline__ bool l2_warm_role(const float *const tabs[3], int groups)
{
  if ((int)blockIdx.x < groups) return false;
  if (blockIdx.x % 8 != 0) return true;
  const int slice = blockIdx.x / 8 - 1, nsl = (gridDim.x - groups) / 8;
  constexpr int per_table = 256 * GA_ROWS / 4; /* float4 */
  uint32_t acc = 0;
  for (int t = 0; t < 3; t++) {
    const uint4 *p = (const uint4 *)tabs[t];
    for (int o = slice * blockDim.x + threadIdx.x; o < per_table; o += nsl * blockDim.x) {
      const uint4 v = p[o];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  asm volatile("" ::"v"(acc)); /* the loads must land */
  return true;
}

}  // namespace lpcnet_mi355x

#endif
