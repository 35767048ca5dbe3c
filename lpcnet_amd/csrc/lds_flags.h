/*
 * lds_flags.h -- workgroup-local producer/consumer flags in LDS, used by the
 * barrier-free sample kernels (fp_kernel, mf_kernel) in place of workgroup
 * barriers.  The data a flag publishes is in LDS, so ordering needs only the
 * writer's LDS queue drained before the flag store (lgkmcnt) and the
 * reader's dependent branch before its data reads.
 */
#ifndef LPCNET_LDS_FLAGS_H
#define LPCNET_LDS_FLAGS_H

#include <hip/hip_runtime.h>

namespace lpcnet_mi355x {

__device__ __forceinline__ int flag_load(const int *p)
{
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

/* Spin until *p >= v.  A wait that outlives `limit` polls (a bug, never a
 * legal schedule) sets the workgroup's abort word, after which every wait
 * returns at once: the kernel finishes instead of hanging the device, and
 * reports the abort through SampleArgs::status (the host call returns -1). */
/* SLEEP > 0: s_sleep between polls (64 clocks per unit) -- for long waits,
 * so idle waves do not flood the LDS the working waves depend on. */
template <int SLEEP = 0>
__device__ __forceinline__ void flag_wait(const int *p, int v, int *abort_w, int limit)
{
  for (int it = 0; flag_load(p) < v; it++) {
    if (flag_load(abort_w)) break;
    if (it > limit) {
      __hip_atomic_store(abort_w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      break;
    }
    if (SLEEP > 0) __builtin_amdgcn_s_sleep(SLEEP);
  }
  asm volatile("" ::: "memory");
}

/* Publish v after every LDS write this wave issued before the call. */
__device__ __forceinline__ void flag_publish(int *p, int v)
{
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

}  // namespace lpcnet_mi355x

#endif
