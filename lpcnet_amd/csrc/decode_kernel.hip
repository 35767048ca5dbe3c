/*
 * decode_kernel.hip -- the 1.6 kb/s packet decoder (decode_packet,
 * /root/reference/src/lpcnet_dec.c:81-156, with perform_double_interp,
 * common.c:36-65) on the device, feeding the synthesis kernels.
 *
 * One 8-byte packet per stream per 40 ms carries 4 feature frames: a
 * 3-stage VQ of the last frame's cepstrum, a signed 4096-entry difference
 * codebook for frame 1 (predicted from the previous packet's last frame,
 * vq_mem, and / or frame 3), an interpolation choice for frames 0 and 2,
 * and one pitch / modulation / correlation triple for all four.  The work is
 * byte unpacking, 3 + 1 codebook row gathers and a few adds per band:
 * HBM-light integer/gather work, so the layout is one 32-lane half-wave
 * per stream (lane = band, lanes 18..21 = the four frames' pitch and
 * correlation), every packet of a stream decoded in order by the same lanes
 * (vq_mem chains packets), features written straight into the
 * [frame][stream][NB_FEATURES] layout lpcnet_batch_synthesize_frames reads,
 * so they never leave HBM.
 *
 * Arithmetic: every float expression is the reference's, in its order,
 * compiled with -ffp-contract=off.  pow(2, main_pitch/21.) (double, glibc)
 * is the one transcendental; its 64 possible values come from the host
 * (engine.cpp), computed with the reference's own expression.
 */
#include "lpcnet_engine.h"

namespace lpcnet_mi355x {

constexpr int DEC_LANES = 32;                 /* lanes per stream */
constexpr int DEC_THREADS = 256;
constexpr int DEC_STREAMS = DEC_THREADS / DEC_LANES;
constexpr int NB1 = NBANDS - 1;               /* freq.h:49 NB_BANDS_1 */

/* lpcnet_dec.c:52-72 bits_unpack: MSB-first bit reader; the 9 fields of a
 * packet (lpcnet_dec.c:97-105) fill its 64 bits exactly */
__device__ __forceinline__ unsigned field(unsigned long long v, int off, int len)
{
  return (unsigned)((v >> (64 - off - len)) & ((1ull << len) - 1));
}

__global__ __launch_bounds__(DEC_THREADS) void decode_kernel(DecodeArgs A)
{
  const int lane = threadIdx.x % DEC_LANES;
  const int sid = blockIdx.x * DEC_STREAMS + threadIdx.x / DEC_LANES;
  if (sid >= A.nstreams) return;
  float mem = lane < NBANDS ? A.st[sid].vq_mem[lane] : 0.f;
  for (int p = 0; p < A.npackets; p++) {
    const unsigned char *buf = A.packets + ((size_t)p * A.nstreams + sid) * 8;
    unsigned long long v = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) v = (v << 8) | buf[k];
    const int c0_id = (int)field(v, 0, 7);
    const int main_pitch = (int)field(v, 7, 6);
    int modulation = (int)field(v, 13, 3);
    const int corr_id = (int)field(v, 16, 2);
    const int vq_end0 = (int)field(v, 18, 10), vq_end1 = (int)field(v, 28, 10), vq_end2 = (int)field(v, 38, 10);
    int vq_mid = (int)field(v, 48, 13);
    const int interp_id = (int)field(v, 61, 3);
    float *out = A.features + (size_t)4 * p * A.nstreams * NF + (size_t)sid * NF;
    const size_t fstride = (size_t)A.nstreams * NF; /* next frame of this stream */
    if (lane < NBANDS) {
      /* features[3]: c0 and the 3-stage VQ sum (lpcnet_dec.c:126-129) */
      float f3;
      if (lane == 0) f3 = (c0_id - 64) / 4.f;
      else
        f3 = A.cb1[vq_end0 * NB1 + lane - 1] + A.cb2[vq_end1 * NB1 + lane - 1] + A.cb3[vq_end2 * NB1 + lane - 1];
      /* features[1]: signed difference codebook + prediction (:131-145) */
      float sign = 1;
      if (vq_mid >= 4096) {
        vq_mid -= 4096;
        sign = -1;
      }
      float f1 = sign * A.cbd[vq_mid * NBANDS + lane];
      if ((vq_mid & 3) < 2) f1 += .5f * (mem + f3);
      else if ((vq_mid & 3) == 2) f1 += mem;
      else f1 += f3;
      /* perform_double_interp (common.c:58-65 -> single_interp :36-56) */
      int best = interp_id;
      best += (best >= 7); /* FORBIDDEN_INTERP */
      const int id0 = best / 3, id1 = best % 3;
      const float f0 = id0 == 0 ? .5f * (mem + f1) : (id0 == 1 ? mem : f1);
      const float f2 = id1 == 0 ? .5f * (f1 + f3) : (id1 == 1 ? f1 : f3);
      out[0 * fstride + lane] = f0;
      out[1 * fstride + lane] = f1;
      out[2 * fstride + lane] = f2;
      out[3 * fstride + lane] = f3;
      mem = f3; /* RNN_COPY(vq_mem, features[3], NB_BANDS) (:155) */
    } else if (lane < NBANDS + 4) {
      /* pitch and correlation of frame `sub` (lpcnet_dec.c:110-124) */
      const int sub = lane - NBANDS;
      int voiced = 1;
      modulation -= 4;
      if (modulation == -4) {
        voiced = 0;
        modulation = 0;
      }
      const float frame_corr = voiced ? 0.3875f + .175f * corr_id : 0.0375f + .075f * corr_id;
      float pp = A.pitch[main_pitch];
      pp *= 1.f + modulation / 16.f / 7.f * (2 * sub - 3);
      pp = 33 > pp ? 33 : pp;   /* MAX16(33, p) */
      pp = 255 < pp ? 255 : pp; /* MIN16(255, .) */
      out[sub * fstride + NBANDS] = .02f * (pp - 100.f);
      out[sub * fstride + NBANDS + 1] = frame_corr - .5f;
    }
  }
  if (lane < NBANDS) A.st[sid].vq_mem[lane] = mem;
}

int launch_decode(const DecodeArgs &a, void *stream)
{
  if (a.nstreams <= 0 || a.npackets <= 0) return 0;
  const int grid = (a.nstreams + DEC_STREAMS - 1) / DEC_STREAMS;
  hipLaunchKernelGGL(decode_kernel, dim3(grid), dim3(DEC_THREADS), 0, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lpcnet_mi355x
