"""DPM clock-ramp probe: the bench workload (fresh batch, warmup W frames,
20 timed frames) after holding the GPU busy for P ms (then resetting the
streams, so the timed frames compute the same PCM).  Prints the timed
ms/step, the sample kernel's ms/frame and the PCM checksum per P."""
import sys, os, zlib
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
import lpcnet_amd as L

blob = L.synthetic_model(1, 0)
B = int(os.environ.get("B", "1024"))
for p in [float(x) for x in os.environ.get("PREHEATS", "0 30 100 300 0 1000").split()]:
    dt, (ks, kn, kf, fs, fn), info, pcm = bench.run_batch(L, blob, B, 0, 5, 20, preheat_ms=p)
    print("preheat %5.0f ms: %.4f ms/step, sample kernel %.4f ms/frame, pcm crc %08x" %
          (p, dt / 20 * 1e3, ks / max(kf, 1), zlib.crc32(pcm[5:].tobytes())), flush=True)
