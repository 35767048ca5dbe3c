#!/usr/bin/env python3
"""bench.py -- LPCNet synthesis throughput on MI355X (BASELINE.json metric).

One "step" = one 10 ms frame (160 samples) for every stream of the batch:
frame network + 160 recurrent samples, device-resident features and PCM,
lpc_from_cepstrum on host threads pipelined ahead (its 64 B/stream H2D upload
is inside the timed region).  Workload: BASELINE.json configs[3] -- int8 path,
1024 streams per GPU (configs[4] shards 1024 streams per GPU, weak scaling).
The batch=1 line (configs[1]) is reported alongside.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
I8_PEAK_TOPS = 5000.0  # MI355X_MICROARCH.md: int8 MFMA dense = 2x the ~2.5 PF bf16 rate


def measured_pmc(kernel_prefix):
    """PMC record of the sample kernel from the committed rocprofv3 passes of
    this same command (tools/gpu_profile.sh -> tools/pmc_summary.py ->
    profiles/<round>/pmc_traffic.json: HBM bytes per launch from
    FETCH_SIZE/WRITE_SIZE, MFMA busy fraction); PMC counters cannot be read
    in-process.  ({}, None) when no profile matches the kernel."""
    import glob
    # a pass just made on this box (tools/gpu_evidence.sh) first, then the committed ones
    cands = [os.path.join(ROOT, "gpurun_out", "pmc_traffic.json")]
    cands += sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")), reverse=True)
    for f in cands:
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        for k, v in d.items():
            if kernel_prefix in k:
                return v, os.path.relpath(f, ROOT)
    return {}, None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30, help="timed frames")
    p.add_argument("--warmup", type=int, default=3, help="untimed frames")
    p.add_argument("--streams", type=int, default=1024, help="streams per GPU")
    p.add_argument("--variant", choices=["int8", "fp32"], default="int8")
    p.add_argument("--no-batch1", action="store_true")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--timers", type=int, default=1,
                   help="HIP events in the timed region: 0 none, 1 around the sample kernel, 2 both kernels")
    return p.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # RCCL over xGMI carries only the barrier and the max-reduction of the
        # timed interval (no data-path collective); LPCNET_DIST_BACKEND=gloo
        # rehearses several ranks on one GPU
        backend = os.environ.get("LPCNET_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return world, rank, local, dist


def barrier_sync(dist, lib_batch):
    lib_batch.sync()
    if dist is not None:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dist.barrier()


def max_over_ranks(dist, x):
    if dist is None:
        return x
    import torch
    dev = "cuda" if torch.cuda.is_available() and dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def run_batch(L, blob, B, stream_base, warmup, steps, timed_dist=None, timers=1):
    """Returns (seconds for `steps` frames, kernel ms / launches, info).
    The timed region carries HIP events around each sample-kernel launch
    (timers=1; 2 adds the frame kernel); the frame kernel's own time comes
    from a short untimed pass with both kernels timed."""
    F = warmup + steps
    extra = min(steps, 8)
    feats = np.stack([L.synthetic_features(stream_base + s, F)[:, :20] for s in range(B)], 1)
    feats = np.ascontiguousarray(feats, np.float32)  # [F][B][20]
    ndev = max(1, L.device_count())
    b = L.LPCNetBatch(B, int(os.environ.get("LOCAL_RANK", "0")) % ndev, blob)
    d_feat = b.device_alloc(feats.nbytes)
    d_pcm = b.device_alloc((F + extra) * B * 160 * 2)
    b.h2d(d_feat, feats)
    if warmup:
        b.synthesize_frames(feats[:warmup], d_feat, d_pcm, warmup)
    barrier_sync(timed_dist, b)
    b.reset_timers(timers)
    t0 = time.perf_counter()
    b.synthesize_frames(np.ascontiguousarray(feats[warmup:]), d_feat + warmup * B * 20 * 4, d_pcm + warmup * B * 160 * 2,
                        steps)
    barrier_sync(timed_dist, b)
    dt = time.perf_counter() - t0
    ks, kn = b.kernel_ms(0)
    pcm = np.zeros((F, B, 160), np.int16)
    b.d2h(pcm, d_pcm)
    b.reset_timers(2)
    b.synthesize_frames(np.ascontiguousarray(feats[warmup:warmup + extra]), d_feat + warmup * B * 20 * 4,
                        d_pcm + F * B * 160 * 2, extra)
    b.sync()
    fs, fn = b.kernel_ms(1)
    info = b.info()
    b.device_free(d_feat)
    b.device_free(d_pcm)
    b.close()
    return dt, (ks, kn, fs, fn), info, pcm


def cpu_baseline(seconds):
    """The reference's own AVX2 kernels (oracle/_ref) driven by the oracle's
    lpcnet.c/nnet.c restatement, one stream per thread on the host cores."""
    import lpcnet_amd as L
    import oracle_lib as O
    kind = "reference" if O.have_ref() else "port"
    kernels = O.ref_kernels() if O.have_ref() else None
    blob = L.synthetic_model(1, 0)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    # warm the lazily built tables on one thread first
    O.Oracle(blob, 0, kernels).synthesize(L.synthetic_features(0, 1)[0])
    frames_done = [0] * threads
    stop = [False]

    def work(t):
        o = O.Oracle(blob, 0, kernels)
        f = L.synthetic_features(1000 + t, 64)
        k = 0
        while not stop[0]:
            o.synthesize(f[k % 64])
            k += 1
            frames_done[t] = k

    ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    time.sleep(seconds)
    stop[0] = True
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    frames = sum(frames_done)
    return {"value": frames * 160 / dt, "unit": "samples/s", "cores": threads, "kind": kind,
            "sample": f"{threads} threads x 1 stream each, int8 synthetic model, {frames} frames in {dt:.1f}s "
                      f"({'reference vec_avx.h/kiss99/freq.c kernels compiled from /root/reference/src' if kind == 'reference' else 'portable oracle'}"
                      f" + oracle restatement of lpcnet.c/nnet.c)"}


def main():
    args = parse()
    world, rank, local, dist = dist_setup(args)
    import lpcnet_amd as L
    variant = L.VARIANT_INT8 if args.variant == "int8" else L.VARIANT_FP32
    blob = L.synthetic_model(1, variant)
    B = args.streams
    from lpcnet_amd.shard import weak_shard
    dt, (ks, kn, fs, fn), info, pcm = run_batch(L, blob, B, weak_shard(rank, B).start, args.warmup, args.steps, dist, args.timers)
    dt = max_over_ranks(dist, dt)
    samples = world * B * 160 * args.steps
    value = samples / dt
    # roofline of the dominant kernel (sample network), algorithmic bytes per launch
    sample_ms = ks / kn if kn else dt / args.steps * 1e3  # timers off: the frame step bounds the launch
    bytes_launch = 160 * info.bytes_shared_per_sample + B * 160 * info.bytes_per_stream_sample
    achieved = bytes_launch / (sample_ms * 1e-3) / 1e9
    kname = info.kernel_name
    pmc, tsrc = measured_pmc(kname) if B == 1024 else ({}, None)
    traffic = pmc.get("hbm_bytes_per_launch_corrected")
    out = {
        "metric": "real-time 16 kHz streams/GPU; samples/s at batch=1 and batch=1024",
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8" if variant == 0 else "f32",
        "data": "synthetic (deterministic kiss99 model of the default LPCNet size + synthetic features)",
        "config": {"workload": f"BASELINE configs[3]: {args.variant} path, {B} streams/GPU x 160-sample frames",
                   "streams_per_gpu": B, "global_streams": world * B, "frame_samples": 160,
                   "parallelism": f"stream shards x{world}, no collective"},
        "rt_streams_per_gpu": value / world / 16000.0,
        "frame_step_ms": dt / args.steps * 1e3,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc,
                     "kernel": kname, "avg_launch_ms": sample_ms, "launches": kn,
                     "algorithmic_bytes_per_launch": bytes_launch},
        "frame_kernel_avg_ms": fs / max(fn, 1),
        # matrix-core work of the sample kernel (north_star: MFMA at batch >= 256):
        # int8 ops issued per launch / launch time, and the PMC busy fraction
        "mfma": ({"achieved_tops": info.mfma_ops_per_group_sample * ((B + info.streams_per_workgroup - 1)
                                                                    // info.streams_per_workgroup) * 160
                                   / (sample_ms * 1e-3) / 1e12,
                  "peak_tops": I8_PEAK_TOPS, "busy_frac_pmc": pmc.get("mfma_util"),
                  "ops_per_launch": info.mfma_ops_per_group_sample * ((B + info.streams_per_workgroup - 1)
                                                                     // info.streams_per_workgroup) * 160}
                 if info.mfma_ops_per_group_sample > 0 else None),
        "kernel_config": {"streams_per_workgroup": info.streams_per_workgroup, "quad_path": info.quad_path,
                          "lds_bytes": info.lds_bytes, "gru_a_blocks": info.gru_a_blocks},
        "pcm_checksum": int(np.abs(pcm[-1].astype(np.int64)).sum()),
    }
    if rank == 0 and world == 1 and not args.no_batch1:
        dt1, (k1, n1, _, _), _, _ = run_batch(L, blob, 1, 0, args.warmup, max(args.steps, 20), None, args.timers)
        s1 = max(args.steps, 20) * 160 / dt1
        out["batch1"] = {"samples_per_s": s1, "x_realtime": s1 / 16000.0, "ms_per_frame": dt1 / max(args.steps, 20) * 1e3,
                         "sample_kernel_avg_ms": k1 / max(n1, 1), "path": "int8"}
        # BASELINE configs[1]: batch=1 with the fp32 (--disable-dot-product) GRU_A weights
        blob32 = L.synthetic_model(1, L.VARIANT_FP32)
        nf = max(args.steps, 20)
        dt2, (k2, n2, _, _), _, _ = run_batch(L, blob32, 1, 0, args.warmup, nf, None, args.timers)
        out["batch1_fp32"] = {"samples_per_s": nf * 160 / dt2, "x_realtime": nf * 160 / dt2 / 16000.0,
                              "ms_per_frame": dt2 / nf * 1e3, "sample_kernel_avg_ms": k2 / max(n2, 1)}
        # BASELINE configs[2]: 256 streams on one GPU (int8 products on the matrix cores)
        dt3, (k3, n3, _, _), info3, _ = run_batch(L, blob, 256, 0, args.warmup, nf, None, args.timers)
        out["batch256"] = {"samples_per_s": 256 * nf * 160 / dt3, "rt_streams": 256 * nf * 160 / dt3 / 16000.0,
                           "ms_per_frame": dt3 / nf * 1e3, "sample_kernel_avg_ms": k3 / max(n3, 1),
                           "kernel": info3.kernel_name}
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
