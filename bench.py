#!/usr/bin/env python3
"""bench.py -- LPCNet synthesis throughput on MI355X (BASELINE.json metric).

One "step" = one 10 ms frame (160 samples) for every stream of the batch:
lpc_from_cepstrum + frame network + 160 recurrent samples, device-resident
features and PCM (lpcnet_batch_synthesize_frames; everything inside the timed
region runs on the GPU).  Workload: BASELINE.json configs[3] -- int8 path,
1024 streams per GPU (configs[4] shards 1024 streams per GPU, weak scaling).
configs[1] (batch=1, fp32 and int8) and configs[2] (batch=256) are reported
alongside in `batch1`, `batch1_fp32`, `batch256`.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints one JSON line.

Roofline: algorithmic bytes per stream-sample = the shared
weight bytes of one sample step (GRU_A/GRU_B weights + idx + biases, plus the
frame network's 1.08 MB / 160) / B + 15,009 per-stream bytes (3 embedding rows,
the dual_fc path, conditioning share, PCM), recomputed from the loaded index;
per launch x 160 x B, over the sample kernel's HIP-event launch time.  `bound`
stays "hbm" as the contract prescribes, and the line says what actually
binds: `hbm_actual_GBs` / `l2_hit` from the PMC passes of this same source
tree (tools/gpu_evidence.sh -> pmc_traffic.json, used only when its
source_sha256 matches), and `latency` from an untimed s_memtime-stamped run
(critical-path cycles per sample x 160 / clock vs the measured launch).
"""
import argparse
import glob
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
I8_PEAK_TOPS = 5000.0  # MI355X_MICROARCH.md: int8 MFMA dense = 2x the ~2.5 PF bf16 rate
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md: L2 aggregate, measured
# MI355X_MICROARCH.md "Indexed rows: gather into LDS": 1,152-B rows shared by
# every workgroup (served by the XCD's L2) gather at 16.8-18.8 TB/s chip-wide;
# the upper figure is the peak the sample kernel's embedding gathers are priced at
L2_GATHER_PEAK_GBS = 18800.0
# VALU issue: 4 SIMD-32 per CU, one wave64 instruction per 2 cycles each
# (MI355X_MICROARCH.md "Wave scheduling") = 2 wave64 VALU instructions per
# CU-cycle, 256 CUs
VALU_ISSUE_PER_CU_CYCLE = 2.0
N_CU = 256
GATHER_BYTES_PER_STREAM_SAMPLE = 3 * 1152 * 4  # three embedding rows, nnet.c:484-491


def measured_pmc(config, kernel_name):
    """PMC record (tools/pmc_summary.py) of `kernel_name` in bench configuration
    `config` from the passes of THIS source tree: gpurun_out/ first (a pass
    just made on this box), then the committed profiles/r*/ (newest round
    first).  ({}, None) when no record matches the source hash."""
    from pmc_summary import source_sha256
    want = source_sha256(ROOT)
    cands = [os.path.join(ROOT, "gpurun_out", "pmc_traffic.json")]
    cands += sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")), reverse=True)
    for f in cands:
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("source_sha256") != want:
            continue
        for k, v in d.get("configs", {}).get(config, {}).items():
            if kernel_name in k:
                return v, os.path.relpath(f, ROOT)
    return {}, None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30, help="timed frames")
    p.add_argument("--warmup", type=int, default=3, help="untimed frames")
    p.add_argument("--streams", type=int, default=1024, help="streams per GPU")
    p.add_argument("--variant", choices=["int8", "fp32"], default="int8")
    p.add_argument("--no-batch1", action="store_true", help="skip the batch1 / batch1_fp32 / batch256 lines")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-dropin", action="store_true", help="skip the drop-in API real-time check (dropin_rt)")
    p.add_argument("--no-latency", action="store_true", help="skip the stamped latency run")
    p.add_argument("--no-capacity", action="store_true", help="skip the measured real-time capacity ladder")
    p.add_argument("--live-only", action="store_true",
                   help="headline, then only the live (per-frame host I/O) line and its capacity ladder")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--preheat-ms", type=float, default=100.0,
                   help="untimed load before the warmup (DPM clock ramp), then every stream is reset")
    p.add_argument("--detail", default=None,
                   help="side file for the full record (default gpurun_out/bench_detail.json)")
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


def run_batch(L, blob, B, stream_base, warmup, steps, timed_dist=None, timers=1, preheat_ms=0.0, kernel=0,
              rcp_table=None):
    """Returns (seconds for `steps` frames, kernel ms / launches, info, pcm).
    The timed region carries HIP events around each sample-kernel launch
    (timers=1; 2 adds the frame kernel); the frame kernel's own time comes
    from a short untimed pass with both kernels timed."""
    F = warmup + steps
    extra = min(steps, 32)  # one chunk of the chunked frame network (B > 128)
    feats = np.stack([L.synthetic_features(stream_base + s, F)[:, :20] for s in range(B)], 1)
    feats = np.ascontiguousarray(feats, np.float32)  # [F][B][20]
    ndev = max(1, L.device_count())
    b = L.LPCNetBatch(B, int(os.environ.get("LOCAL_RANK", "0")) % ndev, blob)
    if kernel:
        b.set_kernel(kernel)
    if rcp_table is not None:
        b.set_rcp_table(rcp_table)
    d_feat = b.device_alloc(feats.nbytes)
    d_pcm = b.device_alloc((F + extra) * B * 160 * 2)
    b.h2d(d_feat, feats)
    if preheat_ms > 0:
        # hold the GPU busy with this very workload until its clocks reach the
        # steady state of a continuously serving GPU, then reset every stream:
        # the warmup and timed frames below compute exactly what they would
        # without the preheat (same PCM)
        # (calls of `steps` frames: the same multi-frame launches as the
        # timed call, so a kernel trace of the run averages one population)
        t_end = time.perf_counter() + preheat_ms * 1e-3
        while time.perf_counter() < t_end:
            b.synthesize_frames(None, d_feat, d_pcm, steps)
            b.sync()
        b.reset()
    if warmup:
        b.synthesize_frames(None, d_feat, d_pcm, warmup)
    barrier_sync(timed_dist, b)
    b.reset_timers(timers)
    t0 = time.perf_counter()
    b.synthesize_frames(None, d_feat + warmup * B * 20 * 4, d_pcm + warmup * B * 160 * 2, steps)
    barrier_sync(timed_dist, b)
    dt = time.perf_counter() - t0
    ks, kn = b.kernel_ms(0)
    kf = b.kernel_frames(0)
    pcm = np.zeros((F, B, 160), np.int16)
    b.d2h(pcm, d_pcm)
    b.reset_timers(2)
    b.synthesize_frames(None, d_feat + warmup * B * 20 * 4, d_pcm + F * B * 160 * 2, extra)
    b.sync()
    fs, fn = b.kernel_ms(1)
    info = b.info()
    b.device_free(d_feat)
    b.device_free(d_pcm)
    b.close()
    return dt, (ks, kn, kf, fs / max(extra, 1), fn), info, pcm


def algorithmic_bytes_per_launch(info, B):
    """SURVEY 8d per stream-sample figure x 160 x B (one frame)"""
    per = (info.bytes_shared_per_sample + info.bytes_shared_per_frame / 160.0) / B + info.bytes_per_stream_sample
    return per * 160 * B, per


def roofline(info, B, frame_ms, config, frames_per_launch=1.0):
    """frame_ms: sample-kernel time per frame (a multi-frame launch of F
    frames takes F x frame_ms); bytes and ops per launch = per frame x F"""
    bytes_frame, per = algorithmic_bytes_per_launch(info, B)
    launch_ms = frame_ms * frames_per_launch
    bytes_launch = bytes_frame * frames_per_launch
    achieved = bytes_launch / (launch_ms * 1e-3) / 1e9
    pmc, src = measured_pmc(config, info.kernel_name)
    # HBM bytes per launch of frames_per_launch frames (the PMC passes may
    # have run launches of another length: scale their per-frame figure)
    traffic = (pmc["hbm_bytes_per_frame"] * frames_per_launch if "hbm_bytes_per_frame" in pmc
               else pmc.get("hbm_bytes_per_launch"))
    r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
         "traffic": traffic, "kernel": info.kernel_name, "avg_launch_ms": launch_ms,
         "frames_per_launch": frames_per_launch, "ms_per_frame": frame_ms,
         "algorithmic_bytes_per_launch": bytes_launch, "algorithmic_bytes_per_stream_sample": per,
         "pmc_source": src,
         # what the counters say actually moves: HBM bytes / launch time, and the
         # L2 hit rate of the gathers (the algorithmic bytes are served by L2)
         "hbm_actual_GBs": traffic / (launch_ms * 1e-3) / 1e9 if traffic else None,
         "l2_hit": pmc.get("l2_hit"),
         "l2_frac": achieved / L2_PEAK_GBS,
         "pmc_frames_per_launch": pmc.get("frames_per_launch")}
    # the resource that serves the algorithmic bytes: the gathered embedding
    # rows come from the XCD's L2 (l2_hit ~0.99), priced at the guide's
    # shared-row gather rate
    gath = GATHER_BYTES_PER_STREAM_SAMPLE * 160 * B * frames_per_launch
    r["roofline_l2"] = {"bound": "l2_gather", "achieved": gath / (launch_ms * 1e-3) / 1e9,
                        "peak": L2_GATHER_PEAK_GBS, "unit": "GB/s",
                        "frac": gath / (launch_ms * 1e-3) / 1e9 / L2_GATHER_PEAK_GBS,
                        "bytes_per_stream_sample": GATHER_BYTES_PER_STREAM_SAMPLE,
                        "what": "3 embedding rows per stream-sample (nnet.c:484-491) against the 16.8-18.8 TB/s "
                                "shared-row gather rate of MI355X_MICROARCH.md"}
    # VALU issue from the PMC pass of this tree (SQ_INSTS_VALU per frame)
    if "valu_insts_per_frame" in pmc or "valu_insts_per_launch" in pmc:
        per_frame = pmc.get("valu_insts_per_frame")
        if per_frame is None:
            per_frame = pmc["valu_insts_per_launch"] / max(pmc.get("frames_per_launch") or frames_per_launch, 1)
        insts = per_frame * frames_per_launch
        peak = VALU_ISSUE_PER_CU_CYCLE * N_CU * (clock_ghz() * 1e9)
        r["valu"] = {"bound": "valu_issue", "insts_per_stream_sample": per_frame / (160 * B),
                     "achieved_insts_per_s": insts / (launch_ms * 1e-3), "peak_insts_per_s": peak,
                     "frac": insts / (launch_ms * 1e-3) / peak, "frac_pmc_busy_cycles": pmc.get("valu_issue_frac"),
                     "what": "wave64 VALU instructions (SQ_INSTS_VALU) against 2 per CU-cycle x 256 CUs at the "
                             "2.4 GHz spec clock"}
    r["binding"] = binding_text(r, pmc)
    mf = None
    if info.mfma_ops_per_group_sample > 0:
        groups = (B + info.streams_per_workgroup - 1) // info.streams_per_workgroup
        ops = info.mfma_ops_per_group_sample * groups * 160 * frames_per_launch
        mf = {"achieved_tops": ops / (launch_ms * 1e-3) / 1e12, "peak_tops": I8_PEAK_TOPS,
              "ops_per_launch": ops, "busy_frac_pmc": pmc.get("mfma_util")}
    return r, mf


def clock_ghz():
    """shader clock of the VALU peak: the 2.4 GHz spec maximum (the measured
    clock under load is lower, so the fraction is a lower bound)"""
    return 2.4


def binding_text(r, pmc):
    """What actually binds the sample kernel, beside the contract's HBM figure."""
    parts = []
    if r.get("hbm_actual_GBs"):
        parts.append(f"HBM traffic {r['hbm_actual_GBs']:.0f} GB/s = {r['hbm_actual_GBs'] / HBM_PEAK_GBS:.3f} of peak "
                     f"(weights in registers/LDS, tables in L2, l2_hit {pmc.get('l2_hit', 0):.3f})")
    parts.append(f"L2 gathers {r['roofline_l2']['frac']:.2f} of the shared-row rate")
    if "valu" in r:
        parts.append(f"VALU issue {r['valu']['frac']:.2f} of peak")
    if pmc.get("mfma_util") is not None:
        parts.append(f"MFMA busy {pmc['mfma_util']:.2f}")
    parts.append("none saturated: the per-sample recurrence (walk -> gathers -> GRU_A elementwise -> GRU_B) "
                 "is a latency chain; see `latency`")
    return "; ".join(parts)


def latency(L, blob, B, measured_ms):
    """Critical path of the sample kernel from s_memtime phase stamps (one
    untimed stamped frame): cycles per sample x 160 / clock, against the
    measured (unstamped) launch.  The stamped launch itself runs ~5-10 %
    slower (instrumentation)."""
    F = 4
    b = L.LPCNetBatch(B, int(os.environ.get("LOCAL_RANK", "0")) % max(1, L.device_count()), blob)
    allf = np.stack([L.synthetic_features(s, F)[:, :20] for s in range(B)], 1)
    for f in range(F - 1):
        b.synthesize(allf[f])
    b.set_stamps(True)
    b.reset_timers(1)
    b.synthesize(allf[F - 1])
    kms, kn = b.kernel_ms(0)
    st = b.get_stamps().astype(np.float64)  # [groups][8 waves][16]
    info = b.info()
    b.close()
    n = max(st[:, :, 7].max(), 1)
    per = st / n
    loop = per[:, :, 6].max(axis=1).mean()
    stamped_ms = kms / max(kn, 1)
    clock = st[:, :, 6].max() / (stamped_ms * 1e-3) / 1e9
    out = {"kernel": info.kernel_name, "cycles_per_sample": loop, "clock_ghz_stamped": clock,
           "stamped_launch_ms": stamped_ms, "predicted_launch_ms": loop * 160 / (clock * 1e9) * 1e3,
           "measured_ms_per_frame": measured_ms,
           "cycles_per_sample_at_measured": loop * measured_ms / stamped_ms}
    if info.quad_path == 4:
        ga = per[:, :6, :].mean(axis=0)   # GRU_A waves [6][16]
        sm = per[:, 6, :].mean(axis=0)    # sampler wave 6
        out["critical_path_cycles"] = {
            "gru_a_gathers": float(ga[:, 10].max()),
            "gru_a_elementwise_slowest_wave": float(ga[:, 0].max()),
            "gru_a_elementwise_fastest_wave": float(ga[:, 0].min()),
            "sampler_gru_b": float(sm[8] + sm[10] + sm[14]),
            "sampler_walk": float(sm[11]),
            "sampler_post": float(sm[12]),
            "sampler_wait_at_Y": float(sm[1]),
            "sampler_wait_at_X": float(sm[5]),
            "gru_a_recurrent_slowest_wave": float(ga[:, 2].max()),
            "gru_a_wait_at_X_fastest_wave": float(ga[:, 5].min()),
        }
    elif info.quad_path == 5:
        # fp_kernel (fp32, one stream per workgroup): hardware wave
        # FP_SAMPLER_HW = 3 is the sampler, the other six run GRU_A units
        ga = np.delete(per[:, :7, :], 3, axis=1).mean(axis=0)  # [6][16]
        sm = per[:, 3, :].mean(axis=0)
        out["critical_path_cycles"] = {
            "gru_a_wait_indices": float(ga[:, 0].max()),
            "gru_a_gathers": float(ga[:, 1].max()),
            "gru_a_zr_chains_slowest_wave": float(ga[:, 2].max()),
            "gru_a_elementwise": float(ga[:, 3].max()),
            "gru_a_h_chain_next": float(ga[:, 8].max()),
            "sampler_bookkeeping_gru_b_recurrent": float(sm[0]),
            "sampler_wait_first_units": float(sm[1]),
            "sampler_gru_b_input_chain": float(sm[2]),
            "sampler_gru_b_update": float(sm[3]),
            "sampler_walk": float(sm[4]),
        }
    if info.quad_path == 4:
        if os.environ.get("LPCNET_WALK_STAMPS"):
            out["walk_cycles"] = {"level0_3_logit": float(sm[2]), "level0_3_decide_and_w47": float(sm[3]),
                                  "level4_7_logit": float(sm[15]), "decide_select": float(sm[11])}
        if os.environ.get("LPCNET_FINE_STAMPS"):
            out["gru_a_waves"] = {f"w{w}": {"gathers": float(ga[w, 10]), "inputs": float(ga[w, 11]), "sigmoid": float(ga[w, 12]),
                                            "tanh_update": float(ga[w, 13]), "quant_store": float(ga[w, 0]),
                                            "waitY": float(ga[w, 1]), "recurrent": float(ga[w, 2]), "waitX": float(ga[w, 5])}
                                  for w in range(6)}
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def physical_cores():
    """Distinct (physical id, core id) pairs of /proc/cpuinfo (SMT siblings
    counted once); os.cpu_count() if unreadable."""
    ids, phys = set(), None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":", 1)[1].strip()
            elif line.startswith("core id"):
                ids.add((phys, line.split(":", 1)[1].strip()))
    except OSError:
        pass
    return len(ids) or os.cpu_count()


# the calibration of this baseline against the
# compiled reference, measured in the build container (tools/cpu_calibrate.py)
CPU_CALIBRATION = ("restatement glue at the reference's -O3 -mavx2 -mfma flags + the reference's own kernels: "
                   "189-233 K samples/s/core on the build container's Xeon = 0.88-1.09x the survey's "
                   "-O2 -mavx2 -mfma reference build (214 K) and 0.65-0.80x its -O3 -march=native build (290 K), "
                   "two runs of best-of-6 alternating rounds (BASELINE.md section 3, profiles/r04/cpu_calibration.json)")


def cpu_baseline(seconds, variant=0):
    """The reference's own AVX2 kernels (oracle/_ref, compiled from the
    reference sources) driven by the oracle's lpcnet.c/nnet.c restatement
    built with the reference's optimisation flags (oracle/Makefile
    BASE_CFLAGS: -O3 -mavx2 -mfma -ffp-contract=off; bit-identical to the
    portable build), one stream per worker thread, one worker pinned per host
    core this process may use.  On the GPU box that is the harness's CPU
    share for one GPU (OMP_NUM_THREADS = 16 there; the affinity mask shows
    the whole machine), so `per_core` is the number to scale to a node
    (`node_extrapolated`: per_core x the machine's physical cores).
    variant 1: the reference's --disable-dot-product build (fp32 GRU weights,
    vec_avx.h:861-904 compiled with DISABLE_DOT_PROD), beside configs[1]'s
    batch1_fp32 line."""
    import lpcnet_amd as L
    import oracle_lib as O
    kind = "reference" if O.have_ref() else "port"
    kernels = O.ref_kernels() if O.have_ref() else None
    avx2 = O.have_avx2_build()
    blob = L.synthetic_model(1, variant)
    cpus = sorted(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(len(cpus), share) if share > 0 else len(cpus))
    # warm the lazily built tables on one thread first
    O.Oracle(blob, variant, kernels, avx2_build=avx2).synthesize(L.synthetic_features(0, 1)[0])
    frames_done = [0] * threads
    stop = [False]

    def work(t):
        try:
            os.sched_setaffinity(threading.get_native_id(), {cpus[t % len(cpus)]})
        except OSError:
            pass
        o = O.Oracle(blob, variant, kernels, avx2_build=avx2)
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
    value = frames * 160 / dt
    pc = physical_cores()
    return {"value": value, "unit": "samples/s", "cores": threads, "kind": kind,
            "per_core": value / threads, "physical_cores": pc, "node_extrapolated": value / threads * pc,
            "cpu_model": cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": len(cpus),
            "glue_build": "-O3 -mavx2 -mfma -ffp-contract=off" if avx2 else "-O2 portable",
            "sample": f"{threads} pinned threads x 1 stream each (one per core of this process's CPU share), "
                      f"{'fp32 (--disable-dot-product)' if variant else 'int8'} "
                      f"synthetic model, {frames} frames in {dt:.1f}s "
                      f"({'reference vec_avx.h/kiss99/freq.c kernels compiled from /root/reference/src' if kind == 'reference' else 'portable oracle'}"
                      f" + oracle restatement of lpcnet.c/nnet.c; calibration: {CPU_CALIBRATION})"}


def side_line(L, blob, B, args, config, variant_name):
    nf = max(args.steps, 20)
    dt, (k, n, kf, _, _), info, _ = run_batch(L, blob, B, 0, args.warmup, nf, None, args.timers, args.preheat_ms)
    frame_ms = k / max(kf, 1)
    rf, mf = roofline(info, B, frame_ms, config, kf / max(n, 1))
    out = {"samples_per_s": B * nf * 160 / dt, "rt_streams": B * nf * 160 / dt / 16000.0, "x_realtime_per_stream":
           nf * 160 / dt / 16000.0, "ms_per_frame": dt / nf * 1e3, "sample_kernel_ms_per_frame": frame_ms,
           "sample_kernel_avg_launch_ms": k / max(n, 1),
           "kernel": info.kernel_name, "path": variant_name, "roofline": rf}
    if mf:
        out["mfma"] = mf
    if not args.no_latency:
        # what binds at this size: the stamped per-sample critical path
        out["latency"] = latency(L, blob, B, frame_ms)
    return out


def capacity(L, blob, args, ladder=(1024, 1025, 1536, 2048, 4096, 8192, 16384, 24576, 28672, 32768, 36864, 40960,
                                     49152, 57344)):
    """Throughput ceiling of one GPU (not a real-time figure: see
    capacity_live): the whole frame step (LPC, frame network, 160 samples
    of every stream; device-resident I/O, 6-frame launches, i.e. 60 ms of
    features handed over in advance) timed at each batch size of the
    ladder, including the non-multiples 1025 and 1536 of the
    4-streams-per-workgroup, 1024-streams-per-round layout; the largest
    batch whose mean frame step stays <= 10 ms is bracketed by bisection
    (multiples of 256)."""
    steps = 6
    rows = {}

    def run(B):
        dt, _, info, _ = run_batch(L, blob, B, 0, 2, steps, None, 0, 0.0)
        ms = dt / steps * 1e3
        rows[B] = {"frame_step_ms": ms, "samples_per_s": B * 160 * steps / dt, "realtime": ms <= 10.0,
                   "streams_per_workgroup": info.streams_per_workgroup}
        return ms

    ok, bad = 0, None
    for B in ladder:
        if run(B) <= 10.0:
            ok = max(ok, B)
        else:
            bad = B
            break
    if bad is not None:
        lo, hi = ok, bad
        while hi - lo > 256:
            mid = (lo + hi) // 2 // 256 * 256
            if mid <= lo:
                break
            if run(mid) <= 10.0:
                lo = mid
            else:
                hi = mid
        ok = lo
    return {"max_streams": ok,
            "criterion": "throughput ceiling: mean frame step of 6-frame device-resident launches "
                         "(10 ms of audio for every stream) <= 10 ms",
            "steps_per_point": steps, "ladder": {str(k): v for k, v in sorted(rows.items())}}


def run_live(L, blob, B, warmup, steps, preheat_ms=0.0, engine_buffers=True, distinct_frames=None):
    """A live server's tick, frame by frame: every 10 ms of audio the host
    hands over B feature frames (host memory) and takes back B x 160 PCM
    samples (host memory) -- lpcnet_batch_synthesize once per frame
    (lpcnet_demo.c:208-219's loop for B streams at once; PCIe copies, the
    LPC, frame and sample kernels and the synchronisation all inside the
    timed region).  engine_buffers: the features are written into the
    batch's feature buffer (host-visible VRAM on large-BAR devices, else
    pinned host memory) and the PCM is read from its pinned PCM buffer
    (lpcnet_batch_host_features / _pcm: no staging copies, the sample
    kernel stores the PCM over PCIe itself); otherwise the caller's
    own numpy arrays in and out.  distinct_frames: the streams' feature
    frames cycle with this period (long tick runs at large B without
    generating every frame).  Returns (seconds per frame for each timed
    frame, pcm of the last frame)."""
    F = warmup + steps
    nd = min(F, distinct_frames) if distinct_frames else F
    feats = np.ascontiguousarray(np.stack([L.synthetic_features(s, nd)[:, :20] for s in range(B)], 1), np.float32)
    b = L.LPCNetBatch(B, int(os.environ.get("LOCAL_RANK", "0")) % max(1, L.device_count()), blob)
    if engine_buffers:
        hf = b.host_features()

        def tick(f):
            np.copyto(hf, feats[f % nd])
            return b.synthesize_host()
    else:
        def tick(f):
            return b.synthesize(feats[f % nd])
    if preheat_ms > 0:
        t_end = time.perf_counter() + preheat_ms * 1e-3
        k = 0
        while time.perf_counter() < t_end:
            tick(k % F)
            k += 1
        b.reset()
    for f in range(warmup):
        tick(f)
    per = []
    pcm = None
    for f in range(warmup, F):
        t0 = time.perf_counter()
        pcm = tick(f)
        per.append(time.perf_counter() - t0)
    pcm = np.array(pcm)
    b.close()
    return np.array(per), pcm


def _json_scalar(o):
    """numpy scalars (np.bool_, np.float64 ...) in the line as their Python values"""
    if isinstance(o, np.generic):
        return o.item()
    raise TypeError(f"bench line: {type(o).__name__} is not JSON serialisable")


def live_line(L, blob, B, args, device_resident_value):
    nf = max(args.steps, 20)
    out = {}
    for key, eb in (("engine_buffers", True), ("caller_buffers", False)):
        per, _ = run_live(L, blob, B, args.warmup, nf, args.preheat_ms, engine_buffers=eb)
        v = float(B * 160 * len(per) / per.sum())
        out[key] = {"samples_per_s": v, "ms_per_frame": float(per.mean()) * 1e3,
                    "ms_per_frame_p50": float(np.median(per)) * 1e3,
                    "ms_per_frame_p99": float(np.percentile(per, 99)) * 1e3, "ms_per_frame_max": float(per.max()) * 1e3,
                    "frames": len(per),
                    "vs_device_resident": v / device_resident_value if device_resident_value else None}
    res = dict(out["engine_buffers"])
    res["caller_buffers"] = out["caller_buffers"]
    res["what"] = ("host features in, host PCM out, one lpcnet_batch_synthesize per 10 ms frame (PCIe-inclusive; "
                   "the headline `value` keeps the inputs resident in HBM); top level: features written into the "
                   "batch's feature buffer (host-visible VRAM on large-BAR devices) and PCM read from its pinned PCM "
                   "buffer (lpcnet_batch_host_features / _pcm); caller_buffers: "
                   "the caller's own arrays, staged through pinned memory by the engine")
    return res


def capacity_live(L, blob, ticks=100, warmup=10,
                  ladder=(1024, 2048, 4096, 8192, 16384, 24576, 28672, 32768, 36864, 40960, 49152, 57344)):
    """Real-time capacity of one GPU (lpcnet_demo.c:208-219: one frame of
    every stream handed over each 10 ms, a stream that misses a tick
    underruns): the largest batch whose per-frame host-I/O step
    (lpcnet_batch_synthesize: features from host memory, PCM to host
    memory, one call per frame) keeps its p99 over `ticks` consecutive
    ticks <= 10 ms, after `warmup` untimed ticks (the clocks of a serving
    GPU); bracketed by bisection in steps of 256.  Mean and max beside it
    (the max of 100 ticks is the 1 % tail's worst frame)."""
    rows = {}

    def run(B):
        per, _ = run_live(L, blob, B, warmup, ticks, distinct_frames=16)
        per = per * 1e3
        p99 = float(np.percentile(per, 99))
        rows[B] = {"frame_step_ms_p99": p99, "frame_step_ms_max": float(per.max()),
                   "frame_step_ms_mean": float(per.mean()), "samples_per_s": float(B * 160 / per.mean() * 1e3),
                   "realtime_p99": bool(p99 <= 10.0), "realtime_max": bool(per.max() <= 10.0)}
        return p99

    ok, bad = 0, None
    for B in ladder:
        if run(B) <= 10.0:
            ok = max(ok, B)
        else:
            bad = B
            break
    if bad is not None:
        lo, hi = ok, bad
        while hi - lo > 256:
            mid = (lo + hi) // 2 // 256 * 256
            if mid <= lo:
                break
            if run(mid) <= 10.0:
                lo = mid
            else:
                hi = mid
        ok = lo
    ok_max = max([B for B, r in rows.items() if r["realtime_max"] and all(
        rows[b]["realtime_max"] for b in rows if b < B)] or [0])
    return {"max_realtime_streams": ok, "max_realtime_streams_on_max": ok_max,
            "criterion": f"p99 of {ticks} consecutive per-frame host-I/O ticks (features in / PCM out over PCIe, "
                         f"one lpcnet_batch_synthesize per 10 ms frame, after {warmup} untimed ticks) <= 10 ms",
            "ticks_per_point": ticks, "ladder": {str(k): v for k, v in sorted(rows.items())}}


def dropin_rt(threads=(256, 960), frames=300):
    """The drop-in API (include/lpcnet.h, one LPCNetState per stream,
    lpcnet.c:213-219, 279-281) paced in real time from C threads
    (tools/dropin_bench rt): each thread calls lpcnet_synthesize once per 10
    ms tick, phases spread over the tick and all on one phase ("burst");
    per-call latency p50 / p99 / max and deadline misses.  Runs as a child
    process before this process touches the GPU; None when the binary is
    absent (make dropin).  The thread counts stop at 960: one thread per
    stream is the reference's calling pattern, and the GPU box limits a
    job's tasks."""
    import subprocess
    exe = os.path.join(ROOT, "tools", "dropin_bench")
    if not os.path.exists(exe):
        return None
    pts = []
    for T in threads:
        for mode in ("spread", "burst"):
            try:
                r = subprocess.run([exe, str(T), str(frames), "rt", mode], capture_output=True, text=True, timeout=120)
                pts.append(json.loads(r.stdout.strip().splitlines()[-1]))
            except (subprocess.SubprocessError, ValueError, IndexError, OSError) as e:
                pts.append({"threads": T, "mode": mode, "error": str(e)[:200]})
    # a thread count is real-time when both pacings are (spread and burst)
    ok = [T for T in threads if all(p.get("realtime_p99") is True for p in pts if p.get("threads") == T)
          and any(p.get("threads") == T for p in pts)]
    worst = {m: max((p for p in pts if p.get("mode") == m and "latency_ms_p99" in p), key=lambda p: p["threads"],
                    default=None) for m in ("spread", "burst")}
    return {"max_threads_realtime_p99": max(ok) if ok else 0, "max_threads_measured": max(threads),
            "criterion": "p99 per-call latency of lpcnet_synthesize <= 10 ms, one C thread per stream paced at one "
                         "frame per 10 ms", "points": pts,
            "at_max": {m: {k: w[k] for k in ("latency_ms_p50", "latency_ms_p99", "latency_ms_max", "deadline_misses",
                                             "calls", "mean_coalesced_streams")} for m, w in worst.items() if w}}


def skewed_lines(L, args):
    """A trained-model-like sparsity pattern (Sparsify's global per-gate
    threshold over skewed block energies, training_tf2/lpcnet.py:140-160:
    block rows of up to 76 (z/r) and 96 (h) blocks): which kernel runs it and
    its throughput at the three batch sizes of the default-model lines."""
    blob = L.synthetic_model(1, L.VARIANT_INT8, skewed=True)
    out = {}
    for B in (1, 256, 1024, 2048, 8192):
        nf = max(args.steps, 20)
        dt, (k, n, kf, _, _), info, _ = run_batch(L, blob, B, 0, args.warmup, nf, None, args.timers, args.preheat_ms)
        out[f"b{B}"] = {"samples_per_s": B * nf * 160 / dt, "sample_kernel_ms_per_frame": k / max(kf, 1),
                        "kernel": info.kernel_name, "quad_path": info.quad_path}
    return out


def host_rcpps_lines(L, args):
    """Same-box numerics: the engine with THIS host's rcpps table
    (lpcnet_batch_set_rcp_table; LPCNET_RCP=host for the drop-in API), i.e.
    the PCM the reference prints on this CPU (vec_avx.h:408,437), beside the
    default (Intel-table) numerics of the headline, at 1 and 1024 streams:
    the fast kernels' table-only forms."""
    tab, bad = L.host_rcp_table()
    out = {"host_table_exact": bad == 0}
    blob = L.synthetic_model(1, L.VARIANT_INT8)
    for B in (1, 1024):
        nf = max(args.steps, 20)
        dt, (k, n, kf, _, _), info, _ = run_batch(L, blob, B, 0, args.warmup, nf, None, args.timers, args.preheat_ms,
                                                  rcp_table=tab)
        out[f"b{B}"] = {"samples_per_s": B * nf * 160 / dt, "sample_kernel_ms_per_frame": k / max(kf, 1),
                        "kernel": info.kernel_name, "quad_path": info.quad_path}
    return out


def lockstep_lines(L, args):
    """The lockstep sample kernel (kernels.hip, mode 1): the kernel of every
    model the fast kernels do not take -- saturating int8 models (int16
    maddubs saturation emulated), fp32 models with a sparse GRU_B -- and of
    the same-box parity mode.  Measured on the saturating int8 model at 1024
    streams (automatic selection), and forced on the default int8 model at
    1024 streams and the default fp32 model at batch 1, beside the fast
    kernels' lines for the same models."""
    out = {}
    cases = (("sat_int8_b1024", L.synthetic_model(1, L.VARIANT_INT8, saturating=True), 1024, 0),
             ("int8_b1024_forced", L.synthetic_model(1, L.VARIANT_INT8), 1024, 1),
             ("fp32_b1_forced", L.synthetic_model(1, L.VARIANT_FP32), 1, 1))
    for name, blob, B, mode in cases:
        nf = max(args.steps, 20)
        dt, (k, n, kf, _, _), info, _ = run_batch(L, blob, B, 0, args.warmup, nf, None, args.timers, args.preheat_ms,
                                                  kernel=mode)
        out[name] = {"samples_per_s": B * nf * 160 / dt, "sample_kernel_ms_per_frame": k / max(kf, 1),
                     "kernel": info.kernel_name, "quad_path": info.quad_path}
    return out


def _r(x, nd=4):
    """a float rounded to `nd` significant digits (None passes)"""
    if x is None:
        return None
    x = float(x)
    return float(f"{x:.{nd}g}")


def _roof_short(rf):
    if not rf:
        return None
    o = {k: _r(rf.get(k)) if isinstance(rf.get(k), float) else rf.get(k)
         for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "avg_launch_ms",
                   "frames_per_launch", "algorithmic_bytes_per_launch", "algorithmic_bytes_per_stream_sample",
                   "hbm_actual_GBs", "l2_hit", "pmc_source")}
    if "roofline_l2" in rf:
        o["roofline_l2"] = {"bound": "l2_gather", "achieved": _r(rf["roofline_l2"]["achieved"]),
                            "peak": rf["roofline_l2"]["peak"], "frac": _r(rf["roofline_l2"]["frac"])}
    if "valu" in rf:
        o["valu"] = {"frac": _r(rf["valu"]["frac"]), "frac_pmc_busy_cycles": _r(rf["valu"].get("frac_pmc_busy_cycles")),
                     "insts_per_stream_sample": _r(rf["valu"]["insts_per_stream_sample"])}
    return o


def _side_short(d):
    if not d:
        return None
    o = {"samples_per_s": _r(d["samples_per_s"]), "kernel": d.get("kernel"),
         "sample_kernel_ms_per_frame": _r(d.get("sample_kernel_ms_per_frame"))}
    rf = d.get("roofline")
    if rf:
        o["roofline_frac"] = _r(rf["frac"])
        o["traffic"] = rf.get("traffic")
        o["l2_hit"] = _r(rf.get("l2_hit"))
        if "roofline_l2" in rf:
            o["l2_gather_frac"] = _r(rf["roofline_l2"]["frac"])
        if "valu" in rf:
            o["valu_frac"] = _r(rf["valu"]["frac"])
    if d.get("mfma"):
        o["mfma_busy_pmc"] = _r(d["mfma"].get("busy_frac_pmc"))
    return o


def _cpu_short(c):
    if not c:
        return None
    return {"value": _r(c["value"]), "unit": c["unit"], "cores": c["cores"], "kind": c["kind"],
            "per_core": _r(c["per_core"]), "cpu_model": c.get("cpu_model"),
            "sample": c["sample"].split(" (")[0]}


def compact_line(out, detail_path):
    """The driver's JSON line (<6 KB): the contract keys, the roofline and
    cpu_baseline objects, one-number summaries of every side measurement;
    the full record is in `detail_path`."""
    c = {k: out[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                             "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config") if k in out}
    rf = _roof_short(out.get("roofline"))
    if rf is not None and out.get("roofline", {}).get("binding"):
        rf["binding"] = out["roofline"]["binding"].split("; none saturated")[0]
    c["roofline"] = rf
    if out.get("mfma"):
        c["mfma"] = {"achieved_tops": _r(out["mfma"]["achieved_tops"]), "peak_tops": out["mfma"]["peak_tops"],
                     "busy_frac_pmc": _r(out["mfma"].get("busy_frac_pmc"))}
    for k in ("cpu_baseline", "cpu_baseline_fp32"):
        if k in out:
            c[k] = _cpu_short(out[k])
    cl = out.get("capacity_live")
    if cl:
        # the real-time figure: tail criterion on consecutive live ticks
        c["realtime_streams_per_gpu"] = cl["max_realtime_streams"]
    c["throughput_rt_equiv_streams_per_gpu"] = _r(out.get("rt_streams_per_gpu"))
    c["frame_step_ms"] = _r(out.get("frame_step_ms"))
    for k in ("batch1", "batch1_fp32", "batch256", "batch8192"):
        if k in out:
            c[k] = _side_short(out[k])
    if "live" in out:
        lv = out["live"]
        c["live"] = {"streams": out["config"].get("streams_per_gpu"), "samples_per_s": _r(lv["samples_per_s"]),
                     "vs_device_resident": _r(lv["vs_device_resident"]), "ms_per_frame": _r(lv["ms_per_frame"]),
                     "ms_per_frame_p99": _r(lv.get("ms_per_frame_p99")),
                     "caller_buffers_samples_per_s": _r(lv["caller_buffers"]["samples_per_s"])}
    if cl:
        top = cl["ladder"].get(str(cl["max_realtime_streams"]), {})
        c["capacity_live"] = {"max_realtime_streams": cl["max_realtime_streams"],
                              "max_realtime_streams_on_max": cl.get("max_realtime_streams_on_max"),
                              "ticks_per_point": cl.get("ticks_per_point"),
                              "at_max": {k: _r(v) for k, v in top.items() if isinstance(v, float)},
                              "criterion": cl["criterion"]}
    for k in ("capacity", "capacity_skewed"):
        if k in out:
            cp = out[k]
            top = cp["ladder"].get(str(cp["max_streams"]), {})
            c[k] = {"max_streams": cp["max_streams"], "frame_step_ms_at_max": _r(top.get("frame_step_ms")),
                    "samples_per_s_at_max": _r(top.get("samples_per_s")), "criterion": cp["criterion"]}
    if "skewed_int8" in out:
        c["skewed_int8"] = {k: _r(v["samples_per_s"]) for k, v in out["skewed_int8"].items()}
    if out.get("dropin_rt"):
        d = out["dropin_rt"]
        c["dropin_rt"] = {"max_threads_realtime_p99": d["max_threads_realtime_p99"],
                          "max_threads_measured": d["max_threads_measured"],
                          "at_max": {m: {k: _r(v) if isinstance(v, float) else v for k, v in w.items()}
                                     for m, w in d.get("at_max", {}).items()},
                          "criterion": d["criterion"]}
    if "latency" in out:
        c["latency_cycles_per_sample"] = _r(out["latency"].get("cycles_per_sample_at_measured"))
    c["pcm_checksum"] = out.get("pcm_checksum")
    c["detail"] = detail_path
    return c


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank0 = int(os.environ.get("RANK", "0")) == 0
    # the drop-in real-time check runs as a child process, before this
    # process initialises the GPU
    drt = dropin_rt() if rank0 and world == 1 and not (args.no_batch1 or args.live_only or args.no_dropin) else None
    world, rank, local, dist = dist_setup(args)
    import lpcnet_amd as L
    variant = L.VARIANT_INT8 if args.variant == "int8" else L.VARIANT_FP32
    blob = L.synthetic_model(1, variant)
    B = args.streams
    from lpcnet_amd.shard import weak_shard
    dt, (ks, kn, kf, fs, fn), info, pcm = run_batch(L, blob, B, weak_shard(rank, B).start, args.warmup, args.steps, dist,
                                                args.timers, args.preheat_ms)
    dt = max_over_ranks(dist, dt)
    samples = world * B * 160 * args.steps
    value = samples / dt
    # sample-kernel time per frame (timers off: the frame step bounds it)
    sample_ms = ks / kf if kf else dt / args.steps * 1e3
    config = {1024: "b1024", 256: "b256", 1: "b1"}.get(B, f"b{B}") + ("_fp32" if variant else "")
    rf, mf = roofline(info, B, sample_ms, config, kf / kn if kn else 1.0)
    out = {
        "metric": "real-time 16 kHz streams/GPU; samples/s at batch=1 and batch=1024",
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "preheat_ms": args.preheat_ms,
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
        "roofline": rf,
        "frame_network_ms_per_frame": fs,
        # matrix-core work of the sample kernel (north_star: MFMA at batch >= 256):
        # int8 ops issued per launch / launch time, and the PMC busy fraction
        "mfma": mf,
        "kernel_config": {"streams_per_workgroup": info.streams_per_workgroup, "quad_path": info.quad_path,
                          "lds_bytes": info.lds_bytes, "gru_a_blocks": info.gru_a_blocks},
        "pcm_checksum": int(np.abs(pcm[-1].astype(np.int64)).sum()),
    }
    if rank == 0 and world == 1 and not args.no_latency:
        out["latency"] = latency(L, blob, B, sample_ms)
    if rank == 0 and world == 1 and not args.no_batch1:
        out["batch1"] = side_line(L, blob, 1, args, "b1", "int8")
        # BASELINE configs[1]: batch=1 with the fp32 (--disable-dot-product) GRU_A weights
        out["batch1_fp32"] = side_line(L, L.synthetic_model(1, L.VARIANT_FP32), 1, args, "b1_fp32", "fp32")
        # BASELINE configs[2]: 256 streams on one GPU (int8 products on the matrix cores)
        out["batch256"] = side_line(L, blob, 256, args, "b256", "int8")
        # the wide-batch kernel (mfw_kernel) that carries the capacity figures
        out["batch8192"] = side_line(L, blob, 8192, args, "b8192", "int8")
    if rank == 0 and world == 1 and not args.no_batch1:
        out["skewed_int8"] = skewed_lines(L, args)
        out["lockstep"] = lockstep_lines(L, args)
        out["host_rcpps"] = host_rcpps_lines(L, args)
    if rank == 0 and world == 1 and (not args.no_batch1 or args.live_only):
        # the same workload as a live server runs it: host I/O every frame
        out["live"] = live_line(L, blob, B, args, value)
    if rank == 0 and world == 1 and args.live_only:
        out["capacity_live"] = capacity_live(L, blob)
    if rank == 0 and world == 1 and not args.no_capacity and not args.live_only:
        out["capacity"] = capacity(L, blob, args)
        out["capacity_live"] = capacity_live(L, blob)
        # the same ladder on the trained-like (Sparsify) sparsity pattern
        out["capacity_skewed"] = capacity(L, L.synthetic_model(1, L.VARIANT_INT8, skewed=True), args)
    if drt is not None:
        out["dropin_rt"] = drt
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        # beside batch1_fp32 (configs[1]): the reference's fp32 build on the same cores
        out["cpu_baseline_fp32"] = cpu_baseline(args.cpu_seconds, 1)
    if rank == 0:
        # the full record (ladders, latency objects, PMC-derived objects) goes
        # to a side file; stdout's last line is the compact record the
        # driver parses
        detail = args.detail or os.path.join(ROOT, "gpurun_out", "bench_detail.json")
        try:
            os.makedirs(os.path.dirname(detail), exist_ok=True)
            with open(detail, "w") as f:
                json.dump(out, f, default=_json_scalar, indent=1)
        except OSError as e:
            print(f"bench: detail file not written ({e})", file=sys.stderr)
            detail = None
        print(json.dumps(compact_line(out, detail and os.path.relpath(detail, ROOT)), default=_json_scalar),
              flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
