"""Sharded multi-rank path (streams shard, no data-path
collective), world sizes 2, 4 and 8 over gloo (stream s
gives identical PCM for G in {1, 2, 4, 8}).

* CPU (no GPU needed): the rank/shard plumbing with the CPU ORACLE standing
  in for the per-rank engine -- each rank synthesises its own shard of
  streams, the ranks exchange only checksums, and the result equals the same
  global stream ids synthesised in one process.
* -m gpu: the same with the ENGINE, through bench.py's own run_batch (the
  timed path of `bench.py --gpus N`): each rank runs its weak shard on device
  LOCAL_RANK % device_count() (both ranks share the card on a one-GPU box),
  the PCM of every stream is gathered, and it must equal the single-process
  run of the same global stream ids."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lpcnet_amd.shard import shard_range, weak_shard

TOTAL, FRAMES = 6, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stream_pcm(blob, sid):
    import lpcnet_amd as L
    import oracle_lib as O
    return O.synth_stream(blob, L.synthetic_features(sid, FRAMES)[:, :20], 0)


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import lpcnet_amd as L
    blob = L.synthetic_model(1, 0)
    mine = shard_range(rank, world, TOTAL)
    sums = torch.zeros(TOTAL, dtype=torch.int64)
    for sid in mine:
        sums[sid] = int(np.abs(_stream_pcm(blob, sid).astype(np.int64)).sum())
    dist.all_reduce(sums)  # each slot written by exactly one rank
    t = torch.tensor([float(len(mine))])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        out.put((sums.tolist(), float(t.item())))
    dist.destroy_process_group()


def test_shard_ranges_partition():
    for world in (1, 2, 3, 8):
        for total in (1, 7, 1024, 8192):
            ids = [i for r in range(world) for i in shard_range(r, world, total)]
            assert ids == list(range(total))
    assert list(weak_shard(3, 1024)) == list(range(3072, 4096))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_two_rank_gloo_shard_invariance(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    sums, maxlen = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import lpcnet_amd as L
    blob = L.synthetic_model(1, 0)
    single = [int(np.abs(_stream_pcm(blob, sid).astype(np.int64)).sum()) for sid in range(TOTAL)]
    assert sums == single
    assert maxlen == float(max(len(shard_range(r, world, TOTAL)) for r in range(world)))


def _engine_worker(rank, world, port, out, per_rank, frames):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["LOCAL_RANK"] = str(rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import lpcnet_amd as L
    blob = L.synthetic_model(1, 0)
    _, _, _, pcm = bench.run_batch(L, blob, per_rank, weak_shard(rank, per_rank).start, 2, frames - 2, dist, 1)
    t = torch.from_numpy(np.ascontiguousarray(pcm.astype(np.int32)))
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    if rank == 0:
        out.put(np.concatenate([p.numpy() for p in parts], axis=1))
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,per_rank,frames", [(2, 96, 6), (2, 1024, 10), (4, 128, 6), (8, 64, 6)])
def test_two_rank_engine_shard_invariance(require_gpu, world, per_rank, frames):
    """per_rank 96: mf_kernel<1> with the overlapped per-frame frame kernel
    (<= 128 streams); per_rank 1024 is BASELINE configs[4]'s own per-GPU
    size: each rank runs mf_kernel<4>, the chunked frame network and the
    multi-frame sample launches, exactly as `bench.py --gpus N` does.
    World sizes 4 and 8 (all ranks sharing the one GPU): 128 / 64 streams per
    rank on the overlapped path against one 512-stream process on the chunked
    mf_kernel<2> path, and the oracle on a stream of every shard."""
    import bench
    import lpcnet_amd as L
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_worker, args=(r, world, port, q, per_rank, frames)) for r in range(world)]
    for p in procs:
        p.start()
    sharded = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    blob = L.synthetic_model(1, 0)
    _, (_, kn, kf, _, _), info, single = bench.run_batch(L, blob, world * per_rank, 0, 2, frames - 2, None, 1)
    assert sharded.shape == single.shape == (frames, world * per_rank, 160)
    assert np.array_equal(sharded, single.astype(np.int32))
    assert np.abs(single[2:].astype(np.float64)).mean() > 100
    if world > 2:
        import oracle_lib as O
        for r in range(world):
            sid = r * per_rank + (r * 37) % per_rank
            ref = O.synth_stream(blob, L.synthetic_features(sid, frames)[:, :20], 0)
            assert np.array_equal(single[:, sid], ref), sid
    if per_rank >= 1024:
        # the single-process 2048-stream run takes mfw_kernel (two 4-stream
        # groups per workgroup, dedicated roles), each rank's 1024 streams
        # mf_kernel<4>: two different kernels agree on every stream; one
        # multi-frame launch of the timed frames
        assert info.quad_path == 7 and info.streams_per_workgroup == 8
        assert kn == 1 and kf == frames - 2, (kn, kf)
        # and both agree with the CPU oracle on streams from each shard
        import oracle_lib as O
        for sid in (0, per_rank - 1, per_rank, 2 * per_rank - 1, per_rank + 517):
            ref = O.synth_stream(blob, L.synthetic_features(sid, frames)[:, :20], 0)
            assert np.array_equal(single[:, sid], ref), sid
