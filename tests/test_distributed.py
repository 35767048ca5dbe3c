"""World-size-2 gloo run of the sharded path on CPU: each rank synthesises its
own shard of streams (CPU oracle standing in for the per-rank engine), the
ranks exchange only checksums, and the result is identical to the same global
stream ids synthesised in one process (shard invariance)."""
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


def test_two_rank_gloo_shard_invariance():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
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
    assert maxlen == 3.0
