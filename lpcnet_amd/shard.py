"""Stream sharding across GPUs: streams are independent, so a
global batch of B_total streams is split into contiguous shards, one per rank,
with no data-path collective.  The only cross-rank traffic is the benchmark's
barrier and max-reduction of the timed interval."""
from __future__ import annotations


def shard_range(rank: int, world: int, total_streams: int) -> range:
    """Contiguous shard of global stream ids owned by ``rank``."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(total_streams, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def weak_shard(rank: int, per_rank: int) -> range:
    """Weak scaling: every rank owns ``per_rank`` streams (bench configs[4])."""
    return range(rank * per_rank, (rank + 1) * per_rank)
