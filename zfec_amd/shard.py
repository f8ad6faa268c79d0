"""Static sharding of independent stripes across GPUs (one process per GPU).

Stripes of an erasure-coded object are independent (zfec/fec.c:494-503 touches
only column range [k0, k0+stride) of each block), so a batch of nstripes is
split into contiguous, balanced ranges, one per rank; each rank encodes /
decodes its range on its own GPU with no data exchange.  The only collectives
a driver needs are for timing (barrier, max over ranks) -- see bench.py.
"""


def shard_range(nstripes, world, rank):
    """Contiguous [start, stop) of stripes owned by `rank`; sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank %r of world %r" % (rank, world))
    base, extra = divmod(nstripes, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def rank_env():
    """(rank, world, local_rank) from the torchrun environment (1 process if unset)."""
    import os

    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def encode_shard(encode_stripes, nstripes, world, rank):
    """Apply `encode_stripes(start, stop)` to this rank's range; returns (start, stop, result)."""
    start, stop = shard_range(nstripes, world, rank)
    return start, stop, (encode_stripes(start, stop) if stop > start else None)
