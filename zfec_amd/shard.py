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


def slab_range(sz, world, rank, align=256):
    """Contiguous byte range [start, stop) of a block owned by `rank` when one huge
    stripe is split across GPUs ("split the byte range into slabs").

    Byte i of every output block depends only on byte i of the input blocks
    (zfec/fec.c:494-503 encodes column range [k0, k0+stride) of each block;
    fec_decode, zfec/fec.c:545-556, is column-wise too), so rank r encodes or
    decodes columns [start, stop) of all k blocks on its own GPU -- the same
    fec_encode / fec_decode call with every block pointer advanced by `start`
    and sz = stop - start -- and no data is exchanged.  Slab boundaries fall on
    multiples of `align` bytes (whole 128-byte lines for the kernels' stores);
    the last rank takes the remainder, and ranks past the end get empty slabs."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank %r of world %r" % (rank, world))
    if align < 1 or sz < 0:
        raise ValueError("bad slab size %r / alignment %r" % (sz, align))
    units = -(-sz // align)
    u0, u1 = shard_range(units, world, rank)
    return min(sz, u0 * align), min(sz, u1 * align)
