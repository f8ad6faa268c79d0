"""Multi-process sharding on CPU (gloo, world_size 2 and 3): the stripe
partition used by bench.py's multi-GPU path covers every stripe exactly once,
and the per-rank results gathered back equal the single-process result.  The
per-stripe work here is the CPU oracle (this suite has no GPU); on the GPU
box the same partition feeds fec_encode_batch per rank."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from zfec_amd.shard import encode_shard, shard_range


def test_shard_range_partition():
    for n in [0, 1, 7, 1024, 1000001]:
        for w in [1, 2, 3, 8]:
            ranges = [shard_range(n, w, r) for r in range(w)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, nstripes, k, m, sz, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle

    rng = np.random.default_rng(42)
    data = rng.integers(0, 256, size=(nstripes, k, sz), dtype=np.uint8)  # every rank sees the same object

    def enc(start, stop):
        return [hashlib.sha256(oracle.encode(k, m, data[s]).tobytes()).hexdigest() for s in range(start, stop)]

    start, stop, digests = encode_shard(enc, nstripes, world, rank)
    gathered = [None] * world
    dist.all_gather_object(gathered, (start, stop, digests or []))
    # timing reduction used by bench.py: max over ranks
    import torch

    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((gathered, float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_encode_matches_single_process(world):
    nstripes, k, m, sz = 13, 3, 10, 257
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nstripes, k, m, sz, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert tmax == float(world)
    from oracle import oracle

    rng = np.random.default_rng(42)
    data = rng.integers(0, 256, size=(nstripes, k, sz), dtype=np.uint8)
    expect = [hashlib.sha256(oracle.encode(k, m, data[s]).tobytes()).hexdigest() for s in range(nstripes)]
    got = []
    for start, stop, digests in sorted(gathered):
        assert len(digests) == stop - start
        got.extend(digests)
    assert got == expect
