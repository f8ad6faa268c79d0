"""Multi-process sharding on CPU (gloo, world_size 2 and 3): the stripe
partition used by bench.py's multi-GPU path covers every stripe exactly once,
and the per-rank results gathered back equal the single-process result.  The
per-stripe work here is the CPU oracle (this suite has no GPU); on the GPU
box the same partition feeds fec_encode_batch per rank."""
import hashlib
import json
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from zfec_amd.shard import encode_shard, shard_range

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


def test_slab_range_partition():
    from zfec_amd.shard import slab_range

    for sz in [0, 1, 255, 256, 257, 4099, 22369622]:
        for w in [1, 2, 3, 8]:
            ranges = [slab_range(sz, w, r) for r in range(w)]
            assert ranges[0][0] == 0 and ranges[-1][1] == sz
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c and (c % 256 == 0 or c == sz)
    with pytest.raises(ValueError):
        slab_range(10, 2, 2)


def _slab_worker(rank, world, port, k, m, sz, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    from zfec_amd.shard import slab_range

    data = np.random.default_rng(7).integers(0, 256, size=(k, sz), dtype=np.uint8)
    c0, c1 = slab_range(sz, world, rank)
    par = oracle.encode(k, m, np.ascontiguousarray(data[:, c0:c1])) if c1 > c0 else np.zeros((m - k, 0), np.uint8)
    gathered = [None] * world
    dist.all_gather_object(gathered, (c0, c1, par.tobytes()))
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_slab_sharded_encode_matches_single_process(world):
    """One stripe split into byte-range slabs across ranks (the multi-GPU split of a
    single huge stripe, bench.py --slabs): the slabs' parity put together equals the
    whole stripe's.  The per-slab work is the CPU oracle here; on the GPU box it is
    fec_encode with offset block pointers (test_slab_split_equals_whole_stripe)."""
    k, m, sz = 3, 10, 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slab_worker, args=(r, world, port, k, m, sz, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from oracle import oracle

    data = np.random.default_rng(7).integers(0, 256, size=(k, sz), dtype=np.uint8)
    whole = oracle.encode(k, m, data)
    got = np.zeros_like(whole)
    for c0, c1, b in gathered:
        got[:, c0:c1] = np.frombuffer(b, np.uint8).reshape(m - k, c1 - c0)
    assert (got == whole).all()


def _barrier_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    import time

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    nb = bench.NodeBarrier(dist, rank, world)
    assert nb.flags is not None
    seen = []
    for i in range(200):
        if rank == i % world:
            time.sleep(0.001)  # one late rank per round: nobody may leave before it arrives
        nb.wait()
        seen.append(int(nb.flags[:, 0].min()))
    dist.barrier()
    q.put((rank, seen == list(range(1, 201)), nb.epoch))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_node_barrier_shared_memory(world):
    """bench.py's NodeBarrier (shared-memory spin barrier bracketing the timed
    steps): no rank leaves a round before every rank has arrived at it, over
    200 rounds with a different late rank each round; the backing file is
    unlinked after set-up."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_barrier_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(r for r, _, _ in res) == list(range(world))
    assert all(ok and epoch == 200 for _, ok, epoch in res)
    assert not [f for f in os.listdir("/dev/shm") if f.startswith("zfec_bench_barrier_")]


def test_rw_ceiling_bounds():
    """bench.py's read-then-write ceiling: between the stores-only and the
    loads-only rate, equal to each at the extremes, and the achieved fraction
    is the achieved rate over it."""
    import bench

    c = bench.rw_ceiling(3, 7, 5000.0)
    assert bench.HBM_WRITE_GBPS < c["GBps"] < bench.HBM_READ_GBPS
    assert abs(bench.rw_ceiling(1, 0, 1.0)["GBps"] - bench.HBM_READ_GBPS) < 0.1
    assert abs(bench.rw_ceiling(0, 1, 1.0)["GBps"] - bench.HBM_WRITE_GBPS) < 0.1
    assert abs(c["achieved_frac_of_ceiling"] - 5000.0 / c["GBps"]) < 1e-3
    assert abs(c["frac_of_peak"] - c["GBps"] / bench.HBM_PEAK_GBPS) < 1e-3


def _bench(args, env_extra=None):
    import subprocess
    import sys

    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=240, cwd=ROOT)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_bench_gpus_flag_starts_that_many_ranks(n):
    """`python bench.py --gpus N` (the driver's command shape) starts N ranks
    itself when no launcher set WORLD_SIZE, and the process group has N ranks
    (--dry-run: gloo, no GPU call)."""
    res = _bench(["--gpus", str(n), "--dry-run"])
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["ranks_seen"] == n and out["ranks_reduced"] == n


def test_bench_world_size_mismatch_fails_loudly():
    """Under a launcher whose WORLD_SIZE differs from --gpus, bench.py exits
    non-zero before any GPU work instead of measuring another number of GPUs."""
    res = _bench(["--gpus", "3", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert res.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 3" in res.stderr
    res = _bench(["--gpus", "0"])
    assert res.returncode != 0
