"""Multi-process sharding THROUGH THE HIP PATH: two ranks (gloo for the
collectives, both on the box's one GPU, as bench.py's rehearsal runs them)
each encode their shard of a batch of stripes with fec_encode_batch and decode
it back with fec_decode_batch, then the gathered per-stripe parity digests must
equal a single-process run and the oracle.  Also the slab split of one stripe
(zfec_amd.shard.slab_range) across the two ranks.  Complements
tests/test_multiproc_gloo.py, whose per-rank work is the CPU oracle."""
import hashlib
import os
import socket

import numpy as np
import pytest

import zfec_amd

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if zfec_amd.device_count() < 1:
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _place(nums, k):
    slots = [None] * k
    sec = iter([n for n in nums if n >= k])
    for n in nums:
        if n < k:
            slots[n] = n
    return [s if s is not None else next(sec) for s in slots]


def _worker(rank, world, port, k, m, sz, nstripes, q):
    import torch
    import torch.distributed as dist

    from zfec_amd import capi
    from zfec_amd.shard import shard_range, slab_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, size=(nstripes, k, sz), dtype=np.uint8)  # every rank builds the same batch
    s0, s1 = shard_range(nstripes, world, rank)
    r = m - k
    code = capi.Code(k, m)
    st = torch.cuda.current_stream().cuda_stream
    src = torch.from_numpy(np.ascontiguousarray(data[s0:s1])).cuda()
    par = torch.empty((s1 - s0, r, sz), dtype=torch.uint8, device="cuda")
    if s1 > s0:
        code.encode_batch(src.data_ptr(), sz, k * sz, par.data_ptr(), sz, r * sz, list(range(k, m)), sz, s1 - s0,
                          stream=st)
        slots = _place(list(range(m - k, m)), k)
        allb = torch.cat([src, par], dim=1)
        recv = allb[:, slots, :].contiguous()
        miss = [i for i in range(k) if slots[i] >= k]
        rec = torch.empty((s1 - s0, len(miss), sz), dtype=torch.uint8, device="cuda")
        code.decode_batch(recv.data_ptr(), sz, k * sz, rec.data_ptr(), sz, len(miss) * sz, slots, sz, s1 - s0,
                          stream=st)
        torch.cuda.synchronize()
        assert torch.equal(rec, src[:, miss, :])
    p = par.cpu().numpy()
    digests = [hashlib.sha256(p[i].tobytes()).hexdigest() for i in range(s1 - s0)]
    # slab split of stripe 0's blocks: this rank encodes columns [c0, c1)
    c0, c1 = slab_range(sz, world, rank)
    ins = [torch.from_numpy(np.ascontiguousarray(data[0, j, c0:c1])).cuda() for j in range(k)]
    slab = zfec_amd.Encoder(k, m).encode(ins)
    slab_par = torch.stack(slab[k:]).cpu().numpy() if c1 > c0 else np.zeros((r, 0), np.uint8)
    gathered = [None] * world
    dist.all_gather_object(gathered, (s0, s1, digests, c0, c1, slab_par.tobytes()))
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("k,m,sz,nstripes", [(3, 10, 4096, 37), (20, 60, 52429, 9)])
def test_two_ranks_through_hip(k, m, sz, nstripes):
    import torch.multiprocessing as mp

    from oracle import oracle

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, k, m, sz, nstripes, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, size=(nstripes, k, sz), dtype=np.uint8)
    got = []
    for s0, s1, dg, _, _, _ in sorted(gathered):
        assert len(dg) == s1 - s0
        got.extend(dg)
    assert len(got) == nstripes
    want = [hashlib.sha256(oracle.encode(k, m, data[s]).tobytes()).hexdigest() for s in range(nstripes)]
    assert got == want
    # the ranks' slabs, joined, are stripe 0's parity
    r = m - k
    par0 = oracle.encode(k, m, data[0])
    for _, _, _, c0, c1, slab in gathered:
        assert (np.frombuffer(slab, np.uint8).reshape(r, c1 - c0) == par0[:, c0:c1]).all()
