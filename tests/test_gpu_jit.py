"""GPU parity of the run-time specialised bit-sliced kernels
(zfec_amd/csrc/bitslice.cpp): bit-exact against the CPU oracle across code
shapes, block sizes around the 2 KiB unit and its overlapping last chunk,
batched strided stripes at misaligned bases (with guard bytes that must stay
untouched), and the auto policy (background compile; the table kernels serve
until it is ready, with identical results)."""
import numpy as np
import pytest

import zfec_amd
from zfec_amd import capi
from oracle import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if zfec_amd.device_count() < 1:
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")


@pytest.fixture
def force_jit():
    prev = capi.jit_mode(capi.JIT_FORCE)
    yield
    capi.jit_mode(prev)


def place(nums, k):
    """slot order with primary i at slot i (zfec/_fecmodule.c:482-493)."""
    slots = [None] * k
    sec = iter([n for n in nums if n >= k])
    for n in nums:
        if n < k:
            slots[n] = n
    return [s if s is not None else next(sec) for s in slots]


# (k, m): few/many inputs and outputs; one row tile, or 2-5 tiles on the waves of a workgroup; more
# than 32 inputs in one kernel (94/100: benchmark-zfec/Main.hs:17); double-buffered LDS-DMA
# phases of 4 with a short last one (14, 17, 30 inputs on 2 tiles, 23 on 3)
JIT_SHAPES = [(3, 10), (2, 40), (5, 9), (10, 16), (16, 32), (20, 60), (32, 40), (10, 58), (94, 100), (40, 48),
              (14, 30), (17, 35), (23, 50), (30, 45), (30, 70)]


@pytest.mark.parametrize("k,m", JIT_SHAPES)
def test_jit_encode_decode_vs_oracle(force_jit, k, m):
    rng = np.random.default_rng(k * 100 + m)
    for sz in [2048, 2049, 3000, 4096, 65536 + 17]:
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
        out = zfec_amd.Encoder(k, m).encode(ins)
        assert capi.last_kernel_name().startswith("zfec_hip_bitslice"), capi.last_kernel_name()
        par = torch.stack(out[k:]).cpu().numpy()
        assert (par == oracle.encode(k, m, data)).all(), (k, m, sz)
        nums = list(range(m - k, m))
        dec = zfec_amd.Decoder(k, m).decode([out[n] for n in nums], nums)
        if any(n >= k for n in nums):
            assert capi.last_kernel_name().startswith("zfec_hip_bitslice"), capi.last_kernel_name()
        assert (torch.stack(dec).cpu().numpy() == data).all(), (k, m, sz)


@pytest.mark.parametrize("k,m,sz,ns", [(10, 16, 5000, 7), (20, 60, 52429, 3), (4, 12, 2048, 33)])
def test_jit_batched_strided_misaligned(force_jit, k, m, sz, ns):
    """Stripes at an odd row stride from odd base offsets; the gaps between rows
    and the bytes around the buffers must stay zero (the overlapping last chunk
    writes only inside [0, sz) of each row)."""
    r = m - k
    ld = sz + 13
    rng = np.random.default_rng(sz + ns)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    host = np.zeros(5 + ns * k * ld + 64, dtype=np.uint8)
    rows = host[5:5 + ns * k * ld].reshape(ns, k, ld)
    rows[:, :, :sz] = data
    src = torch.from_numpy(host).cuda()
    dst = torch.zeros(3 + ns * r * ld + 64, dtype=torch.uint8, device="cuda")
    code = capi.Code(k, m)
    st = torch.cuda.current_stream().cuda_stream
    code.encode_batch(src.data_ptr() + 5, ld, k * ld, dst.data_ptr() + 3, ld, r * ld, list(range(k, m)), sz, ns,
                      stream=st)
    torch.cuda.synchronize()
    assert capi.last_kernel_name().startswith("zfec_hip_bitslice")
    got = dst.cpu().numpy()
    assert got[:3].sum() == 0 and got[3 + ns * r * ld:].sum() == 0
    out = got[3:3 + ns * r * ld].reshape(ns, r, ld)
    assert out[:, :, sz:].sum() == 0
    for s in range(ns):
        assert (out[s, :, :sz] == oracle.encode(k, m, data[s])).all(), s
    # decode every stripe from its last k blocks, same strided layout
    slots = place(list(range(m - k, m)), k)
    allb = np.concatenate([data, out[:, :, :sz]], axis=1)
    recv_host = np.zeros(7 + ns * k * ld, dtype=np.uint8)
    recv_host[7:].reshape(ns, k, ld)[:, :, :sz] = allb[:, slots, :]
    recv = torch.from_numpy(recv_host).cuda()
    missing = [i for i in range(k) if slots[i] >= k]
    rec = torch.zeros(1 + ns * len(missing) * ld + 64, dtype=torch.uint8, device="cuda")
    code.decode_batch(recv.data_ptr() + 7, ld, k * ld, rec.data_ptr() + 1, ld, len(missing) * ld, slots, sz, ns,
                      stream=st)
    torch.cuda.synchronize()
    rg = rec.cpu().numpy()
    assert rg[0] == 0 and rg[1 + ns * len(missing) * ld:].sum() == 0
    rv = rg[1:1 + ns * len(missing) * ld].reshape(ns, len(missing), ld)
    assert (rv[:, :, :sz] == data[:, missing, :]).all()
    assert rv[:, :, sz:].sum() == 0


def test_jit_all_primaries_flag(force_jit):
    """FEC_FLAG_ALL_PRIMARIES through the specialised kernel: identity rows copy."""
    k, m, sz, ns = 6, 14, 4100, 5
    nums = [7, 1, 9, 3, 12, 13]
    code = capi.Code(k, m)
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    allb = np.concatenate([data, np.stack([oracle.encode(k, m, data[s]) for s in range(ns)])], axis=1)
    slots = place(nums, k)
    recv = torch.from_numpy(np.ascontiguousarray(allb[:, slots, :])).cuda()
    out = torch.zeros((ns, k, sz), dtype=torch.uint8, device="cuda")
    code.decode_batch(recv.data_ptr(), sz, k * sz, out.data_ptr(), sz, k * sz, slots, sz, ns,
                      stream=torch.cuda.current_stream().cuda_stream,
                      flags=capi.FEC_FLAG_ASYNC | capi.FEC_FLAG_ALL_PRIMARIES)
    torch.cuda.synchronize()
    assert capi.last_kernel_name().startswith("zfec_hip_bitslice")
    assert (out.cpu().numpy() == data).all()


def test_jit_auto_policy_background_compile():
    """Auto mode: the second large launch of a matrix queues its compile (both
    run the table kernel); after fec_jit_wait the specialised kernel runs;
    same bytes.  (13/22: a code whose kernel is not in the in-tree disk cache,
    so fec_new prefetches nothing.)"""
    prev = capi.jit_mode(capi.JIT_AUTO)
    try:
        k, m, sz = 13, 22, 4 << 20  # (k + r) * sz = 88 MiB per launch: above the auto threshold
        g = torch.Generator(device="cuda").manual_seed(12)
        data = torch.randint(0, 256, (k, sz), dtype=torch.uint8, device="cuda", generator=g)
        enc = zfec_amd.Encoder(k, m)
        out1 = enc.encode([data[i] for i in range(k)])
        first = capi.last_kernel_name()
        capi.jit_wait()  # nothing queued: a matrix is compiled on its second large launch
        enc.encode([data[i] for i in range(k)])
        again = capi.last_kernel_name()
        capi.jit_wait()
        out2 = enc.encode([data[i] for i in range(k)])
        second = capi.last_kernel_name()
        assert first.startswith("matapply") and again.startswith("matapply"), (first, again)
        assert second.startswith("zfec_hip_bitslice"), (first, second)
        for a, b in zip(out1[k:], out2[k:]):
            assert bool(torch.equal(a, b))
        lo, hi = sz // 3, sz // 3 + 50000
        par = torch.stack(out2[k:])[:, lo:hi].cpu().numpy()
        assert (par == oracle.encode(k, m, data[:, lo:hi].cpu().numpy())).all()
    finally:
        capi.jit_mode(prev)


def test_jit_prefetch_first_launch():
    """Auto mode, a code whose compiled encode kernel an earlier process left
    in the disk cache (tools/jit_warm.py compiled 12/21's into
    zfec_amd/jit_cache/): fec_new loads it and its module in the background,
    so the code's FIRST large encode runs it; bytes equal the oracle's."""
    prev = capi.jit_mode(capi.JIT_AUTO)
    try:
        k, m, sz = 12, 21, 4 << 20
        g = torch.Generator(device="cuda").manual_seed(1221)
        data = torch.randint(0, 256, (k, sz), dtype=torch.uint8, device="cuda", generator=g)
        enc = zfec_amd.Encoder(k, m)
        capi.jit_wait()  # the prefetch (a file read and a module load: no compile)
        out = enc.encode([data[i] for i in range(k)])
        assert capi.last_kernel_name().startswith("zfec_hip_bitslice_k12_r9"), capi.last_kernel_name()
        lo, hi = sz // 2, sz // 2 + 40000
        par = torch.stack(out[k:])[:, lo:hi].cpu().numpy()
        assert (par == oracle.encode(k, m, data[:, lo:hi].cpu().numpy())).all()
    finally:
        capi.jit_mode(prev)


def test_jit_off_uses_table_kernels():
    prev = capi.jit_mode(capi.JIT_OFF)
    try:
        k, m, sz = 20, 60, 52429
        data = torch.randint(0, 256, (k, sz), dtype=torch.uint8, device="cuda")
        out = zfec_amd.Encoder(k, m).encode([data[i] for i in range(k)])
        assert capi.last_kernel_name().startswith("matapply"), capi.last_kernel_name()
        par = torch.stack(out[k:]).cpu().numpy()
        assert (par == oracle.encode(k, m, data.cpu().numpy())).all()
    finally:
        capi.jit_mode(prev)


_REMOVED_KNOBS_CHILD = r"""
import json, os, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import torch
from zfec_amd import capi
from oracle import oracle

capi.jit_mode(capi.JIT_FORCE)
k, m, sz, ns = 20, 60, 52429, 2
r = m - k
rng = np.random.default_rng(int(sys.argv[2]))
data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
src = torch.from_numpy(data).cuda()
par = torch.zeros((ns, r, sz), dtype=torch.uint8, device="cuda")
code = capi.Code(k, m)
code.encode_batch(src.data_ptr(), sz, k * sz, par.data_ptr(), sz, r * sz, list(range(k, m)), sz, ns)
enc_kernel = capi.last_kernel_name()
torch.cuda.synchronize()
p = par.cpu().numpy()
ok_enc = all((p[s] == oracle.encode(k, m, data[s])).all() for s in range(ns))
slots = list(range(m - k, m))  # every primary lost
recv = par[:, r - k:].contiguous()
rec = torch.zeros((ns, k, sz), dtype=torch.uint8, device="cuda")
code.decode_batch(recv.data_ptr(), sz, k * sz, rec.data_ptr(), sz, k * sz, slots, sz, ns)
dec_kernel = capi.last_kernel_name()
torch.cuda.synchronize()
ok_dec = bool((rec.cpu().numpy() == data).all())
print(json.dumps({"enc": enc_kernel, "dec": dec_kernel, "ok_enc": bool(ok_enc), "ok_dec": ok_dec}))
"""


@pytest.mark.parametrize("env", [{"ZFEC_HIP_JIT_PROBE": "1"}, {"ZFEC_HIP_JIT_PROBE": "2"},
                                 {"ZFEC_HIP_JIT_TILE": "3", "ZFEC_HIP_JIT_ORDER": "1", "ZFEC_HIP_JIT_PREFETCH": "0",
                                  "ZFEC_HIP_JIT_STORE": "17", "ZFEC_HIP_STORE": "nt", "ZFEC_HIP_BSG_WGS": "1"}])
def test_removed_knobs_cannot_change_bytes(env):
    """Round 3's measurement-only probe variants (ZFEC_HIP_JIT_PROBE=1 read
    zeros, =2 wrote the XOR of the inputs) and the other variant knobs are
    gone from the library: with them set, a forced-JIT K=20/M=60 encode and an
    all-primaries-lost decode in a fresh process still match the oracle, on
    the specialised kernels (zfec/fec.c:487-505, :527-557)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ)
    e.update(env)
    res = subprocess.run([sys.executable, "-c", _REMOVED_KNOBS_CHILD, root, str(len(env))], env=e,
                         capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    out = json.loads([ln for ln in res.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["ok_enc"] and out["ok_dec"], out
    assert out["enc"].startswith("zfec_hip_bitslice_k20_r40") and out["dec"].startswith("zfec_hip_bitslice_k20_r20"), out
