"""GPU parity: the HIP path (through the C-ABI / the Python surface) against the
golden vectors of the real reference and against the CPU oracle on seeded
inputs.  Bit-exact everywhere (integer GF(2^8) arithmetic).

Mirrors the reference's own tests (zfec/test/test_zfec.py): test_from_agl,
hypothesis round trips over all (k, m) with short blocks, random round trips,
easyfec round trips; adds golden-vector and oracle comparisons, ragged and
misaligned sizes, device-resident tensors, the batched entry points, and the
BASELINE config sizes (via round-trip properties and oracle checks)."""
import ctypes
import hashlib
import random

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


def blocks_of(arr):
    return [arr[i].tobytes() for i in range(arr.shape[0])]


def place(nums, k):
    """slot order with primary i at slot i (zfec/_fecmodule.c:482-493)."""
    slots = [None] * k
    sec = [n for n in nums if n >= k]
    for n in nums:
        if n < k:
            slots[n] = n
    it = iter(sec)
    return [s if s is not None else next(it) for s in slots]


# ---- reference self-tests ----------------------------------------------------

def test_from_agl_c():
    assert zfec_amd.test_from_agl()


def test_from_agl_py(golden):
    meta, _ = golden
    e = zfec_amd.Encoder(3, 5)
    b0, b1, b2 = b"\x01" * 8, b"\x02" * 8, b"\x03" * 8
    b3, b4 = e.encode([b0, b1, b2], (3, 4))
    assert b3.hex() == meta["agl"]["parity3"] and b4.hex() == meta["agl"]["parity4"]
    r0, r1, r2 = zfec_amd.Decoder(3, 5).decode((b2, b3, b4), (2, 3, 4))
    assert (r0, r1, r2) == (b0, b1, b2)


# ---- golden vectors from the reference ----------------------------------------

def test_golden_vectors(golden):
    meta, arrays = golden
    for ci, c in enumerate(meta["vectors"]):
        k, m, sz = c["k"], c["m"], c["sz"]
        inp = arrays["vec%d_in" % ci]
        allb = arrays["vec%d_all" % ci]
        ins = blocks_of(inp)
        out = zfec_amd.Encoder(k, m).encode(ins)
        assert len(out) == m
        for i in range(m):
            assert out[i] == allb[i].tobytes(), (c, i)
        for i in range(k):
            assert out[i] is ins[i]  # primaries by reference
        sub = zfec_amd.Encoder(k, m).encode(ins, c["subset_nums"])
        for n, got in zip(c["subset_nums"], sub):
            assert got == allb[n].tobytes()
        for nums in c["decode_nums"]:
            dec = zfec_amd.Decoder(k, m).decode([allb[n].tobytes() for n in nums], nums)
            assert b"".join(dec) == inp.tobytes(), (c, nums)


@pytest.mark.parametrize("idx", range(5))
def test_golden_pattern_kat(golden, idx):
    meta, _ = golden
    c = meta["pattern_kat"][idx]
    k, m, sz = c["k"], c["m"], c["sz"]
    blocks = oracle.pattern_blocks(k, sz)
    out = zfec_amd.Encoder(k, m).encode(blocks_of(blocks))
    par = b"".join(out[k:])
    assert hashlib.sha256(par).hexdigest() == c["parity_sha256"]
    assert out[k][:8].hex() == c["parity0_head"] and out[-1][-8:].hex() == c["parity_last_tail"]


# ---- reference-style round trips (zfec/test/test_zfec.py:37-160) ------------

def _h(k, m, ss, rng):
    out = zfec_amd.Encoder(k, m).encode(ss)
    assert len(out) == m
    pick = rng.sample(list(enumerate(out)), k)
    dec = zfec_amd.Decoder(k, m).decode([b for _, b in pick], [n for n, _ in pick])
    assert dec == list(ss)


def test_small_all_km():
    """test_small: l in [0, 15], 1 <= k <= m <= 256 (seeded sweep instead of hypothesis draws)."""
    rng = random.Random(1234)
    for trial in range(300):
        m = rng.randint(1, 256)
        k = rng.randint(1, m)
        l = rng.randint(0, 15)
        ss = [bytes(rng.getrandbits(8) for _ in range(l // k)) for _ in range(k)]
        _h(k, m, ss, rng)


def test_hypothesis_small():
    hyp = pytest.importorskip("hypothesis")
    from hypothesis import given, settings, HealthCheck
    from hypothesis.strategies import integers, binary, lists, just

    @settings(max_examples=60, deadline=None, suppress_health_check=list(HealthCheck))
    @given(integers(min_value=0, max_value=15).flatmap(
        lambda l: integers(min_value=1, max_value=256).flatmap(
            lambda m: integers(min_value=1, max_value=m).flatmap(
                lambda k: lists(binary(min_size=l // k, max_size=l // k), min_size=k, max_size=k).flatmap(
                    lambda ss: just((k, m, ss)))))))
    def run(kmss):
        k, m, ss = kmss
        _h(k, m, ss, random.Random(len(ss)))

    run()


def test_random_vs_oracle():
    rng = np.random.default_rng(99)
    for trial in range(40):
        m = int(rng.integers(1, 257))
        k = int(rng.integers(1, m + 1))
        sz = int(rng.integers(0, 2 ** 11))
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        out = zfec_amd.Encoder(k, m).encode(blocks_of(data))
        if m > k:
            par = np.frombuffer(b"".join(out[k:]), dtype=np.uint8).reshape(m - k, sz)
            assert (par == oracle.encode(k, m, data)).all(), (k, m, sz)
        nums = sorted(int(x) for x in rng.choice(m, size=k, replace=False))
        slots = place(nums, k)
        dec = zfec_amd.Decoder(k, m).decode([out[n] for n in nums], nums)
        assert b"".join(dec) == data.tobytes()
        rec = oracle.decode(k, m, np.array([np.frombuffer(out[n], np.uint8) for n in slots]).reshape(k, sz), slots)
        missing = [i for i in range(k) if slots[i] >= k]
        for j, i in enumerate(missing):
            assert dec[i] == rec[j].tobytes()


@pytest.mark.parametrize("k,m", [(1, 1), (1, 2), (2, 3), (3, 10), (4, 8), (5, 13), (10, 16), (20, 60),
                                 (32, 64), (33, 64), (40, 100), (64, 128), (128, 256), (200, 256), (255, 256), (256, 256)])
def test_ragged_sizes_vs_oracle(k, m):
    """Block sizes around the 16-byte chunk and tail paths; k > 32 exercises the
    XOR-accumulating multi-pass path, m-k > 48 the row split."""
    rng = np.random.default_rng(k * 1000 + m)
    for sz in [1, 15, 16, 17, 31, 33, 255, 4095, 4097]:
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        out = zfec_amd.Encoder(k, m).encode(blocks_of(data))
        if m > k:
            par = np.frombuffer(b"".join(out[k:]), dtype=np.uint8).reshape(m - k, sz)
            assert (par == oracle.encode(k, m, data)).all(), (k, m, sz)
        nums = list(range(m - k, m))  # as many secondaries as possible
        dec = zfec_amd.Decoder(k, m).decode([out[n] for n in nums], nums)
        assert b"".join(dec) == data.tobytes(), (k, m, sz)


def test_k1_parity_equals_primary():
    """haskell/test/FECTest.hs:107-112: with k = 1 every block is the primary."""
    for m in [1, 2, 7, 256]:
        d = bytes(range(200))
        assert all(b == d for b in zfec_amd.Encoder(1, m).encode([d]))


def test_easyfec_roundtrip():
    rng = random.Random(7)
    for l in list(range(16)) + [rng.randrange(0, 512) for _ in range(5)] + [4096, 10 ** 5 + 3]:
        m = rng.randint(1, 256)
        k = rng.randint(1, m)
        s = bytes(rng.getrandbits(8) for _ in range(l))
        blocks = zfec_amd.easyfec.Encoder(k, m).encode(s)
        pick = rng.sample(list(enumerate(blocks)), k)
        got = zfec_amd.easyfec.Decoder(k, m).decode([b for _, b in pick], [n for n, _ in pick],
                                                    padlen=k * len(blocks[0]) - len(s))
        assert got == s


def test_buffer_types():
    arr = np.arange(3 * 100, dtype=np.uint8).reshape(3, 100)
    kinds = [[bytes(a) for a in arr], [bytearray(a) for a in arr], [memoryview(a.copy()) for a in arr], [a.copy() for a in arr]]
    ref = oracle.encode(3, 10, arr)
    for ins in kinds:
        out = zfec_amd.Encoder(3, 10).encode(ins)
        assert (np.frombuffer(b"".join(out[3:]), np.uint8).reshape(7, 100) == ref).all()


# ---- C-ABI directly ------------------------------------------------------------

def test_c_abi_host_pointers():
    L = capi.lib()
    code = capi.Code(5, 9)
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, size=(5, 1000), dtype=np.uint8)
    out = np.zeros((4, 1000), dtype=np.uint8)
    L.fec_encode(code.ptr, capi.ptr_array([data[i].ctypes.data for i in range(5)]),
                 capi.ptr_array([out[i].ctypes.data for i in range(4)]), capi.uint_array([5, 6, 7, 8]), 4, 1000)
    assert L.fec_last_status() == capi.FEC_OK, L.fec_last_error_message()
    assert (out == oracle.encode(5, 9, data)).all()
    # decode from {6, 1, 8, 3, 5} (primaries 1 and 3 at their own slots)
    slots = [6, 1, 8, 3, 5]
    allb = np.concatenate([data, out])
    ins = [allb[s] for s in slots]
    rec = np.zeros((3, 1000), dtype=np.uint8)
    L.fec_decode(code.ptr, capi.ptr_array([a.ctypes.data for a in ins]),
                 capi.ptr_array([rec[i].ctypes.data for i in range(3)]), capi.uint_array(slots), 1000)
    assert L.fec_last_status() == capi.FEC_OK
    assert (rec == data[[0, 2, 4]]).all()


def test_c_abi_host_memory_flag():
    """FEC_FLAG_HOST_MEMORY (the Python bytes path): no per-pointer queries;
    small calls through the pinned bounce buffer, large ones pinned in place."""
    k, m = 4, 11
    code = capi.Code(k, m)
    rng = np.random.default_rng(31)
    for sz in [1, 700, 100_000, 1_500_001]:
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        out = np.zeros((m - k, sz), dtype=np.uint8)
        code.encode_ptrs([data[i].ctypes.data for i in range(k)], [out[i].ctypes.data for i in range(m - k)],
                         list(range(k, m)), sz, flags=capi.FEC_FLAG_LIBRARY_STREAM | capi.FEC_FLAG_HOST_MEMORY)
        assert (out == oracle.encode(k, m, data)).all(), sz
        slots = [7, 1, 9, 3]
        allb = np.concatenate([data, out])
        rec = np.zeros((2, sz), dtype=np.uint8)
        code.decode_ptrs([allb[s].ctypes.data for s in slots], [rec[i].ctypes.data for i in range(2)], slots, sz,
                         flags=capi.FEC_FLAG_LIBRARY_STREAM | capi.FEC_FLAG_HOST_MEMORY)
        assert (rec == data[[0, 2]]).all(), sz


@pytest.mark.parametrize("env", [{}, {"ZFEC_HIP_STAGE_MIN": str(1 << 60)}, {"ZFEC_HIP_STAGE_MIN": "0"}])
def test_host_small_call_paths(env, knobs):
    """Host calls under 4 MiB: as shipped, the bounce buffer up to 4 MiB
    (staged path off), and the staged path from any size (blocks >= 64 KiB) --
    each bit-exact against the oracle, encode and a mixed primary/secondary
    decode."""
    knobs(**env)
    k, m = 3, 10
    rng = np.random.default_rng(77)
    for sz in [65536, 70_001, 349_525, 1_000_003]:
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        blocks = [data[i].tobytes() for i in range(k)]
        out = zfec_amd.Encoder(k, m).encode(blocks)
        par = np.stack([np.frombuffer(b, np.uint8) for b in out[k:]])
        assert (par == oracle.encode(k, m, data)).all(), sz
        rec = zfec_amd.Decoder(k, m).decode([out[8], out[1], out[4]], [8, 1, 4])
        assert rec == blocks, sz


def _encode_ptrs_check(code, k, m, data, in_addrs, out_addrs, read_out, sz):
    code.encode_ptrs(in_addrs, out_addrs, list(range(k, m)), sz, flags=0)
    got = read_out()
    assert (got == oracle.encode(k, m, data)).all()


def test_c_abi_large_pageable_host_blocks_sharing_pages():
    """> 4 MiB of pageable host blocks sharing pages, at odd offsets with guard
    bytes: staged through the pinned slots (default host path)."""
    k, m = 3, 10
    code = capi.Code(k, m)
    rng = np.random.default_rng(17)
    for sz in [2_500_001, 1 << 21]:
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        buf = np.zeros(k * sz + 11, dtype=np.uint8)  # blocks back to back at an odd offset: neighbours share pages
        buf[5:5 + k * sz] = data.reshape(-1)
        obuf = np.zeros((m - k) * sz + 11, dtype=np.uint8)
        base, obase = buf.ctypes.data + 5, obuf.ctypes.data + 3
        _encode_ptrs_check(code, k, m, data, [base + j * sz for j in range(k)], [obase + i * sz for i in range(m - k)],
                           lambda: obuf[3:3 + (m - k) * sz].reshape(m - k, sz), sz)
        assert obuf[:3].sum() == 0 and obuf[3 + (m - k) * sz:].sum() == 0


def test_c_abi_pinned_and_mixed_blocks():
    """Page-locked host blocks (fec_host_alloc) are used in place; any mix of
    device, pinned and pageable blocks in one call."""
    k, m = 4, 9
    code = capi.Code(k, m)
    L = capi.lib()
    rng = np.random.default_rng(23)
    for sz in [100, 333_333, 3_000_000]:
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        want = oracle.encode(k, m, data)
        pins = [L.fec_host_alloc(sz) for _ in range(k + m - k)]
        try:
            arrs = [np.ctypeslib.as_array((ctypes.c_ubyte * sz).from_address(p)) for p in pins]
            for j in range(k):
                arrs[j][:] = data[j]
            # all pinned
            _encode_ptrs_check(code, k, m, data, pins[:k], pins[k:], lambda: np.stack(arrs[k:]), sz)
            # mixed: input 0 on the device, input 1 pageable, outputs alternate pinned / device / pageable
            dev_in = torch.from_numpy(data[0].copy()).cuda()
            page_in = data[1].copy()
            dev_out = torch.zeros(sz, dtype=torch.uint8, device="cuda")
            page_out = np.zeros(sz, dtype=np.uint8)
            ins = [dev_in.data_ptr(), page_in.ctypes.data, pins[2], pins[3]]
            for a in arrs[k:]:
                a[:] = 0
            outs = [pins[k], dev_out.data_ptr(), page_out.ctypes.data, pins[k + 3], pins[k + 4]]
            code.encode_ptrs(ins, outs, list(range(k, m)), sz, flags=0)
            torch.cuda.synchronize()
            assert (arrs[k] == want[0]).all() and (dev_out.cpu().numpy() == want[1]).all()
            assert (page_out == want[2]).all() and (arrs[k + 3] == want[3]).all() and (arrs[k + 4] == want[4]).all()
        finally:
            for p in pins:
                L.fec_host_free(p)


def test_batch_pinned_host():
    """fec_encode_batch / fec_decode_batch on page-locked host memory."""
    k, m, sz, ns = 3, 10, 4096, 300
    code = capi.Code(k, m)
    L = capi.lib()
    rng = np.random.default_rng(29)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    p_in, p_out = L.fec_host_alloc(data.nbytes), L.fec_host_alloc(ns * (m - k) * sz)
    try:
        a_in = np.ctypeslib.as_array((ctypes.c_ubyte * data.nbytes).from_address(p_in)).reshape(ns, k, sz)
        a_out = np.ctypeslib.as_array((ctypes.c_ubyte * (ns * (m - k) * sz)).from_address(p_out)).reshape(ns, m - k, sz)
        a_in[:] = data
        code.encode_batch(p_in, sz, k * sz, p_out, sz, (m - k) * sz, list(range(k, m)), sz, ns, flags=0)
        for s in [0, 1, ns // 2, ns - 1]:
            assert (a_out[s] == oracle.encode(k, m, data[s])).all(), s
    finally:
        L.fec_host_free(p_in)
        L.fec_host_free(p_out)


def test_c_abi_device_pointers_misaligned():
    code = capi.Code(3, 10)
    rng = np.random.default_rng(11)
    for sz, shift in [(333334, 0), (333334, 1), (1000, 7), (22, 13), (4096, 5)]:
        data = rng.integers(0, 256, size=(3, sz), dtype=np.uint8)
        buf = torch.zeros(3 * sz + 64, dtype=torch.uint8, device="cuda")
        buf[shift:shift + 3 * sz] = torch.from_numpy(data.reshape(-1)).cuda()
        out = torch.zeros(7 * sz + 64, dtype=torch.uint8, device="cuda")
        base, obase = buf.data_ptr() + shift, out.data_ptr() + 3
        code.encode_ptrs([base + j * sz for j in range(3)], [obase + i * sz for i in range(7)], list(range(3, 10)), sz,
                         stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = out[3:3 + 7 * sz].cpu().numpy().reshape(7, sz)
        assert (got == oracle.encode(3, 10, data)).all(), (sz, shift)
        assert int(out[:3].sum()) == 0 and int(out[3 + 7 * sz:].sum()) == 0  # no stray writes


@pytest.mark.parametrize("k,m", [(3, 10), (1, 2), (4, 12), (2, 5)])
def test_misaligned_outputs_aligned_store_path(k, m):
    """Output rows at addresses that are not 16-byte multiples (a C caller's
    packed buffer; the register kernels then store with the nt policy, whose
    straddling stores the L2 merges): bit-exact against the oracle for every
    misalignment 1..15 of the packed rows' base, sizes around the 16-byte unit,
    the 256-lane workgroup and the row end, encode and decode, with guard bytes
    on both sides of the output buffer untouched."""
    r = m - k
    code = capi.Code(k, m)
    rng = np.random.default_rng(k * 100 + m)
    st = torch.cuda.current_stream().cuda_stream
    for sz in (1, 15, 16, 17, 1000, 4096, 4097, 256 * 16 * 2 + 9, 333334):
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        expect = oracle.encode(k, m, data)
        src = torch.from_numpy(data).cuda()
        for d in ([1, 6, 15] if sz > 4096 else range(1, 16)):
            out = torch.full((r * sz + 64,), 0xA5, dtype=torch.uint8, device="cuda")
            base = out.data_ptr() + 16 + d  # torch allocations are 256-byte aligned
            code.encode_ptrs([src[j].data_ptr() for j in range(k)], [base + i * sz for i in range(r)],
                             list(range(k, m)), sz, stream=st)
            name = capi.last_kernel_name()
            torch.cuda.synchronize()
            host = out.cpu().numpy()
            got = host[16 + d:16 + d + r * sz].reshape(r, sz)
            assert (got == expect).all(), (k, m, sz, d, name)
            assert (host[:16 + d] == 0xA5).all() and (host[16 + d + r * sz:] == 0xA5).all(), (sz, d)
            if sz >= 64:
                assert name == "matapply_reg<%d,%d>" % (k, r), name
        # decode into misaligned rows: every primary lost that the code can recover
        nums = list(range(m - k, m)) if r >= k else list(range(r)) + list(range(k, m))[:k - r]
        slots = place(sorted(nums), k)
        allb = torch.from_numpy(np.concatenate([data, expect])).cuda()
        missing = [i for i in range(k) if slots[i] != i]
        rec = torch.full((len(missing) * sz + 64,), 0x5A, dtype=torch.uint8, device="cuda")
        base = rec.data_ptr() + 16 + 9
        code.decode_ptrs([allb[b].data_ptr() for b in slots], [base + i * sz for i in range(len(missing))], slots,
                         sz, stream=st)
        torch.cuda.synchronize()
        host = rec.cpu().numpy()
        assert (host[25:25 + len(missing) * sz].reshape(len(missing), sz) == data[missing]).all(), (k, m, sz)
        assert (host[:25] == 0x5A).all() and (host[25 + len(missing) * sz:] == 0x5A).all()


def test_misaligned_outputs_batches_and_headline_size():
    """Misaligned outputs in batches (stripe strides that are and are not
    16-byte multiples) and at the cfg2 size (64 MiB stripe, outputs at 6 mod
    16; slices at the start, the middle and the end against the oracle)."""
    k, m, r = 3, 10, 7
    code = capi.Code(k, m)
    rng = np.random.default_rng(606)
    st = torch.cuda.current_stream().cuda_stream
    for sz, ns, oss in ((5000, 37, 7 * 5008), (5000, 37, 7 * 5000 + 3)):
        data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
        src = torch.from_numpy(data).cuda()
        out = torch.full((ns * oss + 256,), 0xA5, dtype=torch.uint8, device="cuda")
        base = out.data_ptr() + 16 + 6
        code.encode_batch(src.data_ptr(), sz, k * sz, base, sz, oss, list(range(k, m)), sz, ns, stream=st)
        name = capi.last_kernel_name()
        torch.cuda.synchronize()
        host = out.cpu().numpy()
        assert name == "matapply_reg<3,7>", name
        assert (host[:22] == 0xA5).all()
        for s in range(ns):
            rows = np.stack([host[22 + s * oss + i * sz:][:sz] for i in range(r)])
            assert (rows == oracle.encode(k, m, data[s])).all(), (oss, s)
    sz = -(-(64 << 20) // 3)
    src = torch.randint(0, 256, (k, sz), dtype=torch.uint8, device="cuda")
    out = torch.full((r * sz + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    base = out.data_ptr() + 16 + 6
    code.encode_ptrs([src[j].data_ptr() for j in range(k)], [base + i * sz for i in range(r)], list(range(k, m)), sz,
                     stream=st)
    assert capi.last_kernel_name() == "matapply_reg<3,7>"
    torch.cuda.synchronize()
    got = out[22:22 + r * sz].view(r, sz)
    for a in (0, sz // 2 - 3000, sz - 6000):
        sl = src[:, a:a + 6000].cpu().numpy()
        assert (got[:, a:a + 6000].cpu().numpy() == oracle.encode(k, m, sl)).all(), a
    assert int((out[:22] != 0xA5).sum()) == 0 and int((out[22 + r * sz:] != 0xA5).sum()) == 0


@pytest.mark.parametrize("k,m,sz", [(3, 10, 100003), (10, 16, 65539), (20, 60, 4099)])
def test_slab_split_equals_whole_stripe(k, m, sz):
    """One stripe split into byte-range slabs (zfec_amd.shard.slab_range, the
    multi-GPU split of a single huge stripe): each "rank" encodes
    and decodes its columns with every block pointer advanced to the slab, and
    the slabs put together equal the whole-stripe result and the oracle."""
    from zfec_amd.shard import slab_range

    code = capi.Code(k, m)
    r = m - k
    rng = np.random.default_rng(k * 1000 + m)
    data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
    expect = oracle.encode(k, m, data)
    src = torch.from_numpy(data).cuda()
    st = torch.cuda.current_stream().cuda_stream
    secs = list(range(m - k, m))  # the last k blocks
    for world in (1, 2, 3, 8):
        par = torch.zeros(r, sz, dtype=torch.uint8, device="cuda")
        for rank in range(world):
            c0, c1 = slab_range(sz, world, rank)
            if c1 > c0:
                code.encode_ptrs([src[j].data_ptr() + c0 for j in range(k)],
                                 [par[i].data_ptr() + c0 for i in range(r)], list(range(k, m)), c1 - c0, stream=st)
        torch.cuda.synchronize()
        assert (par.cpu().numpy() == expect).all(), world
        # decode from the last k blocks (secondaries first), slab by slab
        full = torch.cat([src, par])
        slots = place(secs, k)
        missing = [i for i in range(k) if slots[i] != i]
        rec = torch.zeros(len(missing), sz, dtype=torch.uint8, device="cuda")
        for rank in range(world):
            c0, c1 = slab_range(sz, world, rank)
            if c1 > c0:
                code.decode_ptrs([full[b].data_ptr() + c0 for b in slots],
                                 [rec[i].data_ptr() + c0 for i in range(len(missing))], slots, c1 - c0, stream=st)
        torch.cuda.synchronize()
        assert torch.equal(rec, src[missing]), world


# ---- device-resident tensors through the Python surface -----------------------

def test_torch_tensors_roundtrip():
    rng = np.random.default_rng(21)
    for k, m, sz in [(3, 10, 1 << 20), (10, 16, 12345), (20, 60, 52429), (2, 3, 1)]:
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
        out = zfec_amd.Encoder(k, m).encode(ins)
        assert all(out[i] is ins[i] for i in range(k))
        par = torch.stack(out[k:]).cpu().numpy()
        assert (par == oracle.encode(k, m, data)).all()
        nums = list(range(m - k, m))
        dec = zfec_amd.Decoder(k, m).decode([out[n] for n in nums], nums)
        assert (torch.stack(dec).cpu().numpy() == data).all()


def test_torch_tensor_preconditions():
    """Device blocks: non-contiguous, mixed host/device, different lengths -> Error."""
    t = torch.zeros((4, 8), dtype=torch.uint8, device="cuda")
    enc = zfec_amd.Encoder(2, 4)
    with pytest.raises(zfec_amd.Error, match="C-contiguous"):
        enc.encode([t[:, 0], t[:, 1]])
    with pytest.raises(zfec_amd.Error, match="all device tensors"):
        enc.encode([t[0], b"\x00" * 8])
    with pytest.raises(zfec_amd.Error, match="same length"):
        enc.encode([t[0], t[1, :4]])
    with pytest.raises(zfec_amd.Error, match="distinct"):
        zfec_amd.Decoder(2, 4).decode([t[0], t[1]], [3, 3])
    # non-uint8 tensors are encoded as their bytes
    f = torch.arange(8, dtype=torch.float32, device="cuda").reshape(2, 4)
    out = enc.encode([f[0], f[1]])
    ref = zfec_amd.Encoder(2, 4).encode([f[0].cpu().numpy().tobytes(), f[1].cpu().numpy().tobytes()])
    assert [bytes(o.cpu().numpy().tobytes()) for o in out[2:]] == ref[2:]


# ---- batched entry points -------------------------------------------------------

@pytest.mark.parametrize("k,m,sz,ns", [(3, 10, 1366, 2000), (20, 60, 52429, 8), (10, 16, 100, 33), (3, 10, 16, 5)])
def test_batch_encode_decode(k, m, sz, ns):
    code = capi.Code(k, m)
    rng = np.random.default_rng(sz + ns)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    src = torch.from_numpy(data).cuda()
    dst = torch.empty((ns, m - k, sz), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    code.encode_batch(src.data_ptr(), sz, k * sz, dst.data_ptr(), sz, (m - k) * sz, list(range(k, m)), sz, ns, stream=st)
    torch.cuda.synchronize()
    par = dst.cpu().numpy()
    for s in sorted(set([0, ns - 1] + list(rng.integers(0, ns, 5)))):
        assert (par[s] == oracle.encode(k, m, data[s])).all(), s
    # decode every stripe from its last k blocks
    idx = list(range(m - k, m))
    slots = place(idx, k)
    allb = torch.cat([src, dst], dim=1)
    recv = allb[:, slots, :].contiguous()
    nrec = sum(1 for s in slots if s >= k)
    rec = torch.empty((ns, nrec, sz), dtype=torch.uint8, device="cuda")
    code.decode_batch(recv.data_ptr(), sz, k * sz, rec.data_ptr(), sz, nrec * sz, slots, sz, ns, stream=st)
    torch.cuda.synchronize()
    missing = [i for i in range(k) if slots[i] >= k]
    assert (rec.cpu().numpy() == data[:, missing, :]).all()


@pytest.mark.parametrize("k,m,sz,ns", [(3, 10, 1366, 3000), (10, 16, 333, 50), (20, 60, 77, 40), (1, 3, 5, 7)])
def test_batch_block_major_layout(k, m, sz, ns):
    """Block-major batches (block j of every stripe packed back to back: stripe
    stride == sz, block stride >= ns * sz) run as one long stripe of ns * sz
    bytes (fec_abi.cpp run_batch): every stripe against the oracle, decode back,
    and guard bytes between and after the block arrays stay untouched."""
    code = capi.Code(k, m)
    r = m - k
    rng = np.random.default_rng(sz * 7 + ns)
    data = rng.integers(0, 256, size=(k, ns, sz), dtype=np.uint8)
    g = 96  # guard bytes after each block array
    bs = ns * sz + g
    src = torch.zeros(k * bs, dtype=torch.uint8, device="cuda")
    for j in range(k):
        src[j * bs:j * bs + ns * sz] = torch.from_numpy(data[j].reshape(-1)).cuda()
    dst = torch.full((r * bs,), 0xA5, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    code.encode_batch(src.data_ptr(), bs, sz, dst.data_ptr(), bs, sz, list(range(k, m)), sz, ns, stream=st)
    torch.cuda.synchronize()
    out = dst.cpu().numpy().reshape(r, bs)
    assert (out[:, ns * sz:] == 0xA5).all(), "write past a block array"
    par = out[:, :ns * sz].reshape(r, ns, sz)
    for s in sorted(set([0, ns - 1] + [int(x) for x in rng.integers(0, ns, 5)])):
        assert (par[:, s] == oracle.encode(k, m, np.ascontiguousarray(data[:, s]))).all(), s
    # decode every stripe from its last k blocks, same layout
    slots = place(list(range(m - k, m)), k)
    allb = np.concatenate([data, par], axis=0)
    recv = torch.zeros(k * bs, dtype=torch.uint8, device="cuda")
    for i, b in enumerate(slots):
        recv[i * bs:i * bs + ns * sz] = torch.from_numpy(np.ascontiguousarray(allb[b]).reshape(-1)).cuda()
    missing = [i for i in range(k) if slots[i] >= k]
    rec = torch.full((len(missing) * bs,), 0x5A, dtype=torch.uint8, device="cuda")
    code.decode_batch(recv.data_ptr(), bs, sz, rec.data_ptr(), bs, sz, slots, sz, ns, stream=st)
    torch.cuda.synchronize()
    got = rec.cpu().numpy().reshape(len(missing), bs)
    assert (got[:, ns * sz:] == 0x5A).all(), "write past a recovered block array"
    assert (got[:, :ns * sz].reshape(len(missing), ns, sz) == data[missing]).all()


_LAYOUTS = {
    # block-major, the input block arrays overlapping (block stride < ns * sz):
    # the collapse runs them as one long stripe per block
    "block_major_aliased_inputs": dict(k=3, m=10, sz=1366, ns=3000, in_bs=1366 * 1500 + 5, in_ss=1366,
                                       out_bs=1366 * 3000 + 64, out_ss=1366, seed=11, guard=96),
    # block-major with FEC_FLAG_ROW_PADDING: the collapsed row must not run past
    # the grant of the last stripe (the flag's per-row room is absent here)
    "block_major_row_padding": dict(k=3, m=10, sz=1366, ns=3000, in_bs=1366 * 3000, in_ss=1366,
                                    out_bs=1366 * 3000, out_ss=1366, seed=12, guard=128, flags=16),
    # one long stripe and many object-major stripes, cut into many launches
    # when the per-launch unit limit is lowered
    "one_stripe": dict(k=10, m=16, sz=3 * 1024 * 1024 + 77, ns=1, in_bs=3 * 1024 * 1024 + 128, in_ss=0,
                       out_bs=3 * 1024 * 1024 + 128, out_ss=0, seed=13, guard=96),
    "object_major": dict(k=4, m=9, sz=5000, ns=700, in_bs=5000, in_ss=4 * 5000, out_bs=5000, out_ss=5 * 5000,
                         seed=14, guard=96),
    # one long K=3/M=10 stripe on the register kernel (nt sc1 stores by default
    # on single-stripe launches), output rows at an odd stride
    "one_stripe_reg": dict(k=3, m=10, sz=5 * 1024 * 1024 + 13, ns=1, in_bs=5 * 1024 * 1024 + 64, in_ss=0,
                           out_bs=5 * 1024 * 1024 + 40, out_ss=0, seed=15, guard=96),
    # many short blocks (the row walk, matapply_rows), rows at odd strides
    "rows_object_major": dict(k=3, m=10, sz=1366, ns=300, in_bs=1400, in_ss=3 * 1400 + 24, out_bs=1390,
                              out_ss=7 * 1390 + 8, seed=16, guard=96),
}


def _run_child(spec, env_extra, tmp_path, tag):
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / ("%s.npy" % tag)
    env = dict(os.environ)
    env.update(env_extra)
    res = subprocess.run([sys.executable, os.path.join(root, "tests", "gpu_batch_child.py"), json.dumps(spec),
                          str(out)], env=env, capture_output=True, text=True, timeout=110)
    assert res.returncode == 0, res.stderr[-2000:]
    return np.load(out), res.stdout.strip()


@pytest.mark.parametrize("layout", sorted(_LAYOUTS))
def test_batch_layout_env_variants(layout, tmp_path):
    """The same fec_encode_batch run two ways, each in its own process (the
    knobs are read once per process): as shipped, and with at most 1024 units
    per launch (ZFEC_HIP_LAUNCH_UNITS=1024: long rows are cut into byte
    ranges, batches into stripe groups).  Both outputs, guard bytes included,
    must be identical, and sampled stripes must equal the oracle's parity."""
    import importlib.util
    import os

    spec = _LAYOUTS[layout]
    base, kern = _run_child(spec, {}, tmp_path, "base")
    split, _ = _run_child(spec, {"ZFEC_HIP_LAUNCH_UNITS": "1024"}, tmp_path, "split")
    assert np.array_equal(base, split), "launch splitting changed the output"
    if layout == "rows_object_major":
        assert "matapply_rows" in kern, kern
    child = importlib.util.spec_from_file_location(
        "gpu_batch_child", os.path.join(os.path.dirname(os.path.abspath(__file__)), "gpu_batch_child.py"))
    mod = importlib.util.module_from_spec(child)
    child.loader.exec_module(mod)
    src = mod.src_bytes(spec)
    k, m, sz, ns = spec["k"], spec["m"], spec["sz"], spec["ns"]
    r = m - k
    end = (ns - 1) * spec["out_ss"] + (r - 1) * spec["out_bs"] + sz
    assert (base[end:] == 0xA5).all(), "write past the last output row"
    rng = np.random.default_rng(spec["seed"])
    for s in sorted(set([0, ns - 1] + [int(x) for x in rng.integers(0, ns, 6)])):
        ins = np.stack([src[s * spec["in_ss"] + j * spec["in_bs"]:][:sz] for j in range(k)])
        want = oracle.encode(k, m, ins)
        for i in range(r):
            o = s * spec["out_ss"] + i * spec["out_bs"]
            assert (base[o:o + sz] == want[i]).all(), (s, i, kern)


@pytest.mark.parametrize("k,m,sz,ns,rows", [(3, 10, 1366, 300, True), (2, 10, 1025, 64, True), (4, 12, 4096, 100, True),
                                            (1, 9, 2049, 80, True), (3, 10, 1024, 100, False), (3, 10, 4097, 70, False),
                                            (3, 10, 1366, 63, False)])
def test_batch_short_rows_walk(k, m, sz, ns, rows):
    """Short blocks of many stripes go through the one-wave-per-stripe walk
    (matapply_rows, 1 KiB < sz <= 4 KiB, >= 64 stripes): every stripe against
    the oracle, rows at an odd stride with guard bytes that must stay zero."""
    r = m - k
    ld = sz + 40
    rng = np.random.default_rng(sz * 7 + ns)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    host = np.zeros((ns, k, ld), dtype=np.uint8)
    host[:, :, :sz] = data
    src = torch.from_numpy(host).cuda()
    dst = torch.zeros((ns, r, ld), dtype=torch.uint8, device="cuda")
    code = capi.Code(k, m)
    st = torch.cuda.current_stream().cuda_stream
    code.encode_batch(src.data_ptr(), ld, k * ld, dst.data_ptr(), ld, r * ld, list(range(k, m)), sz, ns, stream=st)
    torch.cuda.synchronize()
    assert capi.last_kernel_name().startswith("matapply_rows" if rows else "matapply_reg"), capi.last_kernel_name()
    out = dst.cpu().numpy()
    assert out[:, :, sz:].sum() == 0
    for s in range(ns):
        assert (out[s, :, :sz] == oracle.encode(k, m, data[s])).all(), s
    slots = place(list(range(m - k, m)), k)
    allb = np.concatenate([data, out[:, :, :sz]], axis=1)
    recv = np.zeros((ns, k, ld), dtype=np.uint8)
    recv[:, :, :sz] = allb[:, slots, :]
    missing = [i for i in range(k) if slots[i] >= k]
    rec = torch.zeros((ns, len(missing), ld), dtype=torch.uint8, device="cuda")
    code.decode_batch(torch.from_numpy(recv).cuda().data_ptr(), ld, k * ld, rec.data_ptr(), ld, len(missing) * ld,
                      slots, sz, ns, stream=st)
    torch.cuda.synchronize()
    rv = rec.cpu().numpy()
    assert (rv[:, :, :sz] == data[:, missing, :]).all()
    assert rv[:, :, sz:].sum() == 0


@pytest.mark.parametrize("k,m,sz,ns,ld,used", [(3, 10, 1366, 300, 1536, True), (3, 10, 1366, 300, 1400, False),
                                               (2, 6, 5000, 20, 5120, True), (3, 10, 1408, 100, 1536, True),
                                               (3, 10, 777, 3, 1024, True), (20, 60, 1000, 8, 1024, True),
                                               (3, 10, 100_003, 1, 100_096, True), (3, 10, 100_003, 1, 100_100, False),
                                               (10, 16, 70_001, 1, 70_144, True)])
def test_batch_row_padding_flag(k, m, sz, ns, ld, used):
    """FEC_FLAG_ROW_PADDING: the library may run each row out to its next
    128-byte line.  Bytes [0, sz) stay bit-exact against the oracle; bytes from
    the padded end (or from sz when the stride leaves no room and the flag is
    ignored) to the row stride are guard bytes that must stay zero."""
    r = m - k
    pad = -(-sz // 128) * 128 if used else sz
    rng = np.random.default_rng(sz + ld + ns)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    host = np.zeros((ns, k, ld), dtype=np.uint8)
    host[:, :, :sz] = data
    host[:, :, sz:pad] = 0xA5  # input padding the library may read
    src = torch.from_numpy(host).cuda()
    dst = torch.zeros((ns, r, ld), dtype=torch.uint8, device="cuda")
    code = capi.Code(k, m)
    st = torch.cuda.current_stream().cuda_stream
    fl = capi.FEC_FLAG_ASYNC | capi.FEC_FLAG_ROW_PADDING
    code.encode_batch(src.data_ptr(), ld, k * ld, dst.data_ptr(), ld, r * ld, list(range(k, m)), sz, ns, stream=st,
                      flags=fl)
    torch.cuda.synchronize()
    out = dst.cpu().numpy()
    assert out[:, :, pad:].sum() == 0
    for s in range(ns):
        assert (out[s, :, :sz] == oracle.encode(k, m, data[s])).all(), s
    slots = place(list(range(m - k, m)), k)
    allb = np.concatenate([data, out[:, :, :sz]], axis=1)
    recv = np.zeros((ns, k, ld), dtype=np.uint8)
    recv[:, :, :sz] = allb[:, slots, :]
    missing = [i for i in range(k) if slots[i] >= k]
    rec = torch.zeros((ns, len(missing), ld), dtype=torch.uint8, device="cuda")
    code.decode_batch(torch.from_numpy(recv).cuda().data_ptr(), ld, k * ld, rec.data_ptr(), ld, len(missing) * ld,
                      slots, sz, ns, stream=st, flags=fl)
    torch.cuda.synchronize()
    rv = rec.cpu().numpy()
    assert (rv[:, :, :sz] == data[:, missing, :]).all()
    assert rv[:, :, pad:].sum() == 0


def test_north_star_batch_layouts():
    """The four calls bench.py's batched_1MiB leg times (K=3/M=10, 256 stripes
    of 1 MiB, sz = 349,526 per block): object-major rows at a 256-byte stride
    with FEC_FLAG_ROW_PADDING and without it, a dense [256, 3, sz] array and
    block-major rows.  Every layout gives the same parity bytes for every
    stripe, sampled stripes equal the oracle's, and nothing is written past
    what each call may write: the padding past the 128-byte line (flag) or
    past sz (no flag), and guard bytes after the dense and block-major
    arrays."""
    k, m, ns = 3, 10, 256
    r, sz = m - k, -(-(1 << 20) // k)
    ld, pad, g = -(-sz // 256) * 256, -(-sz // 128) * 128, 4096
    rng = np.random.default_rng(2026)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    dev = torch.from_numpy(data).cuda()
    code = capi.Code(k, m)
    st = torch.cuda.current_stream().cuda_stream
    nums = list(range(k, m))
    outs = {}
    for layout in ("object-major", "object-major, rows end mid-line", "dense", "block-major"):
        flags = capi.FEC_FLAG_ASYNC | (capi.FEC_FLAG_ROW_PADDING if layout == "object-major" else 0)
        if layout.startswith("object-major"):
            src = torch.full((ns, k, ld), 0xA5, dtype=torch.uint8, device="cuda")
            src[:, :, :sz] = dev
            dst = torch.zeros((ns, r, ld), dtype=torch.uint8, device="cuda")
            sbs, sss, dbs, dss = ld, k * ld, ld, r * ld
        elif layout == "dense":
            src = dev.clone()
            flat = torch.zeros(ns * r * sz + g, dtype=torch.uint8, device="cuda")
            dst = flat[:ns * r * sz].view(ns, r, sz)
            sbs, sss, dbs, dss = sz, k * sz, sz, r * sz
        else:
            src = dev.transpose(0, 1).contiguous().view(k, ns * sz)
            flat = torch.zeros(r * ns * sz + g, dtype=torch.uint8, device="cuda")
            dst = flat[:r * ns * sz].view(r, ns * sz)
            sbs, sss, dbs, dss = ns * sz, sz, ns * sz, sz
        code.encode_batch(src.data_ptr(), sbs, sss, dst.data_ptr(), dbs, dss, nums, sz, ns, stream=st, flags=flags)
        torch.cuda.synchronize()
        assert capi.last_kernel_name().startswith("matapply_reg<3,7>"), (layout, capi.last_kernel_name())
        if layout == "object-major":
            assert int(dst[:, :, pad:].count_nonzero()) == 0, "written past the padded line"
            view = dst[:, :, :sz]
        elif layout.startswith("object-major"):
            assert int(dst[:, :, sz:].count_nonzero()) == 0, "written past sz without the flag"
            view = dst[:, :, :sz]
        elif layout == "dense":
            assert int(flat[ns * r * sz:].count_nonzero()) == 0, "written past the dense array"
            view = dst
        else:
            assert int(flat[r * ns * sz:].count_nonzero()) == 0, "written past the block-major rows"
            view = dst.view(r, ns, sz).transpose(0, 1)
        outs[layout] = view
        del src
    first = outs["object-major"]
    for layout, v in outs.items():
        assert torch.equal(v, first), layout
    got = first.cpu().numpy()
    for s in sorted({0, 1, 127, 128, 255} | {int(x) for x in rng.integers(0, ns, 3)}):
        assert (got[s] == oracle.encode(k, m, data[s])).all(), s


@pytest.mark.parametrize("k,m,nums", [(3, 10, [7, 1, 9]), (5, 9, [0, 1, 2, 3, 4]), (10, 16, list(range(6, 16)))])
def test_decode_all_primaries_flag(k, m, nums):
    """FEC_FLAG_ALL_PRIMARIES: the k outputs are the primaries in order, present ones copied."""
    code = capi.Code(k, m)
    rng = np.random.default_rng(k * m)
    sz, ns = 999, 7
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    allb = np.concatenate([data, np.stack([oracle.encode(k, m, data[s]) for s in range(ns)])], axis=1)
    slots = place(nums, k)
    recv = torch.from_numpy(np.ascontiguousarray(allb[:, slots, :])).cuda()
    out = torch.zeros((ns, k, sz), dtype=torch.uint8, device="cuda")
    code.decode_batch(recv.data_ptr(), sz, k * sz, out.data_ptr(), sz, k * sz, slots, sz, ns,
                      stream=torch.cuda.current_stream().cuda_stream,
                      flags=capi.FEC_FLAG_ASYNC | capi.FEC_FLAG_ALL_PRIMARIES)
    torch.cuda.synchronize()
    assert (out.cpu().numpy() == data).all()


# ---- BASELINE config sizes ------------------------------------------------------

def test_config2_64mib_vs_oracle():
    """K=3/M=10, 64 MiB stripe: parity bit-exact vs the oracle, then a
    secondary-only decode recovers the input."""
    k, m, S = 3, 10, 64 << 20
    sz = -(-S // k)
    rng = np.random.default_rng(2)
    data = np.zeros((k, sz), dtype=np.uint8)
    flat = data.reshape(-1)
    flat[:S] = rng.integers(0, 256, size=S, dtype=np.uint8)
    ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
    out = zfec_amd.Encoder(k, m).encode(ins)
    par = torch.stack(out[k:]).cpu().numpy()
    assert (par == oracle.encode(k, m, data)).all()
    dec = zfec_amd.Decoder(k, m).decode(out[3:6], [3, 4, 5])
    assert (torch.stack(dec).cpu().numpy() == data).all()


class _kernels(object):
    """Which kernel family serves a full-size launch: "jit" = the run-time
    specialised bit-sliced kernel of the launch's matrix (compiled up front with
    fec_jit_prepare_*, as bench.py times it), "bsr" = matapply_bsr (the
    bit-sliced kernel with the matrix as run-time data, one precompiled routine
    call per coefficient: the default for a first launch of a matrix and for
    every first-seen erasure pattern, generic mode 2), "generic" = matapply_bsg
    (the same with the combination choice as LDS reads, generic mode 1),
    "table" = the table-lookup kernels (JIT and generic kernels off).
    check(what) asserts the last launch's kernel."""

    PREFIX = {"jit": "zfec_hip_bitslice", "bsr": "matapply_bsr", "generic": "matapply_bsg", "table": "matapply_lds"}
    GENERIC = {"jit": 2, "bsr": 2, "generic": 1, "table": 0}

    def __init__(self, kind):
        self.kind = kind

    def __enter__(self):
        self.prev = capi.jit_mode(capi.JIT_AUTO if self.kind == "jit" else capi.JIT_OFF)
        self.prev_g = capi.generic_mode(self.GENERIC[self.kind])
        return self

    def __exit__(self, *exc):
        capi.jit_mode(self.prev)
        capi.generic_mode(self.prev_g)
        return False

    def prepare(self, code, enc_nums=None, dec_slots=None):
        if self.kind == "jit":
            if enc_nums is not None:
                code.jit_prepare_encode(enc_nums)
            if dec_slots is not None:
                code.jit_prepare_decode(dec_slots)

    def check(self, what):
        torch.cuda.synchronize()
        name = capi.last_kernel_name()
        assert name.startswith(self.PREFIX[self.kind]), (what, self.kind, name)
        return name


def _batched_full_size(k, m, S, ns, seed, sample, kernels=None):
    """BASELINE batched configs at full size: one encode launch over all
    stripes ([stripe][block][row] rows 256-byte aligned, as bench.py lays them
    out), a decode from the last k blocks; the decode must return every
    stripe (device-side equality), and sampled stripes' parity and recovered
    blocks must equal the oracle's.  With `kernels`, the kernel family of both
    launches is fixed and asserted."""
    r = m - k
    sz = -(-S // k)
    ld = -(-sz // 256) * 256
    g = torch.Generator(device="cuda").manual_seed(seed)
    data = torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda", generator=g)
    par = torch.zeros((ns, r, ld), dtype=torch.uint8, device="cuda")
    code = capi.Code(k, m)
    slots = place(list(range(m - k, m)), k)
    if kernels:
        kernels.prepare(code, list(range(k, m)), slots)
    st = torch.cuda.current_stream().cuda_stream
    code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld, list(range(k, m)), sz, ns, stream=st)
    if kernels:
        kernels.check("encode")
    recv = torch.empty((ns, k, ld), dtype=torch.uint8, device="cuda")
    for i, s in enumerate(slots):
        recv[:, i].copy_(data[:, s] if s < k else par[:, s - k])
    missing = [i for i in range(k) if slots[i] >= k]
    rec = torch.zeros((ns, len(missing), ld), dtype=torch.uint8, device="cuda")
    code.decode_batch(recv.data_ptr(), ld, k * ld, rec.data_ptr(), ld, len(missing) * ld, slots, sz, ns, stream=st)
    if kernels:
        kernels.check("decode")
    torch.cuda.synchronize()
    assert bool(torch.equal(rec[:, :, :sz], data[:, missing, :sz]))
    assert int(par[:, :, sz:].count_nonzero()) == 0  # nothing written past the block ends
    rng = np.random.default_rng(seed)
    for s in sorted(set(int(x) for x in rng.integers(0, ns, size=sample))) + [0, ns - 1]:
        got = par[s, :, :sz].cpu().numpy()
        assert (got == oracle.encode(k, m, data[s, :, :sz].cpu().numpy())).all(), s
        rv = rec[s, :, :sz].cpu().numpy()
        assert (rv == oracle.decode(k, m, recv[s, :, :sz].cpu().numpy(), slots)).all(), s


@pytest.mark.parametrize("kind", ["jit", "bsr", "generic", "table"])
def test_config4_1024_stripes_of_1mib(kind):
    """cfg4: K=20/M=60, 1024 x 1 MiB stripes in one launch, on the kernel
    bench.py times (the bit-sliced kernel of the matrix), on matapply_bsr (what
    the first launch of the matrix and every first-seen decode run on), on
    matapply_bsg and on the table kernel."""
    with _kernels(kind) as kn:
        _batched_full_size(20, 60, 1 << 20, 1024, 4, sample=6, kernels=kn)


def test_config5_1e6_objects_of_4kib():
    """cfg5: K=3/M=10, 10^6 x 4 KiB objects (1366-byte blocks) in one launch."""
    _batched_full_size(3, 10, 4096, 10 ** 6, 5, sample=200)


@pytest.mark.parametrize("kind", ["jit", "bsr", "generic", "table"])
def test_config3_256mib_roundtrip(kind):
    """K=10/M=16, 256 MiB: encode, drop primaries 0-5, decode; compare by
    equality on the device (size-independent property) and check parity rows
    and recovered blocks against the oracle on slices at the start, middle and
    end (column independence), on the kernel bench.py times, on matapply_bsr
    (the first-launch default: matapply_bsr_solo<6> here), on matapply_bsg and
    on the table kernel."""
    k, m, S = 10, 16, 256 << 20
    sz = -(-S // k)
    g = torch.Generator(device="cuda").manual_seed(3)
    data = torch.randint(0, 256, (k, sz), dtype=torch.uint8, device="cuda", generator=g)
    ins = [data[i] for i in range(k)]
    nums = list(range(10, 16)) + [6, 7, 8, 9]
    slots = place(nums, k)
    with _kernels(kind) as kn:
        kn.prepare(capi.Code(k, m), list(range(k, m)), slots)
        out = zfec_amd.Encoder(k, m).encode(ins)
        kn.check("encode")
        dec = zfec_amd.Decoder(k, m).decode([out[n] for n in nums], nums)
        kn.check("decode")
    assert bool(torch.equal(torch.stack(dec), data))
    allb = torch.stack(out)
    for lo in (0, sz // 2, sz - 100000):
        hi = lo + 100000
        par = allb[k:, lo:hi].cpu().numpy()
        assert (par == oracle.encode(k, m, data[:, lo:hi].cpu().numpy())).all(), lo
        missing = [i for i in range(k) if slots[i] >= k]
        got = torch.stack(dec)[missing, lo:hi].cpu().numpy()
        recv = allb[slots, lo:hi].cpu().numpy()
        assert (got == oracle.decode(k, m, recv, slots)).all(), lo


# ---- the reference's own binding on top of the engine ---------------------------

def _dropin_module():
    import glob
    import importlib.util
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    paths = glob.glob(os.path.join(root, "oracle", "_ref", "dropin", "_fec*.so"))
    if not paths:
        pytest.skip("oracle/_ref/dropin not built (needs /root/reference at build time)")
    spec = importlib.util.spec_from_file_location("zfec_dropin._fec", paths[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_reference_binding_dropin(golden):
    """zfec/_fecmodule.c compiled unmodified against libzfec_hip.so (oracle/Makefile
    `dropin`): the reference's own C self-test and Python API run on the GPU
    engine and reproduce the golden vectors."""
    ref_api = _dropin_module()
    assert ref_api.test_from_agl()
    meta, arrays = golden
    for ci, c in enumerate(meta["vectors"]):
        k, m, sz = c["k"], c["m"], c["sz"]
        inp = arrays["vec%d_in" % ci]
        allb = arrays["vec%d_all" % ci]
        out = ref_api.Encoder(k, m).encode(blocks_of(inp))
        assert [bytes(x) for x in out] == [allb[i].tobytes() for i in range(m)], c
        nums = c["decode_nums"][0]
        dec = ref_api.Decoder(k, m).decode([allb[n].tobytes() for n in nums], nums)
        assert b"".join(bytes(x) for x in dec) == inp.tobytes()


@pytest.mark.parametrize("k,m,sz,ns,block_major", [(3, 10, 1366, 500, False), (3, 10, 1366, 500, True),
                                                   (10, 16, 4000, 9, True), (20, 60, 777, 6, False)])
def test_tensor_batch_api(k, m, sz, ns, block_major):
    """zfec_amd.Encoder.encode_batch / Decoder.decode_batch on [nstripes, k, sz]
    device tensors (object-major, or a transposed block-major array): parity
    against the oracle for sampled stripes, decode back from the last k blocks."""
    rng = np.random.default_rng(ns * 31 + sz)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    t = torch.from_numpy(data).cuda()
    if block_major:
        t = t.transpose(0, 1).contiguous().transpose(0, 1)  # storage [k][ns][sz]
    enc = zfec_amd.Encoder(k, m)
    par = enc.encode_batch(t)
    assert par.shape == (ns, m - k, sz) and (par.stride(0) < par.stride(1)) == block_major
    torch.cuda.synchronize()
    p = par.cpu().numpy()
    for s in sorted(set([0, ns - 1] + [int(x) for x in rng.integers(0, ns, 4)])):
        assert (p[s] == oracle.encode(k, m, data[s])).all(), s
    sub = enc.encode_batch(t, [m - 1, k])
    assert torch.equal(sub[:, 0], par[:, m - 1 - k]) and torch.equal(sub[:, 1], par[:, 0])
    slots = place(list(range(m - k, m)), k)
    allb = torch.cat([t, par], dim=1)
    recv = allb[:, slots, :]
    if block_major:
        recv = recv.transpose(0, 1).contiguous().transpose(0, 1)
    else:
        recv = recv.contiguous()
    rec = zfec_amd.Decoder(k, m).decode_batch(recv, slots)
    torch.cuda.synchronize()
    missing = [i for i in range(k) if slots[i] >= k]
    assert (rec.cpu().numpy() == data[:, missing, :]).all()
    with pytest.raises(zfec_amd.Error):
        enc.encode_batch(t, [0])  # primaries are not produced by the batch call
    if k > 1 and m - k >= 2:
        bad = [1, 0] + list(range(k, k + k - 2)) if k > 2 else [1, 0]
        with pytest.raises(zfec_amd.Error):
            zfec_amd.Decoder(k, m).decode_batch(recv, bad)  # primary off its slot


@pytest.mark.parametrize("chunk", [None, 65536, 3 << 20])
def test_large_pageable_bytes_path(chunk, knobs):
    """Large pageable host blocks (bytes / numpy views sharing pages) are
    staged through pinned slots by the host copy threads (fec_abi.cpp
    run_staged).  Parity and a secondary-only decode bit-exact against the
    oracle, at the default chunk and at chunk sizes that cut blocks at odd page
    offsets (ZFEC_HIP_STAGE_CHUNK)."""
    if chunk:
        knobs(ZFEC_HIP_STAGE_CHUNK=chunk)
    k, m, sz = 3, 10, (5 << 20) + 123
    rng = np.random.default_rng(sz)
    flat = rng.integers(0, 256, size=k * sz, dtype=np.uint8)
    data = flat.reshape(k, sz)
    views = [data[i] for i in range(k)]  # adjacent blocks share pages
    out = zfec_amd.Encoder(k, m).encode(views)
    par = np.stack([np.frombuffer(b, np.uint8) for b in out[k:]])
    assert (par == oracle.encode(k, m, data)).all()
    dec = zfec_amd.Decoder(k, m).decode(out[k:2 * k], list(range(k, 2 * k)))
    assert b"".join(dec) == flat.tobytes()
    sub = zfec_amd.Encoder(k, m).encode([v.tobytes() for v in views], [9, 4])
    assert sub[0] == out[9] and sub[1] == out[4]


def test_staged_host_path_concurrent_threads():
    """Several Python threads (the GIL is released in the call) run large
    host-memory encodes and decodes at once: every call's chunks go through
    its own thread's pinned staging slots while all of them share one host
    copy pool (fec_abi.cpp run_staged, host_pool.cpp).  Bit-exact against the
    oracle, K=3/M=10 and K=20/M=60, sizes that cut the last chunk short."""
    import threading

    cases = [(3, 10, (3 << 20) + 17), (20, 60, (256 << 10) + 3), (3, 10, 700_001), (10, 16, (1 << 20) + 5)]
    rng = np.random.default_rng(2024)
    inputs = [rng.integers(0, 256, size=(k, sz), dtype=np.uint8) for k, m, sz in cases]
    want = [oracle.encode(k, m, d) for (k, m, sz), d in zip(cases, inputs)]
    errors = []

    def work(i):
        try:
            k, m, sz = cases[i % len(cases)]
            data = inputs[i % len(cases)]
            blocks = [data[j].tobytes() for j in range(k)]
            for _ in range(3):
                out = zfec_amd.Encoder(k, m).encode(blocks)
                par = np.stack([np.frombuffer(b, np.uint8) for b in out[k:]])
                assert (par == want[i % len(cases)]).all(), (i, k, m, sz)
                nums = list(range(m - k, m))
                assert zfec_amd.Decoder(k, m).decode([out[n] for n in nums], nums) == blocks, (i, k, m, sz)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    ths = [threading.Thread(target=work, args=(i,)) for i in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ths)
    assert not errors, errors


@pytest.mark.parametrize("k,m", [(5, 9), (10, 16), (20, 60), (32, 80), (40, 50), (4, 16), (12, 13), (200, 256)])
def test_small_launch_kernel_vs_oracle(k, m):
    """Launches too small for the unit kernels (a wave per output row,
    matapply_small): device blocks of 1, 3, 4, 5, 205, 4097 and 16000 bytes,
    encode and a decode from the last k blocks, bit-exact against the oracle;
    k > 32 takes the XOR-accumulating continuation launches."""
    rng = np.random.default_rng(k * 1000 + m)
    for sz in (1, 3, 4, 5, 205, 4097, 16000):
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
        out = zfec_amd.Encoder(k, m).encode(ins)
        torch.cuda.synchronize()
        if not (k <= 4 and m - k <= 8):
            assert capi.last_kernel_name() == "matapply_small", (k, m, sz, capi.last_kernel_name())
        par = torch.stack(out[k:]).cpu().numpy()
        assert (par == oracle.encode(k, m, data)).all(), (k, m, sz)
        nums = list(range(m - k, m))
        dec = zfec_amd.Decoder(k, m).decode([out[n] for n in nums], nums)
        assert (torch.stack(dec).cpu().numpy() == data).all(), (k, m, sz)


def test_small_launch_kernel_batched_strided():
    """matapply_small over a batch of stripes at odd strides and misaligned
    bases; bytes between rows and after the last one stay 0xA5."""
    k, m, sz, ns = 20, 60, 333, 5
    r = m - k
    rng = np.random.default_rng(333)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    ld = sz + 13
    base_in, base_out = 1, 7
    src = torch.zeros(base_in + ns * k * ld, dtype=torch.uint8, device="cuda")
    src[base_in:].view(ns, k, ld)[:, :, :sz] = torch.from_numpy(data).cuda()
    dst = torch.full((base_out + ns * r * ld + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    code = capi.Code(k, m)
    code.encode_batch(src.data_ptr() + base_in, ld, k * ld, dst.data_ptr() + base_out, ld, r * ld,
                      list(range(k, m)), sz, ns, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert capi.last_kernel_name() == "matapply_small", capi.last_kernel_name()
    d = dst.cpu().numpy()
    assert (d[:base_out] == 0xA5).all() and (d[base_out + ns * r * ld:] == 0xA5).all()
    out = d[base_out:base_out + ns * r * ld].reshape(ns, r, ld)
    assert (out[:, :, sz:] == 0xA5).all(), "write past a row"
    for s in range(ns):
        assert (out[s, :, :sz] == oracle.encode(k, m, data[s])).all(), s


@pytest.mark.parametrize("layout", ["packed", "padded_rows", "block_major", "src_device", "dst_device"])
def test_batch_pageable_host_memory(layout):
    """fec_encode_batch / fec_decode_batch on pageable host memory (numpy):
    staged through pinned slots in groups of stripes (fec_abi.cpp
    run_batch_staged).  Object-major packed rows, rows padded with guard bytes
    that must stay untouched, block-major arrays, and one side on the device;
    enough stripes for several groups; parity and decode vs the oracle."""
    k, m, sz, ns = 5, 12, 3001, 2000
    r = m - k
    rng = np.random.default_rng(ns + sz)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    code = capi.Code(k, m)
    pad = 37 if layout == "padded_rows" else 0
    ld = sz + pad
    if layout == "block_major":
        src = np.ascontiguousarray(data.transpose(1, 0, 2))  # [k][ns][sz]
        sptr, sbs, sss = src.ctypes.data, ns * sz, sz
        dst = np.full((r, ns, sz), 0xA5, np.uint8)
        dptr, dbs, dss = dst.ctypes.data, ns * sz, sz
        read_par = lambda: dst.transpose(1, 0, 2)
    else:
        src = np.full((ns, k, ld), 0x5A, np.uint8)
        src[:, :, :sz] = data
        dst = np.full((ns, r, ld), 0xA5, np.uint8)
        sptr, sbs, sss = src.ctypes.data, ld, k * ld
        dptr, dbs, dss = dst.ctypes.data, ld, r * ld
        read_par = lambda: dst[:, :, :sz]
    keep = []
    if layout == "src_device":
        t = torch.from_numpy(src).cuda()
        keep.append(t)
        sptr = t.data_ptr()
    dev_out = None
    if layout == "dst_device":
        dev_out = torch.full(dst.shape, 0xA5, dtype=torch.uint8, device="cuda")
        dptr = dev_out.data_ptr()
    code.encode_batch(sptr, sbs, sss, dptr, dbs, dss, list(range(k, m)), sz, ns, flags=capi.FEC_FLAG_LIBRARY_STREAM)
    torch.cuda.synchronize()
    if dev_out is not None:
        dst[...] = dev_out.cpu().numpy()
    par = read_par()
    for s in list(range(0, ns, 97)) + [ns - 1]:
        assert (par[s] == oracle.encode(k, m, data[s])).all(), (layout, s)
    if pad:
        assert (dst[:, :, sz:] == 0xA5).all(), "a padded row's guard bytes were written"
    # decode every stripe from parity blocks 5..9 (all primaries missing)
    nums = list(range(k, 2 * k))
    recv = np.ascontiguousarray(par[:, :k, :])  # slots hold blocks k..2k-1
    rec = np.full((ns, k, sz), 0x33, np.uint8)
    code.decode_batch(recv.ctypes.data, sz, k * sz, rec.ctypes.data, sz, k * sz, nums, sz, ns,
                      flags=capi.FEC_FLAG_LIBRARY_STREAM)
    assert (rec == data).all(), layout


def test_batch_api_host_numpy_arrays():
    """Encoder.encode_batch / Decoder.decode_batch take host numpy arrays too
    (object-major and transposed block-major), results as numpy arrays."""
    k, m, sz, ns = 3, 10, 1366, 5000
    rng = np.random.default_rng(1366)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    enc, dec = zfec_amd.Encoder(k, m), zfec_amd.Decoder(k, m)
    for blocks in (data, np.ascontiguousarray(data.transpose(1, 0, 2)).transpose(1, 0, 2)):
        par = enc.encode_batch(blocks)
        assert isinstance(par, np.ndarray) and par.shape == (ns, m - k, sz)
        for s in (0, 1, 2500, ns - 1):
            assert (par[s] == oracle.encode(k, m, data[s])).all(), s
        nums = [7, 1, 9]
        recv = np.stack([par[:, 4], data[:, 1], par[:, 6]], axis=1)
        rec = dec.decode_batch(recv, nums)
        assert (rec == data[:, [0, 2], :]).all()


def test_bench_headline_call_vs_oracle():
    """The exact calls bench.py times for its headline (BASELINE configs[1],
    bench.py run_workload): ONE K=3/M=10 stripe of sz = ceil(64 MiB / 3) =
    22,369,622-byte blocks in 22,369,792-byte rows, fec_encode_batch and then
    fec_decode_batch from blocks 7, 8, 9, both with FEC_FLAG_ASYNC |
    FEC_FLAG_ROW_PADDING on a torch stream -- the single-stripe padding grant
    (fec_abi.cpp run_batch) on the nt sc1 register kernels.  Bytes [0, sz)
    against the oracle on slices at the start, middle and end of the blocks
    (every output byte depends only on the same column of the inputs,
    zfec/fec.c:494-503); the bytes past roundup(sz, 128) up to the row stride
    are guard bytes that must stay untouched."""
    k, m = 3, 10
    r = m - k
    sz = -(-(64 << 20) // k)
    ld = -(-sz // 256) * 256
    pad = -(-sz // 128) * 128
    assert (sz, ld) == (22_369_622, 22_369_792)
    g = torch.Generator(device="cuda").manual_seed(2)
    data = torch.randint(0, 256, (1, k, ld), dtype=torch.uint8, device="cuda", generator=g)
    par = torch.full((1, r, ld), 0xA5, dtype=torch.uint8, device="cuda")
    code = capi.Code(k, m)
    st = torch.cuda.current_stream().cuda_stream
    fl = capi.FEC_FLAG_ASYNC | capi.FEC_FLAG_ROW_PADDING
    code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld, list(range(k, m)), sz, 1, stream=st,
                      flags=fl)
    assert capi.last_kernel_name() == "matapply_reg<3,7>", capi.last_kernel_name()
    torch.cuda.synchronize()
    assert bool((par[:, :, pad:] == 0xA5).all()), "encode wrote past the padded row end"
    L = 1 << 20
    for c0 in (0, sz // 2 - L // 2 + 13, sz - L):
        ins = data[0, :, c0:c0 + L].cpu().numpy()
        assert (par[0, :, c0:c0 + L].cpu().numpy() == oracle.encode(k, m, ins)).all(), c0
    # decode from blocks 7, 8, 9 (all secondaries): the received rows as the bench stages them
    slots = [7, 8, 9]
    recv = torch.stack([par[0, s - k] for s in slots]).unsqueeze(0).contiguous()
    rec = torch.full((1, k, ld), 0xA5, dtype=torch.uint8, device="cuda")
    code.decode_batch(recv.data_ptr(), ld, k * ld, rec.data_ptr(), ld, k * ld, slots, sz, 1, stream=st, flags=fl)
    assert capi.last_kernel_name() == "matapply_reg<3,3>", capi.last_kernel_name()
    torch.cuda.synchronize()
    assert bool(torch.equal(rec[:, :, :sz], data[:, :, :sz])), "decode(encode(x)) != x"
    assert bool((rec[:, :, pad:] == 0xA5).all()), "decode wrote past the padded row end"
    for c0 in (0, sz - L):
        got = rec[0, :, c0:c0 + L].cpu().numpy()
        want = oracle.decode(k, m, recv[0, :, c0:c0 + L].cpu().numpy(), slots)
        assert (got == want).all(), c0


@pytest.mark.parametrize("mode", ["signal", "sync"])
def test_small_call_wait_modes(mode, knobs):
    """4 KiB K=3/M=10 stripes from Python bytes: the one-workgroup register
    kernel publishes its completion in pinned host memory and the caller spins
    on it (fec_abi.cpp run_single); ZFEC_HIP_WAIT=sync waits in
    hipStreamSynchronize instead.  Both bit-exact against the oracle, and the
    path actually taken is the one asked for (fec_last_wait)."""
    if mode == "sync":
        knobs(ZFEC_HIP_WAIT="sync")
    k, m = 3, 10
    rng = np.random.default_rng(4096)
    enc, dec = zfec_amd.Encoder(k, m), zfec_amd.Decoder(k, m)
    for sz in (1366, 4096, 1):
        for _ in range(20):
            data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
            out = enc.encode([data[i].tobytes() for i in range(k)])
            assert capi.last_wait() == (1 if mode == "signal" else 0), (mode, sz)
            par = np.stack([np.frombuffer(b, np.uint8) for b in out[k:]])
            assert (par == oracle.encode(k, m, data)).all(), sz
            rec = dec.decode([out[7], out[1], out[9]], [7, 1, 9])
            assert capi.last_wait() == (1 if mode == "signal" else 0), (mode, sz)
            assert b"".join(rec) == data.tobytes(), sz


def test_small_call_signal_under_load():
    """The completion word a one-workgroup small call publishes must never
    overtake its output bytes (kernels.hip matapply_reg: every wave waits for
    its stores, barrier, one lane's system-scope release, then the flag).
    2000 synchronous 4 KiB K=3/M=10 encodes and decodes from bytes, each
    checked against the oracle, while another thread keeps the GPU busy with
    large device-resident encodes on its own stream (MI355X_MICROARCH.md:
    test hand-offs under uneven load)."""
    import threading

    import torch

    k, m = 3, 10
    stop = threading.Event()
    errors = []

    def load():
        try:
            code = capi.Code(20, 60)
            st = torch.cuda.Stream()
            ld = 1 << 20
            src = torch.randint(0, 256, (8, 20, ld), dtype=torch.uint8, device="cuda")
            dst = torch.empty((8, 40, ld), dtype=torch.uint8, device="cuda")
            while not stop.is_set():
                code.encode_batch(src.data_ptr(), ld, 20 * ld, dst.data_ptr(), ld, 40 * ld, list(range(20, 60)),
                                  ld, 8, stream=st.cuda_stream)
                st.synchronize()
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    th = threading.Thread(target=load)
    th.start()
    try:
        rng = np.random.default_rng(2000)
        enc, dec = zfec_amd.Encoder(k, m), zfec_amd.Decoder(k, m)
        for i in range(2000):
            sz = 1366 if i % 3 else int(rng.integers(1, 4097))
            data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
            out = enc.encode([data[j].tobytes() for j in range(k)])
            assert capi.last_wait() == 1
            par = np.stack([np.frombuffer(b, np.uint8) for b in out[k:]])
            assert (par == oracle.encode(k, m, data)).all(), (i, sz)
            rec = dec.decode([out[7], out[8], out[9]], [7, 8, 9])
            assert b"".join(rec) == data.tobytes(), (i, sz)
    finally:
        stop.set()
        th.join()
    assert not errors, errors


def test_small_call_compact_kernel():
    """Synchronous calls from bytes with k <= 4, r <= 8 and blocks of at most
    4 KiB run on the compact one-workgroup kernel (kernels.hip matapply_one,
    whole 16-byte units in the bounce buffer; inputs inside the argument
    block where k x sz fits 4,352 bytes, else read from the bounce buffer):
    bit-exact against the oracle for every such (k, r) at sizes around the
    unit and the 4 KiB limit, both forms; one byte past the limit takes the
    general kernels."""
    rng = np.random.default_rng(77)
    for k in range(1, 5):
        for m in range(k + 1, k + 9):
            enc, dec = zfec_amd.Encoder(k, m), zfec_amd.Decoder(k, m)
            for sz in (1, 15, 16, 17, 1366, 4095, 4096, 4097):
                data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
                out = enc.encode([data[i].tobytes() for i in range(k)])
                name = capi.last_kernel_name()
                ksz = min((sz + 255) // 256 * 256, (sz + 127) // 128 * 128)
                want = "matapply_one<%d,inline>" % k if k * ksz <= 4352 else "matapply_one<%d>" % k
                assert (name == want) == (sz <= 4096), (k, m, sz, name, want)
                par = np.stack([np.frombuffer(b, np.uint8) for b in out[k:]])
                assert (par == oracle.encode(k, m, data)).all(), (k, m, sz)
                nums = list(range(m - k, m))
                rec = dec.decode([out[i] for i in nums], nums)
                assert b"".join(rec) == data.tobytes(), (k, m, sz)


def test_batch_call_and_ctypes_paths_agree():
    """capi's batched calls go through the extension (_fec.batch_call); the
    ctypes binding of the same C-ABI functions must give the same bytes, the
    same kernel and, for a bad call, the same status (a K=3/M=10 batch with
    row padding and a K=20/M=60 batch, encode and decode)."""
    import torch

    capi.lib()
    fast = capi._batch_call
    assert fast is not None
    for k, m, sz, ns in [(3, 10, 4093, 7), (20, 60, 52429, 3)]:
        r, ld = m - k, (sz + 255) // 256 * 256
        code = capi.Code(k, m)
        data = torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda")
        outs, recs, names = [], [], []
        for use_fast in (True, False):
            capi._batch_call = fast if use_fast else None
            try:
                par = torch.zeros((ns, r, ld), dtype=torch.uint8, device="cuda")
                code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld, list(range(k, m)), sz, ns,
                                  flags=capi.FEC_FLAG_ROW_PADDING)
                names.append(capi.last_kernel_name())
                slots = list(range(m - k, m))
                recv = par[:, r - k:].contiguous() if r >= k else None
                rec = torch.zeros((ns, k, ld), dtype=torch.uint8, device="cuda")
                code.decode_batch(recv.data_ptr(), ld, k * ld, rec.data_ptr(), ld, k * ld, slots, sz, ns)
                torch.cuda.synchronize()
                outs.append(par[:, :, :sz].cpu())
                recs.append(rec[:, :, :sz].cpu())
                with pytest.raises(capi.FecError, match="out of range"):
                    code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld, [m], sz, ns)
            finally:
                capi._batch_call = fast
        assert names[0] == names[1], names
        assert torch.equal(outs[0], outs[1]) and torch.equal(recs[0], recs[1]), (k, m)
        assert torch.equal(recs[0], data[:, :, :sz].cpu()), (k, m)
        assert (outs[0][0].numpy() == oracle.encode(k, m, data[0, :, :sz].cpu().numpy())).all(), (k, m)


@pytest.mark.parametrize("mode", ["signal", "sync"])
def test_medium_call_wait_modes(mode, knobs):
    """Synchronous calls from bytes too large for one workgroup: on the
    zero-copy path (the kernel reads and writes the pinned bounce buffer in
    place: up to 1.5 MiB of host blocks for the register shapes k <= 4, r <= 8,
    up to 256 KiB for wider codes; fec_abi.cpp run_single) the stream writes
    the call's sequence number into the pinned completion word after the
    kernel (hipStreamWriteValue32) and the caller spins on it; the copy path
    and ZFEC_HIP_WAIT=sync wait in hipStreamSynchronize.  Bit-exact against
    the oracle either way."""
    if mode == "sync":
        knobs(ZFEC_HIP_WAIT="sync")
    rng = np.random.default_rng(65536)
    for k, m in ((3, 10), (10, 16)):
        enc, dec = zfec_amd.Encoder(k, m), zfec_amd.Decoder(k, m)
        for stripe in (20000, 65536, 131072, 180000):  # all below the staged path (run_staged)
            sz = -(-stripe // k)
            data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
            out = enc.encode([data[i].tobytes() for i in range(k)])
            # in place: the register shapes up to 1.5 MiB of host blocks, wider codes up to 256 KiB
            zero_copy = (sz * m) <= ((3 << 19) if k <= 4 else (256 << 10))
            assert capi.last_wait() == (1 if mode == "signal" and zero_copy else 0), (mode, k, stripe)
            par = np.stack([np.frombuffer(b, np.uint8) for b in out[k:]])
            assert (par == oracle.encode(k, m, data)).all(), (k, m, stripe)
            nums = list(range(m - k, m))
            rec = dec.decode([out[i] for i in nums], nums)
            assert b"".join(rec) == data.tobytes(), (k, m, stripe)


def test_wide_small_calls_bounce_modes():
    """Small calls of wide codes from bytes: up to 256 KiB of host blocks the
    kernel reads and writes the pinned bounce buffer in place over PCIe (the
    stream then publishes completion in the pinned word, fec_last_wait 1);
    past that one H2D and one D2H copy move them (hipStreamSynchronize, 0).
    Bit-exact against the oracle either way, encode and decode."""
    rng = np.random.default_rng(2060)
    for k, m in ((20, 60), (10, 16), (5, 9), (3, 12)):
        enc, dec = zfec_amd.Encoder(k, m), zfec_amd.Decoder(k, m)
        for stripe in (1, 4096, 20000, 65536, 131072):
            sz = -(-stripe // k)
            data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
            out = enc.encode([data[i].tobytes() for i in range(k)])
            in_place = sz * m <= 256 << 10
            if not (k <= 4 and m - k <= 8):  # the register kernels' calls have their own tests
                assert capi.last_wait() == (1 if in_place else 0), (k, m, stripe)
            par = np.stack([np.frombuffer(b, np.uint8) for b in out[k:]])
            assert (par == oracle.encode(k, m, data)).all(), (k, m, stripe, in_place)
            nums = list(range(m - k, m))
            rec = dec.decode([out[i] for i in nums], nums)
            assert b"".join(rec) == data.tobytes(), (k, m, stripe, in_place)
