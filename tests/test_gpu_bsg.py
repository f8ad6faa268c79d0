"""GPU parity of matapply_bsg, the bit-sliced kernel that takes the
coefficient matrix as run-time data (zfec_amd/csrc/kernels.hip): it serves
every wide-code launch no compiled JIT kernel serves -- above all decodes of an
erasure pattern seen for the first time (zfec/fec.c:527-557 decodes every
pattern with one code path).  Bit-exact against the CPU oracle across code
shapes (every rows-per-wave instantiation, rows not a multiple of 4, k up to
32), block sizes around the 4 KiB unit and its overlapping last unit, batched
strided stripes at misaligned bases with guard bytes, and random erasure
patterns; and codes of more than 32 inputs in one pass, their block pointers
and coefficients read from a device-side table (the reference takes any
1 <= k <= m <= 256, zfec/fec.c:437-440; its own benchmark times 94/100,
benchmark-zfec/Main.hs:17)."""

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
def bsg_only(knobs):
    """JIT off, generic kernel on, matapply_small off (these small launches
    would take it)."""
    prev_j, prev_g = capi.jit_mode(capi.JIT_OFF), capi.generic_mode(1)
    knobs(ZFEC_HIP_SMALL_LANES=0)
    yield
    capi.jit_mode(prev_j)
    capi.generic_mode(prev_g)


def place(nums, k):
    slots = [None] * k
    sec = iter([n for n in nums if n >= k])
    for n in nums:
        if n < k:
            slots[n] = n
    return [s if s is not None else next(sec) for s in slots]


# (k, m), k * (m - k) >= 24: rows per wave RT = ceil((m - k) / 4) covers 1, 2, 3, 4, 5, 6, 8, 10, 12
SHAPES = [(7, 11), (6, 12), (6, 13), (10, 16), (4, 16), (5, 20), (7, 24), (20, 40), (8, 31), (6, 37), (20, 60),
          (32, 70), (12, 60)]


@pytest.mark.parametrize("k,m", SHAPES)
def test_bsg_encode_decode_vs_oracle(bsg_only, k, m):
    rng = np.random.default_rng(k * 100 + m)
    for sz in (4096, 4097, 9000):
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
        out = zfec_amd.Encoder(k, m).encode(ins)
        torch.cuda.synchronize()
        assert capi.last_kernel_name().startswith("matapply_bsg"), capi.last_kernel_name()
        par = torch.stack(out[k:]).cpu().numpy()
        assert (par == oracle.encode(k, m, data)).all(), (k, m, sz)
        nums = sorted(int(x) for x in rng.choice(m, size=k, replace=False))
        if all(n < k for n in nums):
            nums = list(range(m - k, m))
        dec = zfec_amd.Decoder(k, m).decode([out[n] for n in nums], nums)
        assert (torch.stack(dec).cpu().numpy() == data).all(), (k, m, sz, nums)


@pytest.mark.parametrize("k,m,sz,ns", [(10, 16, 5000, 9), (20, 60, 52429, 7), (6, 13, 4096, 33), (32, 40, 12345, 3)])
def test_bsg_batched_strided_misaligned(bsg_only, k, m, sz, ns):
    """Batched stripes at odd strides and misaligned bases: every stripe
    against the oracle; bytes between rows and after the last one stay 0xA5."""
    r = m - k
    rng = np.random.default_rng(sz + ns)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    ld = sz + 24
    base_in, base_out = 3, 5
    src = torch.zeros(base_in + ns * k * ld, dtype=torch.uint8, device="cuda")
    view = src[base_in:].view(ns, k, ld)
    view[:, :, :sz] = torch.from_numpy(data).cuda()
    dst = torch.full((base_out + ns * r * ld + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    code = capi.Code(k, m)
    st = torch.cuda.current_stream().cuda_stream
    code.encode_batch(src.data_ptr() + base_in, ld, k * ld, dst.data_ptr() + base_out, ld, r * ld,
                      list(range(k, m)), sz, ns, stream=st)
    torch.cuda.synchronize()
    assert capi.last_kernel_name().startswith("matapply_bsg"), capi.last_kernel_name()
    d = dst.cpu().numpy()
    assert (d[:base_out] == 0xA5).all() and (d[base_out + ns * r * ld:] == 0xA5).all()
    out = d[base_out:base_out + ns * r * ld].reshape(ns, r, ld)
    assert (out[:, :, sz:] == 0xA5).all(), "write past a row"
    for s in range(ns):
        assert (out[s, :, :sz] == oracle.encode(k, m, data[s])).all(), s


def test_bsg_fresh_erasure_patterns(bsg_only):
    """cfg4's code, 20 random erasure patterns, each decoded once (no JIT kernel
    exists for any of them): recovered blocks equal the inputs and the oracle."""
    k, m, sz, ns = 20, 60, 52429, 16
    ld = (sz + 255) // 256 * 256
    g = torch.Generator(device="cuda").manual_seed(20)
    data = torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda", generator=g)
    par = torch.zeros((ns, m - k, ld), dtype=torch.uint8, device="cuda")
    code = capi.Code(k, m)
    st = torch.cuda.current_stream().cuda_stream
    code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, (m - k) * ld, list(range(k, m)), sz, ns,
                      stream=st)
    allb = torch.cat([data, par], dim=1)
    rng = np.random.default_rng(60)
    for p in range(20):
        nums = sorted(int(x) for x in rng.choice(m, size=k, replace=False))
        sl = place(nums, k)
        miss = [i for i in range(k) if sl[i] >= k]
        if not miss:
            continue
        rv = allb[:, sl, :].contiguous()
        rec = torch.zeros((ns, len(miss), ld), dtype=torch.uint8, device="cuda")
        code.decode_batch(rv.data_ptr(), ld, k * ld, rec.data_ptr(), ld, len(miss) * ld, sl, sz, ns, stream=st)
        torch.cuda.synchronize()
        if len(miss) * k >= 24:
            assert capi.last_kernel_name().startswith("matapply_bsg"), capi.last_kernel_name()
        assert bool(torch.equal(rec[:, :, :sz], data[:, miss, :sz])), nums
        s = int(rng.integers(0, ns))
        want = oracle.decode(k, m, rv[s, :, :sz].cpu().numpy(), sl)
        assert (rec[s, :, :sz].cpu().numpy() == want).all(), nums


def test_bsg_off_gives_identical_bytes():
    """generic mode off: the table kernels serve the same launch, same bytes."""
    k, m, sz = 20, 60, 70000  # 8750 eight-byte units: past matapply_small's threshold
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
    ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
    prev_j = capi.jit_mode(capi.JIT_OFF)
    try:
        outs = {}
        for gen in (1, 0):
            prev = capi.generic_mode(gen)
            try:
                outs[gen] = torch.stack(zfec_amd.Encoder(k, m).encode(ins)[k:])
                torch.cuda.synchronize()
                assert capi.last_kernel_name().startswith("matapply_bsg" if gen else "matapply_lds")
            finally:
                capi.generic_mode(prev)
    finally:
        capi.jit_mode(prev_j)
    assert torch.equal(outs[0], outs[1])


# k > 32: one pass with the device-side table (r <= 48 per launch; wider r in
# near-equal row groups), instead of XOR-accumulating passes of 32 inputs
WIDE_SHAPES = [(33, 41), (47, 60), (94, 100), (64, 112), (128, 150), (200, 256), (255, 256)]


@pytest.mark.parametrize("k,m", WIDE_SHAPES)
def test_bsg_wide_k_vs_oracle(bsg_only, k, m):
    rng = np.random.default_rng(k * 1000 + m)
    for sz in (4096, 6001):
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
        out = zfec_amd.Encoder(k, m).encode(ins)
        torch.cuda.synchronize()
        assert capi.last_kernel_name().startswith("matapply_bsg") and capi.last_kernel_name().endswith(",tbl>"), \
            capi.last_kernel_name()
        par = torch.stack(out[k:]).cpu().numpy()
        assert (par == oracle.encode(k, m, data)).all(), (k, m, sz)
        # decode from a random k of the m blocks
        nums = sorted(int(x) for x in rng.choice(m, size=k, replace=False))
        dec = zfec_amd.Decoder(k, m).decode([out[n] for n in nums], nums)
        assert (torch.stack(dec).cpu().numpy() == data).all(), (k, m, sz, nums)


def test_bsg_wide_k_batched_guards(bsg_only):
    """94/100 over strided stripes at misaligned bases: every stripe against the
    oracle, bytes between rows and around the buffer untouched; the same batch
    again with the generic kernel off (XOR-accumulating table passes) gives the
    same bytes."""
    k, m, sz, ns = 94, 100, 5000, 5
    r = m - k
    rng = np.random.default_rng(94)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    ld = sz + 40
    src = torch.zeros(7 + ns * k * ld, dtype=torch.uint8, device="cuda")
    src[7:].view(ns, k, ld)[:, :, :sz] = torch.from_numpy(data).cuda()
    outs = []
    for gen in (1, 0):
        capi.generic_mode(gen)
        dst = torch.full((9 + ns * r * ld + 64,), 0xA5, dtype=torch.uint8, device="cuda")
        code = capi.Code(k, m)
        code.encode_batch(src.data_ptr() + 7, ld, k * ld, dst.data_ptr() + 9, ld, r * ld, list(range(k, m)), sz, ns,
                          stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert capi.last_kernel_name().startswith("matapply_bsg" if gen else "matapply_lds"), capi.last_kernel_name()
        outs.append(dst.cpu().numpy())
    capi.generic_mode(1)
    assert np.array_equal(outs[0], outs[1])
    d = outs[0]
    assert (d[:9] == 0xA5).all() and (d[9 + ns * r * ld:] == 0xA5).all()
    o = d[9:9 + ns * r * ld].reshape(ns, r, ld)
    assert (o[:, :, sz:] == 0xA5).all(), "write past a row"
    for s_ in range(ns):
        assert (o[s_, :, :sz] == oracle.encode(k, m, data[s_])).all(), s_


def test_bsg_wide_k_table_ring_reuse(bsg_only):
    """More wide launches than the table ring has slots, queued back to back on
    one stream with different matrices (every decode pattern a new one): each
    launch must read its own table, so every result is checked."""
    k, m, sz = 40, 60, 8192
    rng = np.random.default_rng(40)
    data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
    ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
    allb = zfec_amd.Encoder(k, m).encode(ins)
    dec = zfec_amd.Decoder(k, m)
    results = []
    for _ in range(20):  # 20 > 8 ring slots
        nums = sorted(int(x) for x in rng.choice(m, size=k, replace=False))
        results.append((nums, dec.decode([allb[n] for n in nums], nums)))
    torch.cuda.synchronize()
    for nums, got in results:
        assert (torch.stack(got).cpu().numpy() == data).all(), nums
