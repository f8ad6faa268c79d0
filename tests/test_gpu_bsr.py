"""GPU parity of matapply_bsr (zfec_amd/csrc/kernels.hip, routines in
gf_routines.inc): the run-time-data bit-sliced kernel that calls one
precompiled multiply-by-constant routine per coefficient.  It serves launches
of k <= 32 inputs and r <= 40 rows that no compiled JIT kernel serves -- above
all decodes of an erasure pattern seen for the first time (zfec/fec.c:527-557
decodes every pattern with one code path).  Bit-exact against the CPU oracle
for every rows-per-wave instantiation (RT = 1..10) and wave count (1..4 row
tiles), block sizes around the 2 KiB unit and its overlapping last unit,
batched strided stripes at misaligned bases with guard bytes, random erasure
patterns, and against matapply_bsg (generic mode 1) on the same launch."""

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
def bsr_only(knobs):
    """JIT off, generic mode 2 (matapply_bsr first), matapply_small off."""
    prev_j, prev_g = capi.jit_mode(capi.JIT_OFF), capi.generic_mode(2)
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


def bsr_name(r, units=0):
    """kernels.hip bsr_tiles: one wave for r <= 10; two for 11-16 rows, and
    for 17-20 rows in launches of >= 2048 units; else four."""
    nw = 1 if r <= 10 else 2 if r <= 16 or (r <= 20 and units * 2 >= 256 * 16) else 4
    return "matapply_bsr<%d>" % (-(-r // nw))


def is_bsr(name, r, units=0):
    """matapply_bsr<RT> for r rows (RT = rows per wave), any variant suffix."""
    want = bsr_name(r, units)[:-1]
    return name.startswith(want) and name[len(want)] in ">,"


# (k, m): r = m - k = 1..10 (one wave, RT = r), 13 / 20 (two waves), 25 (three), 31 / 40 (four);
# odd k on the double-buffered LDS phases (a short last phase: 9 and 15 inputs in phases of 2 on
# two waves, 13 in phases of 4 on four)
SHAPES = [(30, 31), (12, 14), (10, 13), (7, 11), (6, 11), (10, 16), (5, 12), (20, 28), (3, 12), (32, 42),
          (20, 33), (12, 32), (16, 41), (2, 33), (20, 60), (32, 72), (9, 20), (15, 27), (13, 30)]


@pytest.mark.parametrize("k,m", SHAPES)
def test_bsr_encode_decode_vs_oracle(bsr_only, k, m):
    rng = np.random.default_rng(k * 100 + m)
    for sz in (2048, 2049, 4097, 9000):
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
        out = zfec_amd.Encoder(k, m).encode(ins)
        torch.cuda.synchronize()
        assert is_bsr(capi.last_kernel_name(), m - k), (capi.last_kernel_name(), k, m)
        par = torch.stack(out[k:]).cpu().numpy()
        assert (par == oracle.encode(k, m, data)).all(), (k, m, sz)
        nums = sorted(int(x) for x in rng.choice(m, size=k, replace=False))
        if all(n < k for n in nums):
            nums = list(range(m - k, m))
        dec = zfec_amd.Decoder(k, m).decode([out[n] for n in nums], nums)
        assert (torch.stack(dec).cpu().numpy() == data).all(), (k, m, sz, nums)


@pytest.mark.parametrize("k,m,sz,ns", [(10, 16, 5000, 9), (20, 60, 52429, 7), (6, 13, 2048, 33), (32, 40, 12345, 3),
                                       (20, 33, 2100, 50)])
def test_bsr_batched_strided_misaligned(bsr_only, k, m, sz, ns):
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
    assert is_bsr(capi.last_kernel_name(), r), capi.last_kernel_name()
    d = dst.cpu().numpy()
    assert (d[:base_out] == 0xA5).all() and (d[base_out + ns * r * ld:] == 0xA5).all()
    out = d[base_out:base_out + ns * r * ld].reshape(ns, r, ld)
    assert (out[:, :, sz:] == 0xA5).all(), "write past a row"
    for s in range(ns):
        assert (out[s, :, :sz] == oracle.encode(k, m, data[s])).all(), s


def test_bsr_fresh_erasure_patterns(bsr_only):
    """cfg4's code, 20 random erasure patterns, each decoded once: recovered
    blocks equal the inputs and the oracle."""
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
    rng = np.random.default_rng(61)
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
            assert is_bsr(capi.last_kernel_name(), len(miss)), capi.last_kernel_name()
        assert bool(torch.equal(rec[:, :, :sz], data[:, miss, :sz])), nums
        s = int(rng.integers(0, ns))
        want = oracle.decode(k, m, rv[s, :, :sz].cpu().numpy(), sl)
        assert (rec[s, :, :sz].cpu().numpy() == want).all(), nums


def test_bsr_every_coefficient(bsr_only):
    """Every routine: the 32/72 encode (253 of the 255 nonzero coefficients;
    routine 0 runs for the padding rows of a tile) and decodes chosen until
    their matrices have used the remaining ones, each against the oracle."""
    k, m, sz = 32, 72, 4096
    rng = np.random.default_rng(256)
    data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
    ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
    enc = zfec_amd.Encoder(k, m).encode(ins)
    torch.cuda.synchronize()
    assert is_bsr(capi.last_kernel_name(), m - k), capi.last_kernel_name()
    assert (torch.stack(enc[k:]).cpu().numpy() == oracle.encode(k, m, data)).all()
    cov = set(np.asarray(oracle.enc_matrix(k, m)).reshape(m, k)[k:].flatten().tolist())
    dec = zfec_amd.Decoder(k, m)
    tries = 0
    while not cov >= set(range(1, 256)) and tries < 400:
        tries += 1
        nums = sorted(int(x) for x in rng.choice(m, size=k, replace=False))
        sl = place(nums, k)
        miss = [i for i in range(k) if sl[i] >= k]
        if len(miss) * k < 24:
            continue
        dm = np.asarray(oracle.decode_matrix(k, m, sl)).reshape(k, k)
        new = set(dm[miss].flatten().tolist()) - cov
        if not new:
            continue
        cov |= new
        got = dec.decode([enc[n] for n in nums], nums)
        torch.cuda.synchronize()
        assert is_bsr(capi.last_kernel_name(), len(miss)), capi.last_kernel_name()
        assert (torch.stack(got).cpu().numpy() == data).all(), nums
    assert cov >= set(range(1, 256)), sorted(set(range(1, 256)) - cov)


@pytest.mark.parametrize("k,m", [(20, 60), (10, 16), (32, 42)])
def test_bsr_equals_bsg(k, m):
    """The same encode and fresh decode with generic mode 2 (matapply_bsr) and 1
    (matapply_bsg): identical bytes."""
    rng = np.random.default_rng(k + m)
    sz = 70000
    data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
    ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
    nums = sorted(int(x) for x in rng.choice(m, size=k, replace=False))
    prev_j = capi.jit_mode(capi.JIT_OFF)
    res = {}
    try:
        for gen in (2, 1):
            prev = capi.generic_mode(gen)
            try:
                enc = zfec_amd.Encoder(k, m).encode(ins)
                torch.cuda.synchronize()
                assert capi.last_kernel_name().startswith("matapply_bsr" if gen == 2 else "matapply_bsg")
                dec = zfec_amd.Decoder(k, m).decode([enc[n] for n in nums], nums)
                res[gen] = (torch.stack(enc[k:]).cpu(), torch.stack(dec).cpu())
            finally:
                capi.generic_mode(prev)
    finally:
        capi.jit_mode(prev_j)
    assert torch.equal(res[1][0], res[2][0]) and torch.equal(res[1][1], res[2][1])
    assert (res[2][1].numpy() == data).all()


# k > 32 with one row tile: matapply_bsr_ks (inputs split over the waves of a
# workgroup, partial planes XOR-reduced in LDS, pointers and coefficients from
# a device-side table); the reference benchmark's own shape is 94/100
# (benchmark-zfec/Main.hs:17)
WIDE_SHAPES = [(33, 34), (40, 48), (47, 57), (94, 100), (128, 131), (200, 206), (255, 256)]


@pytest.mark.parametrize("k,m", WIDE_SHAPES)
def test_bsr_wide_vs_oracle(bsr_only, k, m):
    rng = np.random.default_rng(k * 7 + m)
    for sz in (4096, 6001, 70000):
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
        out = zfec_amd.Encoder(k, m).encode(ins)
        torch.cuda.synchronize()
        assert capi.last_kernel_name() == "matapply_bsr<%d,ks,tbl>" % (m - k), capi.last_kernel_name()
        par = torch.stack(out[k:]).cpu().numpy()
        assert (par == oracle.encode(k, m, data)).all(), (k, m, sz)
        nums = sorted(int(x) for x in rng.choice(m, size=k, replace=False))
        dec = zfec_amd.Decoder(k, m).decode([out[n] for n in nums], nums)
        assert (torch.stack(dec).cpu().numpy() == data).all(), (k, m, sz, nums)


def test_bsr_wide_batched_guards(bsr_only):
    """94/100 over strided stripes at misaligned bases: every stripe against the
    oracle, bytes between rows and around the buffer untouched."""
    k, m, sz, ns = 94, 100, 5000, 5
    r = m - k
    rng = np.random.default_rng(9400)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    ld = sz + 40
    src = torch.zeros(7 + ns * k * ld, dtype=torch.uint8, device="cuda")
    src[7:].view(ns, k, ld)[:, :, :sz] = torch.from_numpy(data).cuda()
    dst = torch.full((9 + ns * r * ld + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    code = capi.Code(k, m)
    code.encode_batch(src.data_ptr() + 7, ld, k * ld, dst.data_ptr() + 9, ld, r * ld, list(range(k, m)), sz, ns,
                      stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert capi.last_kernel_name() == "matapply_bsr<6,ks,tbl>", capi.last_kernel_name()
    d = dst.cpu().numpy()
    assert (d[:9] == 0xA5).all() and (d[9 + ns * r * ld:] == 0xA5).all()
    o = d[9:9 + ns * r * ld].reshape(ns, r, ld)
    assert (o[:, :, sz:] == 0xA5).all(), "write past a row"
    for s_ in range(ns):
        assert (o[s_, :, :sz] == oracle.encode(k, m, data[s_])).all(), s_


def test_bsr_wide_table_ring_reuse(bsr_only):
    """More wide launches than the table ring has slots, queued back to back on
    one stream with different matrices: each launch must read its own table."""
    k, m, sz = 94, 100, 8192
    rng = np.random.default_rng(941)
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


def test_bsr_table_cache_cross_stream(bsr_only):
    """A matrix's routine-address table is uploaded once, on the stream of its
    first launch (kernels.hip bsr_addr_table); a launch of the same matrix on
    another stream must wait for that upload.  The first stream is held by a
    spin kernel while the second launch is queued, so a missing wait would
    run the second kernel on an empty table."""
    k, m, sz = 94, 100, 8192
    rng = np.random.default_rng(942)
    data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
    ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
    want = oracle.encode(k, m, data)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    enc = zfec_amd.Encoder(k, m)
    outs = []
    for rep in range(3):
        with torch.cuda.stream(s1):
            torch.cuda._sleep(5_000_000)  # the upload on s1 waits behind this
            outs.append(enc.encode(ins)[k:])
        with torch.cuda.stream(s2):
            outs.append(enc.encode(ins)[k:])
    torch.cuda.synchronize()
    assert capi.last_kernel_name() == "matapply_bsr<6,ks,tbl>", capi.last_kernel_name()
    for o in outs:
        assert (torch.stack(o).cpu().numpy() == want).all()


@pytest.mark.parametrize("k,m", [(94, 100), (255, 256)])
def test_bsr_wide_equals_bsg(k, m):
    """Generic mode 2 (matapply_bsr_ks) and 1 (matapply_bsg's table form) on the
    same encode: identical bytes."""
    rng = np.random.default_rng(k)
    sz = 70000
    data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
    ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
    prev_j = capi.jit_mode(capi.JIT_OFF)
    res = {}
    try:
        for gen in (2, 1):
            prev = capi.generic_mode(gen)
            try:
                res[gen] = torch.stack(zfec_amd.Encoder(k, m).encode(ins)[k:]).cpu()
                torch.cuda.synchronize()
                assert capi.last_kernel_name().startswith("matapply_bsr" if gen == 2 else "matapply_bsg")
            finally:
                capi.generic_mode(prev)
    finally:
        capi.jit_mode(prev_j)
    assert torch.equal(res[1], res[2])


def tbl_name(r, units, k):
    """The kernel a launch of k > 32 inputs or > 40 rows takes (kernels.hip
    bsr_wide_ok / launch_bsr_tbl): the ks form for one row tile, or in row groups
    of 8 for k >= 64 when the LDS-phase form would run fewer than 8 waves per CU
    (units x row groups of 64 x waves per group); else the LDS-phase table form
    with tiles of <= 8 rows in row groups of <= 8 tiles."""
    tile = 8
    ng = -(-r // (8 * tile))
    rpg = -(-r // ng)
    nw = 1
    while nw * tile < rpg:
        nw *= 2
    if k > 32 and (r <= 10 or (k >= 64 and units * ng * nw < 256 * 8)):
        ng = 1 if r <= 10 else -(-r // 8)
        return "matapply_bsr<%d,ks,tbl>" % -(-r // ng)
    # 8-wave workgroups share the inputs' combinations through LDS (kernels.hip bsr_cmb)
    return "matapply_bsr<%d,lds,tbl%s>" % (-(-rpg // nw), ",cmb" if nw >= 8 else "")


# table form of the LDS-phase kernel: k > 32 with more than one row tile (row
# groups of <= 64 rows past 64), and k <= 32 with 41..48 rows
TBL_SHAPES = [(33, 50), (40, 60), (47, 60), (64, 112), (128, 150), (128, 256), (200, 256), (32, 74), (20, 68)]


@pytest.mark.parametrize("k,m,sz", [(40, 60, (128 << 20) // 40), (128, 256, (64 << 20) // 128),
                                    (200, 256, 400 * 2048)])
def test_bsr_table_form_large_launch(bsr_only, k, m, sz):
    """Launches large enough for the LDS-phase table form (tiles of <= 8 rows;
    128/256 in two row groups and 200/256 at 400 units on 8-wave workgroups that
    share their inputs' combinations through LDS): against the oracle on
    sampled columns."""
    rng = np.random.default_rng(k + 3 * m)
    data = torch.randint(0, 256, (k, sz), dtype=torch.uint8, device="cuda")
    out = zfec_amd.Encoder(k, m).encode([data[i] for i in range(k)])
    torch.cuda.synchronize()
    units = -(-sz // 2048)
    assert capi.last_kernel_name() == tbl_name(m - k, units, k), capi.last_kernel_name()
    cols = np.sort(rng.choice(sz, size=4096, replace=False))
    got = torch.stack(out[k:])[:, torch.from_numpy(cols).cuda()].cpu().numpy()
    want = oracle.encode(k, m, data[:, torch.from_numpy(cols).cuda()].cpu().numpy())
    assert (got == want).all()


@pytest.mark.parametrize("k,m", TBL_SHAPES)
def test_bsr_table_form_vs_oracle(bsr_only, k, m):
    rng = np.random.default_rng(k * 13 + m)
    for sz in (4096, 6001):
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
        out = zfec_amd.Encoder(k, m).encode(ins)
        torch.cuda.synchronize()
        assert capi.last_kernel_name() == tbl_name(m - k, -(-sz // 2048), k), (capi.last_kernel_name(), k, m)
        par = torch.stack(out[k:]).cpu().numpy()
        assert (par == oracle.encode(k, m, data)).all(), (k, m, sz)
        nums = sorted(int(x) for x in rng.choice(m, size=k, replace=False))
        dec = zfec_amd.Decoder(k, m).decode([out[n] for n in nums], nums)
        assert (torch.stack(dec).cpu().numpy() == data).all(), (k, m, sz, nums)


def test_bsr_table_form_batched_guards(bsr_only):
    """128/256 (two row groups) over strided stripes at misaligned bases: every
    stripe against the oracle, bytes between rows and around the buffer
    untouched."""
    k, m, sz, ns = 128, 256, 4500, 3
    r = m - k
    rng = np.random.default_rng(128256)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    ld = sz + 40
    src = torch.zeros(7 + ns * k * ld, dtype=torch.uint8, device="cuda")
    src[7:].view(ns, k, ld)[:, :, :sz] = torch.from_numpy(data).cuda()
    dst = torch.full((9 + ns * r * ld + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    code = capi.Code(k, m)
    code.encode_batch(src.data_ptr() + 7, ld, k * ld, dst.data_ptr() + 9, ld, r * ld, list(range(k, m)), sz, ns,
                      stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert capi.last_kernel_name() == tbl_name(r, ns * -(-sz // 2048), k), capi.last_kernel_name()
    d = dst.cpu().numpy()
    assert (d[:9] == 0xA5).all() and (d[9 + ns * r * ld:] == 0xA5).all()
    o = d[9:9 + ns * r * ld].reshape(ns, r, ld)
    assert (o[:, :, sz:] == 0xA5).all(), "write past a row"
    for s_ in range(ns):
        assert (o[s_, :, :sz] == oracle.encode(k, m, data[s_])).all(), s_


# Launches past the grid cap (kernels.hip launch_bsr / launch_bsr_wide: at most
# CUs x 1024 workgroups, 262,144 on MI355X) walk their units grid-stride; these
# shapes give each form more units than that: the one-wave form (5/13:
# matapply_bsr<8>), the LDS-phase form (6/20: two tiles of 7) and the ks form
# (33/34: one row, inputs split over the waves).
@pytest.mark.parametrize("k,m,sz,ns", [(5, 13, 2048, 300000), (6, 20, 2048, 270000), (33, 34, 4096, 132000)])
def test_bsr_past_grid_cap(bsr_only, k, m, sz, ns):
    r = m - k
    units = ns * (sz // 2048)
    assert units > 256 * 1024
    g = torch.Generator(device="cuda").manual_seed(k * m)
    data = torch.randint(0, 256, (ns, k, sz), dtype=torch.uint8, device="cuda", generator=g)
    par = torch.full((ns, r, sz), 0xA5, dtype=torch.uint8, device="cuda")
    code = capi.Code(k, m)
    st = torch.cuda.current_stream().cuda_stream
    code.encode_batch(data.data_ptr(), sz, k * sz, par.data_ptr(), sz, r * sz, list(range(k, m)), sz, ns, stream=st)
    torch.cuda.synchronize()
    name = capi.last_kernel_name()
    want = "matapply_bsr<%d,ks,tbl>" % r if k > 32 else bsr_name(r, units)
    assert name == want or (k <= 32 and is_bsr(name, r, units)), name
    # decode from the last k blocks (all the parity there is, plus the highest
    # primaries): recovered blocks must equal the data in every stripe
    nums = list(range(m - k, m))
    sl = place(nums, k)
    miss = [i for i in range(k) if sl[i] >= k]
    allb = torch.cat([data, par], dim=1)
    rv = allb[:, sl, :].contiguous()
    del allb
    rec = torch.full((ns, len(miss), sz), 0x5A, dtype=torch.uint8, device="cuda")
    code.decode_batch(rv.data_ptr(), sz, k * sz, rec.data_ptr(), sz, len(miss) * sz, sl, sz, ns, stream=st)
    torch.cuda.synchronize()
    assert bool(torch.equal(rec, data[:, miss, :])), "a stripe was not recovered"
    rng = np.random.default_rng(ns)
    # stripes on both sides of the first grid-stride step, the last one, random ones
    cap = 256 * 1024 * 2048 // sz
    for s in sorted({0, cap - 1, cap, ns - 1} | set(int(x) for x in rng.integers(0, ns, size=12))):
        got = par[s].cpu().numpy()
        assert (got == oracle.encode(k, m, data[s].cpu().numpy())).all(), s
        want_rec = oracle.decode(k, m, rv[s].cpu().numpy(), sl)
        assert (rec[s].cpu().numpy() == want_rec).all(), s


# Routine addresses travel in the kernel arguments up to 432 of them (kernels.hip
# kBsrArgAddrs: waves x inputs x rows per wave), past that in the cached
# device-side table (written by bsr_table_write on a matrix's first launch):
# 27/43 (2 waves x 27 inputs x 8 rows = 432) and 28/44 (448) sit on either side;
# 20/60 encodes 40 rows (4 x 20 x 10 = 800), 30/70 1200.
@pytest.mark.parametrize("k,m,want", [(27, 43, "matapply_bsr<8,lds>"), (28, 44, "matapply_bsr<8,lds,tbl>"),
                                      (20, 60, "matapply_bsr<10,lds,tbl>"), (30, 70, "matapply_bsr<10,lds,tbl>")])
def test_bsr_argument_and_table_forms(bsr_only, k, m, want):
    rng = np.random.default_rng(k * 7 + m)
    for sz in (2048, 5000, 9000):
        data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
        ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
        out = zfec_amd.Encoder(k, m).encode(ins)
        torch.cuda.synchronize()
        assert capi.last_kernel_name() == want, (sz, capi.last_kernel_name())
        assert (torch.stack(out[k:]).cpu().numpy() == oracle.encode(k, m, data)).all(), sz


@pytest.mark.parametrize("k,m", [(94, 100), (20, 60), (20, 40)])
def test_bsr_graph_capture(bsr_only, k, m):
    """Encodes captured into a HIP graph and replayed: the table forms (device-
    side tables the host fills at enqueue time) decline under capture
    (kernels.hip stream_capturing) and a kernel described wholly by its
    arguments serves; replays and a later eager launch of the same matrix (whose
    address table must not be a slot whose upload was only recorded) are
    bit-exact."""
    rng = np.random.default_rng(k * 31 + m)
    sz = 9000
    data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
    want = oracle.encode(k, m, data)
    ins = [torch.from_numpy(data[i]).cuda() for i in range(k)]
    enc = zfec_amd.Encoder(k, m)
    enc.encode(ins)  # warm-up outside the capture (first launch of the matrix, probe)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            out = enc.encode(ins)
    torch.cuda.synchronize()
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
        assert (torch.stack(out[k:]).cpu().numpy() == want).all()
    eager = enc.encode(ins)
    torch.cuda.synchronize()
    assert (torch.stack(eager[k:]).cpu().numpy() == want).all()
