"""fec_run_batch_jobs (include/zfec_hip.h): several batched encode / decode
calls in one, two register-shaped jobs sharing ONE launch (matapply_pair),
against the CPU oracle (zfec/fec.c:487-505 encode, :527-557 decode).  Every
job's bytes [0, sz) are bit-exact; with FEC_FLAG_ROW_PADDING the bytes past
the 128-byte line a row ends in stay untouched; jobs the paired kernel does
not take (host memory, short-row batches, other k, wide codes) run one at a
time with the same results."""
import numpy as np
import pytest

import zfec_amd
from zfec_amd import capi
from oracle import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

GUARD = 0xA5


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if zfec_amd.device_count() < 1:
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")


def place(nums, k):
    slots = [None] * k
    sec = iter([n for n in nums if n >= k])
    for n in nums:
        if n < k:
            slots[n] = n
    return [s if s is not None else next(sec) for s in slots]


class EncJob(object):
    """An encode job over device buffers [stripe][block][ld], the output
    pre-filled with GUARD bytes."""

    def __init__(self, code, k, m, nums, sz, ns, ld, rng, flags=0):
        self.k, self.m, self.nums, self.sz, self.ns, self.ld = k, m, list(nums), sz, ns, ld
        self.data = rng.integers(0, 256, size=(ns, k, ld), dtype=np.uint8)
        self.src = torch.from_numpy(self.data).cuda()
        self.dst = torch.full((ns, len(nums), ld), GUARD, dtype=torch.uint8, device="cuda")
        self.job = capi.encode_job(code, self.src.data_ptr(), ld, k * ld, self.dst.data_ptr(), ld, len(nums) * ld,
                                   self.nums, sz, ns, flags)

    def check(self, padded_end):
        out = self.dst.cpu().numpy()
        for s in range(self.ns):
            want = oracle.encode(self.k, self.m, self.data[s, :, :self.sz], self.nums)
            assert (out[s, :, :self.sz] == want).all(), ("encode", s)
        assert (out[:, :, padded_end:] == GUARD).all(), "encode wrote past its grant"


class DecJob(object):
    """A decode job: received blocks (slot order) computed by the oracle."""

    def __init__(self, code, k, m, recv_nums, sz, ns, ld, rng, flags=0):
        self.k, self.m, self.sz, self.ns, self.ld = k, m, sz, ns, ld
        self.slots = place(sorted(recv_nums), k)
        self.missing = [i for i in range(k) if self.slots[i] >= k]
        self.data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
        recv = np.zeros((ns, k, ld), dtype=np.uint8)
        for s in range(ns):
            allb = np.concatenate([self.data[s], oracle.encode(k, m, self.data[s])])
            recv[s, :, :sz] = allb[self.slots]
        self.src = torch.from_numpy(recv).cuda()
        nrec = len(self.missing)
        self.dst = torch.full((ns, max(1, nrec), ld), GUARD, dtype=torch.uint8, device="cuda")
        self.job = capi.decode_job(code, self.src.data_ptr(), ld, k * ld, self.dst.data_ptr(), ld, nrec * ld,
                                   self.slots, sz, ns, flags)

    def check(self, padded_end):
        out = self.dst.cpu().numpy()
        nrec = len(self.missing)
        assert (out[:, :nrec, :self.sz] == self.data[:, self.missing, :]).all(), "decode"
        assert (out[:, :, padded_end:] == GUARD).all(), "decode wrote past its grant"


def run(jobs, flags=capi.FEC_FLAG_ASYNC):
    st = torch.cuda.current_stream().cuda_stream
    capi.run_batch_jobs([j.job for j in jobs], stream=st, flags=flags)
    torch.cuda.synchronize()
    return capi.last_kernel_name()


# (k, m, encode block numbers, decode received numbers, sz, stripes)
PAIRS = [
    (3, 10, range(3, 10), range(7, 10), 100003, 1),   # the bench's cfg2 pair, smaller
    (3, 10, [9, 4, 6], [0, 5, 8], 70001, 3),          # decode of one missing primary, unordered numbers
    (1, 3, [1, 2], [2], 5000, 3),
    (2, 4, [2, 3], [1, 3], 4097, 2),
    (4, 12, range(4, 12), range(8, 12), 8191, 5),
    (4, 5, [4], [0, 1, 2, 4], 7000, 1),
    (2, 10, range(2, 10), [5, 9], 65536, 4),
]


@pytest.mark.parametrize("k,m,enc_nums,recv,sz,ns", PAIRS)
def test_pair_one_launch_vs_oracle(k, m, enc_nums, recv, sz, ns):
    code = capi.Code(k, m)
    rng = np.random.default_rng(sz * 7 + ns)
    ld = (sz + 255) // 256 * 256
    e = EncJob(code, k, m, enc_nums, sz, ns, ld, rng)
    d = DecJob(code, k, m, recv, sz, ns, ld, rng)
    name = run([e, d])
    nrec = len(d.missing)
    ra, rb = max(len(e.nums), nrec), min(len(e.nums), nrec)
    assert name == "matapply_pair<%d,%d,%d>" % (k, ra, rb), name
    e.check(sz)
    d.check(sz)
    # the other order of the two jobs: the same launch
    e2 = EncJob(code, k, m, enc_nums, sz, ns, ld, rng)
    d2 = DecJob(code, k, m, recv, sz, ns, ld, rng)
    assert run([d2, e2], flags=0) == name
    e2.check(sz)
    d2.check(sz)


@pytest.mark.parametrize("sz,ns", [(22369622, 1), (100003, 3), (4097, 9)])
def test_pair_row_padding(sz, ns):
    """FEC_FLAG_ROW_PADDING per job: rows run out to the next 128-byte line,
    nothing past it is written (the bench's cfg2 call shape at full size)."""
    k, m = 3, 10
    code = capi.Code(k, m)
    rng = np.random.default_rng(sz)
    ld = (sz + 255) // 256 * 256
    fl = capi.FEC_FLAG_ROW_PADDING
    e = EncJob(code, k, m, range(k, m), sz, ns, ld, rng, flags=fl)
    d = DecJob(code, k, m, range(m - k, m), sz, ns, ld, rng, flags=fl)
    assert run([e, d]) == "matapply_pair<3,7,3>"
    padded = (sz + 127) // 128 * 128
    e.check(padded)
    d.check(padded)


def test_jobs_fallbacks_vs_oracle():
    """Jobs the paired kernel does not take run one at a time, correctly:
    short-row batches (matapply_rows), another k, a wide code, host memory,
    an odd job out."""
    rng = np.random.default_rng(11)
    c3, c4, c20 = capi.Code(3, 10), capi.Code(4, 8), capi.Code(20, 60)
    rows = EncJob(c3, 3, 10, range(3, 10), 1366, 100, 1536, rng)        # matapply_rows shape
    dec3 = DecJob(c3, 3, 10, range(7, 10), 9000, 2, 9216, rng)
    enc4 = EncJob(c4, 4, 8, range(4, 8), 9000, 2, 9216, rng)              # k differs from dec3
    wide = EncJob(c20, 20, 60, range(20, 60), 52429, 2, 52480, rng)
    lone = DecJob(c4, 4, 8, [0, 5, 6, 7], 3333, 3, 3584, rng)
    run([rows, dec3, enc4, wide, lone])
    for j in (rows, dec3, enc4, wide, lone):
        j.check(j.sz)
    # host memory (pageable numpy) next to a device job
    k, m, sz, ns = 3, 10, 50000, 2
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    out = np.zeros((ns, m - k, sz), dtype=np.uint8)
    host = capi.encode_job(c3, data.ctypes.data, sz, k * sz, out.ctypes.data, sz, (m - k) * sz, list(range(k, m)),
                           sz, ns)
    dev = DecJob(c3, 3, 10, range(7, 10), sz, ns, sz, rng)
    st = torch.cuda.current_stream().cuda_stream
    capi.run_batch_jobs([host, dev.job], stream=st, flags=0)
    torch.cuda.synchronize()
    for s in range(ns):
        assert (out[s] == oracle.encode(k, m, data[s])).all(), s
    dev.check(sz)


def test_jobs_prepared_reuse_and_library_stream():
    """A BatchJobs built once and run repeatedly (the bench's form), on the
    caller's stream and on the library's stream (FEC_FLAG_LIBRARY_STREAM)."""
    k, m, sz = 3, 10, 300007
    code = capi.Code(k, m)
    rng = np.random.default_rng(5)
    e = EncJob(code, k, m, range(k, m), sz, 1, sz + 1, rng)
    d = DecJob(code, k, m, [1, 8, 9], sz, 1, sz + 1, rng)
    jobs = capi.BatchJobs([e.job, d.job])
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        jobs.run(stream=st)
    torch.cuda.synchronize()
    e.check(sz)
    d.check(sz)
    jobs.run(flags=capi.FEC_FLAG_LIBRARY_STREAM)
    e.check(sz)
    d.check(sz)


def test_jobs_errors():
    code = capi.Code(3, 10)
    x = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    good = capi.encode_job(code, x.data_ptr(), 16, 48, x.data_ptr() + 1024, 16, 112, list(range(3, 10)), 16, 1)
    bad_num = capi.encode_job(code, x.data_ptr(), 16, 48, x.data_ptr() + 1024, 16, 112, [3, 10], 16, 1)
    with pytest.raises(capi.FecError, match="job 1: block number 10 out of range"):
        capi.run_batch_jobs([good, bad_num])
    bad_kind = (code, 7) + good[2:]
    with pytest.raises(capi.FecError, match="job 0: kind 7"):
        capi.run_batch_jobs([bad_kind])
    dup = capi.decode_job(code, x.data_ptr(), 16, 48, x.data_ptr() + 1024, 16, 48, [7, 7, 9], 16, 1)
    with pytest.raises(capi.FecError, match="job 1: duplicate block number 7"):
        capi.run_batch_jobs([good, dup])
    capi.run_batch_jobs([])
