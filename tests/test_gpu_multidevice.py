"""GPU parity of the single-process multi-GPU batch entry points
(fec_encode_batch_multi / fec_decode_batch_multi, Encoder.encode_batch(...,
devices=...)): a batch's stripes are split into contiguous balanced ranges,
one per listed device, each run by the library's persistent thread for that
device (stripes are independent, zfec/fec.c:494-503).  On the
one-GPU box the device list repeats device 0, so several library threads share
the GPU, each with its own stream and staging slots -- the same code path as
one thread per GPU on an 8-GPU node.  Every stripe is checked against the CPU
oracle (sampled for the larger batches)."""
import ctypes
import threading

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


def place(nums, k):
    slots = [None] * k
    sec = iter([n for n in nums if n >= k])
    for n in nums:
        if n < k:
            slots[n] = n
    return [s if s is not None else next(sec) for s in slots]


def _check_stripes(k, m, data, par, stripes):
    for s in stripes:
        assert (par[s] == oracle.encode(k, m, data[s])).all(), s


@pytest.mark.parametrize("k,m,sz,ns,devices", [(3, 10, 4096, 1000, [0, 0]), (3, 10, 1366, 999, [0, 0, 0]),
                                               (20, 60, 52429, 64, [0, 0]), (10, 16, 70001, 5, [0, 0, 0, 0, 0, 0, 0]),
                                               (4, 9, 3000, 2, [0, 0, 0]), (94, 100, 8192, 6, [0, 0])])
def test_multi_device_host_batch_vs_oracle(k, m, sz, ns, devices):
    rng = np.random.default_rng(k * 7 + ns)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    enc = zfec_amd.Encoder(k, m)
    par = enc.encode_batch(data, devices=devices)
    assert isinstance(par, np.ndarray) and par.shape == (ns, m - k, sz)
    pick = sorted(set([0, ns - 1] + [int(x) for x in rng.integers(0, ns, 8)]))
    _check_stripes(k, m, data, par, pick)
    # the same batch on one device, one call: identical bytes
    assert np.array_equal(par, enc.encode_batch(data))
    # decode from the last k blocks (secondaries at their slots) over the devices
    slots = place(list(range(m - k, m)), k)
    allb = np.concatenate([data, par], axis=1)
    rec = zfec_amd.Decoder(k, m).decode_batch(np.ascontiguousarray(allb[:, slots]), slots, devices=devices)
    missing = [i for i in range(k) if slots[i] >= k]
    assert np.array_equal(rec, data[:, missing])


def test_multi_device_block_major_and_pinned():
    """A block-major host batch ([k, nstripes, sz] transposed) split over the
    devices, and a page-locked (fec_host_alloc) input read in place by each
    device's kernels."""
    k, m, sz, ns = 3, 10, 5000, 301
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
    bm = np.ascontiguousarray(data.transpose(1, 0, 2)).transpose(1, 0, 2)  # block-major storage
    enc = zfec_amd.Encoder(k, m)
    par = enc.encode_batch(bm, devices=[0, 0])
    _check_stripes(k, m, data, par, [0, 150, 300])
    L = capi.lib()
    nbytes = data.nbytes
    p = L.fec_host_alloc(nbytes)
    assert p
    try:
        pinned = np.frombuffer((ctypes.c_uint8 * nbytes).from_address(p), dtype=np.uint8).reshape(ns, k, sz)
        pinned[:] = data
        par2 = enc.encode_batch(pinned, devices=[0, 0, 0])
        assert np.array_equal(par2, par)
    finally:
        L.fec_host_free(p)


def test_multi_device_concurrent_callers():
    """Two Python threads (the GIL is released in the call) each split their
    own batch over the devices at once."""
    k, m, sz, ns = 3, 10, 65536, 40
    rng = np.random.default_rng(11)
    inputs = [rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8) for _ in range(2)]
    errors = []

    def work(i):
        try:
            for _ in range(3):
                par = zfec_amd.Encoder(k, m).encode_batch(inputs[i], devices=[0, 0])
                _check_stripes(k, m, inputs[i], par, [0, ns // 2, ns - 1])
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    ths = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=100)
    assert not errors, errors


def test_multi_device_rejects():
    k, m = 3, 10
    enc = zfec_amd.Encoder(k, m)
    t = torch.zeros((4, k, 100), dtype=torch.uint8, device="cuda")
    with pytest.raises(zfec_amd.Error, match="own device"):
        enc.encode_batch(t, devices=[0, 0])
    assert enc.encode_batch(t, devices=[0]).shape == (4, m - k, 100)  # its own device: a plain call
    host = np.zeros((4, k, 100), dtype=np.uint8)
    with pytest.raises(zfec_amd.Error, match="out of range"):
        enc.encode_batch(host, devices=[0, zfec_amd.device_count()])
    code = capi.Code(k, m)
    with pytest.raises(capi.FecError, match="host memory"):
        code.encode_batch_multi(t.data_ptr(), 100, k * 100, t.data_ptr(), 100, k * 100, [3, 4, 5], 100, 4, [0])
    # a list of device tensors: each encoded on its own device, a list of results
    outs = enc.encode_batch([t, t[:2]])
    assert [o.shape for o in outs] == [(4, m - k, 100), (2, m - k, 100)]
