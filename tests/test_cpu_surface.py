"""CPU-side checks of the product: the C-ABI library loads and exports every
symbol include/zfec_hip.h declares, the host-side matrix algebra matches the
reference's golden vectors, and the Python surface validates arguments with
the reference's error behaviour (zfec/test/test_zfec.py:85-105,162-258).
No kernel launches here."""
import ctypes
import hashlib
import os
import re
import subprocess

import numpy as np
import pytest

import zfec_amd
from zfec_amd import capi
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "zfec_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", src)))


def test_header_symbols_exported():
    names = header_functions()
    assert "fec_encode" in names and "fec_decode" in names and "fec_encode_batch" in names
    out = subprocess.run(["nm", "-D", "--defined-only", capi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    L = capi.lib()
    for n in names:
        assert getattr(L, n) is not None
    assert set(n for n, _, _ in capi.SYMBOLS) == set(names)


def test_reference_fec_h_surface_subset():
    # every function of zfec/fec.h (and the two non-static helpers of fec.c) is exported
    for n in ["fec_init", "fec_new", "fec_free", "fec_encode", "fec_decode",
              "build_decode_matrix_into_space", "_invert_vdm"]:
        assert n in header_functions()


def test_enc_matrix_matches_reference_every_k(golden):
    meta, _ = golden
    for k in range(1, 257):
        E = capi.Code(k, 256).enc_matrix()
        assert hashlib.sha256(E).hexdigest() == meta["enc_matrix_sha256_m256"][str(k)], k


def test_enc_matrix_python_surface(golden):
    _, arrays = golden
    for key, E in arrays.items():
        if key.startswith("enc_k"):
            k, m = (int(x[1:]) for x in key[4:].split("_"))
            got = np.frombuffer(zfec_amd.Encoder(k, m).enc_matrix(), dtype=np.uint8).reshape(m, k)
            assert (got == E).all(), key


def test_decode_matrix_rows(golden):
    meta, arrays = golden
    L = capi.lib()
    for c in meta["decode_rows"]:
        k, m, slots = c["k"], c["m"], c["slot_nums"]
        code = capi.Code(k, m)
        mat = (ctypes.c_ubyte * (k * k))()
        L.build_decode_matrix_into_space(code.ptr, capi.uint_array(slots), k, ctypes.cast(mat, ctypes.c_void_p))
        assert L.fec_last_status() == capi.FEC_OK
        D = np.frombuffer(bytes(mat), dtype=np.uint8).reshape(k, k)
        rows = D[[i for i in range(k) if slots[i] >= k]]
        assert (rows == arrays[c["key"]]).all()


def test_invert_vdm_matches_oracle():
    L = capi.lib()
    rng = np.random.default_rng(5)
    for k in [1, 2, 3, 7, 20, 64]:
        # a Vandermonde matrix of distinct points p_i (row i = p_i^j)
        pts = rng.choice(np.arange(1, 256), size=k, replace=False).astype(np.uint8)
        V = np.zeros((k, k), dtype=np.uint8)
        for i in range(k):
            acc = 1
            for j in range(k):
                V[i, j] = acc
                acc = oracle.gf_mul(acc, int(pts[i]))
        a = V.copy()
        b = V.copy()
        L._invert_vdm(a.ctypes.data_as(ctypes.c_void_p), k)
        oracle.lib().oracle_invert_vdm(b.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)), k)
        assert (a == b).all(), k


def test_fec_new_validation_no_abort():
    L = capi.lib()
    assert not L.fec_new(0, 3)
    assert L.fec_last_status() == capi.FEC_EINVAL
    assert not L.fec_new(4, 3)
    assert not L.fec_new(1, 257)
    p = L.fec_new(3, 10)
    assert p
    L.fec_free(p)


def test_fec_encode_rejects_bad_block_number():
    L = capi.lib()
    code = capi.Code(3, 10)
    src = [ctypes.create_string_buffer(8) for _ in range(3)]
    dst = [ctypes.create_string_buffer(8)]
    st = L.fec_encode_ex(code.ptr, capi.ptr_array([ctypes.addressof(b) for b in src]),
                         capi.ptr_array([ctypes.addressof(b) for b in dst]), capi.uint_array([10]), 1, 8, None, 0)
    assert st == capi.FEC_EINVAL


def test_fec_decode_rejects_duplicates_and_misplaced_primaries():
    L = capi.lib()
    code = capi.Code(3, 10)
    bufs = [ctypes.create_string_buffer(8) for _ in range(3)]
    addrs = capi.ptr_array([ctypes.addressof(b) for b in bufs])
    for idx in ([3, 3, 4], [1, 0, 5], [3, 4, 10]):
        st = L.fec_decode_ex(code.ptr, addrs, addrs, capi.uint_array(idx), 8, None, 0)
        assert st == capi.FEC_EINVAL, idx


# ---- reference test_zfec.py argument tests, on our surface ------------------

def test_instantiate_no_args():
    with pytest.raises(TypeError):
        zfec_amd.Encoder()
    with pytest.raises(TypeError):
        zfec_amd.Decoder()


@pytest.mark.parametrize("cls", [zfec_amd.Encoder, zfec_amd.Decoder])
def test_bad_args_construct(cls):
    with pytest.raises(zfec_amd.Error, match="argument is required to be greater than or equal to 1"):
        cls(-1, -1)
    with pytest.raises(zfec_amd.Error, match="argument is required to be less than or equal to 256"):
        cls(1, 257)
    with pytest.raises(zfec_amd.Error, match="first argument is required to be less than or equal to the second argument"):
        cls(3, 2)


def test_bad_args_dec():
    decer = zfec_amd.Decoder(2, 4)
    with pytest.raises(TypeError, match="First argument was not a sequence"):
        decer.decode(98, [])
    with pytest.raises(zfec_amd.Error, match="Precondition violation: second argument is required to contain int"):
        decer.decode(["a", "b"], ["c", "d"])
    with pytest.raises(TypeError, match="Second argument was not a sequence"):
        decer.decode(["a", "b"], 98)


def test_bad_args_easyfec_dec():
    decer = zfec_amd.easyfec.Decoder(2, 4)
    with pytest.raises(TypeError, match="First argument was not a sequence"):
        decer.decode(98, [0, 1], 0)
    with pytest.raises(zfec_amd.Error, match="Precondition violation: second argument is required to contain int"):
        decer.decode("ab", ["c", "d"], 0)
    with pytest.raises(TypeError, match="Second argument was not a sequence"):
        decer.decode("ab", 98, 0)


def test_decode_rejects_what_reference_mishandles():
    d = zfec_amd.Decoder(3, 5)
    b = [b"x" * 4] * 3
    with pytest.raises(zfec_amd.Error, match="greater than 255"):
        d.decode(b, [0, 1, 256])
    with pytest.raises(zfec_amd.Error, match="less than m"):
        d.decode(b, [0, 1, 7])          # reference reads enc_matrix out of bounds
    with pytest.raises(zfec_amd.Error, match="distinct"):
        d.decode(b, [1, 1, 2])          # reference spins forever (_fecmodule.c:482-493)
    e = zfec_amd.Encoder(3, 5)
    with pytest.raises(zfec_amd.Error):
        e.encode(b, [5])                # reference reads out of bounds
    with pytest.raises(zfec_amd.Error, match="exactly k blocks"):
        e.encode(b[:2])
    with pytest.raises(zfec_amd.Error, match="same length"):
        e.encode([b"a", b"bb", b"c"])


def test_jit_prepare_compiles_without_gpu(tmp_path, monkeypatch):
    """fec_jit_prepare_encode / _decode generate and compile (hipRTC, gfx950)
    the bit-sliced kernels a K=11/M=17 encode and a decode from blocks 6..16
    would launch, and cache the code objects; no GPU involved.  (A code no
    other test compiles: the registry is per process, and fec_new's
    prefetch loads the kernels of codes the in-tree cache holds.)"""
    monkeypatch.setenv("ZFEC_HIP_JIT_CACHE", str(tmp_path))
    code = capi.Code(11, 17)
    code.jit_prepare_encode(list(range(11, 17)))
    code.jit_prepare_decode([11, 12, 13, 14, 15, 16, 6, 7, 8, 9, 10])
    files = sorted(tmp_path.glob("zfec_hip_bitslice_k11_r*.co"))
    assert len(files) == 2, files
    for f in files:
        assert f.read_bytes()[:4] == b"\x7fELF"
    code.jit_prepare_encode(list(range(11, 17)))  # in-memory hit: nothing new
    assert len(list(tmp_path.glob("*.co"))) == 2
    with pytest.raises(capi.FecError):
        code.jit_prepare_decode([0, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9])  # duplicate: rejected before compiling


@pytest.mark.skipif(zfec_amd.device_count() > 0, reason="only meaningful without a GPU")
def test_no_gpu_fails_loudly():
    with pytest.raises(zfec_amd.Error, match="no GPU"):
        zfec_amd.Encoder(3, 10).encode([b"abc", b"def", b"ghi"])
    with pytest.raises(zfec_amd.Error, match="no GPU"):
        zfec_amd.Decoder(3, 10).decode([b"abc", b"def", b"ghi"], [3, 4, 5])
    with pytest.raises(zfec_amd.Error, match="no GPU"):
        zfec_amd.test_from_agl()


def test_jit_prepare_concurrent_threads(tmp_path, monkeypatch):
    """Several threads asking for the same and for different kernels at once
    (ctypes releases the GIL): one compile per matrix, every call succeeds."""
    import threading

    monkeypatch.setenv("ZFEC_HIP_JIT_CACHE", str(tmp_path))
    codes = {km: capi.Code(*km) for km in [(5, 9), (6, 11)]}
    errors = []

    def work(km):
        try:
            k, m = km
            codes[km].jit_prepare_encode(list(range(k, m)))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    ths = [threading.Thread(target=work, args=(km,)) for km in [(5, 9), (6, 11)] * 4]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors
    assert len(list(tmp_path.glob("zfec_hip_bitslice_k5_r4_*.co"))) == 1
    assert len(list(tmp_path.glob("zfec_hip_bitslice_k6_r5_*.co"))) == 1


def test_tensor_batch_api_preconditions():
    """The batched tensor entry points reject host tensors and wrong shapes
    before any GPU work (no GPU needed)."""
    import torch
    import zfec_amd

    enc = zfec_amd.Encoder(3, 10)
    with pytest.raises(zfec_amd.Error):
        enc.encode_batch(torch.zeros((4, 3, 16), dtype=torch.uint8))  # host tensor
    with pytest.raises(zfec_amd.Error):
        enc.encode_batch(torch.zeros((4, 3, 16), dtype=torch.uint8), [1])  # primary requested
    with pytest.raises(zfec_amd.Error):
        zfec_amd.Decoder(3, 10).decode_batch(torch.zeros((4, 3, 16), dtype=torch.uint8), [1, 0, 5])
    with pytest.raises(TypeError):
        zfec_amd.Decoder(3, 10).decode_batch(torch.zeros((4, 3, 16), dtype=torch.uint8), 5)


@pytest.mark.skipif(zfec_amd.device_count() > 0, reason="only meaningful without a GPU")
def test_batch_library_errors_are_zfec_errors():
    """Library failures inside the batched tensor entry points (here: no GPU)
    surface as zfec_amd.Error, not as the ctypes layer's FecError."""
    enc = zfec_amd.Encoder(3, 10)
    with pytest.raises(zfec_amd.Error, match="no GPU"):
        with zfec_amd._as_error():
            zfec_amd._capi_code(enc).encode_batch(0x1000, 16, 48, 0x2000, 16, 112, list(range(3, 10)), 16, 4)
    with pytest.raises(zfec_amd.Error, match="no GPU"):
        with zfec_amd._as_error():
            zfec_amd._capi_code(zfec_amd.Decoder(3, 10)).decode_batch(0x1000, 16, 48, 0x2000, 16, 48, [3, 4, 5],
                                                                     16, 4)


@pytest.mark.skipif(zfec_amd.device_count() > 0, reason="bogus addresses: only without a GPU")
def test_batch_call_matches_ctypes_binding():
    """capi's batched calls go through zfec_amd._fec.batch_call (the C-ABI
    called from C); the ctypes binding of the same functions must report the
    same statuses and messages for the same arguments (host-side validation:
    no GPU needed)."""
    from zfec_amd import _fec

    capi.lib()
    assert capi._batch_call is _fec.batch_call
    code = capi.Code(3, 10)
    L = capi.lib()
    cases = [
        # (kind, src, sbs, sss, dst, dbs, dss, nums, sz, ns)
        (0, 0x1000, 16, 48, 0x2000, 16, 112, [3, 10], 16, 1),  # block number out of range
        (1, 0x1000, 16, 48, 0x2000, 16, 48, [3, 3, 4], 16, 1),  # duplicate
        (1, 0x1000, 16, 48, 0x2000, 16, 48, [1, 0, 5], 16, 1),  # misplaced primary
        (1, 0x1000, 16, 48, 0x2000, 16, 48, [3, 4], 16, 1),  # too few slot numbers
        (0, 0, 16, 48, 0x2000, 16, 112, [3, 4], 16, 1),  # NULL source
    ]
    for kind, src, sbs, sss, dst, dbs, dss, nums, sz, ns in cases:
        st_fast = _fec.batch_call(kind, code.ptr, src, sbs, sss, dst, dbs, dss, nums, sz, ns, 0, capi.FEC_FLAG_ASYNC)
        msg_fast = L.fec_last_error_message()
        arr = capi.uint_array(list(nums) + [0xFFFFFFFF] * (3 - len(nums)) if kind else nums)
        if kind == 0:
            st_ct = L.fec_encode_batch(code.ptr, src, sbs, sss, dst, dbs, dss, arr, len(nums), sz, ns, None,
                                       capi.FEC_FLAG_ASYNC)
        else:
            st_ct = L.fec_decode_batch(code.ptr, src, sbs, sss, dst, dbs, dss, arr, sz, ns, None,
                                       capi.FEC_FLAG_ASYNC)
        assert (st_fast, msg_fast) == (st_ct, L.fec_last_error_message()), (kind, nums)
        assert st_fast != capi.FEC_OK
    with pytest.raises(TypeError):
        _fec.batch_call(0, code.ptr)
    with pytest.raises(zfec_amd.Error, match="at most 256"):
        _fec.batch_call(0, code.ptr, 1, 1, 1, 1, 1, 1, list(range(257)), 1, 1, 0, 0)
    with pytest.raises(OverflowError):
        _fec.batch_call(0, code.ptr, -1, 1, 1, 1, 1, 1, [3], 1, 1, 0, 0)
    with pytest.raises(TypeError):
        _fec.batch_call(0, code.ptr, 1, 1, 1, 1, 1, 1, 3, 1, 1, 0, 0)
    with pytest.raises(ValueError, match="kind"):
        _fec.batch_call(2, code.ptr, 1, 1, 1, 1, 1, 1, [3], 1, 1, 0, 0)


def test_batch_jobs_validation():
    """fec_run_batch_jobs checks every job before anything runs; a failing
    job's message names it (host logic: no GPU needed)."""
    code = capi.Code(3, 10)
    good = capi.encode_job(code, 0x1000, 16, 48, 0x2000, 16, 112, list(range(3, 10)), 16, 1)
    with pytest.raises(capi.FecError, match="job 1: block number 10 out of range"):
        capi.run_batch_jobs([good, capi.encode_job(code, 0x1000, 16, 48, 0x2000, 16, 32, [3, 10], 16, 1)])
    with pytest.raises(capi.FecError, match="job 0: kind 7"):
        capi.run_batch_jobs([(code, 7) + good[2:]])
    with pytest.raises(capi.FecError, match="job 0: block_nums is NULL"):
        arr = (capi.BatchJob * 1)(capi.BatchJob(code.ptr, capi.FEC_JOB_ENCODE, 0, 0x1000, 16, 48, 0x2000, 16, 112,
                                                None, 7, 16, 1))
        capi.check(capi.lib().fec_run_batch_jobs(arr, 1, None, 0))
    assert capi.lib().fec_run_batch_jobs(None, 1, None, 0) == capi.FEC_EINVAL


@pytest.mark.skipif(zfec_amd.device_count() > 0, reason="only meaningful without a GPU")
def test_batch_jobs_no_gpu_fails_loudly():
    code = capi.Code(3, 10)
    with pytest.raises(capi.FecError, match="no GPU"):
        capi.run_batch_jobs([capi.encode_job(code, 0x1000, 16, 48, 0x2000, 16, 112, list(range(3, 10)), 16, 1)])


_DROPIN_CHILD = r"""
import glob, importlib.util, sys
spec = importlib.util.spec_from_file_location("zfec_dropin._fec", sys.argv[1])
mod = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mod)
for _ in range(2):
    out = mod.Encoder(3, 10).encode([b"abc", b"def", b"ghi"])
    assert len(out) == 10
    dec = mod.Decoder(3, 10).decode([b"abc", b"def", b"ghi"], [3, 4, 5])
print("returned")
"""


@pytest.mark.skipif(zfec_amd.device_count() > 0, reason="only meaningful without a GPU")
@pytest.mark.parametrize("quiet", [False, True])
def test_void_entry_points_report_failures(quiet):
    """fec_encode / fec_decode return void (zfec/fec.h:49,57) and the
    reference's own binding never asks for a status: with no GPU, the
    reference's unmodified _fecmodule.c linked to libzfec_hip.so must see a
    diagnostic on stderr, once per entry point (ZFEC_HIP_QUIET=1 silences it)."""
    import glob
    import sys

    paths = glob.glob(os.path.join(ROOT, "oracle", "_ref", "dropin", "_fec*.so"))
    if not paths:
        pytest.skip("oracle/_ref/dropin not built (needs /root/reference at build time)")
    env = dict(os.environ)
    env.pop("ZFEC_HIP_QUIET", None)
    if quiet:
        env["ZFEC_HIP_QUIET"] = "1"
    res = subprocess.run([sys.executable, "-c", _DROPIN_CHILD, paths[0]], env=env, capture_output=True, text=True,
                         timeout=120)
    assert res.returncode == 0, res.stderr[-2000:]
    assert "returned" in res.stdout
    enc = [ln for ln in res.stderr.splitlines() if "zfec_hip: fec_encode failed" in ln]
    dec = [ln for ln in res.stderr.splitlines() if "zfec_hip: fec_decode failed" in ln]
    if quiet:
        assert not enc and not dec, res.stderr
    else:
        assert len(enc) == 1 and len(dec) == 1, res.stderr
        assert "status 2" in enc[0] and "no GPU" in enc[0]


def test_reuse_host_memory_opt_in():
    """zfec_amd.reuse_host_memory sets glibc's mmap / trim thresholds (process-wide,
    opt-in): accepted values return True, and the library keeps
    working with it (host logic only here, no GPU)."""
    assert zfec_amd.reuse_host_memory() is True
    assert zfec_amd.reuse_host_memory(keep_bytes=64 << 20, mmap_threshold=1 << 20) is True
    assert "reuse_host_memory" in zfec_amd.__all__


_MALLOPT_CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
from zfec_amd import _fec
blocks = [bytes(2 << 20)] * 3
for _ in range(2):
    try:
        _fec.Encoder(3, 10).encode(blocks)
    except _fec.Error:
        pass  # no GPU here: the call fails after the allocator hook ran
print("mallopt_calls=%d" % _fec._mallopt_calls())
"""


@pytest.mark.parametrize("policy", [None, "default", "reuse"])
def test_bytes_calls_leave_allocator_policy_alone(policy):
    """A 2 MiB-block `bytes` encode changes glibc's allocator policy only when
    the caller opts in with ZFEC_AMD_MALLOC=reuse (the reference module never
    calls mallopt, zfec/_fecmodule.c:206-217); by default nothing is set."""
    import sys

    env = dict(os.environ)
    env.pop("ZFEC_AMD_MALLOC", None)
    if policy:
        env["ZFEC_AMD_MALLOC"] = policy
    res = subprocess.run([sys.executable, "-c", _MALLOPT_CHILD, ROOT], env=env, capture_output=True, text=True,
                         timeout=120)
    assert res.returncode == 0, res.stderr[-2000:]
    want = 2 if policy == "reuse" else 0
    assert ("mallopt_calls=%d" % want) in res.stdout, res.stdout + res.stderr[-2000:]


def test_package_exports_like_reference():
    """`import zfec` makes Encoder, Decoder, Error, __version__ and the modules
    easyfec, filefec, cmdline_zfec, cmdline_zunfec available
    (/root/reference/zfec/__init__.py); so does `import zfec_amd`."""
    for name in ["Encoder", "Decoder", "Error", "__version__", "easyfec", "filefec", "cmdline_zfec",
                 "cmdline_zunfec"]:
        assert hasattr(zfec_amd, name), name
    assert issubclass(zfec_amd.filefec.CorruptedShareFilesError, zfec_amd.Error)
