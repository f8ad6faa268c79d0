"""ctypes binding of the C-ABI (include/zfec_hip.h) of libzfec_hip.so.

This is the binding a ctypes/FFI user of zfec's fec.h would write (see
INTEGRATION.md); tests use it to exercise the C entry points directly and
bench.py uses the batched, stream-ordered extensions with device buffers.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# ZFEC_HIP_LIB: another build of the library (make asan-py: the host code built
# with AddressSanitizer); the default is the in-tree build next to this file
LIB_PATH = os.environ.get("ZFEC_HIP_LIB") or os.path.join(_HERE, "libzfec_hip.so")

FEC_OK, FEC_EINVAL, FEC_ENODEV, FEC_EHIP, FEC_ENOMEM, FEC_ESINGULAR, FEC_EUNINIT = range(7)
FEC_FLAG_ASYNC = 1
FEC_FLAG_LIBRARY_STREAM = 2
FEC_FLAG_ALL_PRIMARIES = 4
FEC_FLAG_HOST_MEMORY = 8
FEC_FLAG_ROW_PADDING = 16
FEC_FLAG_NO_POPULATE = 32

# (name, restype, argtypes) for every symbol declared in include/zfec_hip.h
_P = ctypes.c_void_p
_SZ = ctypes.c_size_t
_U = ctypes.c_uint
_UP = ctypes.POINTER(ctypes.c_uint)
_PP = ctypes.POINTER(ctypes.c_void_p)
_IP = ctypes.POINTER(ctypes.c_int)
SYMBOLS = [
    ("fec_init", None, []),
    ("fec_new", _P, [ctypes.c_ushort, ctypes.c_ushort]),
    ("fec_free", None, [_P]),
    ("fec_encode", None, [_P, _PP, _PP, _UP, _SZ, _SZ]),
    ("fec_decode", None, [_P, _PP, _PP, _UP, _SZ]),
    ("build_decode_matrix_into_space", None, [_P, _UP, _U, _P]),
    ("_invert_vdm", None, [_P, _U]),
    ("fec_last_status", ctypes.c_int, []),
    ("fec_last_error_message", ctypes.c_char_p, []),
    ("fec_encode_ex", ctypes.c_int, [_P, _PP, _PP, _UP, _SZ, _SZ, _P, _U]),
    ("fec_decode_ex", ctypes.c_int, [_P, _PP, _PP, _UP, _SZ, _P, _U]),
    ("fec_encode_batch", ctypes.c_int, [_P, _P, _SZ, _SZ, _P, _SZ, _SZ, _UP, _SZ, _SZ, _SZ, _P, _U]),
    ("fec_decode_batch", ctypes.c_int, [_P, _P, _SZ, _SZ, _P, _SZ, _SZ, _UP, _SZ, _SZ, _P, _U]),
    ("fec_host_alloc", _P, [_SZ]),
    ("fec_host_free", None, [_P]),
    ("fec_device_count", ctypes.c_int, []),
    ("fec_version", ctypes.c_char_p, []),
    ("fec_kernel_name", ctypes.c_char_p, [_U, _U]),
    ("fec_last_kernel_name", ctypes.c_char_p, []),
    ("fec_jit_mode", ctypes.c_int, [ctypes.c_int]),
    ("fec_jit_wait", ctypes.c_int, []),
    ("fec_generic_mode", ctypes.c_int, [ctypes.c_int]),
    ("fec_jit_prepare_encode", ctypes.c_int, [_P, _UP, _SZ]),
    ("fec_jit_prepare_decode", ctypes.c_int, [_P, _UP, _U]),
    ("fec_encode_batch_multi", ctypes.c_int, [_P, _P, _SZ, _SZ, _P, _SZ, _SZ, _UP, _SZ, _SZ, _SZ, _IP, _SZ, _U]),
    ("fec_decode_batch_multi", ctypes.c_int, [_P, _P, _SZ, _SZ, _P, _SZ, _SZ, _UP, _SZ, _SZ, _IP, _SZ, _U]),
    ("fec_reload_config", ctypes.c_int, []),
    ("fec_last_wait", ctypes.c_int, []),
    ("fec_run_batch_jobs", ctypes.c_int, [_P, _SZ, _P, _U]),
]

JIT_OFF, JIT_AUTO, JIT_FORCE = 0, 1, 2
FEC_JOB_ENCODE, FEC_JOB_DECODE = 0, 1


class FecT(ctypes.Structure):
    """Layout of fec_t (zfec/fec.h:11-15 prefix + priv)."""

    _fields_ = [("magic", ctypes.c_ulong), ("k", ctypes.c_ushort), ("n", ctypes.c_ushort),
                ("enc_matrix", ctypes.POINTER(ctypes.c_ubyte)), ("priv", ctypes.c_void_p)]


_lib = None
# zfec_amd._fec.batch_call: the batched entry points called from C (the ctypes
# conversion of their thirteen arguments is ~2 us of host cost per call).  Only
# with the in-tree library, which the extension links: with ZFEC_HIP_LIB set
# (another build) every call stays on that library through ctypes.
_batch_call = None


def lib():
    global _lib, _batch_call
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libzfec_hip.so is not built (run `make` or __graft_entry__.build())")
        from . import _runtime

        _runtime.preload()
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SYMBOLS:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        L.fec_init()
        _lib = L
        if not os.environ.get("ZFEC_HIP_LIB") and not os.environ.get("ZFEC_CAPI_CTYPES"):
            try:
                from . import _fec
            except ImportError:
                _fec = None
            _batch_call = getattr(_fec, "batch_call", None)
    return _lib


class FecError(RuntimeError):
    pass


def check(status):
    if status != FEC_OK:
        raise FecError("zfec-hip status %d: %s" % (status, lib().fec_last_error_message().decode()))


def variant_name(k, r):
    """Kernel variant used for k inputs and r outputs (fec_kernel_name)."""
    return lib().fec_kernel_name(k, r).decode()


def last_kernel_name():
    """Kernel the calling thread launched last (fec_last_kernel_name)."""
    return lib().fec_last_kernel_name().decode()


def jit_mode(mode=-1):
    """Set the bit-sliced JIT mode (JIT_OFF / JIT_AUTO / JIT_FORCE); returns the previous one."""
    return lib().fec_jit_mode(mode)


def generic_mode(mode=-1):
    """Run-time-data bit-sliced kernels for wide-code launches no JIT kernel
    serves: 2 = matapply_bsr where it fits, else matapply_bsg (default);
    1 = matapply_bsg only; 0 = off (table kernels).  Returns the previous mode."""
    return lib().fec_generic_mode(mode)


def jit_wait():
    """Wait for background JIT compiles; number of compiled kernels."""
    return lib().fec_jit_wait()


def reload_config():
    """Re-read the ZFEC_HIP_* environment knobs (read once per process
    otherwise; tests and A/B runs)."""
    check(lib().fec_reload_config())


def last_wait():
    """1 if the calling thread's last synchronous small-object call waited on
    the completion word its kernel wrote, 0 if on hipStreamSynchronize."""
    return lib().fec_last_wait()


def ptr_array(addrs):
    return (ctypes.c_void_p * max(1, len(addrs)))(*addrs)


def uint_array(vals):
    return (ctypes.c_uint * max(1, len(vals)))(*vals)


_UINT_CACHE = {}


def _nums(vals):
    """uint_array(vals), cached per tuple of values: a batched call's block
    numbers are usually the same every call (the ctypes array construction
    is about a microsecond of the per-call host cost)."""
    key = tuple(vals)
    a = _UINT_CACHE.get(key)
    if a is None:
        if len(_UINT_CACHE) > 4096:
            _UINT_CACHE.clear()
        a = _UINT_CACHE[key] = uint_array(key)
    return a


class Code(object):
    """RAII wrapper around fec_t* (fec_new / fec_free)."""

    def __init__(self, k, m):
        self.k, self.m = k, m
        self.ptr = lib().fec_new(k, m)
        if not self.ptr:
            raise FecError("fec_new(%d, %d) failed: %s" % (k, m, lib().fec_last_error_message().decode()))

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.fec_free(self.ptr)
            self.ptr = None

    def enc_matrix(self):
        s = ctypes.cast(self.ptr, ctypes.POINTER(FecT)).contents
        return bytes(s.enc_matrix[: self.k * self.m])

    def jit_prepare_encode(self, block_nums):
        check(lib().fec_jit_prepare_encode(self.ptr, uint_array(block_nums), len(block_nums)))

    def jit_prepare_decode(self, index, flags=0):
        check(lib().fec_jit_prepare_decode(self.ptr, uint_array(index), flags))

    def encode_batch(self, src, sbs, sss, dst, dbs, dss, block_nums, sz, nstripes, stream=0, flags=FEC_FLAG_ASYNC):
        if _batch_call is not None:
            st = _batch_call(0, self.ptr, src, sbs, sss, dst, dbs, dss, block_nums, sz, nstripes, stream or 0, flags)
            if st:
                check(st)
            return
        st = _lib.fec_encode_batch(self.ptr, src, sbs, sss, dst, dbs, dss, _nums(block_nums), len(block_nums), sz,
                                   nstripes, stream or None, flags)
        if st:
            check(st)

    def decode_batch(self, src, sbs, sss, dst, dbs, dss, index, sz, nstripes, stream=0, flags=FEC_FLAG_ASYNC):
        if _batch_call is not None:
            st = _batch_call(1, self.ptr, src, sbs, sss, dst, dbs, dss, index, sz, nstripes, stream or 0, flags)
            if st:
                check(st)
            return
        st = _lib.fec_decode_batch(self.ptr, src, sbs, sss, dst, dbs, dss, _nums(index), sz, nstripes,
                                   stream or None, flags)
        if st:
            check(st)

    def encode_batch_multi(self, src, sbs, sss, dst, dbs, dss, block_nums, sz, nstripes, devices, flags=0):
        """fec_encode_batch_multi: the stripes split over `devices` (host memory)."""
        devs = (ctypes.c_int * max(1, len(devices)))(*devices)
        check(lib().fec_encode_batch_multi(self.ptr, src, sbs, sss, dst, dbs, dss, uint_array(block_nums),
                                           len(block_nums), sz, nstripes, devs, len(devices), flags))

    def decode_batch_multi(self, src, sbs, sss, dst, dbs, dss, index, sz, nstripes, devices, flags=0):
        """fec_decode_batch_multi: the stripes split over `devices` (host memory)."""
        devs = (ctypes.c_int * max(1, len(devices)))(*devices)
        check(lib().fec_decode_batch_multi(self.ptr, src, sbs, sss, dst, dbs, dss, uint_array(index), sz, nstripes,
                                           devs, len(devices), flags))

    def encode_ptrs(self, in_addrs, out_addrs, block_nums, sz, stream=0, flags=FEC_FLAG_ASYNC):
        check(lib().fec_encode_ex(self.ptr, ptr_array(in_addrs), ptr_array(out_addrs), uint_array(block_nums),
                                  len(block_nums), sz, stream or None, flags))

    def decode_ptrs(self, in_addrs, out_addrs, index, sz, stream=0, flags=FEC_FLAG_ASYNC):
        check(lib().fec_decode_ex(self.ptr, ptr_array(in_addrs), ptr_array(out_addrs), uint_array(index),
                                  sz, stream or None, flags))


class BatchJob(ctypes.Structure):
    """fec_batch_job (include/zfec_hip.h)."""

    _fields_ = [("code", _P), ("kind", _U), ("flags", _U), ("src", _P), ("src_block_stride", _SZ),
                ("src_stripe_stride", _SZ), ("dst", _P), ("dst_block_stride", _SZ), ("dst_stripe_stride", _SZ),
                ("nums", _UP), ("num_nums", _SZ), ("sz", _SZ), ("nstripes", _SZ)]


def encode_job(code, src, sbs, sss, dst, dbs, dss, block_nums, sz, nstripes, flags=0):
    """One fec_run_batch_jobs job: Code.encode_batch's arguments."""
    return (code, FEC_JOB_ENCODE, flags, src, sbs, sss, dst, dbs, dss, tuple(block_nums), sz, nstripes)


def decode_job(code, src, sbs, sss, dst, dbs, dss, index, sz, nstripes, flags=0):
    """One fec_run_batch_jobs job: Code.decode_batch's arguments."""
    return (code, FEC_JOB_DECODE, flags, src, sbs, sss, dst, dbs, dss, tuple(index), sz, nstripes)


class BatchJobs(object):
    """A fec_run_batch_jobs call built once (the ctypes job array and block
    number arrays) and run any number of times."""

    def __init__(self, jobs):
        lib()
        self._codes = [j[0] for j in jobs]  # keep the fec_t objects alive
        self._nums = [uint_array(j[9]) for j in jobs]
        self.n = len(jobs)
        self._arr = (BatchJob * max(1, self.n))()
        for i, (code, kind, flags, src, sbs, sss, dst, dbs, dss, nums, sz, ns) in enumerate(jobs):
            self._arr[i] = BatchJob(code.ptr, kind, flags, src, sbs, sss, dst, dbs, dss,
                                    ctypes.cast(self._nums[i], _UP), len(nums), sz, ns)

    def run(self, stream=0, flags=FEC_FLAG_ASYNC):
        st = _lib.fec_run_batch_jobs(self._arr, self.n, stream or None, flags)
        if st:
            check(st)


def run_batch_jobs(jobs, stream=0, flags=FEC_FLAG_ASYNC):
    """fec_run_batch_jobs over encode_job / decode_job tuples."""
    BatchJobs(jobs).run(stream, flags)
