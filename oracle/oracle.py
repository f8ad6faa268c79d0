"""ctypes front end for the CPU oracle (oracle/fec_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker.  The product package
(zfec_amd) never imports this module and has no CPU fallback.

Also exposes the real reference (oracle/_ref, compiled from
/root/reference/zfec/fec.c by oracle/Makefile) when it has been built, for
golden-vector generation and the "reference" CPU baseline.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_DIR = os.path.join(HERE, "_ref")

_lib = None


def build(quiet=True):
    """Compile liboracle.so (gcc) if missing or stale."""
    src = os.path.join(HERE, "fec_oracle.c")
    if os.path.exists(LIB_PATH) and os.path.getmtime(LIB_PATH) >= os.path.getmtime(src):
        return
    subprocess.run(["make", "-C", HERE, "liboracle.so"], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_ubyte)
        uip = ctypes.POINTER(ctypes.c_uint)
        L.oracle_init.restype = None
        L.oracle_gf_mul.restype = ctypes.c_ubyte
        L.oracle_gf_mul.argtypes = [ctypes.c_ubyte, ctypes.c_ubyte]
        L.oracle_gf_inv.restype = ctypes.c_ubyte
        L.oracle_gf_inv.argtypes = [ctypes.c_ubyte]
        L.oracle_gf_exp.restype = ctypes.c_ubyte
        L.oracle_gf_exp.argtypes = [ctypes.c_int]
        L.oracle_gf_log.restype = ctypes.c_int
        L.oracle_gf_log.argtypes = [ctypes.c_ubyte]
        L.oracle_enc_matrix.argtypes = [ctypes.c_uint, ctypes.c_uint, u8p]
        L.oracle_invert_vdm.argtypes = [u8p, ctypes.c_uint]
        L.oracle_invert_mat.argtypes = [u8p, ctypes.c_uint]
        L.oracle_invert_mat.restype = ctypes.c_int
        L.oracle_decode_matrix.argtypes = [u8p, ctypes.c_uint, uip, u8p]
        L.oracle_decode_matrix.restype = ctypes.c_int
        L.oracle_encode_flat.argtypes = [u8p, ctypes.c_uint, u8p, u8p, uip, ctypes.c_size_t, ctypes.c_size_t]
        L.oracle_decode_flat.argtypes = [u8p, ctypes.c_uint, u8p, u8p, uip, ctypes.c_size_t]
        L.oracle_decode_flat.restype = ctypes.c_int
        L.oracle_init()
        _lib = L
    return _lib


def _u8(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte))


def _ui(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint))


def gf_mul(a, b):
    return lib().oracle_gf_mul(a, b)


def gf_inv(a):
    return lib().oracle_gf_inv(a)


def enc_matrix(k, m):
    """n x k systematic encoding matrix (zfec/fec.c:430-479)."""
    out = np.zeros((m, k), dtype=np.uint8)
    lib().oracle_enc_matrix(k, m, _u8(out))
    return out


def decode_matrix(k, m, index):
    """Inverse of the received-rows matrix (zfec/fec.c:512-525)."""
    enc = enc_matrix(k, m)
    idx = np.ascontiguousarray(index, dtype=np.uint32)
    out = np.zeros((k, k), dtype=np.uint8)
    if lib().oracle_decode_matrix(_u8(enc), k, _ui(idx), _u8(out)) != 0:
        raise ValueError("singular decode matrix")
    return out


def encode(k, m, blocks, block_nums=None):
    """blocks: (k, sz) uint8.  Returns (len(block_nums), sz) uint8 parity
    (block_nums default k..m-1), computed as zfec/fec.c:487-505."""
    blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
    assert blocks.shape[0] == k
    sz = blocks.shape[1]
    if block_nums is None:
        block_nums = list(range(k, m))
    nums = np.ascontiguousarray(block_nums, dtype=np.uint32)
    enc = enc_matrix(k, m)
    out = np.zeros((len(nums), sz), dtype=np.uint8)
    lib().oracle_encode_flat(_u8(enc), k, _u8(blocks), _u8(out), _ui(nums), len(nums), sz)
    return out


def decode(k, m, blocks, index):
    """blocks: (k, sz) uint8 in slot order (primary i at slot i), index: block
    numbers per slot.  Returns the recovered primaries in ascending order
    (zfec/fec.c:527-557)."""
    blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
    sz = blocks.shape[1]
    idx = np.ascontiguousarray(index, dtype=np.uint32)
    enc = enc_matrix(k, m)
    out = np.zeros((k, sz), dtype=np.uint8)
    if lib().oracle_decode_flat(_u8(enc), k, _u8(blocks), _u8(out), _ui(idx), sz) != 0:
        raise ValueError("singular decode matrix")
    nrec = int(sum(1 for i in index if i >= k))
    return out[:nrec]


def pattern_blocks(k, sz):
    """Deterministic KAT pattern from SURVEY.md Appendix B:
    block j byte i = ((i*31 + j*17 + 7) ^ (i >> 8)) & 0xFF, i as uint32."""
    i = np.arange(sz, dtype=np.uint64) & np.uint64(0xFFFFFFFF)
    out = np.empty((k, sz), dtype=np.uint8)
    for j in range(k):
        out[j] = (((i * np.uint64(31) + np.uint64(j * 17 + 7)) & np.uint64(0xFFFFFFFF)) ^ (i >> np.uint64(8))).astype(np.uint64) & np.uint64(0xFF)
    return out


def ref_bench_lib():
    """oracle/_ref/libref_bench.so (ref_bench.c + the reference's fec.c): the
    reference's CPU path driven from C threads, or None if unbuilt."""
    import ctypes

    path = os.path.join(REF_DIR, "libref_bench.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.ref_bench.argtypes = [ctypes.c_uint, ctypes.c_uint, ctypes.c_size_t, ctypes.c_int, ctypes.c_double,
                              ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double)]
    lib.ref_bench.restype = ctypes.c_int
    return lib


def ref_bench(lib, k, m, sz, threads, seconds):
    """(steps, seconds) of `threads` C threads each repeating encode + last-k
    decode of its own K/M stripe of k*sz bytes for ~`seconds` (ref_bench.c)."""
    import ctypes

    st, el = ctypes.c_uint64(), ctypes.c_double()
    if lib.ref_bench(k, m, sz, threads, seconds, ctypes.byref(st), ctypes.byref(el)) != 0:
        raise RuntimeError("ref_bench failed (allocation, threads, or a wrong decode)")
    return st.value, el.value


def ref_module():
    """The real reference extension (oracle/_ref/_fec*.so) or None if unbuilt."""
    if not os.path.isdir(REF_DIR):
        return None
    if REF_DIR not in sys.path:
        sys.path.insert(0, REF_DIR)
    try:
        import _fec  # noqa: the reference's own module name (zfec/_fecmodule.c:667)
    except ImportError:
        return None
    return _fec
