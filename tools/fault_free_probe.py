#!/usr/bin/env python3
"""Host-side cost of fresh output buffers on this machine: transparent huge
page settings, then for 7 x 22.4 MB (the K=3/M=10 64 MiB encode's outputs):
allocate + fault in (one thread) + free, with and without MADV_HUGEPAGE, and
the free alone.  No GPU."""
import ctypes
import mmap
import os
import statistics
import time

libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
MADV_HUGEPAGE = 14


def thp():
    out = {}
    for f in ("enabled", "defrag", "khugepaged/defrag"):
        try:
            out[f] = open("/sys/kernel/mm/transparent_hugepage/" + f).read().strip()
        except OSError as e:
            out[f] = repr(e)
    return out


def run(huge, n=7, sz=22369622, reps=7):
    ta, tf, tfr = [], [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        bufs = [mmap.mmap(-1, sz) for _ in range(n)]
        if huge:
            for b in bufs:
                addr = ctypes.addressof(ctypes.c_char.from_buffer(b))
                libc.madvise(addr, sz, MADV_HUGEPAGE)
        t1 = time.perf_counter()
        for b in bufs:
            for off in range(0, sz, 4096):
                b[off] = 1
        t2 = time.perf_counter()
        for b in bufs:
            b.close()
        t3 = time.perf_counter()
        ta.append(t1 - t0)
        tf.append(t2 - t1)
        tfr.append(t3 - t2)
    return {"alloc_ms": round(statistics.median(ta) * 1e3, 2), "fault_ms": round(statistics.median(tf) * 1e3, 2),
            "free_ms": round(statistics.median(tfr) * 1e3, 2)}


if __name__ == "__main__":
    print("thp", thp())
    print("4k/default", run(False))
    print("madv_hugepage", run(True))
