#!/usr/bin/env python3
"""Where the time of the staged host path goes (K=3/M=10 encode and decode of
one stripe from pageable host memory, 4 / 16 / 64 MiB):

  bytes        Python bytes in, fresh bytes out (the drop-in API)
  reused       C-ABI call on pageable numpy arrays reused across calls (output
               pages already mapped: no page faults)
  fresh_np     C-ABI call into fresh np.empty outputs each call (faults)

Median ms and GB/s of input over --reps calls; with ZFEC_HIP_TRACE_HOST=1 the
library adds per-phase times on stderr."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import zfec_amd  # noqa: E402
from zfec_amd import capi  # noqa: E402


def med(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--sizes", default="4,16,64")
    ap.add_argument("--reuse", action="store_true", help="call zfec_amd.reuse_host_memory() first")
    a = ap.parse_args()
    if a.reuse:
        assert zfec_amd.reuse_host_memory()
    k, m = 3, 10
    code = capi.Code(k, m)
    for mib in [int(x) for x in a.sizes.split(",")]:
        sz = -(-(mib << 20) // k)
        data = np.random.default_rng(mib).integers(0, 256, size=(k, sz), dtype=np.uint8)
        blocks = [data[i].tobytes() for i in range(k)]
        enc = zfec_amd.Encoder(k, m)
        out = np.empty((m - k, sz), np.uint8)
        ins = [data[i].ctypes.data for i in range(k)]

        def reused():
            code.encode_ptrs(ins, [out[i].ctypes.data for i in range(m - k)], list(range(k, m)), sz,
                             flags=capi.FEC_FLAG_LIBRARY_STREAM | capi.FEC_FLAG_HOST_MEMORY)

        def fresh_np():
            o = [np.empty(sz, np.uint8) for _ in range(m - k)]
            code.encode_ptrs(ins, [x.ctypes.data for x in o], list(range(k, m)), sz,
                             flags=capi.FEC_FLAG_LIBRARY_STREAM | capi.FEC_FLAG_HOST_MEMORY)

        row = {"stripe_MiB": mib}
        for name, fn in (("bytes", lambda: enc.encode(blocks)), ("reused", reused), ("fresh_np", fresh_np)):
            sys.stderr.write(f"== {mib} MiB {name}\n")
            t = med(fn, a.reps)
            row[name + "_ms"] = round(t * 1e3, 3)
            row[name + "_GBps"] = round(k * sz / t / 1e9, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
