#!/usr/bin/env python3
"""Batches in pageable host memory (numpy) through the batched entry points
(staged through pinned slots, fec_abi.cpp run_batch_staged): the cfg5 shape
(K=3/M=10, 10^6 objects of 4 KiB, 1366-byte blocks) and the cfg4 shape
(K=20/M=60, 1024 x 1 MiB stripes), object-major [stripe][block][sz] and
block-major.  Per layout: Encoder.encode_batch into a fresh numpy array (page
faults of the output included), and the C-ABI call into a preallocated,
already-faulted output array; GB/s of input (1e9).  Median of --reps."""
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
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--shapes", default="cfg5,cfg4")
    a = ap.parse_args()
    shapes = {"cfg5": (3, 10, 4096, 1000000), "cfg4": (20, 60, 1 << 20, 1024)}
    for name in a.shapes.split(","):
        k, m, stripe, ns = shapes[name]
        r = m - k
        sz = -(-stripe // k)
        rng = np.random.default_rng(0)
        data = rng.integers(0, 256, size=(ns, k, sz), dtype=np.uint8)
        enc = zfec_amd.Encoder(k, m)
        code = capi.Code(k, m)
        row = {"shape": name, "k": k, "m": m, "sz": sz, "stripes": ns, "input_bytes": ns * k * sz}
        for layout in ("object-major", "block-major"):
            blocks = data if layout == "object-major" else np.ascontiguousarray(
                data.transpose(1, 0, 2)).transpose(1, 0, 2)
            t = med(lambda: enc.encode_batch(blocks), a.reps)
            row[layout + " encode_batch_GBps"] = round(ns * k * sz / t / 1e9, 2)
            out = enc.encode_batch(blocks)  # allocated and faulted once
            sbs, sss = blocks.strides[1], blocks.strides[0]
            obs, oss = out.strides[1], out.strides[0]

            def into():
                code.encode_batch(blocks.ctypes.data, sbs, sss, out.ctypes.data, obs, oss, list(range(k, m)), sz, ns,
                                  flags=capi.FEC_FLAG_LIBRARY_STREAM)

            t = med(into, a.reps)
            row[layout + " into_faulted_GBps"] = round(ns * k * sz / t / 1e9, 2)
            del out
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
