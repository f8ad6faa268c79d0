#!/usr/bin/env python3
"""A/B of the large pageable `bytes` path (K=3/M=10, one 64 MiB stripe,
encode and secondary-only decode from Python bytes), interleaved rounds:

  ZFEC_HIP_PAGEABLE_CHUNK  bytes of every block per chunk of pages locked
                         at a time (32 MiB: the whole 22 MiB block at once)
  populate               1: each chunk's fresh outputs pre-faulted from 4
                         threads right before it is locked
                         (ZFEC_HIP_POPULATE=1); 0 (default): the locking
                         faults them.  (A third variant, background threads
                         faulting the outputs chunk by chunk ahead of the
                         locking, measured no better and was dropped:
                         profiles/r02_host_ab.log)

Prints one line per variant (median / best GB/s of input over the rounds) and
a JSON summary.  ZFEC_HIP_TRACE_HOST=1 in the environment adds the library's
per-phase times on stderr.

    python tools/host_phases.py [--rounds 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import zfec_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    k, m, S = 3, 10, 64 << 20
    sz = -(-S // k)
    blocks = [np.random.default_rng(i).integers(0, 256, size=sz, dtype=np.uint8).tobytes() for i in range(k)]
    enc, dec = zfec_amd.Encoder(k, m), zfec_amd.Decoder(k, m)
    ref = enc.encode(blocks)
    variants = []
    for chunk in (2 << 20, 4 << 20, 8 << 20):
        for pop in ("0", "1"):
            variants.append(("zerocopy", chunk, pop))
    res = {v: {"enc": [], "dec": []} for v in variants}
    for _ in range(a.rounds):
        for v in variants:
            os.environ["ZFEC_HIP_PAGEABLE_CHUNK"] = str(v[1])
            os.environ["ZFEC_HIP_POPULATE"] = "1" if v[2] == "1" else "0"
            t0 = time.perf_counter()
            out = enc.encode(blocks)
            t1 = time.perf_counter()
            assert out == ref
            del out
            t2 = time.perf_counter()
            got = dec.decode(ref[3:6], [3, 4, 5])
            t3 = time.perf_counter()
            assert got == blocks
            del got
            res[v]["enc"].append(k * sz / (t1 - t0) / 1e9)
            res[v]["dec"].append(k * sz / (t3 - t2) / 1e9)
    summary = {}
    for v in variants:
        key = "chunk=%dMiB populate=%s" % (v[1] >> 20, v[2])
        e, d = sorted(res[v]["enc"]), sorted(res[v]["dec"])
        summary[key] = {"encode_GBps_median": round(e[len(e) // 2], 2), "encode_GBps_best": round(e[-1], 2),
                        "decode_GBps_median": round(d[len(d) // 2], 2), "decode_GBps_best": round(d[-1], 2)}
        print("%-34s encode median %6.2f best %6.2f | decode median %6.2f best %6.2f GB/s" % (
            key, e[len(e) // 2], e[-1], d[len(d) // 2], d[-1]), flush=True)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
