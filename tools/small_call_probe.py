#!/usr/bin/env python3
"""Small host calls under a kernel trace: N encodes (and secondary-only
decodes) of one stripe from Python bytes, per (k, m, stripe) given on the
command line, e.g. `python tools/small_call_probe.py 20,60,4096 3,10,4096`.
Prints wall microseconds per call; run under rocprofv3 --kernel-trace --stats
to split each call into kernel time and host overhead."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import zfec_amd  # noqa: E402


def main():
    n = int(os.environ.get("N", "200"))
    for spec in sys.argv[1:]:
        k, m, stripe = (int(x) for x in spec.split(","))
        sz = -(-stripe // k)
        blocks = [np.random.default_rng(i).integers(0, 256, sz, dtype=np.uint8).tobytes() for i in range(k)]
        enc, dec = zfec_amd.Encoder(k, m), zfec_amd.Decoder(k, m)
        out = enc.encode(blocks)
        nums = list(range(m - k, m))
        sec = [out[i] for i in nums]
        t0 = time.perf_counter()
        for _ in range(n):
            enc.encode(blocks)
        t1 = time.perf_counter()
        for _ in range(n):
            dec.decode(sec, nums)
        t2 = time.perf_counter()
        print(json.dumps({"k": k, "m": m, "stripe": stripe, "encode_us": round((t1 - t0) / n * 1e6, 1),
                          "decode_us": round((t2 - t1) / n * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
