#!/usr/bin/env python3
"""Per-call latency of the Python bytes API (host buffers in, bytes out) for
small and medium stripes: zfec_amd.Encoder.encode / Decoder.decode against the
reference's C module (oracle/_ref, when built) on the same inputs, 1 thread."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import zfec_amd  # noqa: E402


def per_call_us(fn, n):
    fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    try:
        from oracle import oracle
        ref = oracle.ref_module()
    except Exception:
        ref = None
    rng = np.random.default_rng(0)
    res = []
    for k, m in [(3, 10), (20, 60)]:
        for stripe in [4096, 65536, 131072, 1 << 20, 4 << 20]:  # 128 KiB: a tahoe-lafs segment
            sz = -(-stripe // k)
            blocks = [rng.integers(0, 256, sz, dtype=np.uint8).tobytes() for _ in range(k)]
            n = 2000 if stripe <= 131072 else (200 if stripe <= 1 << 20 else 50)
            row = {"k": k, "m": m, "stripe": stripe}
            impls = [("gpu", zfec_amd)] + ([("cpu_ref", ref)] if ref is not None else [])
            for name, mod in impls:
                enc, dec = mod.Encoder(k, m), mod.Decoder(k, m)
                out = enc.encode(blocks)
                nums = list(range(m - k, m))
                sec = [out[i] for i in nums]
                row[name + "_encode_us"] = round(per_call_us(lambda: enc.encode(blocks), n), 1)
                row[name + "_decode_us"] = round(per_call_us(lambda: dec.decode(sec, nums), n), 1)
            print(json.dumps(row), flush=True)
            res.append(row)


if __name__ == "__main__":
    main()
