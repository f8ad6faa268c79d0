#!/usr/bin/env python3
"""Where the time of the pageable `bytes` API goes (K=3/M=10, one 64 MiB stripe):
first touch of fresh host pages, hipHostRegister / Unregister of the blocks,
and the zero-copy kernel over PCIe on already page-locked buffers.
Prints one JSON line (ms per call, medians of 5)."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import zfec_amd  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]


def med(fn, n=5):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return round(sorted(ts)[n // 2], 2)


def main():
    k, m, S = 3, 10, 64 << 20
    sz = -(-S // k)
    r = m - k
    torch.cuda.init()
    rng = np.random.default_rng(1)
    blocks = [rng.integers(0, 256, size=sz, dtype=np.uint8).tobytes() for _ in range(k)]
    enc = zfec_amd.Encoder(k, m)
    enc.encode(blocks)
    res = {"k": k, "m": m, "block_bytes": sz}
    res["encode_call_ms"] = med(lambda: enc.encode(blocks))
    res["alloc_outputs_ms"] = med(lambda: [bytes(sz) for _ in range(r)])
    res["alloc_touch_outputs_ms"] = med(lambda: [np.ones(sz, np.uint8) for _ in range(r)])

    def reg(arrs):
        for a in arrs:
            assert hip.hipHostRegister(a.ctypes.data, a.nbytes, 2) == 0
        for a in arrs:
            hip.hipHostUnregister(a.ctypes.data)

    ins = [np.frombuffer(b, np.uint8) for b in blocks]
    outs = [np.ones(sz, np.uint8) for _ in range(r)]
    res["register_inputs_ms"] = med(lambda: reg(ins))
    res["register_outputs_touched_ms"] = med(lambda: reg(outs))
    res["register_outputs_fresh_ms"] = med(lambda: reg([np.empty(sz, np.uint8) for _ in range(r)]))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
