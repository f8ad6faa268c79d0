#!/usr/bin/env python3
"""In-process A/B of the small synchronous call's variants: blocks of N calls
(4 KiB K=3/M=10 encode and secondary-only decode from Python bytes) alternate
between ZFEC_HIP_* settings re-read with fec_reload_config, so the drift of
the host's launch rate within a process hits every variant alike.  Medians of
the per-block means over the rounds (us per call).

    python tools/small_ab_inproc.py [--rounds 12] [--n 2000] [--set kernel|wait] [--stripe 4096]

--set kernel: the small-call kernels (inline / bounce buffer / matapply_reg);
--set wait:   the completion wait (completion word / hipStreamSynchronize);
--set zc:     how far the kernel reads and writes the bounce buffer in place;
--set stage:  larger calls staged through the host pool, or packed into the
              bounce buffer (kernel in place / with copies);
--set pool:   the bounce buffer's copies on the calling thread or on the host pool;
--set zcwide: wide codes (k > 4 or r > 8) with the bounce buffer's copies or in place.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import zfec_amd  # noqa: E402
from zfec_amd import capi  # noqa: E402

SETS = {"kernel": {"inline": {}, "pinned": {"ZFEC_HIP_SMALL_INLINE": "0"}, "reg": {"ZFEC_HIP_SMALL_ONE": "0"}},
        "wait": {"signal": {}, "sync": {"ZFEC_HIP_WAIT": "sync"}},
        "zc": {"zc256k": {"ZFEC_HIP_ZC_LIMIT": str(256 << 10)}, "zc1m": {"ZFEC_HIP_ZC_LIMIT": str(1 << 20)},
               "zc2m": {}},
        "stage": {"default": {},
                  "staged": {"ZFEC_HIP_ZC_LIMIT": str(256 << 10)},
                  "bounce_inplace": {"ZFEC_HIP_STAGE_MIN": str(64 << 20), "ZFEC_HIP_PACK_LIMIT": str(64 << 20),
                                     "ZFEC_HIP_ZC_LIMIT": str(64 << 20)},
                  "bounce_copies": {"ZFEC_HIP_STAGE_MIN": str(64 << 20), "ZFEC_HIP_PACK_LIMIT": str(64 << 20)}},
        "zcwide": {"copies": {}, "inplace256k": {"ZFEC_HIP_ZC_WIDE_LIMIT": str(256 << 10)},
                   "inplace": {"ZFEC_HIP_ZC_WIDE": "1"}},
        "pool": {"thread": {}, "pool64k": {"ZFEC_HIP_POOL_COPY_MIN": str(64 << 10)},
                 "pool256k": {"ZFEC_HIP_POOL_COPY_MIN": str(256 << 10)}}}
KNOBS = ("ZFEC_HIP_SMALL_INLINE", "ZFEC_HIP_SMALL_ONE", "ZFEC_HIP_WAIT", "ZFEC_HIP_ZC_LIMIT", "ZFEC_HIP_STAGE_MIN",
         "ZFEC_HIP_PACK_LIMIT", "ZFEC_HIP_POOL_COPY_MIN", "ZFEC_HIP_ZC_WIDE",
         "ZFEC_HIP_ZC_WIDE_LIMIT")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--set", default="kernel", choices=sorted(SETS))
    ap.add_argument("--stripe", type=int, default=4096)
    ap.add_argument("--km", default="3,10", help="k,m")
    a = ap.parse_args()
    VARIANTS = SETS[a.set]
    k, m = (int(x) for x in a.km.split(","))
    sz = -(-a.stripe // k)
    blocks = [np.random.default_rng(i).integers(0, 256, sz, dtype=np.uint8).tobytes() for i in range(k)]
    enc, dec = zfec_amd.Encoder(k, m), zfec_amd.Decoder(k, m)
    out = enc.encode(blocks)
    nums = list(range(m - k, m))
    sec = [out[i] for i in nums]

    def setv(env):
        for key in KNOBS:
            os.environ.pop(key, None)
        os.environ.update(env)
        capi.reload_config()

    res = {v: {"enc": [], "dec": []} for v in VARIANTS}
    for _ in range(a.n * 5):  # warm-up
        enc.encode(blocks)
    for r in range(a.rounds):
        for v, env in VARIANTS.items():
            setv(env)
            assert enc.encode(blocks)[k:] == out[k:]
            t0 = time.perf_counter()
            for _ in range(a.n):
                enc.encode(blocks)
            t1 = time.perf_counter()
            for _ in range(a.n):
                dec.decode(sec, nums)
            t2 = time.perf_counter()
            res[v]["enc"].append((t1 - t0) / a.n * 1e6)
            res[v]["dec"].append((t2 - t1) / a.n * 1e6)
            if r == 0:
                res[v]["kernel"] = capi.last_kernel_name()
    setv({})
    summary = {v: {"kernel": d["kernel"], "encode_us_median": round(float(np.median(d["enc"])), 2),
                   "decode_us_median": round(float(np.median(d["dec"])), 2),
                   "encode_us_min": round(float(np.min(d["enc"])), 2)} for v, d in res.items()}
    print(json.dumps({"k": k, "m": m, "stripe": a.stripe, "rounds": a.rounds, "calls_per_block": a.n,
                      "variants": summary}, indent=1))


if __name__ == "__main__":
    main()
