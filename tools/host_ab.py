#!/usr/bin/env python3
"""A/B of the host paths for large pageable calls (the drop-in `bytes` API):
ZFEC_HIP_HOST_PATH = stage (pinned staging slots + host copy threads),
lock (page-lock the caller's blocks chunk by chunk), copy (DMA pipeline).

K=3/M=10, one 64 MiB stripe from Python bytes (zfec_amd.Encoder.encode /
Decoder.decode from three parity blocks), interleaved rounds, median and best
GB/s of stripe input bytes.  Each output is checked against the first one.

  python tools/host_ab.py [--reps 7] [--rounds 3] [--chunks 0,1048576] [--threads 16]
--threads runs one child process per thread count (the pool is sized once per
process, ZFEC_HIP_HOST_THREADS).
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(args):
    import zfec_amd

    k, m = args.k, args.m
    sz = -(-(args.mib << 20) // k)
    rng = np.random.default_rng(1)
    data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
    blocks = [data[i].tobytes() for i in range(k)]
    enc, dec = zfec_amd.Encoder(k, m), zfec_amd.Decoder(k, m)
    os.environ["ZFEC_HIP_HOST_PATH"] = "lock"
    ref = enc.encode(blocks)
    par = list(ref[k:2 * k]) if m >= 2 * k else list(ref[m - k:])
    nums = list(range(k, 2 * k)) if m >= 2 * k else list(range(m - k, m))
    assert dec.decode(par, nums) == blocks
    modes = args.modes.split(",")
    chunks = [int(c) for c in args.chunks.split(",")]
    res = {}
    for _ in range(args.rounds):
        for mode in modes:
            for ch in (chunks if mode == "stage" else [0]):
                os.environ["ZFEC_HIP_HOST_PATH"] = mode
                if ch:
                    os.environ["ZFEC_HIP_STAGE_CHUNK"] = str(ch)
                else:
                    os.environ.pop("ZFEC_HIP_STAGE_CHUNK", None)
                tag = mode + (f"_c{ch >> 10}k" if ch else "")
                out = enc.encode(blocks)
                assert out == ref, tag
                assert dec.decode(par, nums) == blocks, tag
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    out = enc.encode(blocks)
                    res.setdefault(tag + "_enc", []).append(time.perf_counter() - t0)
                    del out
                    t0 = time.perf_counter()
                    rec = dec.decode(par, nums)
                    res.setdefault(tag + "_dec", []).append(time.perf_counter() - t0)
                    del rec
    line = {"k": k, "m": m, "stripe_bytes": k * sz, "threads": os.environ.get("ZFEC_HIP_HOST_THREADS", "auto")}
    for key, ts in res.items():
        line[key + "_GBps_median"] = round(k * sz / statistics.median(ts) / 1e9, 2)
        line[key + "_GBps_best"] = round(k * sz / min(ts) / 1e9, 2)
    print(json.dumps(line), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=3)
    p.add_argument("--m", type=int, default=10)
    p.add_argument("--mib", type=int, default=64)
    p.add_argument("--reps", type=int, default=7)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--modes", default="stage,lock")
    p.add_argument("--chunks", default="0")
    p.add_argument("--threads", default="")
    p.add_argument("--child", action="store_true")
    args = p.parse_args()
    if args.child or not args.threads:
        child(args)
        return
    for t in args.threads.split(","):
        env = dict(os.environ, ZFEC_HIP_HOST_THREADS=t)
        argv = [sys.executable, __file__, "--child"] + [a for a in sys.argv[1:] if not a.startswith("--threads")]
        # drop the value that followed --threads
        if "--threads" in sys.argv:
            i = sys.argv.index("--threads")
            argv = [sys.executable, __file__, "--child"] + sys.argv[1:i] + sys.argv[i + 2:]
        r = subprocess.run(argv, env=env, timeout=600)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
