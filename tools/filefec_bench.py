#!/usr/bin/env python3
"""End-to-end share-file throughput of zfec_amd.filefec (file -> m share files
-> file), on tmpfs when available.  Reports input bytes / wall second for
encode_to_files and decode_from_files (k shares, worst case: parity only when
m-k >= k), and, with --cpu, the same files through the reference's C module
via oracle/_ref (the per-segment easyfec loop the reference's filefec runs).

    python tools/filefec_bench.py [--mib 1024] [--k 3] [--m 10] [--cpu]
"""
import argparse
import hashlib
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import zfec_amd  # noqa: E402
from zfec_amd import filefec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--m", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    base = "/dev/shm" if os.path.isdir("/dev/shm") else None
    td = tempfile.mkdtemp(prefix="ffb", dir=base)
    try:
        n = a.mib << 20
        data = np.random.default_rng(1).integers(0, 256, size=n, dtype=np.uint8)
        src = os.path.join(td, "in.bin")
        data.tofile(src)
        digest = hashlib.sha256(data).hexdigest()
        del data
        res = {"k": a.k, "m": a.m, "bytes": n, "fs": base or "tmp", "encode_s": [], "decode_s": []}
        for rep in range(a.reps):
            od = os.path.join(td, "sh")
            shutil.rmtree(od, ignore_errors=True)
            os.mkdir(od)
            t0 = time.perf_counter()
            with open(src, "rb") as f:
                filefec.encode_to_files(f, n, od, "in.bin", a.k, a.m, ".fec")
            res["encode_s"].append(time.perf_counter() - t0)
            names = sorted(os.listdir(od))[-a.k:]  # the last k: parity shares when m-k >= k
            outp = os.path.join(td, "out.bin")
            files = [open(os.path.join(od, x), "rb") for x in names]
            t0 = time.perf_counter()
            with open(outp, "wb") as outf:
                filefec.decode_from_files(outf, files)
            res["decode_s"].append(time.perf_counter() - t0)
            for f in files:
                f.close()
            h = hashlib.sha256()
            with open(outp, "rb") as f:
                for blk in iter(lambda: f.read(1 << 24), b""):
                    h.update(blk)
            assert h.hexdigest() == digest, "round trip mismatch"
            os.remove(outp)
        res["encode_GBps"] = n / min(res["encode_s"]) / 1e9
        res["decode_GBps"] = n / min(res["decode_s"]) / 1e9
        print(json.dumps(res))
    finally:
        shutil.rmtree(td, ignore_errors=True)


if __name__ == "__main__":
    main()
