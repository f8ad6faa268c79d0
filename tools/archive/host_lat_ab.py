#!/usr/bin/env python3
"""Per-call time of the Python bytes API at 1-16 MiB stripes (pinned bounce
buffer below 4 MiB of host blocks, staged path above), A/B of host-path knobs
in one process, interleaved rounds, median microseconds per call.  Run it
under GLIBC_TUNABLES=glibc.malloc.mmap_threshold=33554432:glibc.malloc.trim_threshold=1073741824
to take the freeing and re-faulting of the output bytes out of the figures.

Variants: default (staged from 512 KiB of host blocks when blocks are >= 64
KiB, from 4 MiB otherwise; bounce-buffer copies on the calling thread);
pack_to_4MiB (ZFEC_HIP_STAGE_MIN=inf: the bounce buffer up to 4 MiB);
pool_copy (ZFEC_HIP_POOL_COPY_MIN=512 KiB: bounce-buffer copies on the host
pool); one_chunk (ZFEC_HIP_STAGE_CHUNK=<16 MiB / blocks>: no quarter-block cap)
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import zfec_amd  # noqa: E402


def main():
    rng = np.random.default_rng(0)
    for k, m in [(3, 10), (20, 60)]:
        for stripe in [256 << 10, 1 << 20, 2 << 20, 4 << 20, 16 << 20]:
            sz = -(-stripe // k)
            blocks = [rng.integers(0, 256, sz, dtype=np.uint8).tobytes() for _ in range(k)]
            enc, dec = zfec_amd.Encoder(k, m), zfec_amd.Decoder(k, m)
            ref = enc.encode(blocks)
            nums = list(range(m - k, m))
            sec = [ref[i] for i in nums]
            one_chunk = str(((16 << 20) // m) // 65536 * 65536)
            variants = {"default": {}, "pack_to_4MiB": {"ZFEC_HIP_STAGE_MIN": str(1 << 60)},
                        "pool_copy": {"ZFEC_HIP_POOL_COPY_MIN": str(512 << 10)},
                        "one_chunk": {"ZFEC_HIP_STAGE_CHUNK": one_chunk}}
            times = {}
            n = 40 if stripe <= (4 << 20) else 10
            for _ in range(3):
                for name, env in variants.items():
                    for key in ("ZFEC_HIP_POOL_COPY_MIN", "ZFEC_HIP_STAGE_CHUNK", "ZFEC_HIP_STAGE_MIN"):
                        os.environ.pop(key, None)
                    os.environ.update(env)
                    assert enc.encode(blocks) == ref and dec.decode(sec, nums) == blocks, name
                    for _ in range(n):
                        t0 = time.perf_counter()
                        enc.encode(blocks)
                        t1 = time.perf_counter()
                        dec.decode(sec, nums)
                        t2 = time.perf_counter()
                        times.setdefault(name + "_enc", []).append(t1 - t0)
                        times.setdefault(name + "_dec", []).append(t2 - t1)
            row = {"k": k, "m": m, "stripe": stripe}
            for key, ts in times.items():
                row[key + "_us"] = round(statistics.median(ts) * 1e6, 1)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
