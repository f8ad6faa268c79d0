#!/usr/bin/env python3
"""A/B of the table kernels against the bit-sliced JIT kernels
(zfec_amd/csrc/bitslice.cpp) on device-resident stripes, interleaved rounds,
medians.  Shapes: the bench workloads cfg3 (K=10/M=16, one 256 MiB stripe)
and cfg4 (K=20/M=60, 1024 x 1 MiB stripes), encode and last-k decode.
Variants (ZFEC_HIP_JIT_* knobs): table kernels; bit-sliced JIT kernels with
the default options, Gray-code combination order, waves-per-SIMD register
bounds, row tiles split across the waves of a workgroup, bit-planes shared
through LDS (ZFEC_HIP_JIT_SHARE) at several tile heights, 64-bit shifts in
the bit transposes (ZFEC_HIP_JIT_SHIFT64).  Earlier rounds of
this A/B: profiles/r01_jit_ab.log (tile heights, store cache policies),
profiles/r01_jit_ab2.log (split).

Per launch time = events around `reps` back-to-back launches on the launch
stream / reps; HBM GB/s = (k + r) * sz * stripes / time.  Every variant's
output is compared with the table kernel's.

usage: python tools/jit_bench.py [--shapes cfg3,cfg4] [--rounds 5]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from zfec_amd import capi  # noqa: E402

SHAPES = {"cfg3": (10, 16, 256 << 20, 1), "cfg4": (20, 60, 1 << 20, 1024)}
VARIANTS = [
    ("table", capi.JIT_OFF, {}),
    ("share", capi.JIT_FORCE, {"ZFEC_HIP_JIT_SHARE": "1", "ZFEC_HIP_JIT_SHIFT64": "0"}),
    ("shift64", capi.JIT_FORCE, {"ZFEC_HIP_JIT_SHARE": "1", "ZFEC_HIP_JIT_SHIFT64": "1"}),
]
KNOBS = ("ZFEC_HIP_JIT_TILE", "ZFEC_HIP_JIT_PREFETCH", "ZFEC_HIP_JIT_BARRIER", "ZFEC_HIP_JIT_STORE",
         "ZFEC_HIP_JIT_ORDER", "ZFEC_HIP_JIT_WAVES", "ZFEC_HIP_JIT_SPLIT", "ZFEC_HIP_JIT_SHARE",
         "ZFEC_HIP_JIT_ARGLOAD", "ZFEC_HIP_JIT_SHIFT64")


def place(nums, k):
    slots = [None] * k
    sec = iter([n for n in nums if n >= k])
    for n in nums:
        if n < k:
            slots[n] = n
    return [s if s is not None else next(sec) for s in slots]


def set_variant(mode, env):
    for key in KNOBS:
        os.environ.pop(key, None)
    os.environ.update(env)
    capi.jit_mode(mode)
    capi.generic_mode(0)  # "table" = the table kernels, not matapply_bsg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="cfg3,cfg4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    st = torch.cuda.current_stream()
    res = {}
    for shape in args.shapes.split(","):
        k, m, S, ns = SHAPES[shape]
        r = m - k
        sz = -(-S // k)
        ld = (sz + 255) // 256 * 256
        g = torch.Generator(device="cuda").manual_seed(k)
        data = torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda", generator=g)
        code = capi.Code(k, m)
        slots = place(list(range(m - k, m)), k)
        nrec = sum(1 for s in slots if s >= k)
        outs = {name: torch.zeros((ns, r, ld), dtype=torch.uint8, device="cuda") for name, _, _ in VARIANTS}
        recs = {name: torch.zeros((ns, nrec, ld), dtype=torch.uint8, device="cuda") for name, _, _ in VARIANTS}
        recv = None
        times = {(name, d): [] for name, _, _ in VARIANTS for d in ("enc", "dec")}
        kern = {}
        for rnd in range(args.rounds):
            for name, mode, env in VARIANTS:
                set_variant(mode, env)
                out, rec = outs[name], recs[name]

                def enc():
                    code.encode_batch(data.data_ptr(), ld, k * ld, out.data_ptr(), ld, r * ld, list(range(k, m)), sz,
                                      ns, stream=st.cuda_stream)

                def dec():
                    code.decode_batch(recv.data_ptr(), ld, k * ld, rec.data_ptr(), ld, nrec * ld, slots, sz, ns,
                                      stream=st.cuda_stream)

                enc()
                kern[(name, "enc")] = capi.last_kernel_name()
                if recv is None:  # received blocks: primaries / parity per slot, from the table kernel's output
                    torch.cuda.synchronize()
                    recv = torch.empty((ns, k, ld), dtype=torch.uint8, device="cuda")
                    for i, s in enumerate(slots):
                        recv[:, i].copy_(data[:, s] if s < k else out[:, s - k])
                dec()
                kern[(name, "dec")] = capi.last_kernel_name()
                for d, fn in (("enc", enc), ("dec", dec)):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for _ in range(args.reps):
                        fn()
                    e1.record(st)
                    torch.cuda.synchronize()
                    times[(name, d)].append(e0.elapsed_time(e1) / args.reps)
        base = outs["table"][:, :, :sz]
        missing = [i for i in range(k) if slots[i] >= k]
        for name, _, _ in VARIANTS:
            ok_enc = bool(torch.equal(outs[name][:, :, :sz], base))
            ok_dec = bool(torch.equal(recs[name][:, :, :sz], data[:, missing, :sz]))
            for d, nb in (("enc", k + r), ("dec", k + nrec)):
                ms = float(np.median(times[(name, d)]))
                row = {"kernel": kern[(name, d)], "ms": round(ms, 4),
                       "hbm_GBps": round(nb * sz * ns / (ms * 1e-3) / 1e9, 1),
                       "input_GBps": round(k * sz * ns / (ms * 1e-3) / 1e9, 1),
                       "bitexact": ok_enc if d == "enc" else ok_dec}
                res["%s %s %s" % (shape, d, name)] = row
                print(shape, d, "%-14s" % name, json.dumps(row), flush=True)
    set_variant(capi.JIT_AUTO, {})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
