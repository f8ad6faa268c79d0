#!/usr/bin/env python3
"""North-star shape A/B: K=3/M=10 encode of 1 MiB stripes,
object-major [stripe][block][row] (rows 256-byte aligned), timed like bench.py's
batched_1MiB leg (back-to-back launches over a rotation of disjoint buffer sets
spanning >= 768 MiB: cold = HBM), for several stripes-per-launch counts.  Run it
in two trees to A/B a kernel change; every launch's output is checked once
against the oracle on sampled stripes.

    python tools/batch_ab.py [--stripes 256,1024] [--steps 20] [--rounds 2]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(sys.argv[0])))
sys.path.insert(0, os.getcwd())

import bench  # noqa: E402  (the tree this runs in)
from zfec_amd import capi  # noqa: E402


def one(ns, steps, k=3, m=10, flags=capi.FEC_FLAG_ASYNC, sz=None):
    sz = sz or -(-(1 << 20) // k)
    ld = bench.row_stride(sz)
    code = capi.Code(k, m)
    st = torch.cuda.current_stream()
    nums = list(range(k, m))
    fp = m * ld * ns
    nsets = max(2, -(-bench.COLD_SPAN // fp))
    src = [torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda") for _ in range(nsets)]
    dst = [torch.empty((ns, m - k, ld), dtype=torch.uint8, device="cuda") for _ in range(nsets)]

    def enc_i(i):
        def f(sh):
            code.encode_batch(src[i].data_ptr(), ld, k * ld, dst[i].data_ptr(), ld, (m - k) * ld, nums, sz, ns,
                              stream=sh, flags=flags)
        return f

    enc_i(0)(st.cuda_stream)
    torch.cuda.synchronize()
    from oracle import oracle  # the checker, after nothing is timed
    for s in (0, ns // 2, ns - 1):
        want = oracle.encode(k, m, src[0][s, :, :sz].cpu().numpy())
        assert np.array_equal(dst[0][s, :, :sz].cpu().numpy(), want), s
    warm, _ = bench.back_to_back([enc_i(0)], steps, st, "batch_ab warm")
    cold, _ = bench.back_to_back([enc_i(i) for i in range(nsets)], steps, st, "batch_ab cold")
    kern = capi.last_kernel_name()
    hbm = lambda ms: ns * m * sz / (ms * 1e-3) / 1e9
    del src, dst
    torch.cuda.empty_cache()
    return {"stripes": ns, "sz": sz, "kernel": kern, "nsets": nsets, "ms_cold": round(cold, 4), "ms_warm": round(warm, 4),
            "frac_cold": round(hbm(cold) / bench.HBM_PEAK_GBPS, 4), "frac_warm": round(hbm(warm) / bench.HBM_PEAK_GBPS, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", default="256,1024")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--sz", type=int, default=0, help="block size (default: a third of 1 MiB, 349,526 bytes)")
    ap.add_argument("--row-padding", action="store_true", help="pass FEC_FLAG_ROW_PADDING (rows run to their next 128-byte line)")
    args = ap.parse_args()
    rows = []
    for rnd in range(args.rounds):
        for ns in map(int, args.stripes.split(",")):
            r = one(ns, args.steps, flags=capi.FEC_FLAG_ASYNC | (capi.FEC_FLAG_ROW_PADDING if args.row_padding else 0),
                    sz=args.sz or None)
            r["row_padding"] = args.row_padding
            r["round"] = rnd
            rows.append(r)
            print(json.dumps(r), file=sys.stderr, flush=True)
    print(json.dumps({"tree": os.getcwd(), "rows": rows}))


if __name__ == "__main__":
    main()
