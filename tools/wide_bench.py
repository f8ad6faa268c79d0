#!/usr/bin/env python3
"""Wide codes (k > 32) on the device: one 64 MiB stripe of
94/100 (the reference's own benchmark shape, benchmark-zfec/Main.hs:17),
128/256, 200/256 and 255/256, encode and a decode of the first min(k, m-k)
primaries from secondaries, device-resident, timed like bench.py's cold legs:
back-to-back launches (a spin kernel holds the stream while they are queued)
over a rotation of disjoint buffer sets spanning >= 768 MiB.

Variants: "shipped" -- the library as shipped in auto mode, after its
background compiles (jit_wait): one pass over all k inputs per row group of
<= 48 (matapply_bsg's device-side table, or a specialised JIT kernel up to
1600 coefficients); "generic" -- JIT off, what serves a first-seen matrix
(generic mode 2: matapply_bsr where it fits, else matapply_bsg); "bsg" -- JIT
off, matapply_bsg only; "passes" -- round 2's path, the table kernels in
XOR-accumulating passes of 32 inputs (generic kernel and JIT off).  The
decodes are checked against the stripe every time.

    python tools/wide_bench.py [--shapes 94/100,128/256,200/256] [--launches 10]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (back_to_back, COLD_SPAN, HBM peak)
from zfec_amd import capi  # noqa: E402


# variant -> (JIT mode, generic mode)
VARIANTS = {"shipped": (capi.JIT_AUTO, 2), "generic": (capi.JIT_OFF, 2), "bsg": (capi.JIT_OFF, 1),
            "passes": (capi.JIT_OFF, 0)}


def run_shape(k, m, launches, variant):
    r = m - k
    sz = -(-(64 << 20) // k)
    ld = (sz + 255) // 256 * 256
    nrec = min(k, r)
    # decode: received = the last nrec primaries missing, replaced by the first nrec secondaries
    slots = list(range(k - nrec)) + list(range(k, k + nrec))
    missing = list(range(k - nrec, k))
    fp = (k + r) * ld
    nsets = max(2, -(-bench.COLD_SPAN // fp))
    g = torch.Generator(device="cuda").manual_seed(k)
    data = [torch.randint(0, 256, (1, k, ld), dtype=torch.uint8, device="cuda", generator=g) for _ in range(nsets)]
    par = [torch.empty((1, r, ld), dtype=torch.uint8, device="cuda") for _ in range(nsets)]
    code = capi.Code(k, m)
    nums = list(range(k, m))
    st = torch.cuda.current_stream()
    jit, gen = VARIANTS[variant]
    pj, pg = capi.jit_mode(jit), capi.generic_mode(gen)

    def enc_i(i):
        def f(sh):
            code.encode_batch(data[i].data_ptr(), ld, k * ld, par[i].data_ptr(), ld, r * ld, nums, sz, 1, stream=sh)
        return f

    for i in range(nsets):
        enc_i(i)(st.cuda_stream)
        enc_i(i)(st.cuda_stream)
    capi.jit_wait()
    torch.cuda.synchronize()
    recv = [torch.cat([data[i][:, :k - nrec], par[i][:, :nrec]], dim=1).contiguous() for i in range(nsets)]
    rec = [torch.empty((1, nrec, ld), dtype=torch.uint8, device="cuda") for _ in range(nsets)]

    def dec_i(i):
        def f(sh):
            code.decode_batch(recv[i].data_ptr(), ld, k * ld, rec[i].data_ptr(), ld, nrec * ld, slots, sz, 1,
                              stream=sh)
        return f

    for i in range(nsets):
        dec_i(i)(st.cuda_stream)
        dec_i(i)(st.cuda_stream)
    capi.jit_wait()
    torch.cuda.synchronize()
    for i in range(nsets):
        assert torch.equal(rec[i][:, :, :sz], data[i][:, missing, :sz]), (k, m, variant)
    enc_ms, _ = bench.back_to_back([enc_i(i) for i in range(nsets)], launches, st, "wide encode")
    enc_kern = capi.last_kernel_name()
    dec_ms, _ = bench.back_to_back([dec_i(i) for i in range(nsets)], launches, st, "wide decode")
    dec_kern = capi.last_kernel_name()
    torch.cuda.synchronize()
    for i in range(nsets):
        assert torch.equal(rec[i][:, :, :sz], data[i][:, missing, :sz]), (k, m, variant)
    capi.jit_mode(pj)
    capi.generic_mode(pg)
    gbps = lambda b, ms: b / (ms * 1e-3) / 1e9
    return {"encode": {"kernel": enc_kern, "ms": round(enc_ms, 3), "input_GBps": round(gbps(k * sz, enc_ms), 1),
                       "hbm_frac": round(gbps((k + r) * sz, enc_ms) / bench.HBM_PEAK_GBPS, 4)},
            "decode": {"kernel": dec_kern, "recovered": nrec, "ms": round(dec_ms, 3),
                       "input_GBps": round(gbps(k * sz, dec_ms), 1),
                       "hbm_frac": round(gbps((k + nrec) * sz, dec_ms) / bench.HBM_PEAK_GBPS, 4)},
            "nsets": nsets}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="94/100,128/256,200/256,255/256")
    ap.add_argument("--variants", default="shipped,passes")
    ap.add_argument("--launches", type=int, default=10)
    args = ap.parse_args()
    out = {"stripe": "one 64 MiB stripe, rows 256-byte aligned, device-resident, cold rotation", "shapes": {}}
    for shape in args.shapes.split(","):
        k, m = map(int, shape.split("/"))
        out["shapes"][shape] = {v: run_shape(k, m, args.launches, v) for v in args.variants.split(",")}
        torch.cuda.empty_cache()
        print(shape, json.dumps(out["shapes"][shape]), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
