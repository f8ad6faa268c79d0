#!/usr/bin/env python3
"""What bounds the K=20/M=60 bit-sliced encode (bench cfg4)?

The JIT generator's probe variants (zfec_amd/csrc/bitslice.cpp, BsOptions::probe,
ZFEC_HIP_JIT_PROBE) keep the kernel's structure and change one thing:
  real    the shipped kernel;
  nohbm   no HBM traffic: every buffer resource has num_records = 0, so the same
          loads return zeros and the same stores are dropped (all the
          arithmetic, the LDS sharing and barriers; the data is then zeros);
  noarith the same loads and stores, no arithmetic (no transposes, combinations
          or updates: outputs are an XOR of the raw inputs);
  zero    the shipped kernel on all-zero input blocks: the same instructions and
          traffic, no bit toggling in the data (MI355X_MICROARCH.md, DVFS
          give-back: the clock the chip holds depends on the data).
Each variant runs `reps` launches back to back on cfg4's 1024 x 1 MiB stripes
(rows 256-byte aligned, as bench.py lays them out), after `warm` untimed ones,
timed by HIP events, in interleaved rounds so clock and power state are shared
between variants.  Under rocprofv3 --pmc the same run gives each variant's
counters (tools/jit_probe_pmc.sh).  Only `real` produces the code's bytes
(checked against the table kernels on the first stripes).

usage: python tools/jit_probe.py [--shape cfg4|cfg3] [--rounds 3] [--reps 40] [--warm 40]
                                 [--variants real,nohbm,noarith]
(--shape cfg3: K=10/M=16, one 256 MiB stripe; launches rotate over buffer sets
spanning >= 768 MiB so every launch reads and writes HBM, as bench.py's cold legs.)
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

PROBES = {"real": 0, "nohbm": 1, "noarith": 2, "zero": 0, "lds2": 0, "lds1": 0}
# residency caps of the real kernel by extra dynamic LDS per workgroup (160 KiB per CU;
# the kernel's own 40 KiB of planes): 2 or 1 workgroups per CU instead of 3
EXTRA_LDS = {"lds2": 40 << 10, "lds1": 100 << 10}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="cfg4", choices=["cfg4", "cfg3"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--warm", type=int, default=300)
    ap.add_argument("--variants", default="real,zero,nohbm,noarith")
    ap.add_argument("--legs-out", default=None, help="JSON of the dispatch order per variant (tools/jit_probe_summary.py)")
    ap.add_argument("--prepare-only", action="store_true", help="compile the probe kernels (no GPU) and exit")
    args = ap.parse_args()
    k, m, ns, stripe = {"cfg4": (20, 60, 1024, 1 << 20), "cfg3": (10, 16, 1, 256 << 20)}[args.shape]
    r = m - k
    sz = -(-stripe // k)
    ld = (sz + 255) // 256 * 256
    nsets = max(1, -(-(768 << 20) // ((k + r) * ld * ns)))
    nums = list(range(k, m))
    code = capi.Code(k, m)
    names = args.variants.split(",")
    if args.prepare_only:
        for name in names:
            os.environ["ZFEC_HIP_JIT_PROBE"] = str(PROBES[name])
            capi.reload_config()
            code.jit_prepare_encode(nums)
        print("prepared", names)
        return
    capi.jit_mode(capi.JIT_FORCE)
    g = torch.Generator(device="cuda").manual_seed(20)
    datas = [torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda", generator=g) for _ in range(nsets)]
    data = datas[0]
    zeros = [torch.zeros((ns, k, ld), dtype=torch.uint8, device="cuda") for _ in range(nsets)]
    pars = [torch.zeros((ns, r, ld), dtype=torch.uint8, device="cuda") for _ in range(nsets)]
    par = pars[0]
    st = torch.cuda.current_stream()
    src = [datas]
    turn = [0]
    legs = []

    def leg(name, n):
        if legs and legs[-1][0] == name:
            legs[-1][1] += n
        else:
            legs.append([name, n])

    def launch():
        i = turn[0] % nsets
        turn[0] += 1
        code.encode_batch(src[0][i].data_ptr(), ld, k * ld, pars[i].data_ptr(), ld, r * ld, nums, sz, ns,
                          stream=st.cuda_stream)

    # the real kernel's bytes against the table kernels on a few stripes
    os.environ["ZFEC_HIP_JIT_PROBE"] = "0"
    capi.reload_config()
    launch()
    leg("check", 1)
    torch.cuda.synchronize()
    nchk = min(4, ns)
    want = torch.zeros((nchk, r, ld), dtype=torch.uint8, device="cuda")
    capi.jit_mode(capi.JIT_OFF)
    prev_g = capi.generic_mode(0)
    code.encode_batch(data.data_ptr(), ld, k * ld, want.data_ptr(), ld, r * ld, nums, sz, nchk,
                      stream=st.cuda_stream)
    torch.cuda.synchronize()
    capi.generic_mode(prev_g)
    capi.jit_mode(capi.JIT_FORCE)
    assert torch.equal(want[:, :, :sz], par[:nchk, :, :sz]), "real JIT kernel != table kernel"

    res = {n: [] for n in names}
    kern = {}
    for rnd in range(args.rounds):
        for name in names:
            os.environ["ZFEC_HIP_JIT_PROBE"] = str(PROBES[name])
            os.environ["ZFEC_HIP_JIT_LDS"] = str(EXTRA_LDS.get(name, 0))
            capi.reload_config()
            src[0] = zeros if name == "zero" else datas
            for _ in range(args.warm):
                launch()
            leg(name + " (warm)", args.warm)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(args.reps):
                launch()
            b.record(st)
            leg(name, args.reps)
            torch.cuda.synchronize()
            kern[name] = capi.last_kernel_name()
            res[name].append(a.elapsed_time(b) / args.reps * 1e3)  # us per launch
    os.environ["ZFEC_HIP_JIT_PROBE"] = "0"
    os.environ["ZFEC_HIP_JIT_LDS"] = "0"
    capi.reload_config()
    hbm = (k + r) * sz * ns
    out = {"shape": "K=%d/M=%d encode, %d x %d-byte stripes, rows %d B, %d buffer sets" % (k, m, ns, stripe, ld, nsets),
           "rounds": args.rounds,
           "reps": args.reps, "warm": args.warm, "algorithmic_bytes_per_launch": hbm, "variants": {}}
    for name in names:
        us = res[name]
        out["variants"][name] = {"kernel": kern[name], "us_per_launch": [round(x, 1) for x in us],
                                 "us_median": round(float(np.median(us)), 1),
                                 "hbm_frac_if_real": round(hbm / (float(np.median(us)) * 1e-6) / 8e12, 4)}
    print(json.dumps(out, indent=1))
    if args.legs_out:
        with open(args.legs_out, "w") as f:
            json.dump({"legs": legs, "kernels": kern}, f)


if __name__ == "__main__":
    main()
