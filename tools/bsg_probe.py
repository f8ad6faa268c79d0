#!/usr/bin/env python3
"""Short, profiler-friendly run of one wide-code launch shape for counter
passes (tools/bsg_pmc.sh): cfg4's decode from the last k blocks (K=20/M=60,
1024 x 1 MiB stripes, r = 20) on the chosen kernel family, `--reps` launches.

usage: python tools/bsg_probe.py --kind bsg|jit|table [--op dec|enc] [--reps 10]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from zfec_amd import capi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="bsg", choices=["bsg", "jit", "table"])
    ap.add_argument("--op", default="dec", choices=["dec", "enc"])
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    k, m, ns = 20, 60, 1024
    sz = -(-(1 << 20) // k)
    ld = (sz + 255) // 256 * 256
    r = m - k
    capi.jit_mode(capi.JIT_FORCE if a.kind == "jit" else capi.JIT_OFF)
    capi.generic_mode(0 if a.kind == "table" else 1)
    code = capi.Code(k, m)
    data = torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda")
    par = torch.empty((ns, r, ld), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    slots = list(range(m - k, m))
    rec = torch.empty((ns, k, ld), dtype=torch.uint8, device="cuda")
    for _ in range(a.reps):
        if a.op == "enc":
            code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld, list(range(k, m)), sz, ns,
                              stream=st)
        else:
            code.decode_batch(data.data_ptr(), ld, k * ld, rec.data_ptr(), ld, k * ld, slots, sz, ns, stream=st)
    torch.cuda.synchronize()
    print("kernel", capi.last_kernel_name())


if __name__ == "__main__":
    main()
