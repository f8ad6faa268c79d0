"""K=3/M=10 encode of one 64 MiB stripe (the cfg2 shape) with the output rows
16-byte aligned against rows at 6 (mod 16) -- packed [block][sz] rows, the
layout a C caller with one output buffer has -- through fec_encode_ex on
device memory.  Back-to-back launches between HIP events after warm-up
launches, aligned / misaligned interleaved over several rounds, each over a
rotation of buffer sets spanning >= 768 MiB (cold: every launch reads and
writes HBM).  Prints one JSON line.

    python tools/misaligned_bench.py [--rounds 3] [--n 40]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zfec_amd import capi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--n", type=int, default=40)
    ap.add_argument("--offset", type=int, default=6)
    args = ap.parse_args()
    k, m, r = 3, 10, 7
    sz = -(-(64 << 20) // k)
    code = capi.Code(k, m)
    st = torch.cuda.current_stream()
    nsets = max(2, -(-(768 << 20) // (m * sz)))
    srcs = [torch.randint(0, 256, (k, sz), dtype=torch.uint8, device="cuda") for _ in range(nsets)]
    outs = [torch.empty(r * sz + 256, dtype=torch.uint8, device="cuda") for _ in range(nsets)]
    nums = list(range(k, m))

    def launch(i, off):
        base = outs[i].data_ptr() + off
        # aligned: rows at a 16-byte multiple stride (sz rounded up), misaligned: packed rows
        stride = (sz + 15) // 16 * 16 if off == 0 else sz
        code.encode_ptrs([srcs[i][j].data_ptr() for j in range(k)], [base + q * stride for q in range(r)], nums, sz,
                         stream=st.cuda_stream)

    res = {"aligned": [], "misaligned": []}
    names = {}
    for _ in range(args.rounds):
        for tag, off in (("aligned", 0), ("misaligned", args.offset)):
            for i in range(3 * nsets):
                launch(i % nsets, off)
            names[tag] = capi.last_kernel_name()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(10_000_000)
            a.record(st)
            for i in range(args.n):
                launch(i % nsets, off)
            b.record(st)
            torch.cuda.synchronize()
            res[tag].append(a.elapsed_time(b) / args.n)
    tb = lambda ms: round(m * sz / (ms * 1e-3) / 1e12, 3)
    out = {"shape": "K=3/M=10, one %d-byte-block stripe, outputs at offset %d (mod 16), cold rotation of %d sets"
                    % (sz, args.offset, nsets),
           "kernels": names,
           "ms": {t: [round(x, 4) for x in v] for t, v in res.items()},
           "TBps_hbm": {t: [tb(x) for x in v] for t, v in res.items()},
           "misaligned_over_aligned": round(min(res["aligned"]) / min(res["misaligned"]), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
