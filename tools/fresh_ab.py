"""Decodes of first-seen erasure patterns (bench.py decode_fresh) on one
shape, in this process: cfg4 (K=20/M=60, 1024 x 1 MiB) or cfg3, N random
patterns, each launch timed between events, every result checked against the
stripe.  Prints one JSON line; run it in several processes to compare
builds or variants.

    python tools/fresh_ab.py [--shape cfg4] [--patterns 20] [--tag name]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from zfec_amd import capi  # noqa: E402

SHAPES = {"cfg4": (20, 60, 1 << 20, 1024), "cfg3": (10, 16, 256 << 20, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="cfg4")
    ap.add_argument("--patterns", type=int, default=20)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    k, m, stripe, ns = SHAPES[args.shape]
    r = m - k
    sz = -(-stripe // k)
    ld = bench.row_stride(sz)
    g = torch.Generator(device="cuda").manual_seed(99)
    data = torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda", generator=g)
    par = torch.empty((ns, r, ld), dtype=torch.uint8, device="cuda")
    recv = torch.empty((ns, k, ld), dtype=torch.uint8, device="cuda")
    code = capi.Code(k, m)
    st = torch.cuda.current_stream()
    code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld, list(range(k, m)), sz, ns,
                      stream=st.cuda_stream)
    torch.cuda.synchronize()
    res = bench.decode_fresh(code, k, m, sz, ns, ld, data, par, recv, args.patterns, st)
    res.update({"shape": args.shape, "tag": args.tag, "generic": os.environ.get("ZFEC_HIP_GENERIC", "2")})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
