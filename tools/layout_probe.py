#!/usr/bin/env python3
"""cfg5 (10^6 K=3/M=10 objects of 4 KiB, sz = 1366) in two HBM layouts, same
encode + last-k decode step as bench.py:

  object-major  [stripe][block][row]: bench.py's layout (256-byte rows,
                FEC_FLAG_ROW_PADDING) -- every stripe is 10 short rows;
  block-major   [block][stripe * sz]: block j of every object packed back to
                back, so the batch is one stripe of 10^6 * 1366 bytes per block
                (fec_abi.cpp run_batch collapses it into one long-stream launch).

GB/s = 2 * k * sz * stripes / (step time), events around `steps` steps after
warmup.  Both layouts are checked against each other (decode(encode(x)) == x).

--shape cfg4 runs the same comparison for 1024 K=20/M=60 stripes of 1 MiB
(sz = 52,429; bench rows of 52,480 bytes).

usage: python tools/layout_probe.py [--shape cfg5|cfg4] [--stripes N] [--steps 20] [--rounds 3]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from zfec_amd import capi  # noqa: E402


def place(nums, k):
    slots = [None] * k
    sec = iter([n for n in nums if n >= k])
    for n in nums:
        if n < k:
            slots[n] = n
    return [s if s is not None else next(sec) for s in slots]


def timed(step, steps, warmup):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(steps):
        step()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--shape", default="cfg5", choices=["cfg5", "cfg4"])
    p.add_argument("--stripes", type=int, default=0)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    k, m, stripe, ns = {"cfg5": (3, 10, 4096, 1000000), "cfg4": (20, 60, 1 << 20, 1024)}[a.shape]
    ns = a.stripes or ns
    r = m - k
    sz = -(-stripe // k)
    code = capi.Code(k, m)
    slots = place(list(range(m - k, m)), k)
    missing = [i for i in range(k) if slots[i] >= k]
    st = torch.cuda.current_stream().cuda_stream
    gen = torch.Generator(device="cuda").manual_seed(5)
    fl = capi.FEC_FLAG_ASYNC

    # object-major, as bench.py
    ld = -(-sz // 256) * 256  # bench.py row_stride
    o_data = torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda", generator=gen)
    o_par = torch.empty((ns, r, ld), dtype=torch.uint8, device="cuda")
    o_recv = torch.empty((ns, k, ld), dtype=torch.uint8, device="cuda")
    o_rec = torch.empty((ns, len(missing), ld), dtype=torch.uint8, device="cuda")
    ofl = fl | capi.FEC_FLAG_ROW_PADDING

    def o_step():
        code.encode_batch(o_data.data_ptr(), ld, k * ld, o_par.data_ptr(), ld, r * ld, list(range(k, m)), sz, ns,
                          stream=st, flags=ofl)
        code.decode_batch(o_recv.data_ptr(), ld, k * ld, o_rec.data_ptr(), ld, len(missing) * ld, slots, sz, ns,
                          stream=st, flags=ofl)

    code.encode_batch(o_data.data_ptr(), ld, k * ld, o_par.data_ptr(), ld, r * ld, list(range(k, m)), sz, ns,
                      stream=st, flags=ofl)
    for i, s in enumerate(slots):
        o_recv[:, i].copy_(o_data[:, s] if s < k else o_par[:, s - k])

    # block-major: the same objects
    b_data = o_data[:, :, :sz].permute(1, 0, 2).contiguous()  # [k][ns][sz]
    b_par = torch.empty((r, ns, sz), dtype=torch.uint8, device="cuda")
    b_recv = torch.empty((k, ns, sz), dtype=torch.uint8, device="cuda")
    b_rec = torch.empty((len(missing), ns, sz), dtype=torch.uint8, device="cuda")
    bs = ns * sz

    def b_step():
        code.encode_batch(b_data.data_ptr(), bs, sz, b_par.data_ptr(), bs, sz, list(range(k, m)), sz, ns, stream=st,
                          flags=fl)
        code.decode_batch(b_recv.data_ptr(), bs, sz, b_rec.data_ptr(), bs, sz, slots, sz, ns, stream=st, flags=fl)

    code.encode_batch(b_data.data_ptr(), bs, sz, b_par.data_ptr(), bs, sz, list(range(k, m)), sz, ns, stream=st,
                      flags=fl)
    for i, s in enumerate(slots):
        b_recv[i].copy_(b_data[s] if s < k else b_par[s - k])
    o_step()
    b_step()
    torch.cuda.synchronize()
    assert torch.equal(b_par, o_par[:, :, :sz].permute(1, 0, 2)), "layouts disagree on parity"
    assert torch.equal(b_rec, b_data[missing]), "block-major decode(encode(x)) != x"
    assert torch.equal(o_rec[:, :, :sz], o_data[:, missing, :sz]), "object-major decode(encode(x)) != x"

    # wide codes: the second large launch of a matrix queues its bit-sliced
    # kernel's compile (as in bench.py); wait for it, then check again
    o_step()
    b_step()
    capi.jit_wait()
    b_par.zero_()
    o_step()
    b_step()
    torch.cuda.synchronize()
    assert torch.equal(b_par, o_par[:, :, :sz].permute(1, 0, 2)), "layouts disagree on parity (JIT kernels)"
    assert torch.equal(b_rec, b_data[missing]), "block-major decode(encode(x)) != x (JIT kernels)"
    res = {"object_major_ms": [], "block_major_ms": []}
    for _ in range(a.rounds):
        res["object_major_ms"].append(round(timed(o_step, a.steps, a.warmup), 4))
        res["block_major_ms"].append(round(timed(b_step, a.steps, a.warmup), 4))
    code.encode_batch(b_data.data_ptr(), bs, sz, b_par.data_ptr(), bs, sz, list(range(k, m)), sz, ns, stream=st,
                      flags=fl)
    kb = capi.last_kernel_name()
    code.encode_batch(o_data.data_ptr(), ld, k * ld, o_par.data_ptr(), ld, r * ld, list(range(k, m)), sz, ns,
                      stream=st, flags=ofl)
    ko = capi.last_kernel_name()
    torch.cuda.synchronize()
    byts = 2 * k * sz * ns
    for key in ("object_major", "block_major"):
        ms = sorted(res[key + "_ms"])[len(res[key + "_ms"]) // 2]
        res[key + "_GBps"] = round(byts / (ms * 1e-3) / 1e9, 1)
    res.update({"collapse": os.environ.get("ZFEC_HIP_BATCH_COLLAPSE", "1"), "shape": a.shape, "k": k, "m": m, "stripes": ns, "sz": sz, "encode_kernel_object_major": ko, "encode_kernel_block_major": kb})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
