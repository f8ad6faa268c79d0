#!/usr/bin/env python3
"""A/B of the three kernel families that can serve a wide-code launch, on
device-resident stripes (interleaved rounds, medians):

  table   matapply_lds (v_perm table lookups; JIT off, generic mode 0)
  bsg     matapply_bsg<RT,2> (bit-sliced, coefficients as run-time data; generic mode 1)
  bsr     matapply_bsr (bit-sliced, one precompiled routine call per coefficient; generic mode 2)
  jit     zfec_hip_bitslice_* (bit-sliced, the matrix compiled in; hipRTC)

(Round 2's bsg_sb / bsg_bb / bsg_p4 variants and the knobs that selected them
were removed with the code in round 4; profiles/r02_bsg_ab*.log keeps their
figures.)

Shapes: cfg3 (K=10/M=16, one 256 MiB stripe) and cfg4 (K=20/M=60, 1024 x
1 MiB stripes), encode and last-k decode.  Then decode_fresh: cfg4 decodes,
each from a new random set of k received blocks (every launch a matrix the
process has not seen: no JIT kernel exists for it), timed one launch at a
time between events; mean input GB/s over the patterns and a bit-exact check
of every one against the table kernel.

Per launch time = events around `reps` back-to-back launches / reps;
HBM GB/s = (k + r) * sz * stripes / time; input GB/s = k * sz * stripes / time.

usage: python tools/bsg_bench.py [--shapes cfg3,cfg4] [--rounds 5] [--fresh 20]
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
VARIANTS = [("table", capi.JIT_OFF, 0), ("bsg", capi.JIT_OFF, 1), ("bsr", capi.JIT_OFF, 2),
            ("jit", capi.JIT_FORCE, 2)]


def place(nums, k):
    slots = [None] * k
    sec = iter([n for n in nums if n >= k])
    for n in nums:
        if n < k:
            slots[n] = n
    return [s if s is not None else next(sec) for s in slots]


def set_variant(jit, gen):
    capi.jit_mode(jit)
    capi.generic_mode(gen)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="cfg3,cfg4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--fresh", type=int, default=20)
    args = ap.parse_args()
    st = torch.cuda.current_stream()
    res = {}
    for shape in [s for s in args.shapes.split(",") if s]:
        k, m, S, ns = SHAPES[shape]
        r = m - k
        sz = -(-S // k)
        ld = (sz + 255) // 256 * 256
        g = torch.Generator(device="cuda").manual_seed(k)
        data = torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda", generator=g)
        code = capi.Code(k, m)
        slots = place(list(range(m - k, m)), k)
        nrec = sum(1 for s in slots if s >= k)
        outs = {v[0]: torch.zeros((ns, r, ld), dtype=torch.uint8, device="cuda") for v in VARIANTS}
        recs = {v[0]: torch.zeros((ns, nrec, ld), dtype=torch.uint8, device="cuda") for v in VARIANTS}
        recv = None
        times = {(v[0], d): [] for v in VARIANTS for d in ("enc", "dec")}
        kern = {}
        for rnd in range(args.rounds):
            for name, jit, gen in VARIANTS:
                set_variant(jit, gen)
                out, rec = outs[name], recs[name]

                def enc():
                    code.encode_batch(data.data_ptr(), ld, k * ld, out.data_ptr(), ld, r * ld, list(range(k, m)), sz,
                                      ns, stream=st.cuda_stream)

                def dec():
                    code.decode_batch(recv.data_ptr(), ld, k * ld, rec.data_ptr(), ld, nrec * ld, slots, sz, ns,
                                      stream=st.cuda_stream)

                enc()
                kern[(name, "enc")] = capi.last_kernel_name()
                if recv is None:
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
                print(shape, d, "%-8s" % name, json.dumps(row), flush=True)
        if shape == "cfg4" and args.fresh:
            allb = torch.cat([data, outs["table"]], dim=1)  # [ns, m, ld]
            rng = np.random.default_rng(99)
            ms_b, ms_t, ms_r, names, ok = [], [], [], {"bsg": set(), "bsr": set()}, True
            out_r = torch.empty((ns, k, ld), dtype=torch.uint8, device="cuda")
            out_b = torch.empty((ns, k, ld), dtype=torch.uint8, device="cuda")
            out_t = torch.empty((ns, k, ld), dtype=torch.uint8, device="cuda")
            for p in range(args.fresh):
                nums = sorted(int(x) for x in rng.choice(m, size=k, replace=False))
                sl = place(nums, k)
                nr = sum(1 for s in sl if s >= k)
                if nr == 0:
                    continue
                rv = allb[:, sl, :].contiguous()
                for name, tgt, lst in (("bsr", out_r, ms_r), ("bsg", out_b, ms_b), ("table", out_t, ms_t)):
                    set_variant(capi.JIT_OFF, {"bsr": 2, "bsg": 1, "table": 0}[name])
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    code.decode_batch(rv.data_ptr(), ld, k * ld, tgt.data_ptr(), ld, k * ld, sl, sz, ns,
                                      stream=st.cuda_stream)
                    e1.record(st)
                    if name in names:
                        names[name].add(capi.last_kernel_name())
                    torch.cuda.synchronize()
                    lst.append((e0.elapsed_time(e1), nr))
                miss = [i for i in range(k) if sl[i] >= k]
                ok = ok and bool(torch.equal(out_b[:, :nr, :sz], out_t[:, :nr, :sz]))
                ok = ok and bool(torch.equal(out_r[:, :nr, :sz], out_t[:, :nr, :sz]))
                ok = ok and bool(torch.equal(out_b[:, :nr, :sz], data[:, miss, :sz]))
            for name, lst in (("bsr", ms_r), ("bsg", ms_b), ("table", ms_t)):
                gbps = [k * sz * ns / (t * 1e-3) / 1e9 for t, _ in lst]
                row = {"patterns": len(lst), "mean_recovered": round(float(np.mean([n for _, n in lst])), 1),
                       "input_GBps_mean": round(float(np.mean(gbps)), 1),
                       "input_GBps_min": round(float(np.min(gbps)), 1),
                       "kernels": sorted(names[name]) if name in names else "table", "bitexact": ok}
                res["cfg4 decode_fresh %s" % name] = row
                print("cfg4 decode_fresh", "%-6s" % name, json.dumps(row), flush=True)
    set_variant(capi.JIT_AUTO, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
