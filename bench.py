#!/usr/bin/env python3
"""bench.py -- device-resident Reed-Solomon encode+decode throughput on MI355X.

Metric (BASELINE.json): "encode+decode GB/s (device-resident input) at K/M;
% of HBM roofline".  Workload (BASELINE.json configs[1]): K=3, M=10, one
64 MiB stripe per GPU (block size sz = ceil(64 MiB / 3) = 22,369,622 B).

One step = encode the stripe (3 primaries -> 7 secondaries, one launch) +
secondary-only decode (blocks 3,4,5 -> primaries 0,1,2, one launch), both
through the C-ABI (fec_encode_batch / fec_decode_batch) on torch's current
stream, inputs resident in HBM.  value = (encode input + decode input bytes)
= 2*k*sz per step per GPU, summed over GPUs, / wall time of the K timed steps
(max over ranks), in GB/s (1e9).

Multi-GPU (torchrun, one rank per GPU): each rank encodes/decodes its own
stripe -- stripes are independent, no data-path collective (weak scaling);
the only collectives are the timing barrier and the max-over-ranks reduce.

Also reported: the dominant kernel's roofline (encode: (k+r)*sz algorithmic
HBM bytes per launch / mean launch time from HIP events on the launch
stream), the decode kernel's, a batched 1 MiB-stripe encode (the north-star
target shape), and a bounded CPU baseline (rank 0, N=1) of the reference's
own C code (oracle/_ref, kind "reference") or the oracle restatement (kind
"port").
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from zfec_amd import capi  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

K, M = 3, 10
STRIPE = 64 << 20


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-extra", action="store_true", help="skip the 1 MiB-stripe batched leg")
    return p.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return dist, rank, world, local
    torch.cuda.set_device(0)
    return None, 0, 1, 0


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, x):
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, x):
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def pmc_traffic():
    """Per-launch HBM bytes of the encode kernel from the committed PMC summary
    (profiles/pmc_summary.json, made by tools/pmc.sh + tools/pmc_summary.py)."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("encode_cfg2", {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(seconds, sz):
    """Bounded CPU sample of the same workload (encode + secondary-only decode
    of one K=3/M=10 stripe of 3*sz bytes per step), one stripe per thread."""
    from oracle import oracle

    ref = oracle.ref_module()
    try:
        threads = len(os.sched_getaffinity(0))
    except AttributeError:
        threads = os.cpu_count() or 1
    threads = max(1, min(16, threads))
    rng = np.random.default_rng(7)
    proto = [rng.integers(0, 256, size=sz, dtype=np.uint8).tobytes() for _ in range(K)]
    counts = [0] * threads
    stop = threading.Event()

    if ref is not None:
        kind = "reference"

        def work(t):
            enc, dec = ref.Encoder(K, M), ref.Decoder(K, M)
            blocks = [bytes(b) for b in proto]
            while not stop.is_set():
                out = enc.encode(blocks)
                dec.decode(out[K:2 * K], list(range(K, 2 * K)))
                counts[t] += 1
    else:
        kind = "port"
        data = np.frombuffer(b"".join(proto), dtype=np.uint8).reshape(K, sz)

        def work(t):
            while not stop.is_set():
                par = oracle.encode(K, M, data)
                oracle.decode(K, M, par[:K], list(range(K, 2 * K)))
                counts[t] += 1

    ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    time.sleep(seconds)
    stop.set()
    for th in ths:
        th.join()
    el = time.perf_counter() - t0
    steps = sum(counts)
    gbps = steps * 2 * K * sz / el / 1e9
    return {"value": round(gbps, 4), "unit": "GB/s", "cores": threads, "kind": kind,
            "sample": "%d steps (encode+secondary-only decode of a K=3/M=10 %d-byte stripe) in %.1f s, "
                      "one stripe per thread; %s" % (
                          steps, K * sz, el,
                          "reference zfec/fec.c+_fecmodule.c compiled by oracle/Makefile (-O2 -march=x86-64-v2)"
                          if kind == "reference" else "oracle/fec_oracle.c restatement")}


def align_up(x, a):
    return (x + a - 1) // a * a


def run_stripe_bench(code, k, m, sz, steps, warmup, dist):
    """Returns (elapsed_s, enc_ms_mean, dec_ms_mean) over `steps` timed steps.

    HBM layout: each stripe is a [block][row_stride] array whose row stride is
    sz rounded up to 256 bytes, so every block starts 256-byte aligned (the
    blocks of the reference's API are separate buffers, i.e. aligned too)."""
    r = m - k
    ld = align_up(sz, 256)
    g = torch.Generator(device="cuda").manual_seed(1234 + k)
    data = torch.randint(0, 256, (k, ld), dtype=torch.uint8, device="cuda", generator=g)
    par = torch.empty((r, ld), dtype=torch.uint8, device="cuda")
    rec = torch.empty((k, ld), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    enc_nums = list(range(k, m))
    dec_slots = list(range(k, 2 * k))  # blocks 3,4,5: no primaries present

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        code.encode_batch(data.data_ptr(), ld, 0, par.data_ptr(), ld, 0, enc_nums, sz, 1, stream=sh)
        if ev is not None:
            ev[1].record(stream)
        code.decode_batch(par.data_ptr(), ld, 0, rec.data_ptr(), ld, 0, dec_slots, sz, 1, stream=sh)
        if ev is not None:
            ev[2].record(stream)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    # correctness of the timed configuration (size-independent property)
    assert torch.equal(rec[:, :sz], data[:, :sz]), "decode(encode(x)) != x"
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    barrier(dist)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(evs[i])
    torch.cuda.synchronize()
    barrier(dist)
    el = time.perf_counter() - t0
    step_enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    step_dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))

    # Per-kernel launch duration for the roofline: the same launches back to
    # back on the same stream, bracketed by one pair of HIP events (the
    # in-step brackets above also contain each launch's dispatch latency).
    def b2b(fn, n=20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(n):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    enc_ms = b2b(lambda: code.encode_batch(data.data_ptr(), ld, 0, par.data_ptr(), ld, 0, enc_nums, sz, 1, stream=sh))
    dec_ms = b2b(lambda: code.decode_batch(par.data_ptr(), ld, 0, rec.data_ptr(), ld, 0, dec_slots, sz, 1, stream=sh))
    return el, enc_ms, dec_ms, step_enc_ms, step_dec_ms


def run_batched_1mib(steps):
    """North-star shape: K=3/M=10 encode of 1 MiB stripes, 256 stripes per
    launch (block rows 256-byte aligned, as in the main workload)."""
    k, m, ns = 3, 10, 256
    sz = -(-(1 << 20) // k)
    ld = align_up(sz, 256)
    code = capi.Code(k, m)
    src = torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda")
    dst = torch.empty((ns, m - k, ld), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    nums = list(range(k, m))
    for _ in range(3):
        code.encode_batch(src.data_ptr(), ld, k * ld, dst.data_ptr(), ld, (m - k) * ld, nums, sz, ns, stream=st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(steps):
        code.encode_batch(src.data_ptr(), ld, k * ld, dst.data_ptr(), ld, (m - k) * ld, nums, sz, ns, stream=st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    in_gbps = ns * k * sz / (ms * 1e-3) / 1e9
    hbm = in_gbps * m / k
    return {"shape": "K=3/M=10 encode, 256 x 1 MiB stripes per launch", "input_GBps": round(in_gbps, 1),
            "hbm_GBps": round(hbm, 1), "frac_of_peak": round(hbm / HBM_PEAK_GBPS, 4), "ms_per_launch": round(ms, 4)}


def main():
    args = parse()
    dist, rank, world, local = dist_setup(args)
    sz = -(-STRIPE // K)
    code = capi.Code(K, M)
    el, enc_ms, dec_ms, step_enc_ms, step_dec_ms = run_stripe_bench(code, K, M, sz, args.steps, args.warmup, dist)
    el = max_over_ranks(dist, el)
    total_bytes = sum_over_ranks(dist, float(args.steps * 2 * K * sz))
    value = total_bytes / el / 1e9
    enc_bytes = (K + (M - K)) * sz       # read k blocks, write m-k blocks
    dec_bytes = (K + K) * sz             # read k blocks, write k recovered
    enc_ach = enc_bytes / (enc_ms * 1e-3) / 1e9
    dec_ach = dec_bytes / (dec_ms * 1e-3) / 1e9
    out = {
        "metric": "encode+decode GB/s (device-resident input) at K/M; % of HBM roofline",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (torch.randint bytes, resident in HBM)",
        "config": {"workload": "K=3 M=10, one 64 MiB stripe per GPU: encode (3->7 blocks) + secondary-only "
                               "decode (blocks 3,4,5 -> 0,1,2)", "k": K, "m": M, "stripe_bytes": STRIPE,
                   "block_bytes": sz, "block_row_stride": align_up(sz, 256), "parallelism": "stripes sharded across GPUs (dp%d), no collective" % world},
        "roofline": {"bound": "hbm", "achieved": round(enc_ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(enc_ach / HBM_PEAK_GBPS, 4), "traffic": pmc_traffic(),
                     "kernel": "matapply_reg<3,7> (encode)", "algorithmic_bytes_per_launch": enc_bytes,
                     "launch_ms": round(enc_ms, 4), "in_step_event_ms": round(step_enc_ms, 4),
                     "timing": "20 back-to-back launches between two HIP events on the launch stream"},
        "decode_roofline": {"achieved": round(dec_ach, 1), "frac": round(dec_ach / HBM_PEAK_GBPS, 4),
                            "kernel": "matapply_reg<3,3> (decode)", "algorithmic_bytes_per_launch": dec_bytes,
                            "launch_ms": round(dec_ms, 4), "in_step_event_ms": round(step_dec_ms, 4)},
        "encode_input_GBps": round(K * sz / (enc_ms * 1e-3) / 1e9, 1),
        "decode_input_GBps": round(K * sz / (dec_ms * 1e-3) / 1e9, 1),
    }
    if rank == 0 and not args.no_extra:
        out["batched_1MiB"] = run_batched_1mib(20)
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, sz)
        except Exception as e:  # the baseline must never sink the GPU measurement
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
