#!/usr/bin/env python3
"""End-to-end (host memory -> GPU -> host memory) K=3/M=10 encode and decode
of one 64 MiB stripe, the path filefec/cmdline_zfec would take.

Strategies timed (GB/s of stripe input bytes, 1e9):
  bytes_api      zfec_amd.Encoder.encode(list of bytes) -> list of bytes
                 (pageable host buffers; the library stages them), per call
                 with the free of the previous call's outputs; then again
                 after zfec_amd.reuse_host_memory()
  pinned_api     the same C-ABI call with pinned (hipHostMalloc'd) host buffers,
                 e.g. a reader that reads file/socket data straight into pinned
                 memory: the kernel reads and writes them in place over PCIe
                 (zero-copy, both link directions at once; run_single in
                 zfec_amd/csrc/fec_abi.cpp)
  bytes_call     the library call alone: the previous call's output bytes are
                 still alive while the next call runs (their free is outside
                 the timing), after zfec_amd.reuse_host_memory()
  host_batch     Encoder.encode_batch / Decoder.decode_batch on a numpy array
                 of 65,536 K=3/M=10 objects of 4 KiB (256 MiB): one call each,
                 staged through pinned slots by the library's host threads
  h2d/d2h        raw pinned hipMemcpy rates for reference
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import zfec_amd  # noqa: E402
from zfec_amd import capi  # noqa: E402


def gbps(nbytes, s):
    return round(nbytes / s / 1e9, 2)


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    k, m, S = 3, 10, 64 << 20
    sz = -(-S // k)
    rng = np.random.default_rng(1)
    data = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
    blocks = [data[i].tobytes() for i in range(k)]
    res = {"stripe_bytes": k * sz, "k": k, "m": m}

    enc, dec = zfec_amd.Encoder(k, m), zfec_amd.Decoder(k, m)
    out = enc.encode(blocks)

    def bytes_rates(tag):
        # per call, the free of the previous call's output bytes included (as a
        # caller sees it), median of 7
        te, td = [], []
        for _ in range(7):
            t0 = time.perf_counter()
            enc.encode(blocks)
            t1 = time.perf_counter()
            dec.decode(out[3:6], [3, 4, 5])
            td.append(time.perf_counter() - t1)
            te.append(t1 - t0)
        res["bytes_api_encode_GBps" + tag] = gbps(k * sz, sorted(te)[3])
        res["bytes_api_decode_GBps" + tag] = gbps(k * sz, sorted(td)[3])

    # default glibc policy: every call's fresh output pages are faulted in and
    # returned to the kernel on free
    bytes_rates("")
    # zfec_amd.reuse_host_memory(): freed blocks stay in the heap for the next call
    assert zfec_amd.reuse_host_memory()
    bytes_rates("_reuse_host_memory")
    assert dec.decode(out[3:6], [3, 4, 5]) == blocks
    assert enc.encode(blocks) == out

    # the library call alone: outputs of the previous call kept alive, so no
    # free (munmap) falls inside the timing
    te, td, keep = [], [], []
    for _ in range(7):
        t0 = time.perf_counter()
        keep.append(enc.encode(blocks))
        t1 = time.perf_counter()
        keep.append(dec.decode(out[3:6], [3, 4, 5]))
        t2 = time.perf_counter()
        te.append(t1 - t0)
        td.append(t2 - t1)
        if len(keep) > 4:
            del keep[:2]
    res["bytes_call_encode_GBps"] = gbps(k * sz, sorted(te)[3])
    res["bytes_call_decode_GBps"] = gbps(k * sz, sorted(td)[3])
    del keep

    # a host batch of small objects: one encode_batch / decode_batch call each
    nb, osz = 65536, -(-4096 // k)
    hb = rng.integers(0, 256, size=(nb, k, osz), dtype=np.uint8)
    par = enc.encode_batch(hb)
    t = timeit(lambda: enc.encode_batch(hb), 3)
    res["host_batch_encode_GBps"] = gbps(hb.nbytes, t)
    recv = np.ascontiguousarray(np.asarray(par)[:, :k])
    t = timeit(lambda: dec.decode_batch(recv, list(range(k, 2 * k))), 3)
    res["host_batch_decode_GBps"] = gbps(hb.nbytes, t)
    assert np.array_equal(np.asarray(dec.decode_batch(recv, list(range(k, 2 * k)))), hb)
    res["host_batch"] = "%d objects of %d bytes per block (K=3/M=10), numpy in and out" % (nb, osz)

    # pinned host buffers through the C-ABI
    pin_in = torch.from_numpy(data.copy()).pin_memory()
    pin_out = torch.empty((m - k, sz), dtype=torch.uint8).pin_memory()
    pin_rec = torch.empty((k, sz), dtype=torch.uint8).pin_memory()
    code = capi.Code(k, m)
    ins = [pin_in[i].data_ptr() for i in range(k)]
    outs = [pin_out[i].data_ptr() for i in range(m - k)]

    def enc_pinned():
        code.encode_ptrs(ins, outs, list(range(k, m)), sz, flags=capi.FEC_FLAG_LIBRARY_STREAM)

    t = timeit(enc_pinned, 5)
    res["pinned_api_encode_GBps"] = gbps(k * sz, t)
    assert b"".join(pin_out[i].numpy().tobytes() for i in range(m - k)) == b"".join(out[k:])
    rec = [pin_rec[i].data_ptr() for i in range(k)]

    def dec_pinned():
        code.decode_ptrs([pin_out[i].data_ptr() for i in range(3)], rec, [3, 4, 5], sz,
                         flags=capi.FEC_FLAG_LIBRARY_STREAM)

    t = timeit(dec_pinned, 5)
    res["pinned_api_decode_GBps"] = gbps(k * sz, t)
    assert np.array_equal(pin_rec.numpy(), data)

    # raw copy rates
    dev = torch.empty((k, sz), dtype=torch.uint8, device="cuda")
    t = timeit(lambda: dev.copy_(pin_in, non_blocking=True), 5)
    res["raw_h2d_pinned_GBps"] = gbps(k * sz, t)
    t = timeit(lambda: pin_in.copy_(dev, non_blocking=True), 5)
    res["raw_d2h_pinned_GBps"] = gbps(k * sz, t)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
