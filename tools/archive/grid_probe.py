"""Grid-cap policy probe: device-resident encode / decode of batched stripes
through the table kernels (JIT off), timed back to back behind a spin kernel.
Run once per ZFEC_HIP_GRID_MULT value (the library reads it at start-up):

    ZFEC_HIP_GRID_MULT=64 python tools/grid_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from zfec_amd import capi  # noqa: E402

# (k, m, block bytes, stripes, row stride)
SHAPES = [
    (3, 10, 1366, 10 ** 6, 1536),
    (3, 10, 1360, 10 ** 6, 1536),
    (3, 10, 1376, 10 ** 6, 1536),
    (3, 10, 1408, 10 ** 6, 1536),
    (3, 10, 1536, 10 ** 6, 1536),
    (3, 10, 1366, 10 ** 6, 1366),
    (3, 10, 1408, 10 ** 6, 1408),
]


def place(nums, k):
    slots = [None] * k
    sec = iter([n for n in nums if n >= k])
    for n in nums:
        if n < k:
            slots[n] = n
    return [s if s is not None else next(sec) for s in slots]


def timed(fn, n=10):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda._sleep(20_000_000)
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(n):
        fn()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def main():
    capi.jit_mode(capi.JIT_OFF)
    st = torch.cuda.current_stream().cuda_stream
    gm = os.environ.get("ZFEC_HIP_ROWS_MULT", "default")
    for k, m, sz, ns, ld in SHAPES:
        r = m - k
        code = capi.Code(k, m)
        data = torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda")
        par = torch.empty((ns, r, ld), dtype=torch.uint8, device="cuda")
        slots = place(list(range(m - k, m)), k)
        nrec = sum(1 for s in slots if s >= k)
        rec = torch.empty((ns, nrec, ld), dtype=torch.uint8, device="cuda")
        enc = lambda: code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld,
                                        list(range(k, m)), sz, ns, stream=st)
        dec = lambda: code.decode_batch(data.data_ptr(), ld, k * ld, rec.data_ptr(), ld, nrec * ld, slots, sz, ns,
                                        stream=st)
        te, td = timed(enc), timed(dec)
        print("gm=%-7s k=%2d m=%2d sz=%8d ns=%7d ld=%8d  encode %8.4f ms %6.0f GB/s  decode %8.4f ms %6.0f GB/s  (%s)"
              % (gm, k, m, sz, ns, ld, te, (k + r) * sz * ns / te / 1e6, td, (k + nrec) * sz * ns / td / 1e6,
                 capi.last_kernel_name()), flush=True)
        del data, par, rec
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
