#!/usr/bin/env python3
"""Host-side cost of one batched C-ABI call (ctypes + library + launch), with
a tiny workload so the GPU never limits the rate; and the cfg2 encode launched
back to back, timed by HIP events vs the per-call host time."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zfec_amd  # noqa: E402,F401
from zfec_amd import capi  # noqa: E402


def per_call_us(fn, n=3000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / n * 1e6


def main():
    st = torch.cuda.current_stream().cuda_stream
    lib = capi.lib()
    print("ctypes fec_version: %.2f us" % per_call_us(lambda: lib.fec_version()))
    for k, m in [(3, 10), (10, 16), (20, 60)]:
        code = capi.Code(k, m)
        sz = 4096
        src = torch.zeros((k, sz), dtype=torch.uint8, device="cuda")
        dst = torch.zeros((m - k, sz), dtype=torch.uint8, device="cuda")
        nums = list(range(k, m))
        slots = list(range(m - k, m)) if m - k >= k else None
        e = lambda: code.encode_batch(src.data_ptr(), sz, k * sz, dst.data_ptr(), sz, (m - k) * sz, nums, sz, 1,
                                      stream=st)
        print("K=%d/M=%d encode_batch 4 KiB: %.2f us/call" % (k, m, per_call_us(e)))
        if slots:
            d = lambda: code.decode_batch(dst.data_ptr(), sz, k * sz, src.data_ptr(), sz, k * sz, slots, sz, 1,
                                          stream=st)
            print("K=%d/M=%d decode_batch 4 KiB: %.2f us/call" % (k, m, per_call_us(d)))
    # empty kernel launch cost through torch for scale
    x = torch.zeros(16, device="cuda")
    print("torch x.add_(1) launch: %.2f us" % per_call_us(lambda: x.add_(1)))
    # cfg2 encode, 20 back to back: events vs host-side time
    k, m = 3, 10
    sz = -(-(64 << 20) // k)
    ld = (sz + 255) // 256 * 256
    code = capi.Code(k, m)
    src = torch.randint(0, 256, (k, ld), dtype=torch.uint8, device="cuda")
    dst = torch.empty((m - k, ld), dtype=torch.uint8, device="cuda")
    nums = list(range(k, m))
    e = lambda: code.encode_batch(src.data_ptr(), ld, k * ld, dst.data_ptr(), ld, (m - k) * ld, nums, sz, 1, stream=st)
    for _ in range(5):
        e()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    t0 = time.perf_counter()
    for _ in range(100):
        e()
    t1 = time.perf_counter()
    b.record()
    torch.cuda.synchronize()
    print("cfg2 encode x100: events %.2f us/launch, host enqueue %.2f us/call" % (a.elapsed_time(b) * 10, (t1 - t0) * 1e4))


if __name__ == "__main__":
    main()
