#!/usr/bin/env python3
"""Host cost of bringing a compiled (JIT) kernel of the disk cache into use:
fec_new (which queues the prefetch), the prefetch itself (generate the
kernel source, hash it, read the cached code object, load the module on the
current device: no compile), and the first launch after it, against later
launches of the same kernel.  K=20/M=60 full encode, 8 stripes of 1 MiB (a small launch, so the
host figures are the load, not the kernel).

    python tools/jit_load_probe.py
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from zfec_amd import capi  # noqa: E402


def main():
    k, m, ns = 20, 60, 64
    r = m - k
    sz = -(-(1 << 20) // k)
    ld = (sz + 255) // 256 * 256
    data = torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda")
    par = torch.empty((ns, r, ld), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    code = capi.Code(k, m)  # fec_new: the prefetch of the compiled kernel starts
    t1 = time.perf_counter()
    capi.jit_wait()  # the prefetch: source hash, cached code object, module load
    t2 = time.perf_counter()
    nums = list(range(k, m))
    code.jit_prepare_encode(nums)  # in memory by now
    t3 = time.perf_counter()
    res = {"fec_new_ms": round((t1 - t0) * 1e3, 3), "prefetch_wait_ms": round((t2 - t1) * 1e3, 3),
           "prepare_ms": round((t3 - t2) * 1e3, 3)}
    for tag in ("first_launch", "second_launch", "third_launch"):
        torch.cuda.synchronize()
        a = time.perf_counter()
        code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld, nums, sz, ns,
                          stream=st.cuda_stream, flags=capi.FEC_FLAG_ASYNC)
        b = time.perf_counter()
        torch.cuda.synchronize()
        res[tag] = {"host_ms": round((b - a) * 1e3, 3), "kernel": capi.last_kernel_name()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
