#!/usr/bin/env python3
"""Compile (hipRTC, no GPU needed) the bit-sliced kernels the GPU tests and the
bench workloads launch, into zfec_amd/jit_cache/ next to libzfec_hip.so, so a
fresh GPU box loads them instead of compiling."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from zfec_amd import capi  # noqa: E402


def place(nums, k):
    slots = [None] * k
    sec = iter([n for n in nums if n >= k])
    for n in nums:
        if n < k:
            slots[n] = n
    return [s if s is not None else next(sec) for s in slots]


# (k, m): tests/test_gpu_jit.py shapes, the auto-policy shape, bench cfg3 / cfg4, the wide-k shapes
SHAPES = [(3, 10), (2, 40), (5, 9), (10, 16), (16, 32), (20, 60), (32, 40), (10, 58), (4, 12), (12, 21), (94, 100),
          (40, 48), (255, 256), (14, 30), (17, 35), (23, 50), (30, 45), (30, 70)]


def main():
    t0 = time.time()
    for k, m in SHAPES:
        code = capi.Code(k, m)
        code.jit_prepare_encode(list(range(k, m)))
        code.jit_prepare_decode(place(list(range(m - k, m)), k))
    code = capi.Code(6, 14)
    code.jit_prepare_decode(place([7, 1, 9, 3, 12, 13], 6), capi.FEC_FLAG_ALL_PRIMARIES)
    print("jit_warm: %d kernels ready in %.1f s" % (capi.jit_wait(), time.time() - t0))


if __name__ == "__main__":
    main()
