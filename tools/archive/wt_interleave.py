"""Interleaved encode + decode steps (bench.py's cfg2 pattern) at several K=3/M=10
stripe sizes: the store-policy check of the register kernels (ZFEC_HIP_WT_MAX
selects the footprint up to which they store write-through).

    python tools/wt_interleave.py            # library default
    ZFEC_HIP_WT_MAX=0 python tools/wt_interleave.py   # streaming stores only
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from zfec_amd import capi  # noqa: E402


def main():
    k, m = 3, 10
    r = m - k
    code = capi.Code(k, m)
    st = torch.cuda.Stream()
    for mib in [2, 4, 8, 16, 32, 64]:
        sz = -(-(mib << 20) // k)
        ld = -(-sz // 256) * 256
        src = torch.randint(0, 256, (k, ld), dtype=torch.uint8, device="cuda")
        par = torch.empty((r, ld), dtype=torch.uint8, device="cuda")
        rec = torch.empty((k, ld), dtype=torch.uint8, device="cuda")
        nums = list(range(k, m))
        slots = [7, 8, 9]

        def step():
            code.encode_batch(src.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld, nums, sz, 1, stream=st.cuda_stream)
            code.decode_batch(par.data_ptr() + 4 * ld, ld, k * ld, rec.data_ptr(), ld, k * ld, slots, sz, 1,
                              stream=st.cuda_stream)

        with torch.cuda.stream(st):
            for _ in range(10):
                step()
            names = capi.last_kernel_name()
            res = []
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                n = 50
                a.record(st)
                for _ in range(n):
                    step()
                b.record(st)
                b.synchronize()
                res.append(a.elapsed_time(b) / n)
        assert torch.equal(rec[:, :sz], src[:, :sz])
        t = sorted(res)[2]
        print("%3d MiB stripe  %8.4f ms/step  %7.1f GB/s (input both directions)  decode kernel %s"
              % (mib, t, 2 * k * sz / (t * 1e-3) / 1e9, names), flush=True)


if __name__ == "__main__":
    main()
