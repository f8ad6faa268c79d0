"""Per-launch durations of the cfg2 encode kernel launched back to back, with a
HIP event after every launch: does the duration drift over a long run of
launches (clocks, power), and how does it compare with the interleaved
encode/decode pattern of bench.py's timed loop?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from zfec_amd import capi  # noqa: E402


def main():
    k, m = 3, 10
    r = m - k
    sz = -(-(64 << 20) // k)
    ld = -(-sz // 256) * 256
    code = capi.Code(k, m)
    st = torch.cuda.current_stream()
    data = torch.randint(0, 256, (k, ld), dtype=torch.uint8, device="cuda")
    par = torch.empty((r, ld), dtype=torch.uint8, device="cuda")
    recv = torch.empty((k, ld), dtype=torch.uint8, device="cuda")
    rec = torch.empty((k, ld), dtype=torch.uint8, device="cuda")
    nums = list(range(k, m))

    def enc():
        code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld, nums, sz, 1, stream=st.cuda_stream)

    def dec():
        code.decode_batch(recv.data_ptr(), ld, k * ld, rec.data_ptr(), ld, k * ld, [7, 8, 9], sz, 1,
                          stream=st.cuda_stream)

    def series(pattern, n):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n * len(pattern) + 1)]
        for _ in range(3):
            for f in pattern:
                f()
        ev[0].record(st)
        i = 1
        for _ in range(n):
            for f in pattern:
                f()
                ev[i].record(st)
                i += 1
        torch.cuda.synchronize()
        return np.array([ev[j].elapsed_time(ev[j + 1]) * 1e3 for j in range(len(ev) - 1)])

    def steps(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(n):
            enc()
            dec()
        b.record(st)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / n * 1e3

    # bench.py's order: a few warmup steps, then the timed steps, right after start-up
    enc()
    dec()
    torch.cuda.synchronize()
    for _ in range(5):
        enc()
        dec()
    torch.cuda.synchronize()
    print("fresh process: 50 enc/dec steps %.1f us/step; again %.1f; again %.1f" % (steps(50), steps(50), steps(50)),
          flush=True)
    for _ in range(400):
        enc()
        dec()
    torch.cuda.synchronize()
    print("after 400 more steps: 50 enc/dec steps %.1f us/step" % steps(50), flush=True)
    for rep in range(2):
        d = series([enc], 300)
        print("encode b2b x300 (us): mean %.1f median %.1f; per 30: %s" % (
            d.mean(), np.median(d), " ".join("%.1f" % x.mean() for x in d.reshape(10, 30))), flush=True)
        d = series([enc, dec], 150).reshape(150, 2)
        print("enc/dec pairs x150 (us): enc mean %.1f dec mean %.1f; enc per 15: %s" % (
            d[:, 0].mean(), d[:, 1].mean(), " ".join("%.1f" % x.mean() for x in d[:, 0].reshape(10, 15))), flush=True)
        # no per-launch events: plain back-to-back average
        for n in (20, 50, 200):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                enc()
            a.record(st)
            for _ in range(n):
                enc()
            b.record(st)
            torch.cuda.synchronize()
            print("encode b2b x%d, two events: %.1f us" % (n, a.elapsed_time(b) / n * 1e3), flush=True)


if __name__ == "__main__":
    main()
