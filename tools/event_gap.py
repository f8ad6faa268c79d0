#!/usr/bin/env python3
"""How HIP event placement changes the measured duration of the cfg2 encode
kernel: n launches with one event pair vs an event between every launch,
alternating with the decode kernel or not."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import zfec_amd  # noqa: E402,F401
from zfec_amd import capi  # noqa: E402

k, m = 3, 10
sz = -(-(64 << 20) // k)
ld = (sz + 255) // 256 * 256
code = capi.Code(k, m)
data = torch.randint(0, 256, (1, k, ld), dtype=torch.uint8, device="cuda")
par = torch.empty((1, m - k, ld), dtype=torch.uint8, device="cuda")
rec = torch.empty((1, k, ld), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
enc = lambda: code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, (m - k) * ld, list(range(k, m)), sz, 1,
                                stream=st.cuda_stream)
dec = lambda: code.decode_batch(par.data_ptr(), ld, k * ld, rec.data_ptr(), ld, k * ld, [7, 8, 9], sz, 1,
                                stream=st.cuda_stream)
E = lambda: torch.cuda.Event(enable_timing=True)
for _ in range(10):
    enc(), dec()
torch.cuda.synchronize()
for trial in range(3):
    n = 100
    a, b = E(), E()
    a.record(st)
    for _ in range(n):
        enc()
    b.record(st)
    torch.cuda.synchronize()
    pair = a.elapsed_time(b) / n * 1e3
    ev = [E() for _ in range(n + 1)]
    for i in range(n):
        ev[i].record(st)
        enc()
    ev[n].record(st)
    torch.cuda.synchronize()
    per = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(n)]
    # alternating enc/dec with events around each encode
    ev2 = [(E(), E()) for _ in range(n)]
    for i in range(n):
        ev2[i][0].record(st)
        enc()
        ev2[i][1].record(st)
        dec()
    torch.cuda.synchronize()
    alt = [x.elapsed_time(y) * 1e3 for x, y in ev2]
    a, b = E(), E()
    a.record(st)
    for _ in range(n):
        enc(), dec()
    b.record(st)
    torch.cuda.synchronize()
    step = a.elapsed_time(b) / n * 1e3
    print("trial %d: 1 pair / %d enc: %.2f us | event between each: median %.2f min %.2f | alternating enc/dec, "
          "events around enc: median %.2f min %.2f | enc+dec step %.2f us" % (
              trial, n, pair, np.median(per), min(per), np.median(alt), min(alt), step))
