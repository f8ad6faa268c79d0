"""Encode and decode of independent stripes on one stream vs two streams.

bench.py's step is an encode of one stripe and a decode of another (disjoint
buffers), launched in order on one stream, so each launch's ramp-up and drain
(~5 us, tools/mb_cold.hip sweep intercept) is exposed.  Here the same K steps run

  one      encode, decode, encode, ... on one stream (bench.py's loop)
  two      all encodes on stream A, all decodes on stream B, joined once at the
           end (independent requests of a server on two streams)
  joined   as `two`, but both streams join the main stream after every step
           (the shape round 2's --overlap experiment measured)

each enqueued while a spin kernel holds the streams, timed between HIP events.

    python tools/stream_probe.py [cfg2|cfg3] [steps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from zfec_amd import capi  # noqa: E402

SHAPES = {"cfg2": (3, 10, 64 << 20), "cfg3": (10, 16, 256 << 20)}


def main():
    w = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    k, m, total = SHAPES[w]
    r = m - k
    sz = -(-total // k)
    ld = -(-sz // 256) * 256
    code = capi.Code(k, m)
    main_st = torch.cuda.current_stream()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    data = torch.randint(0, 256, (k, ld), dtype=torch.uint8, device="cuda")
    par = torch.empty((r, ld), dtype=torch.uint8, device="cuda")
    nums = list(range(k, m))
    code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld, nums, sz, 1,
                      stream=main_st.cuda_stream)
    # receive the last k blocks; a primary sits at its own index (zfec/fec.c:527-557)
    present = list(range(m - k, m))
    prim = [b for b in present if b < k]
    sec = [b for b in present if b >= k]
    rnums, rows = [], []
    for i in range(k):
        b = i if i in prim else sec.pop(0)
        rnums.append(b)
        rows.append(data[b] if b < k else par[b - k])
    recv = torch.stack(rows).contiguous()
    missing = [i for i in range(k) if i not in prim]
    rec = torch.empty((len(missing), ld), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    def enc(st):
        code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld, nums, sz, 1, stream=st.cuda_stream)

    def dec(st):
        code.decode_batch(recv.data_ptr(), ld, k * ld, rec.data_ptr(), ld, len(missing) * ld, rnums, sz, 1,
                          stream=st.cuda_stream)

    def run(mode):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(20_000_000)  # hold the main stream while the host enqueues
        a.record(main_st)
        if mode == "one":
            for _ in range(n):
                enc(main_st)
                dec(main_st)
        else:
            sa.wait_stream(main_st)
            sb.wait_stream(main_st)
            for _ in range(n):
                enc(sa)
                dec(sb)
                if mode == "joined":
                    main_st.wait_stream(sa)
                    main_st.wait_stream(sb)
                    sa.wait_stream(main_st)
                    sb.wait_stream(main_st)
            main_st.wait_stream(sa)
            main_st.wait_stream(sb)
        b.record(main_st)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / n * 1e3

    for mode in ("one", "two", "joined"):
        run(mode)  # warm-up
    in_bytes = 2 * k * sz  # bench.py's value: input bytes of both directions
    for rep in range(3):
        for mode in ("one", "two", "joined"):
            us = run(mode)
            print("%s %-7s %8.1f us/step  %7.1f GB/s of input" % (w, mode, us, in_bytes / us / 1e3), flush=True)
    # the decode is bit-exact after all that
    torch.cuda.synchronize()
    assert torch.equal(rec[:, :sz], data[missing, :sz]), "decode mismatch"
    print("decode check ok")


if __name__ == "__main__":
    main()
