#!/usr/bin/env python3
"""Interleaved A/B of library variants (tools/ab_build.sh builds them into
abuild/<name>/) on the shapes the bit-sliced run-time-data kernels serve.
Each (round, variant) pair is its own process, loading its variant through
ZFEC_HIP_LIB, so every variant runs on the same box in turns:
A B C .. A B C ..

Cases (every launch device-resident, timed like bench.py's cold legs:
back-to-back launches over a rotation of buffer sets spanning >= 768 MiB;
every case's output is checked -- against the CPU oracle on a sample of
stripes / a column slice, or decode(encode(x)) == x):
  cfg4_enc    K=20/M=60, 1024 x 1 MiB stripes, encode of all 40 parity rows,
              JIT off: what a process's first launch of that code runs
              (matapply_bsr<10,lds,tbl>)
  cfg4_dec    the same stripes, decode of all 20 primaries from parity
              blocks 20..39 (r = 20), JIT off (matapply_bsr<10,lds>)
  w128        128/256, one 64 MiB stripe, encode of all 128 parity rows, JIT
              off (matapply_bsr<8,lds,tbl,cmb>)
  w94         94/100, one 64 MiB stripe, encode, JIT off (the ks form)
  s64         K=3/M=10, one 64 MiB stripe, encode (cfg2's matapply_reg<3,7>)
  wide:K/M    K/M, one 64 MiB stripe, encode, JIT off
  cfg4_fl     cfg4_enc as first launches: 6 new row orders, one launch each
              between events (bench.py's first_launch_encode leg)
  cfg4_jit    cfg4_enc with the JIT as shipped after its compile (the
              compiled kernel: the reference point of cfg4_enc)
  jit:K/M, bsr:K/M
              K/M encode over 1024 x 1 MiB stripes, compiled (JIT) kernel /
              JIT off
  b1m_om / b1m_omp / b1m_dense / b1m_bm
              the north-star batch, K=3/M=10 encode of 256 x 1 MiB stripes per
              launch, in four layouts (batch_case)

    python tools/ab_bsr.py --variants r05,new --cases cfg4_enc,w128 --rounds 2 \\
        --out gpurun_out/ab.json
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(cases, launches):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    import bench
    from oracle import oracle
    from zfec_amd import capi

    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    res = {}
    check = not os.environ.get("ZFEC_AB_NOCHECK")  # timing-only variants (e.g. form=trunc64) give wrong bytes

    def timed(fns, leg):
        ms, _ = bench.back_to_back(fns, launches, st, leg)
        return ms, capi.last_kernel_name()

    for case in cases:
        if case == "cfg4_fl":
            res[case] = first_launch_case(check)
            continue
        if case.startswith("b1m_"):
            res[case] = batch_case(case, launches, check)
            continue
        jit_case = case == "cfg4_jit" or case.startswith("jit:")
        if case.startswith(("jit:", "bsr:")):  # K/M encode over 1024 x 1 MiB stripes
            k, m = map(int, case[4:].split("/"))
            ns = 1024
            sz = -(-(1 << 20) // k)
        elif case in ("cfg4_enc", "cfg4_dec", "cfg4_jit"):
            k, m, ns = 20, 60, 1024
            sz = -(-(1 << 20) // k)
        elif case == "w128" or case.startswith("wide:"):  # one 64 MiB stripe, JIT off
            k, m = (128, 256) if case == "w128" else map(int, case[5:].split("/"))
            ns = 1
            sz = -(-(64 << 20) // k)
        elif case == "w94":
            k, m, ns = 94, 100, 1
            sz = -(-(64 << 20) // k)
        elif case == "s64":  # cfg2's stripe: K=3/M=10, one 64 MiB stripe (matapply_reg<3,7>)
            k, m, ns = 3, 10, 1
            sz = -(-(64 << 20) // k)
        else:
            raise SystemExit("unknown case " + case)
        r = m - k
        ld = (sz + 255) // 256 * 256
        code = capi.Code(k, m)
        capi.jit_mode(capi.JIT_AUTO if jit_case else capi.JIT_OFF)
        capi.generic_mode(2)
        nsets = max(2, -(-bench.COLD_SPAN // ((k + r) * ld * ns)))
        g = torch.Generator(device="cuda").manual_seed(k * 1000 + m)
        data = [torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda", generator=g) for _ in range(nsets)]
        par = [torch.empty((ns, r, ld), dtype=torch.uint8, device="cuda") for _ in range(nsets)]
        nums = list(range(k, m))

        def enc_i(i):
            def f(sh):
                code.encode_batch(data[i].data_ptr(), ld, k * ld, par[i].data_ptr(), ld, r * ld, nums, sz, ns,
                                  stream=sh, flags=capi.FEC_FLAG_ASYNC)
            return f

        for i in range(nsets):
            enc_i(i)(st.cuda_stream)
            enc_i(i)(st.cuda_stream)
        capi.jit_wait()
        torch.cuda.synchronize()
        out = {}
        if case != "cfg4_dec":
            ms, kern = timed([enc_i(i) for i in range(nsets)], case)
            out.update(kernel=kern, ms=round(ms, 4),
                       hbm_frac=round((k + r) * sz * ns / (ms * 1e-3) / 1e9 / bench.HBM_PEAK_GBPS, 4))
            # oracle check: 4 stripes, or a 4 KiB column slice of a single stripe
            for i in ((0, nsets - 1) if check else ()):
                if ns > 1:
                    for s in (0, 1, ns // 2, ns - 1):
                        want = oracle.encode(k, m, data[i][s, :, :sz].cpu().numpy())
                        assert np.array_equal(par[i][s, :, :sz].cpu().numpy(), want), (case, i, s)
                else:
                    for c0 in (0, sz // 2, sz - 4096):
                        want = oracle.encode(k, m, data[i][0, :, c0:c0 + 4096].cpu().numpy())
                        assert np.array_equal(par[i][0, :, c0:c0 + 4096].cpu().numpy(), want), (case, i, c0)
        else:
            slots = list(range(k, 2 * k))  # every primary lost: parity blocks 20..39
            recv = [par[i][:, :k].contiguous() for i in range(nsets)]
            rec = [torch.empty((ns, k, ld), dtype=torch.uint8, device="cuda") for _ in range(nsets)]

            def dec_i(i):
                def f(sh):
                    code.decode_batch(recv[i].data_ptr(), ld, k * ld, rec[i].data_ptr(), ld, k * ld, slots, sz, ns,
                                      stream=sh, flags=capi.FEC_FLAG_ASYNC)
                return f

            ms, kern = timed([dec_i(i) for i in range(nsets)], case)
            torch.cuda.synchronize()
            for i in range(nsets if check else 0):
                assert torch.equal(rec[i][:, :, :sz], data[i][:, :, :sz]), (case, i)
            out.update(kernel=kern, ms=round(ms, 4),
                       hbm_frac=round(2 * k * sz * ns / (ms * 1e-3) / 1e9 / bench.HBM_PEAK_GBPS, 4))
        res[case] = out
        del data, par
        torch.cuda.empty_cache()
    print("ABRESULT " + json.dumps(res), flush=True)


def first_launch_case(check):
    """cfg4's shape, K=20/M=60 encodes of 1024 x 1 MiB stripes in 6 row orders
    the process has not launched (rotations of the 40 parity numbers: each a new
    matrix), JIT off, one launch per order between HIP events (as bench.py's
    first_launch_encode leg): the kernel and the host work of a first launch."""
    import numpy as np
    import torch

    import bench
    from oracle import oracle
    from zfec_amd import capi

    k, m, ns = 20, 60, 1024
    r = m - k
    sz = -(-(1 << 20) // k)
    ld = (sz + 255) // 256 * 256
    capi.jit_mode(capi.JIT_OFF)
    code = capi.Code(k, m)
    st = torch.cuda.current_stream()
    data = torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda")
    par = torch.empty((ns, r, ld), dtype=torch.uint8, device="cuda")
    nums = list(range(k, m))
    rows = []
    for i in range(7):
        order = nums[i:] + nums[:i]
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(st)
        code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld, order, sz, ns,
                          stream=st.cuda_stream, flags=capi.FEC_FLAG_ASYNC)
        b.record(st)
        torch.cuda.synchronize()
        if i:
            rows.append(a.elapsed_time(b))
        if check and i == 6:
            for s_ in (0, ns - 1):
                want = oracle.encode(k, m, data[s_, :, :sz].cpu().numpy(), order)
                assert np.array_equal(par[s_, :, :sz].cpu().numpy(), want), s_
    ms = float(np.mean(rows))
    del data, par
    torch.cuda.empty_cache()
    return {"kernel": capi.last_kernel_name(), "ms": round(ms, 4),
            "hbm_frac": round((k + r) * sz * ns / (ms * 1e-3) / 1e9 / bench.HBM_PEAK_GBPS, 4)}


def batch_case(case, launches, check):
    """North-star batch (K=3/M=10 encode, 256 x 1 MiB stripes per launch) in one
    layout: b1m_om object-major rows 256-byte aligned, no row-padding flag (rows
    end mid-line); b1m_omp the same with FEC_FLAG_ROW_PADDING; b1m_dense a
    contiguous [256, 3, sz] tensor (rows back to back, no slack: easyfec's
    blocks, zfec/easyfec.py:28-39); b1m_bm block-major [3, 256 * sz]."""
    import numpy as np
    import torch

    import bench
    from oracle import oracle
    from zfec_amd import capi

    k, m, ns = 3, 10, 256
    r = m - k
    sz = -(-(1 << 20) // k)
    ld = bench.row_stride(sz)
    code = capi.Code(k, m)
    st = torch.cuda.current_stream()
    nums = list(range(k, m))
    flags = capi.FEC_FLAG_ASYNC | (capi.FEC_FLAG_ROW_PADDING if case == "b1m_omp" else 0)
    if case in ("b1m_om", "b1m_omp"):
        shp_i, shp_o, sbs, sss, dbs, dss = (ns, k, ld), (ns, r, ld), ld, k * ld, ld, r * ld
    elif case == "b1m_dense":
        shp_i, shp_o, sbs, sss, dbs, dss = (ns, k, sz), (ns, r, sz), sz, k * sz, sz, r * sz
    elif case == "b1m_bm":
        shp_i, shp_o, sbs, sss, dbs, dss = (k, ns * sz), (r, ns * sz), ns * sz, sz, ns * sz, sz
    else:
        raise SystemExit("unknown case " + case)
    fp = (shp_i[0] * shp_i[1] * shp_i[2]) + (shp_o[0] * shp_o[1] * shp_o[2]) if len(shp_i) == 3 else m * ns * sz
    nsets = max(2, -(-bench.COLD_SPAN // fp))
    src = [torch.randint(0, 256, shp_i, dtype=torch.uint8, device="cuda") for _ in range(nsets)]
    dst = [torch.empty(shp_o, dtype=torch.uint8, device="cuda") for _ in range(nsets)]

    def enc_i(i):
        def f(sh):
            code.encode_batch(src[i].data_ptr(), sbs, sss, dst[i].data_ptr(), dbs, dss, nums, sz, ns, stream=sh,
                              flags=flags)
        return f

    enc_i(0)(st.cuda_stream)
    torch.cuda.synchronize()
    if check:
        flat_i, flat_o = src[0].reshape(-1), dst[0].reshape(-1)
        for s_ in (0, 1, ns // 2, ns - 1):
            blocks = np.stack([flat_i[s_ * sss + j * sbs:s_ * sss + j * sbs + sz].cpu().numpy() for j in range(k)])
            got = np.stack([flat_o[s_ * dss + i * dbs:s_ * dss + i * dbs + sz].cpu().numpy() for i in range(r)])
            assert np.array_equal(got, oracle.encode(k, m, blocks)), (case, s_)
    cold, _ = bench.back_to_back([enc_i(i) for i in range(nsets)], launches, st, case)
    kern = capi.last_kernel_name()
    del src, dst
    torch.cuda.empty_cache()
    return {"kernel": kern, "ms": round(cold, 4), "hbm_frac": round(ns * m * sz / (cold * 1e-3) / 1e9 / bench.HBM_PEAK_GBPS, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True, help="names under abuild/ (or 'tree': the in-tree library)")
    ap.add_argument("--cases", default="cfg4_enc,cfg4_dec,w128")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--worker", action="store_true")
    args = ap.parse_args()
    cases = args.cases.split(",")
    if args.worker:
        worker(cases, args.launches)
        return
    variants = args.variants.split(",")
    rows = {v: [] for v in variants}
    for rnd in range(args.rounds):
        for v in variants:
            env = dict(os.environ)
            if os.path.exists(os.path.join(ROOT, "abuild", v, "NOCHECK")):
                env["ZFEC_AB_NOCHECK"] = "1"
            if v != "tree":
                env["ZFEC_HIP_LIB"] = os.path.join(ROOT, "abuild", v, "libzfec_hip.so")
            t0 = time.time()
            p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--worker", "--cases", args.cases,
                                "--launches", str(args.launches), "--variants", v], env=env, capture_output=True,
                               text=True, timeout=600)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("ABRESULT ")]
            if p.returncode != 0 or not line:
                print(p.stdout[-2000:], p.stderr[-4000:], file=sys.stderr)
                raise SystemExit("variant %s failed (rc %d)" % (v, p.returncode))
            r = json.loads(line[0][len("ABRESULT "):])
            rows[v].append(r)
            print("round %d %-8s %5.1fs %s" % (rnd, v, time.time() - t0,
                                               " ".join("%s=%.4f(%s)" % (c, r[c]["ms"], r[c]["kernel"]) for c in cases)),
                  flush=True)
    summary = {}
    for v in variants:
        summary[v] = {}
        for c in cases:
            ms = [r[c]["ms"] for r in rows[v]]
            summary[v][c] = {"kernel": rows[v][0][c]["kernel"], "ms": ms, "ms_mean": round(sum(ms) / len(ms), 4),
                             "hbm_frac_mean": round(sum(r[c]["hbm_frac"] for r in rows[v]) / len(ms), 4)}
        spec = os.path.join(ROOT, "abuild", v, "SPEC")
        summary[v]["spec"] = open(spec).read().strip() if os.path.exists(spec) else "in-tree build"
    doc = {"tool": "tools/ab_bsr.py (variants: tools/ab_build.sh)", "cases": cases, "rounds": args.rounds,
           "launches": args.launches, "variants": summary}
    text = json.dumps(doc, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text)
    print(text)


if __name__ == "__main__":
    main()
