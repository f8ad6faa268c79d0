#!/usr/bin/env python3
"""Summarise tools/jit_probe_pmc.sh TAG into one JSON (profiles/):
per variant of tools/jit_probe.py (real / zero / nohbm / noarith), the kernel
time of its timed dispatches, the effective clock GRBM_GUI_ACTIVE / 8 / time
(MI355X_MICROARCH.md, DVFS give-back: rocprofv3 sums the counter over the 8
XCDs), VALU instructions per dispatch and their issue rate, and HBM bytes
(2 * FETCH_SIZE + WRITE_SIZE, KiB; gfx950 FETCH_SIZE counts half of a wide
coalesced read stream).  Dispatches are paired with the variants through the
run's --legs-out order.

    python tools/jit_probe_summary.py TAG OUT.json [cfg4|cfg3]
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows_by_dispatch(d):
    """{dispatch id: {"name", "us", counters...}} of the bit-sliced JIT dispatches in pass dir d."""
    out = {}
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Kernel_Name"].startswith("zfec_hip_bitslice"):
                out.setdefault(int(r["Dispatch_Id"]), {})["name"] = r["Kernel_Name"]
                out[int(r["Dispatch_Id"])]["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Kernel_Name"].startswith("zfec_hip_bitslice"):
                e = out.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"]})
                e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [out[key] for key in sorted(out)]


def by_variant(d, legs_path):
    legs = json.load(open(legs_path))["legs"]
    rows = rows_by_dispatch(d)
    res, i = {}, 0
    for leg, n in legs:
        part = rows[i:i + n]
        i += n
        if leg == "check" or leg.endswith("(warm)"):
            continue
        res.setdefault(leg, []).extend(part)
    return res, len(rows), i


def mean(xs):
    return sum(xs) / len(xs) if xs else None


def main():
    tag, out_path = sys.argv[1], sys.argv[2]
    base = os.path.join(ROOT, "gpurun_out", tag)
    clk, n_clk, used = by_variant(os.path.join(base, "clk"), os.path.join(base, "clk_legs.json"))
    fet, _, _ = by_variant(os.path.join(base, "fetch"), os.path.join(base, "fetch_legs.json"))
    wri, _, _ = by_variant(os.path.join(base, "write"), os.path.join(base, "write_legs.json"))
    shape = sys.argv[3] if len(sys.argv) > 3 else "cfg4"
    k, m, ns, stripe = {"cfg4": (20, 60, 1024, 1 << 20), "cfg3": (10, 16, 1, 256 << 20)}[shape]
    sz = -(-stripe // k)
    alg = (k + (m - k)) * sz * ns
    res = {"source": "tools/jit_probe_pmc.sh %s; tools/jit_probe_summary.py" % tag,
           "shape": "K=%d/M=%d encode, %d x %d-byte stripes (bench %s), kernel %s" % (k, m, ns, stripe, shape,
               clk.get("real", [{}])[0].get("name") if clk.get("real") else None),
           "algorithmic_bytes_per_launch": alg, "dispatches_paired": [n_clk, used],
           "clock_formula": "GRBM_GUI_ACTIVE / 8 / kernel time (profiled pass)",
           "traffic_formula": "(2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes per dispatch", "variants": {}}
    for name, rs in clk.items():
        us = mean([r["us"] for r in rs if "us" in r])
        grbm = mean([r.get("GRBM_GUI_ACTIVE", 0.0) for r in rs])
        valu = mean([r.get("SQ_INSTS_VALU", 0.0) for r in rs])
        e = {"dispatches": len(rs), "kernel_us_mean": round(us, 1), "effective_clock_GHz": round(grbm / 8 / (us * 1e3), 3),
             "SQ_INSTS_VALU": round(valu), "SQ_BUSY_CYCLES": round(mean([r.get("SQ_BUSY_CYCLES", 0.0) for r in rs])),
             "SQ_WAVE_CYCLES": round(mean([r.get("SQ_WAVE_CYCLES", 0.0) for r in rs])),
             "valu_wave_insts_per_ns": round(valu / (us * 1e3), 2),
             "valu_issue_cycles_per_SIMD_per_clock": round(valu * 4 / 1024 / (grbm / 8), 3)}
        f = mean([r.get("FETCH_SIZE", 0.0) for r in fet.get(name, [])])
        w = mean([r.get("WRITE_SIZE", 0.0) for r in wri.get(name, [])])
        if f is not None and w is not None:
            e["hbm_bytes"] = round((2 * f + w) * 1024)
            e["hbm_over_algorithmic"] = round((2 * f + w) * 1024 / alg, 3)
        res["variants"][name] = e
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
