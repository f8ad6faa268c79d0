"""Rooflines of the wide-code kernels from tools/pmc_wide.sh's passes: per
kernel, the trace's mean duration, VALU wave-instructions and LDS-array
cycles per dispatch, and their fractions of the chip's VALU-issue and LDS
ceilings next to HBM.

    python tools/pmc_wide_summary.py TAG ROUND   -> profiles/<ROUND>_wide_rooflines.json

VALU ceiling: 1024 SIMDs x clock / 4.25 cycles per VOP3 wave-instruction (the
measured v_bitop3 rate, tools/mb_valu.hip; VOP2 issue faster, so this is
conservative for a mix).  LDS ceiling: one LDS-array cycle per CU per clock
(SQ_LDS_IDX_ACTIVE counts array cycles, MI355X_MICROARCH.md §LDS).  The clock
is the kernel's own: GRBM_GUI_ACTIVE / 8 XCDs / duration.  HBM: algorithmic
bytes (k + r) * sz per launch / duration against 8 TB/s.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NCU, NSIMD = 256, 1024


def per_kernel(path, value="Counter_Value"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                n = r["Kernel_Name"]
                if "zfec" not in n and "matapply" not in n or "probe" in n:
                    continue
                if "bitslice" in n and r.get("Grid_Size") == r.get("Workgroup_Size"):
                    continue  # a JIT prefetch's no-work warm launch (bitslice.cpp warm_launch)
                agg[(n, r.get("Dispatch_Id"))][r["Counter_Name"]].append(float(r[value]))
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for (n, _), cs in agg.items():
        for c, v in cs.items():
            out[n][c].append(sum(v))  # a dispatch's value summed over its instances
    return {n: {c: sum(v) / len(v) for c, v in cs.items()} for n, cs in out.items()}


def trace_means(path):
    d = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                n = r["Kernel_Name"]
                if "bitslice" in n and r.get("Grid_Size_X") == r.get("Workgroup_Size_X"):
                    continue  # (the prefetch's warm launch)
                if "zfec" in n or "matapply" in n:
                    d[n].append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9)
    return {n: (sum(v) / len(v), len(v)) for n, v in d.items()}


def short(n):
    n = n.replace("void ", "").replace("zfec_hip::(anonymous namespace)::", "").replace("zfec_hip::", "")
    return n.split("(")[0]


def main():
    tag, rnd = sys.argv[1], sys.argv[2]
    base = os.path.join(ROOT, "gpurun_out", tag)
    tr = trace_means(os.path.join(base, "kt"))
    sq, lds = per_kernel(os.path.join(base, "sq")), per_kernel(os.path.join(base, "lds"))
    out = {"source": "tools/pmc_wide.sh %s (tools/wide_bench.py --variants shipped); per-dispatch means" % tag,
           "basis": __doc__.split("\n\n")[1], "kernels": {}}
    for n, (t, cnt) in sorted(tr.items()):
        c = dict(sq.get(n, {}))
        c.update(lds.get(n, {}))
        row = {"dispatches": cnt, "ms_mean": round(t * 1e3, 4)}
        g = c.get("GRBM_GUI_ACTIVE")
        clk = g / 8 / t if g else None
        if clk:
            row["clock_GHz"] = round(clk / 1e9, 3)
        if c.get("SQ_INSTS_VALU") is not None and clk:
            row["valu_insts"] = int(c["SQ_INSTS_VALU"])
            row["valu_frac"] = round(c["SQ_INSTS_VALU"] * 4.25 / (NSIMD * clk * t), 4)
        if c.get("SQ_LDS_IDX_ACTIVE") is not None and clk:
            row["lds_array_cycles"] = int(c["SQ_LDS_IDX_ACTIVE"])
            row["lds_frac"] = round(c["SQ_LDS_IDX_ACTIVE"] / (NCU * clk * t), 4)
            row["lds_bank_conflict_cycles"] = int(c.get("SQ_LDS_BANK_CONFLICT", 0))
        for key in ("SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                    "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if key in c:
                row[key] = int(c[key])
        out["kernels"][short(n)] = row
    with open(os.path.join(ROOT, "profiles", "%s_wide_rooflines.json" % rnd), "w") as f:
        json.dump(out, f, indent=1)
    for n, row in out["kernels"].items():
        print(n, row.get("ms_mean"), row.get("valu_frac"), row.get("lds_frac"), row.get("clock_GHz"))


if __name__ == "__main__":
    main()
