#!/usr/bin/env python3
"""Per-kernel means per dispatch of tools/pmc_ab.sh's counter passes:
    python tools/pmc_ab_summary.py gpurun_out/TAG [OUT.json]
Derived: valu_issue = SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / 8 x 4 SIMDs x
256 CUs / 4) (quad-cycles per SIMD), wait_inst_frac = SQ_WAIT_INST_ANY /
SQ_WAVE_CYCLES, wait_any_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES (both in the
counters' quad-cycle units)."""
import csv
import glob
import json
import os
import sys


def main():
    root = sys.argv[1]
    res = {}
    for var in sorted(os.listdir(root)):
        vd = os.path.join(root, var)
        if not os.path.isdir(vd):
            continue
        per = {}
        for f in glob.glob(os.path.join(vd, "p*", "**", "*counter_collection.csv"), recursive=True):
            disp = {}
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    n = r["Kernel_Name"]
                    if "zfec" not in n or "probe" in n:
                        continue
                    if "bitslice" in r["Kernel_Name"] and r.get("Grid_Size") == r.get("Workgroup_Size"):
                        continue  # a JIT prefetch's no-work warm launch (bitslice.cpp warm_launch)
                    d = disp.setdefault((n, r["Dispatch_Id"]), {})
                    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            for (n, _), cv in disp.items():
                k = n.replace("void zfec_hip::(anonymous namespace)::", "").split("(")[0]
                e = per.setdefault(k, {})
                for c, v in cv.items():
                    e.setdefault(c, []).append(v)
        out = {}
        for k, e in per.items():
            m = {c: sum(v) / len(v) for c, v in e.items()}
            m["dispatches"] = max(len(v) for v in e.values())
            if "GRBM_GUI_ACTIVE" in m and "SQ_ACTIVE_INST_VALU" in m:
                simd_quads = m["GRBM_GUI_ACTIVE"] / 8 * 1024 / 4
                m["valu_issue"] = m["SQ_ACTIVE_INST_VALU"] / simd_quads
            if "SQ_WAVE_CYCLES" in m:
                for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
                    if c in m:
                        m[c.lower() + "_frac"] = m[c] / m["SQ_WAVE_CYCLES"]
            out[k] = {c: (round(v, 4) if isinstance(v, float) and v < 100 else int(v)) for c, v in sorted(m.items())}
        res[var] = out
    txt = json.dumps({"source": "tools/pmc_ab.sh + tools/pmc_ab_summary.py", "variants": res}, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
