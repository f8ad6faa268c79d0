#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run into profiles/.

Reads gpurun_out/<tag>/{ktrace,fetch,write}/*.csv (rocprofv3 --output-format
csv) and writes:
  profiles/<tag>_kernel_stats.csv   rocprofv3's own --stats summary (copied)
  profiles/<tag>_pmc.json           per (kernel, grid) dispatch group: calls,
                                    mean duration, FETCH/WRITE per launch
  profiles/pmc_summary.json         the bench's dominant kernels (read by bench.py)

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE (KiB) reads exactly half
of a wide coalesced stream on gfx950, so it is doubled; WRITE_SIZE (KiB) is
exact for 16-byte-per-lane stores.  traffic = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = name.replace("void zfec_hip::(anonymous namespace)::", "")
    return name.split("(zfec_hip::MatJob)")[0][:80]


def load(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", tag)
    groups = defaultdict(lambda: {"calls": 0, "dur_ns": [], "fetch_kib": [], "write_kib": []})
    for r in load(os.path.join(src, "ktrace", "kt_kernel_trace.csv")):
        key = (r["Kernel_Name"], int(r["Grid_Size"]) if "Grid_Size" in r else int(r["Grid_Size_X"]))
        g = groups[key]
        g["calls"] += 1
        g["dur_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for sub, col in (("fetch", "fetch_kib"), ("write", "write_kib")):
        d = os.path.join(src, sub)
        f = [x for x in os.listdir(d) if x.endswith("counter_collection.csv")][0]
        for r in load(os.path.join(d, f)):
            groups[(r["Kernel_Name"], int(r["Grid_Size"]))][col].append(float(r["Counter_Value"]))
    out = []
    for (name, grid), g in groups.items():
        if "zfec_hip" not in name:
            continue
        mean = lambda v: sum(v) / len(v) if v else None
        fetch, write = mean(g["fetch_kib"]), mean(g["write_kib"])
        traffic = None if fetch is None or write is None else 2 * fetch * 1024 + write * 1024
        out.append({"kernel": short(name), "grid_threads": grid, "calls": g["calls"],
                    "mean_us": round(mean(g["dur_ns"]) / 1e3, 3) if g["dur_ns"] else None,
                    "fetch_kib_raw": fetch, "write_kib": write, "hbm_bytes_per_launch": traffic})
    out.sort(key=lambda x: (x["kernel"], x["grid_threads"]))
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", tag + "_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    shutil.copy(os.path.join(src, "ktrace", "kt_kernel_stats.csv"), os.path.join(ROOT, "profiles", tag + "_kernel_stats.csv"))
    summ = {"source": "profiles/%s_pmc.json (tools/profile_round.sh %s)" % (tag, tag),
            "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KiB*1024), MI355X_MICROARCH.md HBM section"}
    for e in out:
        if e["kernel"].startswith("matapply_reg<3, 7") and e["grid_threads"] == 1398272:
            summ["encode_cfg2"] = e
        if e["kernel"].startswith("matapply_reg<3, 3") and e["grid_threads"] == 1398272:
            summ["decode_cfg2"] = e
    with open(os.path.join(ROOT, "profiles", "pmc_summary.json"), "w") as f:
        json.dump(summ, f, indent=1)
    for e in out:
        print(e)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "prof")
