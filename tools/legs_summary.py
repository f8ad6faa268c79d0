#!/usr/bin/env python3
"""Combine a tools/profile_r02.sh run into profiles/: per workload and bench.py
leg, the kernel-trace mean duration and the PMC traffic per launch.

    python tools/legs_summary.py TAG ROUND [WORKLOAD ...]

Reads gpurun_out/TAG/<w>/{legs_kt.json, ktrace/kt_kernel_trace.csv,
legs_f.json, fetch/*counter_collection.csv, legs_w.json,
write/*counter_collection.csv}; writes profiles/ROUND_legs_<w>.json and
copies rocprofv3's --stats summary to profiles/ROUND_<w>_kernel_stats.csv.

Traffic per launch follows MI355X_MICROARCH.md (HBM section): FETCH_SIZE (KiB)
counts half of a wide coalesced read stream on gfx950 and is doubled;
WRITE_SIZE (KiB) is exact for 16-byte-per-lane stores:
bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TL = os.path.join(ROOT, "tools", "trace_legs.py")


def legs_of(legs, csvs):
    if not csvs or not os.path.exists(legs):
        return None
    out = subprocess.run([sys.executable, TL, legs, csvs[0]], capture_output=True, text=True, check=True).stdout
    return json.loads(out)


def main():
    tag, rnd = sys.argv[1], sys.argv[2]
    wls = sys.argv[3:] or ["cfg2", "cfg3", "cfg4", "cfg5"]
    for w in wls:
        d = os.path.join(ROOT, "gpurun_out", tag, w)
        kt = legs_of(os.path.join(d, "legs_kt.json"), glob.glob(os.path.join(d, "ktrace", "*kernel_trace.csv")))
        fe = legs_of(os.path.join(d, "legs_f.json"), glob.glob(os.path.join(d, "fetch", "*counter_collection.csv")))
        wr = legs_of(os.path.join(d, "legs_w.json"), glob.glob(os.path.join(d, "write", "*counter_collection.csv")))
        if kt is None:
            print("no trace for", w)
            continue
        res = {"workload": w, "source": "tools/profile_r02.sh %s %s; tools/legs_summary.py" % (tag, w),
               "traffic_formula": "(2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes per launch",
               "pairing": {"kernel_trace": [kt["dispatches"], kt["paired"], kt["name_mismatches"]],
                           "fetch": fe and [fe["dispatches"], fe["paired"], fe["name_mismatches"]],
                           "write": wr and [wr["dispatches"], wr["paired"], wr["name_mismatches"]]},
               "legs": {}}
        for key, v in kt["legs"].items():
            e = dict(v)
            f = fe and fe["legs"].get(key, {}).get("FETCH_SIZE")
            x = wr and wr["legs"].get(key, {}).get("WRITE_SIZE")
            if f is not None and x is not None:
                e["traffic_bytes"] = round((2 * f + x) * 1024)
            res["legs"][key] = e
        with open(os.path.join(ROOT, "profiles", "%s_legs_%s.json" % (rnd, w)), "w") as fh:
            json.dump(res, fh, indent=1)
        for st in glob.glob(os.path.join(d, "ktrace", "*kernel_stats.csv")):
            shutil.copy(st, os.path.join(ROOT, "profiles", "%s_%s_kernel_stats.csv" % (rnd, w)))
        print(w)
        for key, e in res["legs"].items():
            print("  %-62s n=%-4d mean %9.2f us  traffic %s" % (key[:62], e["launches"], e["mean_us"],
                                                                e.get("traffic_bytes")))


if __name__ == "__main__":
    main()
