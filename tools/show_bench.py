#!/usr/bin/env python3
"""One-line summary of each bench JSON log given on the command line."""
import json
import sys

for fn in sys.argv[1:]:
    for line in open(fn):
        line = line.strip()
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "metric" not in d:
            print(fn, line[:400])
            continue
        rf, dr = d.get("roofline") or {}, d.get("decode_roofline") or {}
        print("%-34s value %8.1f %s  enc %s %.3f  dec %s %.3f  batched %s  cpu %s" % (
            fn, d["value"], d["unit"], rf.get("kernel"), rf.get("frac") or 0, dr.get("kernel"), dr.get("frac") or 0,
            (d.get("batched_1MiB") or {}).get("frac_of_peak"), (d.get("cpu_baseline") or {}).get("value")))
        fs = d.get("first_seen_decode")
        if fs:
            for tag in ("first_seen", "jit"):
                e = fs[tag]
                v = e.get("valu_roofline") or {}
                print("    %-10s %-28s %.4f ms  HBM %.3f  VALU %s" % (tag, e["kernel"], e["ms_mean"], e["frac_of_peak"],
                                                                  v.get("frac", v.get("error"))))
