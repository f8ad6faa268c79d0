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
        rf, dr = d.get("roofline") or {}, d.get("decode_roofline") or {}
        print("%-34s value %8.1f %s  enc %s %.3f  dec %s %.3f  batched %s  cpu %s" % (
            fn, d["value"], d["unit"], rf.get("kernel"), rf.get("frac") or 0, dr.get("kernel"), dr.get("frac") or 0,
            (d.get("batched_1MiB") or {}).get("frac_of_peak"), (d.get("cpu_baseline") or {}).get("value")))
