#!/usr/bin/env python3
"""Prints the A/B files a round-5 GPU session wrote (first_seen legs, wide_bench
generic shapes, batch_ab rows): python tools/r05_summary.py gpurun_out/r05d"""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "fs_*.json"))):
    x = json.loads(open(f).read().strip().splitlines()[-1])["first_seen_decode"]
    print(os.path.basename(f), x["first_seen"]["kernel"], x["first_seen"]["ms_mean"], x["first_seen"]["frac_of_peak"],
          "jit", x["jit"]["ms_mean"])
for f in sorted(glob.glob(os.path.join(d, "wide_*.json"))):
    x = json.load(open(f))["shapes"]
    print(os.path.basename(f))
    for s, v in x.items():
        g = v["generic"]
        print("   %-8s enc %-26s %.3f  dec %-26s %.3f" % (s, g["encode"]["kernel"], g["encode"]["ms"],
                                                       g["decode"]["kernel"], g["decode"]["ms"]))
for f in sorted(glob.glob(os.path.join(d, "batch_*.json"))):
    x = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), [(r["stripes"], r["ms_cold"], r["frac_cold"], r["frac_warm"]) for r in x["rows"]])
