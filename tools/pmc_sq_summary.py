"""Per-dispatch means of the issue-side counters collected by tools/pmc_sq.sh,
written to profiles/pmc_sq_summary.json (read by bench.py's valu_roofline) and
profiles/<round>_pmc_sq.json.

    python tools/pmc_sq_summary.py TAG ROUND [WORKLOAD ...]   # e.g. sq2 r01 cfg2 cfg3 cfg4 cfg5
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def summarize(tag, workloads):
    from bench import device_tree_hash

    out = {"source": "tools/pmc_sq.sh %s %s (rocprofv3 --pmc, two passes, per-dispatch means)"
                     % ("|".join(workloads), tag),
           "tree": device_tree_hash(),
           "tree_basis": "sha256 of the device sources (bench.py DEVICE_SOURCES) the counters were collected on; "
                         "bench.py's valu_roofline uses this file only when it matches the tree it runs from",
           "workloads": {}}
    for w in workloads:
        ws = {}
        for sub in ("ic", "sq", "lds", "sca"):
            files = glob.glob(os.path.join(ROOT, "gpurun_out", tag, w, sub, "**", "*counter_collection.csv"),
                              recursive=True)
            if not files:
                continue
            agg = collections.defaultdict(lambda: collections.defaultdict(list))
            with open(files[0]) as f:
                for r in csv.DictReader(f):
                    if "zfec" not in r["Kernel_Name"]:
                        continue
                    if "bitslice" in r["Kernel_Name"] and r.get("Grid_Size") == r.get("Workgroup_Size"):
                        continue  # a JIT prefetch's no-work warm launch (bitslice.cpp warm_launch)
                    n = r["Kernel_Name"].replace("zfec_hip::(anonymous namespace)::", "").replace("void ", "", 1).split("(")[0]
                    agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
            for n, v in agg.items():
                ws.setdefault(n, {}).update({c: round(sum(x) / len(x)) for c, x in v.items()})
        out["workloads"][w] = ws
    return out


def main():
    tag, rnd = sys.argv[1], sys.argv[2]
    workloads = sys.argv[3:] or ["cfg2", "cfg3", "cfg4", "cfg5"]
    out = summarize(tag, workloads)
    for name in ("pmc_sq_summary.json", "%s_pmc_sq.json" % rnd):
        with open(os.path.join(ROOT, "profiles", name), "w") as f:
            json.dump(out, f, indent=1)
    for w, v in out["workloads"].items():
        for n, c in v.items():
            print(w, n, c.get("SQ_INSTS_VALU"))


if __name__ == "__main__":
    main()
