#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run into profiles/.

Reads gpurun_out/<tag>/<workload>/{ktrace,fetch,write}/*.csv (rocprofv3
--output-format csv) and writes:
  profiles/<tag>_<workload>_kernel_stats.csv  rocprofv3's own --stats summary (copied)
  profiles/<tag>_pmc.json       per workload and role (encode/decode): launches,
                                mean duration, FETCH/WRITE per launch
  profiles/pmc_summary.json     {"encode_<workload>": ..., "decode_<workload>": ...}
                                (read by bench.py for roofline.traffic)

Roles come from kernel names: bench.py prints the encode and decode kernels it
timed (roofline.kernel / decode_roofline.kernel in its JSON line, captured in
ktrace.log); launches of other kernels (the table kernels that run while a
bit-sliced kernel compiles, torch's own) are left out.  When encode and decode
are the same kernel (one table variant for both), its launches are reported
once as "encode+decode".

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE (KiB) reads exactly half
of a wide coalesced stream on gfx950, so it is doubled; WRITE_SIZE (KiB) is
exact for 16-byte-per-lane stores.  traffic = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = name.replace("zfec_hip::(anonymous namespace)::", "").replace("void ", "", 1)
    return name.split("(")[0][:80]


def load(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def bench_kernels(src):
    """(encode, decode) kernel names from the bench JSON line in ktrace.log."""
    with open(os.path.join(src, "ktrace.log")) as f:
        line = [l for l in f if l.startswith("{")][-1]
    d = json.loads(line)
    strip = lambda s: s.rsplit(" (", 1)[0]
    return strip(d["roofline"]["kernel"]), strip(d["decode_roofline"]["kernel"])


def role_of(name, enc, dec):
    n = short(name)
    if enc == dec:
        return "encode+decode" if n.startswith(enc.split("<")[0]) and _same(n, enc) else None
    if _same(n, enc):
        return "encode"
    if _same(n, dec):
        return "decode"
    return None


def _same(traced, printed):
    """rocprof's demangled template name vs the library's short variant name."""
    if traced == printed:
        return True
    # matapply_reg<3, 7, true, 1> vs matapply_reg<3,7>; matapply_lds<false, true, 6, 2, 2, 1> vs matapply_lds<6,2,2,pad>
    base_t, base_p = traced.split("<")[0], printed.split("<")[0]
    if base_t != base_p or "<" not in traced:
        return False
    targs = [a.strip() for a in traced.split("<", 1)[1].rstrip(">").split(",")]
    pargs = [a.strip() for a in printed.split("<", 1)[1].rstrip(">").split(",") if a.strip() != "pad"]
    nums = [a for a in targs if a.lstrip("-").isdigit()]
    return nums[:len(pargs)] == pargs


def ours(rows):
    rows = [r for r in rows if "zfec_hip" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0))
    return rows


def counter_rows(d):
    f = [x for x in os.listdir(d) if x.endswith("counter_collection.csv")][0]
    rows = ours(load(os.path.join(d, f)))
    return rows


def summarize(src):
    enc, dec = bench_kernels(src)
    kt = ours(load(os.path.join(src, "ktrace", "kt_kernel_trace.csv")))
    fe = counter_rows(os.path.join(src, "fetch"))
    wr = counter_rows(os.path.join(src, "write"))
    res = {}
    for rows, col in ((kt, "dur_ns"), (fe, "fetch_kib"), (wr, "write_kib")):
        for r in rows:
            role = role_of(r["Kernel_Name"], enc, dec)
            if role is None:
                continue
            e = res.setdefault(role, {"kernel": short(r["Kernel_Name"]), "dur_ns": [], "fetch_kib": [], "write_kib": []})
            if col == "dur_ns":
                e[col].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            else:
                e[col].append(float(r["Counter_Value"]))
    out = {}
    for role, e in res.items():
        mean = lambda v: sum(v) / len(v) if v else None
        fetch, write = mean(e["fetch_kib"]), mean(e["write_kib"])
        out[role] = {"kernel": e["kernel"], "launches": len(e["dur_ns"]),
                     "mean_us": round(mean(e["dur_ns"]) / 1e3, 3) if e["dur_ns"] else None,
                     "fetch_kib_raw": fetch, "write_kib": write,
                     "hbm_bytes_per_launch": None if fetch is None or write is None else 2 * fetch * 1024 + write * 1024}
    return out


def main(tag):
    base = os.path.join(ROOT, "gpurun_out", tag)
    allw = {}
    summ = {"source": "profiles/%s_pmc.json (tools/profile_round.sh %s; tools/pmc_summary.py %s)" % (tag, tag, tag),
            "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KiB*1024), MI355X_MICROARCH.md HBM section"}
    for w in sorted(os.listdir(base)):
        if not os.path.isdir(os.path.join(base, w, "ktrace")):
            continue
        allw[w] = summarize(os.path.join(base, w))
        shutil.copy(os.path.join(base, w, "ktrace", "kt_kernel_stats.csv"),
                    os.path.join(ROOT, "profiles", "%s_%s_kernel_stats.csv" % (tag, w)))
        for role, e in allw[w].items():
            summ["%s_%s" % (role, w)] = e
            print(w, role, e)
    with open(os.path.join(ROOT, "profiles", tag + "_pmc.json"), "w") as f:
        json.dump(allw, f, indent=1)
    with open(os.path.join(ROOT, "profiles", "pmc_summary.json"), "w") as f:
        json.dump(summ, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "prof")
