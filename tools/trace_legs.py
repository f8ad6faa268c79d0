#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of a bench.py run into bench.py's legs.

bench.py --legs-out LEGS.json records, in launch order, which leg every
library launch belongs to ("timed loop", "encode cold", "decode warm",
"decode fresh", ...) and the kernel it ran.  The zfec dispatches of the trace
(kernel names in namespace zfec_hip, or zfec_hip_bitslice_*), in start-time
order, are the same launches in the same order; this script pairs them up
(checking every kernel name) and reports per-leg mean / min / max durations,
the figures bench.py's roofline.launch_ms (back-to-back average) is checked
against.

    python tools/trace_legs.py LEGS.json KERNEL_TRACE.csv [OUT.json]
    python tools/trace_legs.py LEGS.json COUNTER_COLLECTION.csv [OUT.json]

With a --pmc counter_collection.csv (one row per dispatch and counter) it
reports per-leg mean counter values instead of durations.

Dispatches the library makes on its own, outside any launch bench.py records,
are skipped: bsr_table_probe (the once-per-device read of the routine table's
address before the first matapply_bsr launch) and the no-work one-workgroup
launch with which a JIT prefetch warms a compiled kernel (fec_new,
bitslice.cpp warm_launch: a zfec_hip_bitslice dispatch whose grid is one
workgroup; a real launch of those kernels is thousands).  Any other name
that differs from the recorded kernel is a pairing error: the script exits 1
(round 5 paired every cfg3/cfg4 launch after the probe with its
predecessor's leg).
"""
import csv
import json
import sys


def short(name):
    """'void zfec_hip::(anonymous namespace)::matapply_reg<3, 7, true, ...>(zfec_hip::MatJob)' ->
    ('matapply_reg', [3, 7]); 'zfec_hip_bitslice_k20_r40_<hash>' -> (itself, [])."""
    n = name.replace("zfec_hip::(anonymous namespace)::", "").replace("void ", "", 1).split("(")[0]
    if "<" not in n:
        return n, []
    base, args = n.split("<", 1)
    return base, [a.strip() for a in args.rstrip(">").split(",")]


def bsr_traced(recorded):
    """The library's printed matapply_bsr names -> (traced base name, template
    arguments): <RT> the one-wave form (matapply_bsr_solo<RT>), <RT,lds> /
    <RT,lds,cmb> / <RT,lds,tbl> / <RT,lds,tbl,cmb> matapply_bsr<RT, TBL, CMB, J>,
    <RT,ks,tbl> matapply_bsr_ks<RT> (kernels.hip fill_bsr*; bench.py
    _bsr_traced_name)."""
    a = recorded[len("matapply_bsr<"):-1].split(",")
    rt, form = a[0], ",".join(a[1:])
    return {"": ("matapply_bsr_solo", [rt]), "lds": ("matapply_bsr", [rt, "false", "false", "BsrJob"]),
            "lds,cmb": ("matapply_bsr", [rt, "false", "true", "BsrJob"]),
            "lds,a32": ("matapply_bsr", [rt, "false", "false", "BsrJob32"]),
            "lds,a32,cmb": ("matapply_bsr", [rt, "false", "true", "BsrJob32"]),
            "lds,tbl": ("matapply_bsr", [rt, "true", "false", "BsrTblJob"]),
            "lds,tbl,cmb": ("matapply_bsr", [rt, "true", "true", "BsrTblJob"]),
            "ks,tbl": ("matapply_bsr_ks", [rt])}.get(form)


def same(traced, recorded):
    tb, ta = short(traced)
    if recorded.startswith("matapply_bsr<"):
        m = bsr_traced(recorded)
        if m is None or tb != m[0] or len(ta) < len(m[1]):
            return False
        # template arguments equal; a job type matches its unqualified name
        return all(t == w or (w.startswith("Bsr") and t.split("::")[-1] == w) for t, w in zip(ta, m[1]))
    rb, ra = short(recorded)
    if tb != rb:
        return False
    nums = [a for a in ta if a.lstrip("-").isdigit()]
    rnums = [a for a in ra if a.lstrip("-").isdigit()]
    return nums[:len(rnums)] == rnums


def internal(r):
    """A library-internal dispatch (see the module docstring)."""
    n = r["Kernel_Name"]
    if "bsr_table_probe" in n:
        return True
    if "zfec_hip_bitslice" in n:
        grid = r.get("Grid_Size") or r.get("Grid_Size_X")
        wg = r.get("Workgroup_Size") or r.get("Workgroup_Size_X")
        return grid is not None and wg is not None and int(grid) == int(wg)
    return False


def dispatches(path):
    """[(order key, kernel name, {duration_us | counter: value})] of the zfec dispatches
    (library-internal ones named "internal:<name>")."""
    with open(path) as f:
        rd = list(csv.DictReader(f))
    if rd and "Counter_Name" in rd[0]:
        by = {}
        for r in rd:
            if "zfec_hip" not in r["Kernel_Name"]:
                continue
            if internal(r):
                r = dict(r, Kernel_Name="internal:" + r["Kernel_Name"])
            d = by.setdefault(int(r["Dispatch_Id"]), (r["Kernel_Name"], {}))
            d[1][r["Counter_Name"]] = d[1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        return [(key, n, v) for key, (n, v) in sorted(by.items())]
    rows = []
    for r in rd:
        n = r["Kernel_Name"]
        if "zfec_hip" in n:
            if internal(r):
                n = "internal:" + n
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            # enqueue order (launches on two streams may start out of it)
            key = int(r["Dispatch_Id"]) if r.get("Dispatch_Id") else t0
            rows.append((key, n, {"duration_us": (t1 - t0) / 1e3}))
    rows.sort(key=lambda x: x[0])
    return rows


def main():
    legs = json.load(open(sys.argv[1]))
    rows = dispatches(sys.argv[2])
    out, i, mismatch, skipped, first_bad = {}, 0, 0, 0, None
    for leg, kern, cnt in legs["legs"]:
        vals = []
        for _ in range(cnt):
            while i < len(rows) and rows[i][1].startswith("internal:"):
                skipped += 1
                i += 1
            if i >= len(rows):
                break
            _, n, v = rows[i]
            if not same(n, kern):
                mismatch += 1
                if first_bad is None:
                    first_bad = {"dispatch": i, "traced": n, "recorded": kern, "leg": leg}
            vals.append(v)
            i += 1
        if not vals:
            continue
        key = "%s | %s" % (leg, kern)
        out.setdefault(key, []).extend(vals)
    res = {"workload": legs.get("workload"), "source": sys.argv[2].split("/")[-1], "dispatches": len(rows),
           "paired": i, "internal_skipped": skipped, "name_mismatches": mismatch, "first_mismatch": first_bad,
           "legs": {}}
    for key, vals in out.items():
        e = {"launches": len(vals)}
        for c in sorted(vals[0]):
            xs = [v[c] for v in vals if c in v]
            if c == "duration_us":
                e.update({"mean_us": round(sum(xs) / len(xs), 2), "min_us": round(min(xs), 2),
                          "max_us": round(max(xs), 2)})
            else:
                e[c] = round(sum(xs) / len(xs), 1)
        res["legs"][key] = e
    txt = json.dumps(res, indent=1)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(txt + "\n")
    print(txt)
    if mismatch:
        sys.exit("trace_legs: %d dispatches do not match their recorded kernel (first: %s)" % (mismatch, first_bad))


if __name__ == "__main__":
    main()
