#!/usr/bin/env python3
"""Check bench.py's HIP-event launch durations against the kernel trace of the
SAME run (tools/profile_r02.sh: the bench line printed under rocprofv3 is in
gpurun_out/TAG/<w>/ktrace.log; the per-leg trace means in
profiles/ROUND_legs_<w>.json, from tools/legs_summary.py).

    python tools/bench_vs_trace.py TAG ROUND [WORKLOAD ...] > profiles/ROUND_bench_vs_trace.txt
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, rnd = sys.argv[1], sys.argv[2]
    worst = 0.0
    for w in sys.argv[3:] or ["cfg2", "cfg3", "cfg4", "cfg5"]:
        log = os.path.join(ROOT, "gpurun_out", tag, w, "ktrace.log")
        d = json.loads([ln for ln in open(log) if ln.startswith('{"metric"')][-1])
        legs = json.load(open(os.path.join(ROOT, "profiles", "%s_legs_%s.json" % (rnd, w))))["legs"]

        def trace(prefix):
            for key, v in legs.items():
                if key.startswith(prefix + " |"):
                    return v["mean_us"]
            return None

        rows = [("encode cold", d["roofline"]["launch_ms"]), ("encode warm", d["roofline"]["launch_ms_warm"]),
                ("decode cold", d["decode_roofline"]["launch_ms"]),
                ("decode warm", d["decode_roofline"]["launch_ms_warm"])]
        for lay, x in d.get("batched_1MiB", {}).get("layouts", {}).items():
            rows += [("batched_1MiB %s cold" % lay, x["ms_per_launch"]),
                     ("batched_1MiB %s warm" % lay, x["ms_per_launch_warm"])]
        # single launches between events (the first-seen / first-launch legs): the
        # events also hold a launch's host-side gaps, so these are reported, not
        # counted in the back-to-back legs' largest deviation
        single = []
        fs = d.get("first_seen_decode") or {}
        fl = d.get("first_launch_encode") or {}
        for key, leg, src in (("first_seen", "first-seen decode", fs), ("jit", "first-seen jit decode", fs),
                              ("first_launch", "first-launch encode", fl), ("jit", "first-launch jit encode", fl)):
            if key in src:
                single.append((leg, src[key]["ms_mean"]))
        for name, ms in single:
            t = trace(name)
            if t:
                print("%s %-34s event %9.2f us  trace %9.2f us  ratio %.3f (single launches)" % (w, name, ms * 1e3, t,
                                                                                             ms * 1e3 / t))
        for name, ms in rows:
            t = trace(name)
            ratio = ms * 1e3 / t
            worst = max(worst, abs(ratio - 1))
            print("%s %-34s bench %9.2f us  trace %9.2f us  ratio %.3f" % (w, name, ms * 1e3, t, ratio))
    print("largest deviation: %.1f %%" % (worst * 100))


if __name__ == "__main__":
    main()
