#!/usr/bin/env python3
"""bench.py -- device-resident Reed-Solomon encode+decode throughput on MI355X.

Metric (BASELINE.json): "encode+decode GB/s (device-resident input) at K/M;
% of HBM roofline".  Default workload = BASELINE.json configs[1]: K=3, M=10,
one 64 MiB stripe per GPU (block size sz = ceil(64 MiB / 3) = 22,369,622 B).
Other configs (--workload cfg3|cfg4|cfg5) are the parity-test cases, timed
the same way for DESIGN.md.

One step = encode every stripe of the workload (k primaries -> m-k
secondaries, one launch of fec_encode_batch) + decode them back from
secondary blocks (one launch of fec_decode_batch), inputs resident in HBM.
value = (encode input + decode input bytes) = 2 * k * sz * stripes per step,
summed over GPUs, / wall time of the K timed steps (max over ranks), GB/s
(1e9).  The step's two launches are plain stream-ordered launches (--graph:
capture them once into a HIP graph and replay it per step; on ROCm 7.2 the
replay measured slower than eager launches).

Multi-GPU (one process per GPU): `python bench.py --gpus N` with no WORLD_SIZE
in the environment starts N ranks itself (torch.distributed.run on 127.0.0.1,
before this process makes any GPU call) and exits with their status; under an
external torchrun WORLD_SIZE must equal --gpus, or the run stops with an error
instead of measuring another number of GPUs.  The line's `ranks_seen` is the
world size the process group reported.  Stripes are independent, so ranks
never exchange data.  cfg2/cfg3: each rank owns its own stripe (weak
scaling); with --slabs the ONE stripe's block byte range is split instead
(zfec_amd.shard.slab_range, strong scaling: rank r holds columns [c0, c1) of
every block).  cfg4/cfg5: the fixed batch is split by
zfec_amd.shard.shard_range (strong scaling).  The only collectives are the timing barrier and the
max/sum reductions.

Also reported: the dominant kernel's roofline (encode: (k+r)*sz*stripes
algorithmic HBM bytes per launch / average launch duration over back-to-back
launches between two HIP events on the launch stream; PMC traffic from
profiles/pmc_summary.json), the decode kernel's, a batched 1 MiB-stripe
encode (the north-star shape), and a bounded CPU baseline (rank 0, N=1) of
the reference's own C code (oracle/_ref, kind "reference") or the oracle
restatement (kind "port").
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(argv):
    """--gpus N without WORLD_SIZE: run this script as N ranks (one process per
    GPU, as the driver's torchrun line does) and return their exit status; None
    when this process is a rank already (or N is 1).  Runs before torch or the
    library is imported, so the parent never touches a GPU."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    n = ap.parse_known_args(argv)[0].gpus
    if n < 1:
        sys.exit("bench.py: --gpus must be >= 1 (got %d)" % n)
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != n:
            sys.exit("bench.py: WORLD_SIZE=%s but --gpus %d: refusing to measure another number of GPUs than asked"
                     % (ws, n))
        return None
    if n == 1:
        return None
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, cwd=ROOT)


if __name__ == "__main__":
    _rc = launch_ranks(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, ROOT)

import zfec_amd  # noqa: E402
from zfec_amd import capi  # noqa: E402
from zfec_amd.shard import shard_range, slab_range  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# Cold-cache HBM rates of loads alone and of stores alone in this library's access pattern
# (tools/mb_cold.exe read3 / write7, best of the runs in profiles/r02_mb_cold.log).  HBM does
# not overlap this pattern's reads with its writes (a cold encode takes read3 + write7), so a
# launch reading R and writing W bytes needs at least R / READ + W / WRITE.
HBM_READ_GBPS, HBM_WRITE_GBPS = 6449.0, 5799.0


def rw_ceiling(read_bytes, write_bytes, achieved_gbps):
    """The read-then-write ceiling of one launch's traffic and the achieved fraction of it."""
    c = (read_bytes + write_bytes) / (read_bytes / HBM_READ_GBPS + write_bytes / HBM_WRITE_GBPS)
    return {"GBps": round(c, 1), "frac_of_peak": round(c / HBM_PEAK_GBPS, 4),
            "achieved_frac_of_ceiling": round(achieved_gbps / c, 4),
            "basis": "(R + W) / (R / %.0f + W / %.0f GB/s): cold loads-only and stores-only rates of the same "
                     "walk (tools/mb_cold.exe read3 / write7, profiles/r02_mb_cold.log)" % (HBM_READ_GBPS,
                                                                                        HBM_WRITE_GBPS)}
METRIC = "encode+decode GB/s (device-resident input) at K/M; % of HBM roofline"

# name: (k, m, stripe bytes, stripes, scaling)
WORKLOADS = {
    "cfg2": (3, 10, 64 << 20, 1, "weak"),
    "cfg3": (10, 16, 256 << 20, 1, "weak"),
    "cfg4": (20, 60, 1 << 20, 1024, "strong"),
    "cfg5": (3, 10, 4 << 10, 1000000, "strong"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS) + ["first_seen"],
                   help="first_seen: only the first_seen_decode leg (cfg4's shape), for the counter runs")
    p.add_argument("--no-first-seen", action="store_true",
                   help="cfg2: skip the first_seen_decode leg (first-seen erasure patterns at cfg4's shape)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-extra", action="store_true", help="skip the 1 MiB-stripe batched leg")
    p.add_argument("--layout", default="256", choices=["odd128", "256"],
                   help="block row stride in HBM: 256-byte multiple (default) or an odd number of 128-byte lines")
    p.add_argument("--no-row-padding", action="store_true",
                   help="do not pass FEC_FLAG_ROW_PADDING (rows then end mid-line where sz is not a multiple of 128)")
    p.add_argument("--slabs", action="store_true",
                   help="cfg2/cfg3 only: split the ONE stripe's block byte range into slabs across the GPUs "
                        "(zfec_amd.shard.slab_range; strong scaling) instead of one stripe per GPU")
    p.add_argument("--fresh", type=int, default=None,
                   help="decodes from fresh random erasure patterns to time (default: 20 for the wide codes cfg3/cfg4, "
                        "0 otherwise)")
    p.add_argument("--legs-out", default=None,
                   help="write the run's launch sequence per leg (JSON) for tools/trace_legs.py")
    p.add_argument("--streams", type=int, default=None, choices=[1, 2],
                   help="2: each step's encode on one stream and its decode (independent buffers) on a second "
                        "stream, joined once after the timed steps, so short launches overlap each other's "
                        "ramp-up and drain (default: 2 for cfg2/cfg4/cfg5, 1 for cfg3, whose bit-sliced launches "
                        "measured 1-2 %% slower side by side while cfg4's gained 0.6-1.3 %%, "
                        "profiles/r06_streams_wide_ab.json)")
    p.add_argument("--paired", action="store_true",
                   help="each step as ONE fec_run_batch_jobs call on one stream: its encode and decode share one "
                        "matapply_pair launch where both are register-kernel shapes (cfg2), else one launch each")
    p.add_argument("--dry-run", action="store_true",
                   help="set up the ranks and the process group (gloo, no GPU call), print rank 0's view of the world "
                        "as one JSON line and exit: the launch path, testable on CPU")
    p.add_argument("--graph", action="store_true",
                   help="replay the step as a captured HIP graph (measured slower than eager launches on ROCm 7.2)")
    return p.parse_args()


def dist_setup(gpus=1):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != gpus:  # launch_ranks checked this already; keep the invariant for importers
        raise SystemExit("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, gpus))
    # ZFEC_BENCH_DIST=1 initialises the process group at world size 1 too, so
    # the RCCL path (init, barrier, max/sum reductions) can be rehearsed under
    # torchrun on a one-GPU box
    if world > 1 or os.environ.get("ZFEC_BENCH_DIST") == "1":
        import torch.distributed as dist

        # ZFEC_BENCH_BACKEND=gloo rehearses the multi-rank path with several
        # ranks on one GPU (the driver's runs use RCCL, one rank per GPU)
        backend = os.environ.get("ZFEC_BENCH_BACKEND", "nccl")
        if backend == "gloo":
            torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
            dist.init_process_group("gloo")
        else:
            ndev = torch.cuda.device_count()
            if local >= ndev:
                raise SystemExit("bench.py: rank %d (LOCAL_RANK %d) has no GPU of its own: %d visible; one rank "
                                 "per GPU over RCCL" % (rank, local, ndev))
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return dist, rank, world
    torch.cuda.set_device(0)
    return None, 0, 1


def barrier(dist):
    if dist is not None:
        dist.barrier()


class NodeBarrier:
    """Barrier of the ranks of one node over a shared-memory page: rank r
    writes the barrier's epoch into its own 64-byte slot and spins until every
    slot has reached it (one writer per slot, so plain stores suffice on x86).
    It brackets the timed steps: a dist.barrier() there (RCCL or gloo) added
    0.1-0.2 ms per timed region on the MI355X box against a few microseconds
    for this (ZFEC_BENCH_BARRIER=dist restores it, for A/B runs).  The process
    group only sets it up.  World size 1: a no-op, as in the plain run."""

    def __init__(self, dist, rank, world):
        self.world, self.rank, self.epoch, self.flags = world, rank, 0, None
        # one node only: every rank must be able to map rank 0's /dev/shm page
        # (torchrun sets LOCAL_WORLD_SIZE; a multi-node job falls back to
        # dist.barrier())
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        if (dist is None or world == 1 or local_world != world
                or os.environ.get("ZFEC_BENCH_BARRIER") == "dist"):
            self.dist = dist if world > 1 else None
            return
        import mmap
        import uuid

        self.dist = None
        name = [None]
        if rank == 0:
            name[0] = "/dev/shm/zfec_bench_barrier_%s" % uuid.uuid4().hex
            with open(name[0], "wb") as f:
                f.truncate(64 * world)
        dist.broadcast_object_list(name, src=0)
        with open(name[0], "r+b") as f:
            self.mm = mmap.mmap(f.fileno(), 64 * world)
        dist.barrier()  # every rank has mapped the page
        if rank == 0:
            os.unlink(name[0])  # the mappings stay valid
        self.flags = np.ndarray((world, 8), dtype=np.int64, buffer=self.mm)

    def wait(self, timeout_s=300.0):
        if self.flags is None:
            barrier(self.dist)
            return
        self.epoch += 1
        self.flags[self.rank, 0] = self.epoch
        col = self.flags[:, 0]
        t_end = time.monotonic() + timeout_s
        while col.min() < self.epoch:
            if time.monotonic() > t_end:
                raise RuntimeError("NodeBarrier: a rank did not arrive within %.0f s" % timeout_s)


def reduce(dist, x, op):
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if dist.get_backend() == "gloo" else "cuda")
    dist.all_reduce(t, op=op)
    return float(t.item())


def align_up(x, a):
    return (x + a - 1) // a * a


def row_stride(sz, rule="256"):
    """Distance between consecutive block rows in HBM.  "256": rows rounded up
    to 256 bytes (default).  "odd128": an odd number of 128-byte lines (in the
    kernel microbenchmark, tools/mb_encode.exe MB_BATCH with 1366-byte rows, 4.78
    vs 4.41 TB/s; in this bench's encode+decode step no difference on any
    workload, 2 runs each)."""
    if rule == "256":
        return align_up(sz, 256)
    lines = -(-sz // 128)
    return 128 * (lines if lines % 2 else lines + 1)


def place(nums, k):
    """Slot order with primary i at slot i (zfec/_fecmodule.c:482-493)."""
    slots = [None] * k
    sec = iter([n for n in nums if n >= k])
    for n in nums:
        if n < k:
            slots[n] = n
    return [s if s is not None else next(sec) for s in slots]


PROFILE_ROUND = "r06"


def pmc_traffic(workload, leg="encode cold"):
    """HBM bytes per launch of one bench leg from the committed per-leg PMC
    summary (profiles/<round>_legs_<workload>.json: tools/profile_r02.sh +
    tools/legs_summary.py; (2 * FETCH_SIZE + WRITE_SIZE) KiB per launch)."""
    try:
        with open(os.path.join(ROOT, "profiles", "%s_legs_%s.json" % (PROFILE_ROUND, workload))) as f:
            legs = json.load(f)["legs"]
        for key, v in legs.items():
            if key.startswith(leg + " |"):
                return v.get("traffic_bytes")
    except (OSError, ValueError, KeyError):
        pass
    return None


# VALU issue ceiling: 256 CUs x 4 SIMDs x ~2.4 GHz / 4.25 cycles per VOP3 wave-instruction
# (the measured v_perm_b32 / v_bitop3_b32 rate, tools/mb_valu.hip)
VALU_PEAK_INSTS = 256 * 4 * 2.4e9 / 4.25


# Device code the committed counter summaries describe: a summary is used only
# when it was collected on these exact sources (tools/pmc_sq_summary.py).
DEVICE_SOURCES = ("zfec_amd/csrc/kernels.hip", "zfec_amd/csrc/kernels.hpp", "zfec_amd/csrc/bitslice.cpp",
                  "zfec_amd/csrc/bitslice.hpp", "zfec_amd/csrc/gf_routines.inc")


def device_tree_hash():
    import hashlib

    h = hashlib.sha256()
    for rel in DEVICE_SOURCES:
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def _bsr_traced_name(printed):
    """The library's matapply_bsr names -> the kernels' demangled names:
    <RT> one-wave form, <RT,lds> LDS-phase form, <RT,lds,a32> its 32-bit
    argument form, <RT,lds,tbl> its table form
    (",cmb": the combination-sharing variant of either),
    <RT,ks,tbl> the input-split form (kernels.hip fill_bsr*)."""
    if not printed.startswith("matapply_bsr<"):
        return None
    a = printed[len("matapply_bsr<"):-1].split(",")
    rt = a[0]
    form = ",".join(a[1:])
    return {"": "matapply_bsr_solo<%s>" % rt, "lds": "matapply_bsr<%s, false, false, BsrJob>" % rt,
            "lds,cmb": "matapply_bsr<%s, false, true, BsrJob>" % rt,
            "lds,a32": "matapply_bsr<%s, false, false, BsrJob32>" % rt,
            "lds,a32,cmb": "matapply_bsr<%s, false, true, BsrJob32>" % rt,
            "lds,tbl": "matapply_bsr<%s, true, false, BsrTblJob>" % rt,
            "lds,tbl,cmb": "matapply_bsr<%s, true, true, BsrTblJob>" % rt,
            "ks,tbl": "matapply_bsr_ks<%s>" % rt}.get(form)


def _same_kernel(traced, printed):
    """rocprof's demangled name vs the library's name: the same name, the
    library's short template name as the leading arguments of the traced one
    (matapply_reg<3,7> vs matapply_reg<3, 7, 3, true, true>), or a
    matapply_bsr form's name (_bsr_traced_name)."""
    if traced == printed or traced == _bsr_traced_name(printed):
        return True
    if printed.startswith("matapply_bsr<"):
        return False
    if "<" not in traced or "<" not in printed or traced.split("<")[0] != printed.split("<")[0]:
        return False
    targs = [a.strip() for a in traced.split("<", 1)[1].rsplit(">", 1)[0].split(",")]
    pargs = [a.strip() for a in printed.split("<", 1)[1].rsplit(">", 1)[0].split(",")]
    return targs[:len(pargs)] == pargs


def valu_roofline(workload, kernel, launch_ms):
    """Second roofline of the dominant kernel: VALU wave-instructions per launch
    (SQ_INSTS_VALU from the committed counter summary, tools/pmc_sq.sh) over the
    launch duration, against the VALU issue ceiling.  Only from a summary
    collected on this tree's device sources, and only when exactly one traced
    kernel of the workload is this one."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_sq_summary.json")) as f:
            summ = json.load(f)
        d = summ["workloads"].get(workload, {})
    except (OSError, ValueError, KeyError):
        return None
    if summ.get("tree") != device_tree_hash():
        return {"error": "profiles/pmc_sq_summary.json was collected on other device sources (tree %s, this tree %s)"
                         % (summ.get("tree"), device_tree_hash())}
    hits = [(n, c) for n, c in d.items() if _same_kernel(n, kernel) and c.get("SQ_INSTS_VALU")]
    if len(hits) != 1:
        return {"error": "%d traced kernels match %s" % (len(hits), kernel)}
    name, c = hits[0]
    n = float(c["SQ_INSTS_VALU"])
    ach = n / (launch_ms * 1e-3)
    return {"bound": "valu-issue", "insts_per_launch": int(n), "achieved": round(ach / 1e9, 1),
            "peak": round(VALU_PEAK_INSTS / 1e9, 1), "unit": "G VALU wave-instructions/s",
            "frac": round(ach / VALU_PEAK_INSTS, 4), "traced_kernel": name, "tree": summ.get("tree"),
            "basis": "SQ_INSTS_VALU per dispatch (profiles/pmc_sq_summary.json, same device sources) / launch_ms; "
                     "peak = 1024 SIMDs x 2.4 GHz / 4.25 cycles per VOP3 wave-instruction (measured)"}


def host_cpus():
    """CPUs this process may use: its affinity mask, capped by a cgroup CPU
    quota when one is set (cpu.max), plus what the host reports."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    return {"usable": usable, "affinity": aff, "cgroup_quota_cpus": quota, "os_cpu_count": os.cpu_count(),
            "model": model}


def cpu_baseline(seconds, k, m, sz):
    """Bounded CPU sample of the same workload (encode + last-k decode of one
    stripe of k*sz bytes per step, decoding from the last k blocks), one
    stripe per thread on every CPU this process may use (no cap), plus a
    1-thread figure.  Stripes are shrunk so all threads' buffers stay within
    ~8 GB of host memory.

    The reference's fec.c (oracle/_ref, built from /root/reference by
    oracle/Makefile) runs from C threads (oracle/ref_bench.c), so neither the
    Python binding's per-call cost nor the GIL caps the CPU figure; the same
    step through the reference's Python binding (zfec/_fecmodule.c, one Python
    thread per CPU) is reported beside it.  Without oracle/_ref the oracle
    restatement runs instead (kind "port")."""
    from oracle import oracle

    cpus = host_cpus()
    threads = cpus["usable"]
    sz = max(1, min(sz, (8 << 30) // (threads * (m + k))))
    nums = place(list(range(m - k, m)), k)  # the same last-k decode set as the GPU leg
    rb = oracle.ref_bench_lib()
    mod = oracle.ref_module()
    rng = np.random.default_rng(7)
    proto = [rng.integers(0, 256, size=sz, dtype=np.uint8).tobytes() for _ in range(k)]

    def py_run(make_work, nthreads, secs):
        counts = [0] * nthreads
        stop = threading.Event()
        work = make_work(counts, stop)
        ths = [threading.Thread(target=work, args=(t,)) for t in range(nthreads)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        time.sleep(secs)
        stop.set()
        for th in ths:
            th.join()
        return sum(counts), time.perf_counter() - t0  # steps in flight at the stop are counted

    def binding_work(counts, stop):
        def work(t):
            enc, dec = mod.Encoder(k, m), mod.Decoder(k, m)
            blocks = [bytes(b) for b in proto]
            while not stop.is_set():
                out = enc.encode(blocks)
                dec.decode([out[n] for n in nums], nums)
                counts[t] += 1
        return work

    def port_work(counts, stop):
        data = np.frombuffer(b"".join(proto), dtype=np.uint8).reshape(k, sz)

        def work(t):
            while not stop.is_set():
                allb = np.concatenate([data, oracle.encode(k, m, data)])
                oracle.decode(k, m, allb[nums], nums)
                counts[t] += 1
        return work

    rate = lambda steps, el: round(steps * 2 * k * sz / el / 1e9, 4)
    extra = {}
    if rb is not None:
        kind, how = "reference", ("reference zfec/fec.c compiled by oracle/Makefile (-O2 -march=x86-64-v2), "
                                  "driven from C threads (oracle/ref_bench.c)")
        steps, el = oracle.ref_bench(rb, k, m, sz, threads, seconds)
        steps1, el1 = oracle.ref_bench(rb, k, m, sz, 1, max(2.0, seconds * 0.3))
        if mod is not None:
            sb, eb = py_run(binding_work, threads, max(2.0, seconds * 0.3))
            extra["value_python_binding"] = rate(sb, eb)
            extra["python_binding"] = ("the same step through the reference's own Python binding (_fecmodule.c) "
                                       "from %d Python threads: %d steps in %.1f s" % (threads, sb, eb))
    elif mod is not None:
        kind, how = "reference", "reference zfec/_fecmodule.c + fec.c (oracle/Makefile), one Python thread per CPU"
        steps, el = py_run(binding_work, threads, seconds)
        steps1, el1 = py_run(binding_work, 1, max(2.0, seconds * 0.3))
    else:
        kind, how = "port", "oracle/fec_oracle.c restatement, one Python thread per CPU"
        steps, el = py_run(port_work, threads, seconds)
        steps1, el1 = py_run(port_work, 1, max(2.0, seconds * 0.3))
    out = {"value": rate(steps, el), "unit": "GB/s", "cores": threads, "kind": kind,
           "value_1thread": rate(steps1, el1),
           "host": cpus,
           "sample": "%d steps (encode + last-k decode of a K=%d/M=%d %d-byte stripe) in %.1f s on %d threads, "
                     "one stripe per thread, every CPU the process may use (affinity %d, cgroup quota %s, "
                     "os.cpu_count %s); 1 thread: %d steps in %.1f s; %s" % (
                         steps, k, m, k * sz, el, threads, cpus["affinity"], cpus["cgroup_quota_cpus"],
                         cpus["os_cpu_count"], steps1, el1, how)}
    out.update(extra)
    return out


def bench_zfec_style(Encoder, Decoder, k=3, m=10, size=10 ** 6, reps=1000):
    """bench/bench_zfec.py:78-117 semantics: 10^6 random bytes split into k
    blocks (last one zero-padded), `reps` encodes of all m blocks, then
    primary-only and secondary-only (blocks k..2k-1) decodes; results in the
    reference's units ("MB/s": encode = input bytes / 2^20 / s, decode = all m
    blocks' bytes / 2^20 / s, README.rst:118-127)."""
    d = os.urandom(size)
    bs = -(-size // k)
    ds = [d[i * bs:(i + 1) * bs] for i in range(k)]
    ds[-1] = ds[-1] + b"\x00" * (len(ds[-2]) - len(ds[-1]))
    enc = Encoder(k, m)
    t0 = time.perf_counter()
    for _ in range(reps):
        enc.encode(ds)
    enc_s = (time.perf_counter() - t0) / reps
    blocks = enc.encode(ds)
    nums = list(range(len(blocks)))
    dec = Decoder(k, m)
    res = {"encode_MBps": size / 2 ** 20 / enc_s}
    for name, sl in (("decode_primary_MBps", slice(0, k)), ("decode_secondary_MBps", slice(k, 2 * k))):
        t0 = time.perf_counter()
        for _ in range(reps):
            dec.decode(blocks[sl], nums[sl])
        el = (time.perf_counter() - t0) / reps
        assert b"".join(dec.decode(blocks[sl], nums[sl]))[:size] == d
        res[name] = sum(len(b) for b in blocks) / 2 ** 20 / el
    return {key: round(v, 1) for key, v in res.items()}


class Legs(object):
    """Order of this process's library launches, run-length encoded per leg,
    so tools/trace_legs.py can split a rocprofv3 kernel trace of this run into
    the same legs (the dispatches of the zfec kernels, in order)."""

    def __init__(self):
        self.runs = []

    def add(self, leg, kernel, count=1):
        if self.runs and self.runs[-1][0] == leg and self.runs[-1][1] == kernel:
            self.runs[-1][2] += count
        else:
            self.runs.append([leg, kernel, count])


LEGS = Legs()

# the 256 MiB Infinity Cache (MALL): buffer rotations for cold launches span
# at least this many bytes, so a launch's buffers were last touched >= 2 x the
# cache's size of traffic ago
COLD_SPAN = 768 << 20


# GPU time of untimed launches before a back-to-back measurement: the chip
# lowers its clock some milliseconds into sustained load and settles after
# that (K=20/M=60 encode: 680-850 us per launch a few milliseconds in, 590 us
# after 180 ms; tools/jit_probe.py), so the timed
# launches start in the settled state
WARM_MS = 200.0


def back_to_back(fns, n, stream, leg):
    """Average GPU duration of n launches queued back to back, fns[i % len]
    for launch i, after untimed launches of the same kind worth WARM_MS of GPU
    time (at most 2000).  The stream is held by a spin kernel while the host
    starts enqueueing them, so the host's per-call cost cannot leave gaps
    between the timed launches.  Returns (ms per launch, host enqueue us per
    launch)."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    fns[0](stream.cuda_stream)
    b.record(stream)
    LEGS.add(leg + " (untimed)", capi.last_kernel_name())
    torch.cuda.synchronize()
    warm = int(min(2000, max(3, WARM_MS / max(1e-3, a.elapsed_time(b)))))
    torch.cuda._sleep(20_000_000)
    # queued behind the spin kernel too: the timed launches start on a busy GPU.  The
    # host's enqueue cost is timed on the first of them, while the spin kernel holds
    # the GPU and the launch queue is still empty (later ones may wait for queue space)
    nh = min(warm, 64)
    h0 = time.perf_counter()
    for i in range(nh):
        fns[(i + 1) % len(fns)](stream.cuda_stream)
    host_us = (time.perf_counter() - h0) / nh * 1e6
    for i in range(nh, warm):
        fns[(i + 1) % len(fns)](stream.cuda_stream)
    LEGS.add(leg + " (untimed)", capi.last_kernel_name(), warm)
    a.record(stream)
    for i in range(n):
        fns[(i + 1 + warm) % len(fns)](stream.cuda_stream)
    b.record(stream)
    kern = capi.last_kernel_name()
    for _ in range(n):
        LEGS.add(leg, kern)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n, host_us


def run_workload(k, m, sz, ns, steps, warmup, dist, use_graph=False, layout="256", row_padding=True, fresh=0,
                 streams=1, paired=False):
    """Encode + decode `ns` stripes per step; returns timings.

    HBM layout: [stripe][block][row_stride] with the row stride = sz rounded up
    to 256 bytes (row_stride), so every block starts 256-byte aligned (the
    reference's API takes separate buffers per block, which are aligned too).
    row_padding: the calls carry FEC_FLAG_ROW_PADDING, letting the library run
    each row out to its next 128-byte line inside that padding (whole-line
    writes; the bytes counted stay k*sz per stripe).
    fresh: that many extra decodes, each from a new random set of k received
    blocks (a matrix never seen before: no specialised kernel exists for it)."""
    r = m - k
    ld = row_stride(sz, layout)
    gen = torch.Generator(device="cuda").manual_seed(1234 + k)
    # decode from the last k blocks (all secondaries when m >= 2k); primaries at their slot
    slots = place(list(range(m - k, m)), k)
    nrec = sum(1 for s in slots if s >= k)
    # rotation sets for the cold legs: set 0 is the timed loop's
    enc_fp, dec_fp = (k + r) * ld * ns, (k + nrec) * ld * ns
    nsets = max(2, -(-COLD_SPAN // min(enc_fp, dec_fp)))
    data = [torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda", generator=gen) for _ in range(nsets)]
    par = [torch.empty((ns, r, ld), dtype=torch.uint8, device="cuda") for _ in range(nsets)]
    recv = [torch.empty((ns, k, ld), dtype=torch.uint8, device="cuda") for _ in range(nsets)]  # slot order
    rec = [torch.empty((ns, nrec, ld), dtype=torch.uint8, device="cuda") for _ in range(nsets)]
    enc_nums = list(range(k, m))
    code = capi.Code(k, m)
    fl = capi.FEC_FLAG_ASYNC | (capi.FEC_FLAG_ROW_PADDING if row_padding else 0)

    # the addresses and strides of each set are fixed: computed once, so the
    # per-call host cost is the library call's (host_enqueue_us), not torch's
    def enc_i(i):
        a = (data[i].data_ptr(), ld, k * ld, par[i].data_ptr(), ld, r * ld, enc_nums, sz, ns)

        def f(sh):
            code.encode_batch(*a, stream=sh, flags=fl)
        return f

    def dec_i(i):
        a = (recv[i].data_ptr(), ld, k * ld, rec[i].data_ptr(), ld, nrec * ld, slots, sz, ns)

        def f(sh):
            code.decode_batch(*a, stream=sh, flags=fl)
        return f

    enc, dec = enc_i(0), dec_i(0)
    stream = torch.cuda.current_stream()
    for i in range(nsets):
        enc_i(i)(stream.cuda_stream)
        LEGS.add("setup", capi.last_kernel_name())
        for j, s in enumerate(slots):  # stage the received blocks once (not part of a step)
            recv[i][:, j].copy_(data[i][:, s] if s < k else par[i][:, s - k])
        dec_i(i)(stream.cuda_stream)
        LEGS.add("setup", capi.last_kernel_name())
    # wide codes: a matrix's second large launch queues the background compile
    # of its bit-sliced kernel (zfec_amd/csrc/bitslice.cpp); wait for it so the
    # warmup and the timed loop run the kernels a long-running user gets
    capi.jit_wait()
    kernels = {}
    for i in range(max(1, warmup)):
        enc(stream.cuda_stream)
        kernels["encode"] = capi.last_kernel_name()
        LEGS.add("warmup", kernels["encode"])
        dec(stream.cuda_stream)
        kernels["decode"] = capi.last_kernel_name()
        LEGS.add("warmup", kernels["decode"])
    torch.cuda.synchronize()
    missing = [i for i in range(k) if slots[i] >= k]
    for i in range(nsets):
        assert torch.equal(rec[i][:, :, :sz], data[i][:, missing, :sz]), "decode(encode(x)) != x"

    launch = "eager"

    def step():
        enc(stream.cuda_stream)
        dec(stream.cuda_stream)

    fork = join = lambda: None
    if streams == 2:
        # a step's encode and decode touch disjoint buffers: encodes in order on
        # one stream, decodes on another, so each launch's ramp-up and drain
        # overlap the other stream's work; the streams fork from the launch
        # stream before the steps and join it after them (no per-step join)
        s_enc, s_dec = torch.cuda.Stream(), torch.cuda.Stream()

        def step():
            enc(s_enc.cuda_stream)
            dec(s_dec.cuda_stream)

        def fork():
            s_enc.wait_stream(stream)
            s_dec.wait_stream(stream)

        def join():
            stream.wait_stream(s_enc)
            stream.wait_stream(s_dec)

        launch = "eager, 2 streams (encodes | decodes)"

    if paired:
        # one fec_run_batch_jobs call per step: the two independent jobs share
        # one launch (matapply_pair) where both are register-kernel shapes
        jobs = capi.BatchJobs([
            capi.encode_job(code, data[0].data_ptr(), ld, k * ld, par[0].data_ptr(), ld, r * ld, enc_nums, sz, ns,
                            flags=fl & capi.FEC_FLAG_ROW_PADDING),
            capi.decode_job(code, recv[0].data_ptr(), ld, k * ld, rec[0].data_ptr(), ld, nrec * ld, slots, sz, ns,
                            flags=fl & capi.FEC_FLAG_ROW_PADDING)])
        jobs.run(stream.cuda_stream)
        kernels["step"] = capi.last_kernel_name()
        torch.cuda.synchronize()

        def step():
            jobs.run(stream.cuda_stream)

        fork = join = lambda: None
        launch = "one fec_run_batch_jobs call per step (%s)" % kernels["step"]

    if use_graph and streams == 1 and not paired:
        try:
            cap = torch.cuda.Stream()
            graph = torch.cuda.CUDAGraph()
            cap.wait_stream(stream)
            with torch.cuda.graph(graph, stream=cap):
                enc(cap.cuda_stream)
                dec(cap.cuda_stream)
            torch.cuda.synchronize()
            rec[0].zero_()
            graph.replay()
            torch.cuda.synchronize()
            assert torch.equal(rec[0][:, :, :sz], data[0][:, missing, :sz]), "graph replay: decode(encode(x)) != x"
            step = graph.replay
            launch = "hipGraph (1 replay per step)"
        except Exception as e:  # capture unsupported: keep eager launches
            launch = "eager (graph capture failed: %s: %s)" % (type(e).__name__, str(e)[:120])
    fork()
    for _ in range(3):
        step()
        if launch.startswith("eager"):
            LEGS.add("warmup", kernels["encode"])
            LEGS.add("warmup", kernels["decode"])
        elif paired:
            LEGS.add("warmup", kernels["step"])
    join()
    torch.cuda.synchronize()
    nbar = NodeBarrier(dist, dist.get_rank() if dist else 0, dist.get_world_size() if dist else 1)
    nbar.wait()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    fork()
    for _ in range(steps):
        step()
    join()
    e1.record(stream)
    torch.cuda.synchronize()
    nbar.wait()
    el = time.perf_counter() - t0
    # the timed steps' results are the code's: decode(encode(x)) == x
    assert torch.equal(rec[0][:, :, :sz], data[0][:, missing, :sz]), "timed loop: decode(encode(x)) != x"
    for j, s in enumerate(slots):  # and the timed encodes rewrote the parity the decodes read
        if s >= k:
            assert torch.equal(par[0][:, s - k, :sz], recv[0][:, j, :sz]), "timed loop: parity changed"
    if launch.startswith("eager"):
        for _ in range(steps):
            LEGS.add("timed loop", kernels["encode"])
            LEGS.add("timed loop", kernels["decode"])
    elif paired:
        for _ in range(steps):
            LEGS.add("timed loop", kernels["step"])

    # Per-kernel launch duration for the rooflines: back-to-back launches of
    # one kernel between two HIP events on the launch stream, (a) "warm": the
    # same buffers every launch (what the timed loop does; footprints under
    # 256 MiB are then partly served by the Infinity Cache), (b) "cold": a
    # rotation of `nsets` disjoint buffer sets spanning >= 768 MiB, so every
    # launch reads and writes HBM.  (c) The timed loop's encode/decode pattern
    # with an event pair around every launch (each event adds ~1 us).
    nb = max(20, steps)
    enc_w, enc_host_us = back_to_back([enc], nb, stream, "encode warm")
    dec_w, dec_host_us = back_to_back([dec], nb, stream, "decode warm")
    enc_c, _ = back_to_back([enc_i(i) for i in range(nsets)], nb, stream, "encode cold")
    dec_c, _ = back_to_back([dec_i(i) for i in range(nsets)], nb, stream, "decode cold")

    def per_launch(n):
        E = lambda: torch.cuda.Event(enable_timing=True)
        ev = [(E(), E(), E()) for _ in range(n)]
        for a, b, c in ev:
            a.record(stream)
            enc(stream.cuda_stream)
            b.record(stream)
            dec(stream.cuda_stream)
            c.record(stream)
            LEGS.add("event pairs", kernels["encode"])
            LEGS.add("event pairs", kernels["decode"])
        torch.cuda.synchronize()
        return (float(np.mean([a.elapsed_time(b) for a, b, _ in ev])),
                float(np.mean([b.elapsed_time(c) for _, b, c in ev])))

    npl = max(50, steps)
    enc_pl, dec_pl = per_launch(npl)
    out = {"elapsed_s": el, "gpu_step_ms": e0.elapsed_time(e1) / steps, "launch": launch,
           "enc_ms": enc_c, "dec_ms": dec_c, "enc_ms_warm": enc_w, "dec_ms_warm": dec_w,
           "enc_ms_pairs": enc_pl, "dec_ms_pairs": dec_pl, "b2b_launches": nb, "nsets": nsets,
           "enqueue_us": (enc_host_us, dec_host_us),
           "pair_launches": npl, "nrec": nrec, "slots": slots, "kernels": kernels}
    if fresh:
        out["decode_fresh"] = decode_fresh(code, k, m, sz, ns, ld, data[0], par[0], recv[0], fresh, stream)
    return out


def decode_fresh(code, k, m, sz, ns, ld, data, par, recv, n, stream):
    """Decodes that each use a new random set of k received blocks: a matrix
    the process has never seen, so no specialised (JIT) kernel exists for it
    and the launch runs on what serves first-seen patterns (matapply_bsr).
    One launch per pattern between events (the staging copy into slot order is
    outside them); every result is checked against the stripe."""
    rng = np.random.default_rng(4321)
    out = torch.empty((ns, k, ld), dtype=torch.uint8, device="cuda")
    rows = []
    for _ in range(n):
        while True:
            nums = sorted(int(x) for x in rng.choice(m, size=k, replace=False))
            sl = place(nums, k)
            miss = [i for i in range(k) if sl[i] >= k]
            if miss:
                break
        for j, s in enumerate(sl):
            recv[:, j].copy_(data[:, s] if s < k else par[:, s - k])
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        code.decode_batch(recv.data_ptr(), ld, k * ld, out.data_ptr(), ld, k * ld, sl, sz, ns,
                          stream=stream.cuda_stream, flags=ROW_PADDING_FLAGS)
        b.record(stream)
        kern = capi.last_kernel_name()
        LEGS.add("decode fresh", kern)
        torch.cuda.synchronize()
        assert torch.equal(out[:, :len(miss), :sz], data[:, miss, :sz]), "fresh-pattern decode != input"
        ms = a.elapsed_time(b)
        rows.append((ms, len(miss), kern))
    gb = [k * sz * ns / (ms * 1e-3) / 1e9 for ms, _, _ in rows]
    hbm = [(k + nr) * sz * ns / (ms * 1e-3) / 1e9 for ms, nr, _ in rows]
    return {"patterns": n, "input_GBps_mean": round(float(np.mean(gb)), 1),
            "input_GBps_min": round(float(np.min(gb)), 1), "hbm_GBps_mean": round(float(np.mean(hbm)), 1),
            "recovered_mean": round(float(np.mean([nr for _, nr, _ in rows])), 2),
            "ms_mean": round(float(np.mean([ms for ms, _, _ in rows])), 4),
            "kernels": sorted(set(kk for _, _, kk in rows)),
            "timing": "one decode launch per pattern between HIP events; no JIT warm-up (JIT mode as shipped: a "
                      "pattern's first launch never runs a specialised kernel)"}


def run_batched_1mib(steps):
    """North-star shape: K=3/M=10 encode of 1 MiB stripes, 256 stripes per
    launch, in two layouts:
      object-major  [stripe][block][row] (rows 256-byte aligned, as in the main
                    workload): one launch walks 256 stripes of 10 rows each;
                    with FEC_FLAG_ROW_PADDING as the main workload's calls
                    (the headline), and without it (every output row's last
                    128-byte line partly written: HBM completes each such line
                    with a read-modify-write, 147 -> 161 us per launch,
                    profiles/r05_rowend_ab.json);
      dense         a contiguous [256, 3, sz] tensor (blocks of exactly sz bytes
                    back to back, no row slack: what Encoder.encode_batch gets
                    from a caller who did not pad; easyfec's blocks,
                    zfec/easyfec.py:28-39), outputs [256, 7, sz]: rows start
                    and end mid-line;
      block-major   block j of every stripe back to back ([block][stripe][sz],
                    stripe stride = sz): fec_encode_batch runs it as ONE stripe
                    of 256 x sz bytes per block, 10 long streams.
    Each is timed back to back on the same buffers ("warm") and over a
    rotation of disjoint buffer sets spanning >= 768 MiB ("cold": HBM, not the
    Infinity Cache).  The top-level figures are object-major cold; the
    layouts' own figures are under "layouts"."""
    k, m, ns = 3, 10, 256
    sz = -(-(1 << 20) // k)
    ld = row_stride(sz)
    code = capi.Code(k, m)
    st = torch.cuda.current_stream()
    nums = list(range(k, m))
    res = {"shape": "K=3/M=10 encode, 256 x 1 MiB stripes per launch", "algorithmic_bytes_per_launch": m * sz * ns,
           "layouts": {}, "row_padding": ("object-major: the calls carry FEC_FLAG_ROW_PADDING, as the main "
                                          "workload's do (rows end on a whole 128-byte line inside their 256-byte "
                                          "padding); 'object-major, rows end mid-line': the same buffers without "
                                          "the flag (each output row's last line is written partially)")}
    for layout in ("object-major", "object-major, rows end mid-line", "dense", "block-major"):
        flags = capi.FEC_FLAG_ASYNC | (capi.FEC_FLAG_ROW_PADDING if layout == "object-major" else 0)
        if layout.startswith("object-major"):
            fp = m * ld * ns
            shape_in, shape_out = (ns, k, ld), (ns, m - k, ld)
            sbs, sss, dbs, dss = ld, k * ld, ld, (m - k) * ld
        elif layout == "dense":
            fp = m * sz * ns
            shape_in, shape_out = (ns, k, sz), (ns, m - k, sz)
            sbs, sss, dbs, dss = sz, k * sz, sz, (m - k) * sz
        else:
            fp = m * sz * ns
            shape_in, shape_out = (k, ns * sz), (m - k, ns * sz)
            sbs, sss, dbs, dss = ns * sz, sz, ns * sz, sz
        nsets = max(2, -(-COLD_SPAN // fp))
        src = [torch.randint(0, 256, shape_in, dtype=torch.uint8, device="cuda") for _ in range(nsets)]
        dst = [torch.empty(shape_out, dtype=torch.uint8, device="cuda") for _ in range(nsets)]

        def enc_i(i):
            def f(sh):
                code.encode_batch(src[i].data_ptr(), sbs, sss, dst[i].data_ptr(), dbs, dss, nums, sz, ns, stream=sh,
                                  flags=flags)
            return f

        warm, _ = back_to_back([enc_i(0)], steps, st, "batched_1MiB %s warm" % layout)
        cold, _ = back_to_back([enc_i(i) for i in range(nsets)], steps, st, "batched_1MiB %s cold" % layout)
        lr = {"kernel": capi.last_kernel_name(), "nsets": nsets}
        for tag, ms in (("", cold), ("_warm", warm)):
            in_gbps = ns * k * sz / (ms * 1e-3) / 1e9
            hbm = in_gbps * m / k
            lr.update({"input_GBps" + tag: round(in_gbps, 1), "hbm_GBps" + tag: round(hbm, 1),
                       "frac_of_peak" + tag: round(hbm / HBM_PEAK_GBPS, 4), "ms_per_launch" + tag: round(ms, 4)})
        res["layouts"][layout] = lr
        del src, dst
        torch.cuda.empty_cache()
    om = res["layouts"]["object-major"]
    res.update({key: om[key] for key in ("kernel", "input_GBps", "hbm_GBps", "frac_of_peak", "ms_per_launch",
                                         "frac_of_peak_warm")})
    return res


FIRST_SEEN_PATTERNS = 5

# Decode legs on the workloads' padded rows carry the same row-padding contract
# as the timed loop (FEC_FLAG_ROW_PADDING: rows end on whole 128-byte lines).
ROW_PADDING_FLAGS = capi.FEC_FLAG_ASYNC | capi.FEC_FLAG_ROW_PADDING


def run_first_seen(npat=FIRST_SEEN_PATTERNS):
    """first_seen_decode leg: cfg4's shape (K=20/M=60, 1024 x 1 MiB stripes,
    rows 256-byte aligned), decoded from `npat` erasure patterns the process
    has never seen, each from 20 of the 40 parity blocks (every primary lost:
    r = 20 rows recovered per stripe), with the JIT policy as shipped: no
    compiled kernel exists for a first-seen matrix, so each runs on
    matapply_bsr (zfec/fec.c:527-557 decodes every pattern on one path).
    Beside it the same decode of the one pattern whose bit-sliced kernel is
    compiled (parity blocks 40..59, fec_jit_prepare_decode).  Every launch is
    one decode between HIP events after the received blocks are staged into
    slot order (outside the events), one untimed launch of each kind first;
    every result is checked against the data."""
    k, m, ns = 20, 60, 1024
    r = m - k
    sz = -(-(1 << 20) // k)
    ld = row_stride(sz)
    # the code first, then its data, as a caller does: fec_new starts loading the
    # code's compiled encode kernel from the JIT disk cache in the background
    t_new = time.perf_counter()
    code = capi.Code(k, m)
    gen = torch.Generator(device="cuda").manual_seed(2060)
    data = torch.randint(0, 256, (ns, k, ld), dtype=torch.uint8, device="cuda", generator=gen)
    par = torch.empty((ns, r, ld), dtype=torch.uint8, device="cuda")
    recv = torch.empty((ns, k, ld), dtype=torch.uint8, device="cuda")
    out = torch.empty((ns, k, ld), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    nums = list(range(k, m))

    host = {}

    def enc_once(order, leg):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(stream)
        h0 = time.perf_counter()
        code.encode_batch(data.data_ptr(), ld, k * ld, par.data_ptr(), ld, r * ld, order, sz, ns,
                          stream=stream.cuda_stream, flags=ROW_PADDING_FLAGS)
        host["ms"] = (time.perf_counter() - h0) * 1e3
        b.record(stream)
        kern = capi.last_kernel_name()
        LEGS.add(leg, kern)
        torch.cuda.synchronize()
        return a.elapsed_time(b), kern

    # the process's first launch of this code's encode matrix (host work of the
    # launch -- the routine table's address probe, the address-table upload --
    # inside the events), then the same launch again
    # the prefetch (source hash, cached code object, module load and a no-work
    # launch on this device: ~10 ms) has finished before the first launch, as it
    # has for a caller whose data takes longer than that to arrive; a launch
    # during it contends with it inside the HIP runtime (5 ms of host time)
    capi.jit_wait()
    prefetch_ms = (time.perf_counter() - t_new) * 1e3
    t_first, k_first = enc_once(nums, "first-launch encode setup")
    h_first = host["ms"]
    t_second, _ = enc_once(nums, "first-launch encode setup")
    ref = par[::97, :, :sz].clone()  # a sample of stripes: the parity every later encode is checked against

    def enc_check(order):
        got = par[::97, :, :sz]
        for j, b in enumerate(order):
            assert torch.equal(got[:, j], ref[:, b - k]), "first-launch encode != the code's parity"

    jit_slots = list(range(m - k, m))
    code.jit_prepare_decode(jit_slots)  # loads (or compiles) the compiled kernel of this one pattern
    rng = np.random.default_rng(5005)
    seen = {tuple(jit_slots)}

    def fresh_slots():
        while True:
            sl = tuple(sorted(int(x) for x in rng.choice(np.arange(k, m), size=k, replace=False)))
            if sl not in seen:
                seen.add(sl)
                return list(sl)

    def one(sl, leg):
        for j, s in enumerate(sl):
            recv[:, j].copy_(par[:, s - k])
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        code.decode_batch(recv.data_ptr(), ld, k * ld, out.data_ptr(), ld, k * ld, sl, sz, ns,
                          stream=stream.cuda_stream, flags=ROW_PADDING_FLAGS)
        b.record(stream)
        kern = capi.last_kernel_name()
        LEGS.add(leg, kern)
        torch.cuda.synchronize()
        assert torch.equal(out[:, :, :sz], data[:, :, :sz]), "first-seen decode != input"
        return a.elapsed_time(b), kern

    res = {"shape": "K=20/M=60, %d x 1 MiB stripes (sz %d, row stride %d), decode of all %d primaries from %d parity "
                    "blocks" % (ns, sz, ld, k, k),
           "algorithmic_bytes_per_launch": (k + k) * sz * ns, "patterns": npat}
    hbm = lambda ms: (k + k) * sz * ns / (ms * 1e-3) / 1e9
    for tag, pick, leg in (("first_seen", fresh_slots, "first-seen decode"),
                           ("jit", lambda: jit_slots, "first-seen jit decode")):
        one(pick(), leg + " (untimed)")
        rows = [one(pick(), leg) for _ in range(npat)]
        ms = [x for x, _ in rows]
        kern = sorted(set(n for _, n in rows))
        mean = float(np.mean(ms))
        e = {"kernel": kern[0] if len(kern) == 1 else kern, "ms_mean": round(mean, 4),
             "ms_min": round(float(np.min(ms)), 4), "ms_max": round(float(np.max(ms)), 4),
             "hbm_GBps": round(hbm(mean), 1), "frac_of_peak": round(hbm(mean) / HBM_PEAK_GBPS, 4),
             "input_GBps": round(k * sz * ns / (mean * 1e-3) / 1e9, 1)}
        if len(kern) == 1:
            e["valu_roofline"] = valu_roofline("first_seen", kern[0], mean)
        res[tag] = e
    res["first_seen_vs_jit"] = round(res["jit"]["ms_mean"] / res["first_seen"]["ms_mean"], 4)
    # first_launch_encode: encodes of all 40 parity rows in `npat` row orders the
    # process has never launched (each order a new matrix, so each launch is a
    # first launch: no compiled kernel exists for it), against the compiled
    # kernel of the natural order (fec_jit_prepare_encode)
    hbm_e = lambda ms: (k + r) * sz * ns / (ms * 1e-3) / 1e9
    fl = {"shape": "K=20/M=60, %d x 1 MiB stripes, encode of all %d parity rows" % (ns, r),
          "algorithmic_bytes_per_launch": (k + r) * sz * ns,
          "process_first_launch": {"kernel": k_first, "ms_incl_host": round(t_first, 4),
                                   "host_ms": round(h_first, 4), "second_launch_ms": round(t_second, 4),
                                   "since_fec_new_ms": round(prefetch_ms, 1),
                                   "note": "the process's first launch of the code's encode (natural row order), "
                                           "between events that also hold its host work, after fec_new's prefetch of "
                                           "the compiled kernel from the JIT disk cache (zfec_amd/jit_cache/, "
                                           "written by tools/jit_warm.py at build) has finished (since_fec_new_ms: "
                                           "construction, 4 GiB of buffers, the prefetch)"}}
    orders = [nums[i:] + nums[:i] for i in range(1, npat + 2)]
    enc_once(orders[0], "first-launch encode (untimed)")
    enc_check(orders[0])
    rows = []
    for o in orders[1:]:
        rows.append(enc_once(o, "first-launch encode"))
        enc_check(o)
    code.jit_prepare_encode(nums)
    enc_once(nums, "first-launch jit encode (untimed)")
    jrows = [enc_once(nums, "first-launch jit encode") for _ in range(npat)]
    enc_check(nums)
    for tag, rr in (("first_launch", rows), ("jit", jrows)):
        ms = [x for x, _ in rr]
        kern = sorted(set(n for _, n in rr))
        mean = float(np.mean(ms))
        e = {"kernel": kern[0] if len(kern) == 1 else kern, "ms_mean": round(mean, 4),
             "ms_min": round(float(np.min(ms)), 4), "ms_max": round(float(np.max(ms)), 4),
             "hbm_GBps": round(hbm_e(mean), 1), "frac_of_peak": round(hbm_e(mean) / HBM_PEAK_GBPS, 4),
             "input_GBps": round(k * sz * ns / (mean * 1e-3) / 1e9, 1)}
        if len(kern) == 1:
            e["valu_roofline"] = valu_roofline("first_seen", kern[0], mean)  # (the same counter run)
        fl[tag] = e
    fl["first_launch_vs_jit"] = round(fl["jit"]["ms_mean"] / fl["first_launch"]["ms_mean"], 4)
    fl["timing"] = ("one encode launch per row order between HIP events, the orders rotations of the 40 parity "
                    "numbers the process has not launched (each a matrix with no compiled kernel), JIT mode as "
                    "shipped; one untimed launch of each kind first; parity checked on a sample of stripes")
    res["first_launch_encode"] = fl
    res["timing"] = ("one decode launch per pattern between HIP events (staging copies outside), JIT mode as "
                     "shipped (auto): a first-seen matrix has no compiled kernel; one untimed launch of each kind "
                     "first")
    del data, par, recv, out
    torch.cuda.empty_cache()
    return res


def dry_run(args):
    """--dry-run: the ranks and their process group, no GPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=int(os.environ.get("RANK", "0")), world_size=world,
                            init_method=None if world > 1 else "tcp://127.0.0.1:%d" % _free_port())
    t = torch.tensor([1.0])
    dist.all_reduce(t)
    if dist.get_rank() == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_seen": dist.get_world_size(),
                          "ranks_reduced": int(t.item())}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    if args.dry_run:
        return dry_run(args)
    dist, rank, world = dist_setup(args.gpus)
    if args.workload == "first_seen":
        if world != 1:
            raise SystemExit("--workload first_seen runs on one GPU")
        fs = run_first_seen()
        if args.legs_out:
            with open(args.legs_out, "w") as f:
                json.dump({"workload": "first_seen", "legs": LEGS.runs}, f)
        print(json.dumps({"first_seen_decode": fs}), flush=True)
        return
    ranks_seen = dist.get_world_size() if dist is not None else 1
    if ranks_seen != args.gpus:
        raise SystemExit("bench.py: the process group has %d ranks, --gpus %d" % (ranks_seen, args.gpus))
    k, m, stripe, nstripes, scaling = WORKLOADS[args.workload]
    r = m - k
    sz = -(-stripe // k)
    sz_block = sz
    if args.slabs:
        if nstripes != 1:
            raise SystemExit("--slabs applies to the single-stripe workloads (cfg2, cfg3)")
        # this rank's columns [c0, c1) of every block; held on its GPU as blocks of c1 - c0 bytes
        c0, c1 = slab_range(sz, world, rank)
        sz, ns, scaling = c1 - c0, 1, "strong"
    elif scaling == "strong":
        s0, s1 = shard_range(nstripes, world, rank)
        ns = s1 - s0
    else:
        ns = nstripes
    fresh = args.fresh if args.fresh is not None else (20 if args.workload in ("cfg3", "cfg4") else 0)
    if args.streams is None:
        args.streams = 1 if args.workload == "cfg3" or args.paired else 2
    t = run_workload(k, m, sz, ns, args.steps, args.warmup, dist, use_graph=args.graph, layout=args.layout,
                     streams=args.streams, paired=args.paired,
                     row_padding=not args.no_row_padding, fresh=fresh if rank == 0 else 0)
    el = reduce(dist, t["elapsed_s"], dist.ReduceOp.MAX if dist else None)
    total_bytes = reduce(dist, float(args.steps * 2 * k * sz * ns), dist.ReduceOp.SUM if dist else None)
    value = total_bytes / el / 1e9
    nrec = t["nrec"]
    enc_bytes = (k + r) * sz * ns    # read k blocks, write m-k blocks, per stripe
    dec_bytes = (k + nrec) * sz * ns  # read k blocks, write the recovered ones
    gbps = lambda nbytes, ms: nbytes / (ms * 1e-3) / 1e9
    desc = {"cfg2": "K=3 M=10, one 64 MiB stripe per GPU",
            "cfg3": "K=10 M=16, one 256 MiB stripe per GPU",
            "cfg4": "K=20 M=60, 1 GiB = 1024 x 1 MiB stripes split across GPUs",
            "cfg5": "K=3 M=10, 1e6 x 4 KiB objects split across GPUs"}[args.workload]
    if args.slabs:
        desc = desc.replace("stripe per GPU", "stripe split into byte-range slabs across GPUs")
    row_padding = not args.no_row_padding
    timing = ("%d launches back to back between two HIP events on the launch stream, enqueued while a spin kernel "
              "holds the stream (average launch duration, no host gaps) after untimed launches worth %.0f ms of GPU "
              "time (the clock the chip settles at under sustained load), over a rotation "
              "of %d disjoint buffer sets spanning >= 768 MiB (3x the 256 MiB Infinity Cache), so every launch "
              "reads and writes HBM; *_warm: the same on one buffer set (as the timed loop runs); "
              "launch_ms_event_pairs: mean of %d encode/decode steps as in the timed loop with a HIP event pair "
              "around each launch" % (t["b2b_launches"], WARM_MS, t["nsets"], t["pair_launches"]))
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "ranks_seen": ranks_seen,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (torch.randint bytes, resident in HBM)",
        "config": {"workload": "%s: encode (%d->%d blocks) + decode from blocks %s" % (desc, k, r, t["slots"]),
                   "name": args.workload, "k": k, "m": m, "stripe_bytes": stripe, "stripes_per_gpu": ns,
                   "block_bytes": sz_block, "slab_bytes_rank0": sz if args.slabs else None,
                   "block_row_stride": row_stride(sz, args.layout), "row_padding": row_padding,
                   "value_counts": "input bytes of both directions per step: the encode reads k*sz and the decode "
                                   "reads k*sz per stripe, so value = 2 x stripe_roundtrip_GBps",
                   "row_padding_contract": ("FEC_FLAG_ROW_PADDING: the caller's block rows have slack up to the next "
                                            "128-byte line (row stride %d >= roundup(sz, 128)); the library may "
                                            "read and write it" % row_stride(sz, args.layout)) if row_padding
                   else "off: rows end at sz",
                   "parallelism": ("block byte range split into %d slabs (%d B on rank 0), one per GPU, no collective"
                                   % (world, sz) if args.slabs else
                                   "stripes sharded across %d GPU(s), no collective" % world)},
        "stripe_roundtrip_GBps": round(value / 2, 2),
        "roofline": {"bound": "hbm", "achieved": round(gbps(enc_bytes, t["enc_ms"]), 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(gbps(enc_bytes, t["enc_ms"]) / HBM_PEAK_GBPS, 4),
                     "traffic": None if args.slabs else pmc_traffic(args.workload),
                     "traffic_warm": None if args.slabs else pmc_traffic(args.workload, "encode warm"),
                     "kernel": "%s (encode)" % t["kernels"]["encode"], "algorithmic_bytes_per_launch": enc_bytes,
                     "launch_ms": round(t["enc_ms"], 4),
                     "achieved_warm": round(gbps(enc_bytes, t["enc_ms_warm"]), 1),
                     "frac_warm": round(gbps(enc_bytes, t["enc_ms_warm"]) / HBM_PEAK_GBPS, 4),
                     "launch_ms_warm": round(t["enc_ms_warm"], 4),
                     "launch_ms_event_pairs": round(t["enc_ms_pairs"], 4),
                     "rw_ceiling": rw_ceiling(k * sz * ns, r * sz * ns, gbps(enc_bytes, t["enc_ms"])),
                     "host_enqueue_us": round(t["enqueue_us"][0], 1),
                     "timing": timing},
        "decode_roofline": {"achieved": round(gbps(dec_bytes, t["dec_ms"]), 1),
                            "frac": round(gbps(dec_bytes, t["dec_ms"]) / HBM_PEAK_GBPS, 4),
                            "kernel": "%s (decode)" % t["kernels"]["decode"],
                            "algorithmic_bytes_per_launch": dec_bytes, "launch_ms": round(t["dec_ms"], 4),
                            "frac_warm": round(gbps(dec_bytes, t["dec_ms_warm"]) / HBM_PEAK_GBPS, 4),
                            "launch_ms_warm": round(t["dec_ms_warm"], 4),
                            "launch_ms_event_pairs": round(t["dec_ms_pairs"], 4),
                            "rw_ceiling": rw_ceiling(k * sz * ns, nrec * sz * ns, gbps(dec_bytes, t["dec_ms"]))},
        "valu_roofline": None if args.slabs else valu_roofline(args.workload, t["kernels"]["encode"], t["enc_ms"]),
        "launch": t["launch"],
        "streams": args.streams, "paired": args.paired,
        "gpu_ms_per_step": round(t["gpu_step_ms"], 4),
        "encode_input_GBps": round(gbps(k * sz * ns, t["enc_ms"]), 1),
        "decode_input_GBps": round(gbps(k * sz * ns, t["dec_ms"]), 1),
    }
    if "decode_fresh" in t:
        out["decode_fresh_pattern"] = t["decode_fresh"]
    if rank == 0 and not args.no_extra and args.workload == "cfg2":
        out["batched_1MiB"] = run_batched_1mib(20)
    if rank == 0 and not args.no_first_seen and args.workload == "cfg2":
        out["first_seen_decode"] = run_first_seen()
        out["first_launch_encode"] = out["first_seen_decode"].pop("first_launch_encode")
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            csz = min(sz, -(-(64 << 20) // k))  # sample stripes of at most 64 MiB (same K/M)
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, k, m, csz)
        except Exception as e:  # the baseline must never sink the GPU measurement
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
        if not args.no_extra and args.workload == "cfg2":
            # configs[0]: the reference's own harness (bench/bench_zfec.py), 1 thread, on the
            # reference C module, next to the same harness on this engine's bytes API
            try:
                from oracle import oracle

                ref = oracle.ref_module()
                bz = {"harness": "bench/bench_zfec.py semantics, K=3 M=10, 10^6 B, 1000 reps, 1 thread, "
                                 "reference units (MB/s = 2^20 B/s)"}
                if ref is not None:
                    bz["cpu_reference"] = bench_zfec_style(ref.Encoder, ref.Decoder)
                bz["gpu_bytes_api"] = bench_zfec_style(zfec_amd.Encoder, zfec_amd.Decoder)
                out["cpu_baseline"]["bench_zfec"] = bz
            except Exception as e:
                out["cpu_baseline"]["bench_zfec"] = {"error": repr(e)}
    if rank == 0:
        if args.legs_out:
            with open(args.legs_out, "w") as f:
                json.dump({"workload": args.workload, "legs": LEGS.runs}, f)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
