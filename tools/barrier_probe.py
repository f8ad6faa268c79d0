#!/usr/bin/env python3
"""Cost of the timing barrier bench.py brackets its timed steps with, under
torchrun (RCCL): dist.barrier(), an all_reduce of a preallocated one-element
device tensor + synchronize, and a barrier on a gloo group.  Median and max
microseconds over 50 calls after 5 warm-up calls.

  ZFEC_BENCH_DIST=1 python -m torch.distributed.run --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29519 tools/barrier_probe.py
"""
import json
import os
import statistics
import time

import torch
import torch.distributed as dist


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    gloo = dist.new_group(backend="gloo")
    t = torch.zeros(1, device="cuda")

    def ar():
        dist.all_reduce(t)
        torch.cuda.synchronize()

    def bar():
        dist.barrier()
        torch.cuda.synchronize()

    def gbar():
        dist.barrier(group=gloo)

    res = {"world": dist.get_world_size()}
    for name, fn in (("dist.barrier", bar), ("all_reduce_1elem_sync", ar), ("gloo_barrier", gbar)):
        for _ in range(5):
            fn()
        ts = []
        for _ in range(50):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        res[name + "_us_median"] = round(statistics.median(ts) * 1e6, 1)
        res[name + "_us_max"] = round(max(ts) * 1e6, 1)
    if dist.get_rank() == 0:
        print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
