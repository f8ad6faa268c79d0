"""bench.py's multi-rank path, run as the driver runs it on an
8-GPU node -- torchrun, one process per rank, rank 0 printing the JSON line --
but with two ranks sharing the one GPU of the test box over gloo
(ZFEC_BENCH_BACKEND=gloo; the driver's runs use RCCL, one rank per GPU).  It
checks the process setup, the shared-memory timing barrier, the max/sum
reductions, the stripe sharding of cfg4 and the byte-range slabs of cfg2, and
that every rank's timed loop passed its own round-trip asserts (a rank that
fails them exits non-zero, and torchrun with it)."""
import json
import math
import os
import socket
import subprocess
import sys

import pytest

import zfec_amd

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if zfec_amd.device_count() < 1:
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(args, launcher=True):
    """launcher=False: a plain `python bench.py --gpus 2`, which starts its two
    ranks itself (bench.py launch_ranks), as the driver's command shape does."""
    env = dict(os.environ)
    env["ZFEC_BENCH_BACKEND"] = "gloo"
    env.setdefault("OMP_NUM_THREADS", "4")
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + args
    if launcher:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
               "127.0.0.1", "--master-port", str(_free_port())] + cmd[1:]
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert res.returncode == 0, (res.stdout[-3000:], res.stderr[-3000:])
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-3000:]  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.timeout(300)
def test_bench_two_ranks_cfg4_sharded():
    out = _torchrun(["--workload", "cfg4", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-extra", "--fresh",
                     "0"])
    assert out["n_gpus"] == 2 and out["ranks_seen"] == 2
    assert out["config"]["stripes_per_gpu"] == 512  # 1024 stripes split over 2 ranks
    assert out["scaling"] == "strong"
    assert math.isfinite(out["value"]) and out["value"] > 0
    assert out["roofline"]["kernel"].startswith("zfec_hip_bitslice_k20_r40"), out["roofline"]["kernel"]


@pytest.mark.timeout(300)
def test_bench_two_ranks_cfg2_slabs():
    out = _torchrun(["--workload", "cfg2", "--steps", "3", "--warmup", "1", "--no-cpu", "--no-extra", "--slabs"])
    assert out["n_gpus"] == 2
    assert out["scaling"] == "strong"
    sz = -(-(64 << 20) // 3)
    # rank 0's slab: the first half of every block, on a 256-byte boundary
    assert out["config"]["slab_bytes_rank0"] == -(-(-(-sz // 256)) // 2) * 256
    assert math.isfinite(out["value"]) and out["value"] > 0


@pytest.mark.timeout(300)
def test_bench_gpus_flag_launches_its_ranks():
    """`python bench.py --gpus 2` with no launcher: bench.py starts the two
    ranks itself, and the line reports the world the process group saw."""
    out = _torchrun(["--workload", "cfg4", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-extra", "--fresh", "0"],
                    launcher=False)
    assert out["n_gpus"] == 2 and out["ranks_seen"] == 2
    assert out["config"]["stripes_per_gpu"] == 512
    assert math.isfinite(out["value"]) and out["value"] > 0
