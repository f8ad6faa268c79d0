"""CPU checks of the generated source of the bit-sliced kernels' double-buffered
LDS-DMA phases (zfec_amd/csrc/bitslice.cpp, the shared-input form of the
zfec/fec.c:487-505 / :527-557 apply): every tile branch meets the same
barriers, every LDS-DMA target and plane read stays inside the declared LDS,
each wave waits for one DMA'd phase per phase of the matrix, and a kernel whose
inputs all fit keeps its single register-loaded phase.  No GPU: the kernels are
generated and compiled for gfx950 by hipRTC here."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def place(nums, k):
    """slot order with primary i at slot i (zfec/_fecmodule.c:482-493)."""
    slots = [None] * k
    sec = iter([n for n in nums if n >= k])
    for n in nums:
        if n < k:
            slots[n] = n
    return [s if s is not None else next(sec) for s in slots]


def generated(tmp_path, monkeypatch, k, m, decode):
    """The generated source of the kernel of a K/M encode (all parity rows) or
    decode (from the last k blocks), compiled in a fresh process: the JIT
    registry is per process, and another test's code may already hold the
    kernel in memory (fec_new prefetches the kernels the in-tree cache holds),
    which would compile -- and dump -- nothing."""
    dump = tmp_path / "dump"
    dump.mkdir()
    env = dict(os.environ, ZFEC_HIP_JIT_CACHE=str(tmp_path / "cache"), ZFEC_HIP_JIT_DUMP=str(dump))
    nums = place(list(range(m - k, m)), k) if decode else list(range(k, m))
    prog = ("import sys; sys.path.insert(0, %r)\n"
            "from zfec_amd import capi\n"
            "c = capi.Code(%d, %d)\n"
            "c.%s(%r)\n" % (ROOT, k, m, "jit_prepare_decode" if decode else "jit_prepare_encode", nums))
    subprocess.run([sys.executable, "-c", prog], env=env, check=True, timeout=300)
    files = list(dump.glob("zfec_hip_bitslice_k%d_r*.hip" % k))
    assert len(files) == 1, files
    return files[0].read_text()


# decodes from the last k blocks: r = 18 / 27 / 20 rows on 2 / 3 / 2 tiles, phases of 4 with a
# short last one for k = 17 and 23; 30/70's decode from its last 30 blocks: r = 30 on 3 tiles,
# 8 phases (the last of 2)
@pytest.mark.parametrize("k,m,decode", [(17, 35, True), (23, 50, True), (20, 60, True), (30, 70, True)])
def test_dma_phase_structure(tmp_path, monkeypatch, k, m, decode):
    src = generated(tmp_path, monkeypatch, k, m, decode=decode)
    size = int(re.search(r"__shared__ u32x4 sh\[(\d+)\]", src).group(1))
    assert size == 2 * 4 * 128, size  # two phases of 4 inputs, 128 u32x4 each
    # every DMA target and every plane access inside the declared LDS
    for off in re.findall(r"sh \+ (\d+)u", src):
        assert int(off) + 64 <= size, off
    for off in re.findall(r"sh\[(\d+)u \+ lane\]", src):
        assert int(off) + 64 <= size, off
    body = src[src.index("while (s < a.nstripes)"):]
    branches = re.split(r"if \(tile == \d+u\) \{", body)[1:]
    nphases = -(-k // 4)
    bars = [b.count("__syncthreads()") for b in branches]
    bars[-1] -= 1  # the unit's closing barrier follows the last branch
    assert len(set(bars)) == 1 and bars[0] == nphases, bars
    for b in branches:
        # one wait per phase, each after the DMA it waits for
        assert b.count("dma_wait()") == nphases
        assert b.index("dma16(") < b.index("dma_wait()")
        assert b.count("dma16(") >= 2 * (nphases - 1)


@pytest.mark.parametrize("k,m", [(20, 60), (30, 70)])
def test_single_phase_kernel_keeps_register_loads(tmp_path, monkeypatch, k, m):
    """4-tile kernels (r = 40 encodes) load through registers in one phase of
    all k inputs: DMA phases lost 2-8 % on K=20/M=60 (profiles/r05_lds_dma_ab.json)
    and 2.3 % on 30/70 (profiles/r06_jit_dma_tiles_ab.json)."""
    src = generated(tmp_path, monkeypatch, k, m, decode=False)
    assert "dma16(ka->" not in src and "dma_wait();" not in src
    assert int(re.search(r"__shared__ u32x4 sh\[(\d+)\]", src).group(1)) == k * 128
