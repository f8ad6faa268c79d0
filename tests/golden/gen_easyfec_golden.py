#!/usr/bin/env python3
"""Golden vectors for easyfec from the REAL reference (zfec/easyfec.py), run in
place from /root/reference over the reference C extension built by
oracle/Makefile (oracle/_ref/_fec*.so).

    make -C oracle ref && python3 tests/golden/gen_easyfec_golden.py

Writes tests/golden/easyfec.json: per case the input (seeded numpy bytes:
seed + size, or literal hex), k, m, the sha256 of each of the m blocks the
reference's easyfec.Encoder.encode returns (full hex for small blocks), and
decode cases (share numbers, padlen) that the reference's easyfec.Decoder
round-trips.  Data only; no reference source is copied.
"""
import hashlib
import importlib.util
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402

REFPKG = "/root/reference/zfec"
_fec = oracle.ref_module()
if _fec is None:
    sys.exit("reference module not built: run `make -C oracle ref` first")

pkg = types.ModuleType("zfec")
pkg.__path__ = [REFPKG]
pkg.Encoder, pkg.Decoder, pkg.Error, pkg._fec = _fec.Encoder, _fec.Decoder, _fec.Error, _fec
sys.modules["zfec"] = pkg
spec = importlib.util.spec_from_file_location("zfec.easyfec", os.path.join(REFPKG, "easyfec.py"))
easyfec = importlib.util.module_from_spec(spec)
sys.modules["zfec.easyfec"] = easyfec
spec.loader.exec_module(easyfec)


def data_of(case):
    if "hex" in case:
        return bytes.fromhex(case["hex"])
    return np.random.default_rng(case["seed"]).integers(0, 256, size=case["size"], dtype=np.uint8).tobytes()


CASES = [
    {"hex": "", "k": 3, "m": 8}, {"hex": b"x".hex(), "k": 1, "m": 1}, {"hex": b"xy".hex(), "k": 1, "m": 3},
    {"hex": b"Yellow Whirled!".hex(), "k": 3, "m": 8}, {"hex": b"Yellow Whirled!".hex(), "k": 4, "m": 16},
    {"hex": b"abcde".hex(), "k": 4, "m": 6}, {"hex": b"ab".hex(), "k": 5, "m": 7},
    {"seed": 1, "size": 1000, "k": 3, "m": 10}, {"seed": 2, "size": 4097, "k": 3, "m": 10},
    {"seed": 3, "size": (1 << 20) + 3, "k": 3, "m": 10}, {"seed": 4, "size": 1 << 20, "k": 20, "m": 60},
    {"seed": 5, "size": 333333, "k": 10, "m": 16}, {"seed": 6, "size": 65537, "k": 7, "m": 7},
    {"seed": 7, "size": 100000, "k": 255, "m": 256}, {"seed": 8, "size": 2 * 1024 * 1024 - 1, "k": 13, "m": 16},
    {"seed": 9, "size": 12345, "k": 2, "m": 3},
]

rng = np.random.default_rng(2024)
out = {"generator": "tests/golden/gen_easyfec_golden.py", "reference": "zfec/easyfec.py", "cases": []}
for case in CASES:
    data = data_of(case)
    k, m = case["k"], case["m"]
    blocks = easyfec.Encoder(k, m).encode(data)
    assert len(blocks) == m
    bs = len(blocks[0])
    rec = dict(case)
    rec["blocksize"] = bs
    rec["padlen"] = bs * k - len(data)
    rec["block_sha256"] = [hashlib.sha256(bytes(b)).hexdigest() for b in blocks]
    if bs <= 64:
        rec["block_hex"] = [bytes(b).hex() for b in blocks]
    rec["decodes"] = []
    for t in range(3):
        nums = sorted(int(x) for x in rng.choice(m, size=k, replace=False)) if t else list(range(m - k, m))
        got = easyfec.Decoder(k, m).decode([blocks[n] for n in nums], nums, rec["padlen"])
        assert bytes(got) == data, case
        rec["decodes"].append(nums)
    out["cases"].append(rec)
with open(os.path.join(HERE, "easyfec.json"), "w") as f:
    json.dump(out, f, indent=1)
print("cases:", len(out["cases"]))
