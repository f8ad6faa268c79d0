#!/usr/bin/env python3
"""Golden callback sequences of the REAL reference's segment API
(zfec/filefec.py encode_file_stringy :450-492 and encode_file_stringy_easyfec
:494-522), run in place from /root/reference over the reference C extension
built by oracle/Makefile (oracle/_ref/_fec*.so), as gen_filefec_golden.py does.

    make -C oracle ref && python3 tests/golden/gen_segments_golden.py

Writes tests/golden/segments.json: per case (function, k, m, chunksize, input
size, input seed) the list of callback arguments, each as [indatasize, number
of blocks, sha256 of the blocks concatenated (first 16 hex digits)].  Data
only; no reference source is copied.  The reference's encode_file /
encode_file_not_really* build arrays with the Python 2 typecode 'c' (and
sha1.new), which Python 3 rejects; the generator records that they raise.
"""
import hashlib
import importlib.util
import io
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


def load(name):
    spec = importlib.util.spec_from_file_location("zfec." + name, os.path.join(REFPKG, name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["zfec." + name] = mod
    spec.loader.exec_module(mod)
    setattr(pkg, name, mod)
    return mod


load("easyfec")
filefec = load("filefec")

# (k, m, chunksize, size): empty and one-byte files, whole segments, a final
# segment of exactly (k-1)*chunksize bytes, ragged sizes, wide codes
CASES = [(3, 10, 4096, 0), (3, 10, 4096, 1), (3, 10, 4096, 3 * 4096 * 5), (3, 10, 4096, 3 * 4096 * 4 + 2 * 4096),
         (3, 10, 4096, 100_003), (5, 9, 1000, 123_456), (1, 3, 512, 5000), (20, 60, 4096, (1 << 20) + 77),
         (2, 3, 1, 17), (4, 4, 333, 9999), (7, 13, 64, 7 * 64 * 3)]


def record(fn, k, m, chunksize, data):
    calls = []

    def cb(res, ind):
        calls.append([ind, len(res), hashlib.sha256(b"".join(bytes(b) for b in res)).hexdigest()[:16]])

    fn(io.BytesIO(data), cb, k, m, chunksize)
    return calls


out = {"generator": "tests/golden/gen_segments_golden.py", "cases": [], "python2_only": {}}
for name in ("encode_file", "encode_file_not_really", "encode_file_not_really_and_hash"):
    try:
        getattr(filefec, name)(io.BytesIO(b"abc"), lambda *a: None, 2, 3, 4)
        out["python2_only"][name] = "ran"
    except Exception as e:  # array typecode 'c' / sha1.new are Python 2
        out["python2_only"][name] = "%s: %s" % (type(e).__name__, e)
for fn in ("encode_file_stringy", "encode_file_stringy_easyfec"):
    for k, m, chunksize, size in CASES:
        seed = size * 31 + k
        data = np.random.default_rng(seed).integers(0, 256, size=size, dtype=np.uint8).tobytes()
        out["cases"].append({"fn": fn, "k": k, "m": m, "chunksize": chunksize, "size": size, "seed": seed,
                             "calls": record(getattr(filefec, fn), k, m, chunksize, data)})
path = os.path.join(HERE, "segments.json")
with open(path, "w") as f:
    json.dump(out, f, indent=0)
print("wrote", path, len(out["cases"]), "cases", out["python2_only"])
