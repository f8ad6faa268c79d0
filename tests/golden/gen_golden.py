#!/usr/bin/env python3
"""Generate golden vectors from the REAL reference (zfec/fec.c + zfec/_fecmodule.c).

Run in the build container, where /root/reference exists:

    make -C oracle ref && python3 tests/golden/gen_golden.py

The reference is compiled from its own sources by oracle/Makefile into
oracle/_ref/_fec*.so and imported here through its own Python API
(zfec/_fecmodule.c: Encoder.encode, Decoder.decode, test_from_agl).  Only
data is written: tests/golden/golden.npz (arrays) and golden.json (digests,
parameters).  These fixtures pin both the CPU oracle and the HIP path.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle  # noqa: E402

ref = oracle.ref_module()
if ref is None:
    sys.exit("reference module not built: run `make -C oracle ref` first")


def sha(b):
    return hashlib.sha256(b).hexdigest()


def ref_enc_matrix(k, m):
    """E (m x k) read back through the reference's public encode: input block
    i is the unit vector e_i (k bytes), so parity block r byte j = E[r][j]."""
    blocks = [bytes(1 if j == i else 0 for j in range(k)) for i in range(k)]
    out = ref.Encoder(k, m).encode(blocks)
    return np.frombuffer(b"".join(out), dtype=np.uint8).reshape(m, k).copy()


def ref_encode(k, m, blocks, nums=None):
    enc = ref.Encoder(k, m)
    bl = [bytes(b) for b in blocks]
    out = enc.encode(bl, nums) if nums is not None else enc.encode(bl)
    return [bytes(x) for x in out]


def ref_decode(k, m, blocks, nums):
    return [bytes(x) for x in ref.Decoder(k, m).decode([bytes(b) for b in blocks], list(nums))]


arrays = {}
meta = {"generator": "tests/golden/gen_golden.py", "reference": "zfec/fec.c + zfec/_fecmodule.c (oracle/_ref)"}

# 1. Encoding matrices.  Parity row r depends on (k, r) only, so (k, 256)
#    covers every m; digests for every k, full matrices for a selection.
meta["enc_matrix_sha256_m256"] = {}
full_ks = [1, 2, 3, 4, 5, 7, 8, 10, 13, 16, 20, 32, 64, 128, 255, 256]
for k in range(1, 257):
    E = ref_enc_matrix(k, 256)
    meta["enc_matrix_sha256_m256"][str(k)] = sha(E.tobytes())
    if k in full_ks:
        arrays["enc_k%d_m256" % k] = E
# prefix property spot checks (rows of (k, m) == first m rows of (k, 256))
for k, m in [(3, 10), (3, 5), (10, 16), (20, 60), (1, 1), (7, 9), (128, 200)]:
    E = ref_enc_matrix(k, m)
    assert (E == ref_enc_matrix(k, 256)[:m]).all(), (k, m)
    arrays["enc_k%d_m%d" % (k, m)] = E

# 2. test_from_agl (zfec/_fecmodule.c:614-659): k=3, n=5, 8-byte blocks.
assert ref.test_from_agl()
b = [b"\x01" * 8, b"\x02" * 8, b"\x03" * 8]
p3, p4 = ref_encode(3, 5, b, (3, 4))
meta["agl"] = {"k": 3, "m": 5, "parity3": p3.hex(), "parity4": p4.hex()}

# 3. Pattern KATs at the config block sizes.
meta["pattern_kat"] = []
for k, m, sz in [(3, 10, 349525), (10, 16, 104858), (20, 60, 52429), (3, 10, 1366), (3, 10, 333334)]:
    blocks = oracle.pattern_blocks(k, sz)
    out = ref_encode(k, m, blocks)
    par = b"".join(out[k:])
    sec = list(range(k, 2 * k)) if 2 * k <= m else list(range(m - k, m))
    dec = ref_decode(k, m, [out[i] for i in sec], sec)
    assert b"".join(dec) == blocks.tobytes()
    meta["pattern_kat"].append({"k": k, "m": m, "sz": sz, "parity_sha256": sha(par),
                                "parity0_head": out[k][:8].hex(), "parity_last_tail": out[-1][-8:].hex()})

# 4. Full small vectors: random inputs, every parity block, and decodes from
#    assorted erasure patterns (including all-secondary and mixed).
rng = np.random.default_rng(20261015)
cases = [(1, 1, 5), (1, 4, 9), (2, 3, 16), (3, 5, 8), (3, 10, 33), (3, 10, 1), (4, 16, 17),
         (5, 8, 64), (10, 16, 100), (13, 16, 31), (20, 60, 40), (32, 64, 19), (64, 255, 7),
         (128, 256, 5), (255, 256, 3), (256, 256, 2), (100, 200, 0)]
meta["vectors"] = []
for ci, (k, m, sz) in enumerate(cases):
    blocks = rng.integers(0, 256, size=(k, sz), dtype=np.uint8)
    out = ref_encode(k, m, blocks)
    arrays["vec%d_in" % ci] = blocks
    arrays["vec%d_all" % ci] = np.frombuffer(b"".join(out), dtype=np.uint8).reshape(m, sz).copy()
    # desired-order / subset encode
    nums = [int(x) for x in rng.permutation(m)[: min(m, 5)]]
    sub = ref_encode(k, m, blocks, nums)
    arrays["vec%d_subset" % ci] = np.frombuffer(b"".join(sub), dtype=np.uint8).reshape(len(nums), sz).copy()
    decs = []
    for trial in range(3):
        pick = sorted(int(x) for x in rng.choice(m, size=k, replace=False))
        if trial == 0 and m >= 2 * k:
            pick = list(range(m - k, m))  # secondary-only
        order = [int(x) for x in rng.permutation(k)]
        got_nums = [pick[i] for i in order]
        dec = ref_decode(k, m, [out[i] for i in got_nums], got_nums)
        assert b"".join(dec) == blocks.tobytes()
        decs.append(got_nums)
    meta["vectors"].append({"k": k, "m": m, "sz": sz, "subset_nums": nums, "decode_nums": decs})

# 5. Decode matrices (rows for the missing primaries), read back through the
#    reference decode of unit-vector blocks: slot c carries e_c, so the
#    recovered primary r has byte c = D[r][c].
meta["decode_rows"] = []
for k, m, nums in [(3, 10, [3, 4, 5]), (3, 10, [0, 7, 9]), (10, 16, [10, 11, 12, 13, 14, 15, 6, 7, 8, 9]),
                   (20, 60, list(range(40, 60))), (5, 8, [7, 1, 6, 3, 5])]:
    slots = [bytes(1 if j == c else 0 for j in range(k)) for c in range(k)]
    # the reference reorders so primary i sits in slot i; build inputs already in that order
    order = [None] * k
    rest = [n for n in nums if n >= k]
    for n in nums:
        if n < k:
            order[n] = n
    it = iter(rest)
    order = [o if o is not None else next(it) for o in order]
    dec = ref_decode(k, m, slots, order)
    rows = [dec[i] for i in range(k) if order[i] >= k]
    arrays["decrows_k%d_m%d_%s" % (k, m, "_".join(map(str, nums)))] = np.frombuffer(b"".join(rows), dtype=np.uint8).reshape(len(rows), k).copy()
    meta["decode_rows"].append({"k": k, "m": m, "slot_nums": order, "key": "decrows_k%d_m%d_%s" % (k, m, "_".join(map(str, nums)))})

np.savez_compressed(os.path.join(HERE, "golden.npz"), **arrays)
with open(os.path.join(HERE, "golden.json"), "w") as f:
    json.dump(meta, f, indent=1, sort_keys=True)
print("wrote", len(arrays), "arrays;", os.path.getsize(os.path.join(HERE, "golden.npz")), "bytes npz")
