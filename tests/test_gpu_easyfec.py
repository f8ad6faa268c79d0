"""easyfec on device tensors and on bytes, against
golden vectors made by the reference's own easyfec.py
(tests/golden/gen_easyfec_golden.py, zfec/easyfec.py:28-39 split/pad,
:45-55 join/strip): every block's sha256 for the encode direction, and the
decoded data for several received-share sets with the reference's padlen.
Device path: the primaries that lie wholly inside the data are zero-copy
views of it, and the result of a decode is a view of one device buffer."""
import hashlib
import json
import os

import numpy as np
import pytest

import zfec_amd
from zfec_amd import easyfec

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "easyfec.json")))


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if zfec_amd.device_count() < 1:
        pytest.fail("no GPU visible: the -m gpu suite must run on an MI355X")


def data_of(case):
    if "hex" in case:
        return bytes.fromhex(case["hex"])
    return np.random.default_rng(case["seed"]).integers(0, 256, size=case["size"], dtype=np.uint8).tobytes()


def sha(b):
    if isinstance(b, (bytes, bytearray)):
        return hashlib.sha256(bytes(b)).hexdigest()
    return hashlib.sha256(b.cpu().numpy().tobytes()).hexdigest()


def ids(case):
    return "k%d_m%d_n%d" % (case["k"], case["m"], case.get("size", len(case.get("hex", "")) // 2))


@pytest.mark.parametrize("case", GOLD["cases"], ids=ids)
def test_easyfec_device_vs_reference(case):
    data = data_of(case)
    k, m = case["k"], case["m"]
    t = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
    blocks = easyfec.Encoder(k, m).encode(t)
    assert len(blocks) == m
    assert all(zfec_amd._is_device_tensor(b) and b.numel() == case["blocksize"] for b in blocks)
    assert [sha(b) for b in blocks] == case["block_sha256"]
    # primaries wholly inside the data are views of it (no copy)
    cs = case["blocksize"]
    for i in range(k):
        if cs and (i + 1) * cs <= len(data):
            assert blocks[i].data_ptr() == t.data_ptr() + i * cs, i
    for nums in case["decodes"]:
        got = easyfec.Decoder(k, m).decode([blocks[n] for n in nums], nums, case["padlen"])
        assert zfec_amd._is_device_tensor(got)
        assert got.numel() == len(data)
        assert got.cpu().numpy().tobytes() == data, nums


@pytest.mark.parametrize("case", GOLD["cases"], ids=ids)
def test_easyfec_bytes_vs_reference(case):
    data = data_of(case)
    k, m = case["k"], case["m"]
    blocks = easyfec.Encoder(k, m).encode(data)
    assert [sha(b) for b in blocks] == case["block_sha256"]
    if "block_hex" in case:
        assert [bytes(b).hex() for b in blocks] == case["block_hex"]
    for nums in case["decodes"]:
        got = easyfec.Decoder(k, m).decode([blocks[n] for n in nums], nums, case["padlen"])
        assert got == data, nums


def test_easyfec_device_non_uint8_and_errors():
    """A float tensor is encoded as its bytes (same blocks as the bytes path);
    a non-contiguous tensor is rejected; a padlen past the data gives what the
    reference's slicing gives (zfec/easyfec.py:53-55), an empty result."""
    x = torch.arange(1001, dtype=torch.float32, device="cuda")
    dev = easyfec.Encoder(4, 7).encode(x)
    host = easyfec.Encoder(4, 7).encode(x.cpu().numpy().tobytes())
    assert [b.cpu().numpy().tobytes() for b in dev] == host
    with pytest.raises(zfec_amd.Error):
        easyfec.Encoder(2, 3).encode(torch.zeros((4, 4), dtype=torch.uint8, device="cuda")[:, 0])
    big = easyfec.Decoder(4, 7).decode([dev[n] for n in (3, 4, 5, 6)], [3, 4, 5, 6], 10 ** 6)
    assert big.numel() == 0
    assert easyfec.Decoder(4, 7).decode([host[n] for n in (3, 4, 5, 6)], [3, 4, 5, 6], 10 ** 6) == b""
