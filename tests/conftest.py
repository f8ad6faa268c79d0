import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def golden():
    import json
    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "golden.json")) as f:
        meta = json.load(f)
    arrays = dict(np.load(os.path.join(d, "golden.npz"), allow_pickle=False))
    return meta, arrays


@pytest.fixture
def knobs(monkeypatch):
    """Set ZFEC_HIP_* environment knobs for one test.  The library reads them
    once per process, so they are re-read (fec_reload_config) after being set
    and again after the test has restored the environment."""
    from zfec_amd import capi

    def set_knobs(**kv):
        for key, val in kv.items():
            monkeypatch.setenv(key, str(val))
        capi.reload_config()

    yield set_knobs
    monkeypatch.undo()
    capi.reload_config()
