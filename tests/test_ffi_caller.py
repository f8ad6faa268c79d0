"""A plain C caller of libzfec_hip.so (tests/c/ffi_caller.c): host buffers,
fec.h entry points only, many threads -- the way the reference's Haskell
binding (haskell/Codec/FEC.hs:79-114) and other FFI callers use the library,
with the properties of haskell/test/FECTest.hs.  Built with gcc at test time."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(tmp_path):
    exe = str(tmp_path / "ffi_caller")
    libdir = os.path.join(ROOT, "zfec_amd")
    subprocess.run(["gcc", "-O2", "-std=c99", "-Wall", "-Werror", os.path.join(ROOT, "tests", "c", "ffi_caller.c"),
                    "-I", os.path.join(ROOT, "include"), "-L", libdir, "-lzfec_hip", "-Wl,-rpath," + libdir,
                    "-lpthread", "-o", exe], check=True)
    return exe


def test_ffi_caller_builds(tmp_path):
    """The header compiles as C99 and the program links against the library (CPU)."""
    assert os.path.exists(build(tmp_path))


@pytest.mark.gpu
def test_ffi_caller_runs(tmp_path):
    exe = build(tmp_path)
    p = subprocess.run([exe, "25"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.startswith("ok:")
