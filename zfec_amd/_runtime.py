"""One HIP runtime per process.

PyTorch-ROCm wheels bundle their own libamdhip64.so / libhsa-runtime64.so
(torch/lib).  libzfec_hip.so is linked against the system ROCm runtime by
SONAME (libamdhip64.so.7).  If both copies end up in one process the second
runtime cannot open the GPU ("No HIP GPUs are available").  When torch is
installed we therefore load torch's runtime first, by path and RTLD_GLOBAL:
libzfec_hip.so's DT_NEEDED then resolves to it by SONAME, and torch's own
later load of the same file is recognised by file identity.  Without torch
the system runtime (/opt/rocm) is used.
"""
import ctypes
import importlib.util
import os

_done = False


def torch_lib_dir():
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return None
    d = os.path.join(list(spec.submodule_search_locations)[0], "lib")
    return d if os.path.isdir(d) else None


def preload():
    global _done
    if _done:
        return
    _done = True
    if os.environ.get("ZFEC_HIP_SYSTEM_RUNTIME") == "1":
        return
    d = torch_lib_dir()
    if d is None:
        return
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        p = os.path.join(d, name)
        if os.path.exists(p):
            ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
