"""Child process of tests/test_gpu_parity.py::test_batch_layout_env_variants.

Runs one fec_encode_batch over a strided layout under whatever ZFEC_HIP_*
environment the parent set (the library reads those knobs once per process)
and saves the whole output buffer, guard bytes included, for the parent to
compare across variants and against the oracle.

usage: python tests/gpu_batch_child.py '<json spec>' out.npy
spec: k, m, sz, ns, in_bs, in_ss, out_bs, out_ss, seed, guard, flags
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def src_bytes(spec):
    n = (spec["ns"] - 1) * spec["in_ss"] + (spec["k"] - 1) * spec["in_bs"] + spec["sz"]
    return np.random.default_rng(spec["seed"]).integers(0, 256, size=n, dtype=np.uint8)


def dst_len(spec):
    r = spec["m"] - spec["k"]
    return (spec["ns"] - 1) * spec["out_ss"] + (r - 1) * spec["out_bs"] + spec["sz"] + spec["guard"]


def main():
    import torch

    from zfec_amd import capi

    spec = json.loads(sys.argv[1])
    k, m = spec["k"], spec["m"]
    src = torch.from_numpy(src_bytes(spec)).cuda()
    dst = torch.full((dst_len(spec),), 0xA5, dtype=torch.uint8, device="cuda")
    code = capi.Code(k, m)
    code.encode_batch(src.data_ptr(), spec["in_bs"], spec["in_ss"], dst.data_ptr(), spec["out_bs"], spec["out_ss"],
                      list(range(k, m)), spec["sz"], spec["ns"], stream=torch.cuda.current_stream().cuda_stream,
                      flags=capi.FEC_FLAG_ASYNC | spec.get("flags", 0))
    torch.cuda.synchronize()
    np.save(sys.argv[2], dst.cpu().numpy())
    print("kernel", capi.last_kernel_name())


if __name__ == "__main__":
    main()
