"""zfec_amd -- zfec's erasure-coding API on AMD MI355X (gfx950).

Drop-in for the reference's Python surface (/root/reference/zfec/__init__.py:12,
zfec/_fecmodule.c): ``Encoder(k, m).encode(inblocks, desired_blocks_nums=None)``,
``Decoder(k, m).decode(blocks, blocknums)``, ``Error``, ``easyfec``.

Bytes-like blocks (bytes, bytearray, memoryview, C-contiguous numpy arrays)
are staged to the GPU and the results come back as ``bytes``, exactly as the
reference returns them.  Device-resident blocks (torch tensors on a ROCm
device) stay on the device: the work is enqueued on the tensor's current
stream and the results are new device tensors.  All GF(2^8) arithmetic runs
in the HIP kernels of libzfec_hip.so; there is no CPU fallback -- importing
fails if the extension is not built, and encode/decode raise ``Error`` when no
GPU is visible.
"""
from . import _runtime

_runtime.preload()  # must precede loading libzfec_hip.so (see _runtime.py)

from . import _fec  # noqa: E402
from ._fec import Error, device_count, test_from_agl, version

__version__ = "0.1.0"

__all__ = ["Encoder", "Decoder", "Error", "easyfec", "filefec", "cmdline_zfec", "cmdline_zunfec", "test_from_agl",
           "device_count", "version", "reuse_host_memory"]


def _is_device_tensor(x):
    return type(x).__module__.startswith("torch") and getattr(x, "is_cuda", False)


def _byte_view(t):
    import torch

    if not t.is_contiguous():
        raise Error("Precondition violation: Input blocks are required to be C-contiguous.")
    return t.reshape(-1) if t.dtype == torch.uint8 else t.reshape(-1).view(torch.uint8)


def _stream_handle(device):
    import torch

    return torch.cuda.current_stream(device).cuda_stream


def _device_blocks(blocks, k):
    for b in blocks:
        if not _is_device_tensor(b):
            raise Error("Precondition violation: blocks are required to be all device tensors or all host buffers")
    bl = [_byte_view(b) for b in blocks]
    if len(bl) != k:
        raise Error(
            "Precondition violation: Wrong length -- first argument (the sequence of input blocks) is required to "
            "contain exactly k blocks.  len(first): %d, k: %d" % (len(bl), k)
        )
    sz = bl[0].numel() if bl else 0
    dev = bl[0].device if bl else None
    for b in bl:
        if b.numel() != sz:
            raise Error(
                "Precondition violation: Input blocks are required to be all the same length.  length of one block "
                "was: %d, length of another block was: %d" % (sz, b.numel())
            )
        if b.device != dev:
            raise Error("Precondition violation: device blocks are required to be on one device")
    return bl, sz, dev


def _is_host_array(x):
    return type(x).__module__ == "numpy" and hasattr(x, "ctypes")


def _batch_view(blocks, nblocks, what):
    """Check a [nstripes, nblocks, sz] uint8 array for the batched entry points:
    a device tensor, or a host numpy array (pageable memory; the library stages
    it through pinned slots, fec_abi.cpp run_batch_staged).  Any strides with
    unit stride along sz, so a transposed block-major [nblocks, nstripes, sz]
    array passes as is (fec_encode_batch runs it as one long stripe).
    Returns (nstripes, sz, block stride, stripe stride, data pointer)."""
    if _is_host_array(blocks):
        import numpy as np

        if blocks.dtype != np.uint8 or blocks.ndim != 3:
            raise Error("Precondition violation: %s is required to be a uint8 array [nstripes, %d, sz]"
                        % (what, nblocks))
        ns, nb, sz = blocks.shape
        strides = blocks.strides
        ptr = blocks.ctypes.data
    else:
        import torch

        if not _is_device_tensor(blocks) or blocks.dtype != torch.uint8 or blocks.dim() != 3:
            raise Error("Precondition violation: %s is required to be a uint8 device tensor or numpy array "
                        "[nstripes, %d, sz]" % (what, nblocks))
        ns, nb, sz = blocks.shape
        strides = (blocks.stride(0), blocks.stride(1), blocks.stride(2))
        ptr = blocks.data_ptr()
    if nb != nblocks:
        raise Error("Precondition violation: %s is required to hold %d blocks per stripe, not %d" % (what, nblocks, nb))
    if sz > 1 and strides[2] != 1:
        raise Error("Precondition violation: %s blocks are required to be contiguous along sz" % what)
    if min(strides[0], strides[1]) < 0:
        raise Error("Precondition violation: %s is required to have non-negative strides" % what)
    return ns, sz, strides[1], strides[0], ptr


def _batch_out(like, like_block_major, ns, nb, sz):
    """Output [ns, nb, sz] where `like` lives (device tensor or numpy array):
    block-major storage when the input was."""
    shape = (nb, ns, sz) if like_block_major else (ns, nb, sz)
    if _is_host_array(like):
        import numpy as np

        out = np.empty(shape, dtype=np.uint8)
        return out.transpose(1, 0, 2) if like_block_major else out
    import torch

    out = torch.empty(shape, dtype=torch.uint8, device=like.device)
    return out.transpose(0, 1) if like_block_major else out


def _batch_strides(out):
    if _is_host_array(out):
        return out.ctypes.data, out.strides[1], out.strides[0]
    return out.data_ptr(), out.stride(1), out.stride(0)


def _batch_call_args(blocks):
    """stream / flags of a batched call: a device tensor's work is enqueued on
    its current stream; host arrays are synchronous."""
    from . import capi

    if _is_host_array(blocks):
        return 0, capi.FEC_FLAG_LIBRARY_STREAM
    return _stream_handle(blocks.device), capi.FEC_FLAG_ASYNC


class _as_error(object):
    """Library failures of the batched entry points (capi.FecError: no GPU,
    cross-device tensors, ...) surface as zfec_amd.Error like every other
    failure of this API."""

    def __enter__(self):
        return self

    def __exit__(self, et, ev, tb):
        from . import capi

        if et is not None and issubclass(et, capi.FecError):
            raise Error(str(ev)) from ev
        return False


def _devices_arg(blocks, devices):
    """None, or the list of devices a host-array batch is split over
    ("all": every visible GPU).  Device tensors stay on their own device."""
    if devices is None:
        return None
    if isinstance(devices, str):
        if devices != "all":
            raise Error("Precondition violation: devices is required to be a list of device indices or 'all'")
        devices = list(range(device_count()))
    devs = [int(d) for d in devices]
    if not devs:
        raise Error("Precondition violation: devices is required to list at least one device")
    if not _is_host_array(blocks):
        if devs != [blocks.device.index if blocks.device.index is not None else 0]:
            raise Error("Precondition violation: a device tensor batch runs on its own device; devices= splits host "
                        "(numpy) batches over several GPUs")
        return None
    return devs


def _capi_code(coder):
    code = getattr(coder, "_batch_code", None)
    if code is None:
        from . import capi

        with _as_error():
            code = coder._batch_code = capi.Code(coder.k, coder.m)
    return code


class Encoder(_fec.Encoder):
    """Encoder(k, m) -- see zfec/_fecmodule.c:40-44."""

    # encode(inblocks, desired_blocks_nums=None) is _fec.Encoder.encode: host
    # buffers run in C; device tensors come back to _encode_device
    # (fecmodule.cpp route_device)

    def encode_batch(self, blocks, desired_blocks_nums=None, devices=None):
        """Encode many independent stripes in one launch (fec_encode_batch).

        blocks: uint8 device tensor [nstripes, k, sz] (any strides with unit
        stride along sz; a transposed block-major [k, nstripes, sz] array is the
        fastest layout), or the same as a host numpy array, or a list of such
        device tensors (one per GPU: each runs on its own device, and a list of
        results comes back).  desired_blocks_nums: secondary block numbers in
        [k, m-1] (default k..m-1).  devices (host arrays only): a list of GPU
        indices, or "all", to split the stripes over (fec_encode_batch_multi:
        one library thread per GPU, each staging its share over its own PCIe
        link).  Returns a new [nstripes, len(desired), sz] tensor (numpy array
        for host input), block-major when the input was; device work is
        enqueued on the current stream, host calls return when done.  A batched
        counterpart of encode() for many small objects;
        no reference equivalent."""
        from . import capi

        if isinstance(blocks, (list, tuple)):
            return [self.encode_batch(b, desired_blocks_nums) for b in blocks]
        k, m = self.k, self.m
        nums = list(range(k, m)) if desired_blocks_nums is None else list(desired_blocks_nums)
        for x in nums:
            if not isinstance(x, int) or x < k or x >= m:
                raise Error("Precondition violation: encode_batch desired block nums are required to be secondary "
                            "block nums in [k, m-1] = [%d, %d], but one was %r" % (k, m - 1, x))
        ns, sz, sbs, sss, ptr = _batch_view(blocks, k, "blocks")
        devs = _devices_arg(blocks, devices)
        out = _batch_out(blocks, sss < sbs, ns, len(nums), sz)
        if nums and ns and sz:
            optr, obs, oss = _batch_strides(out)
            with _as_error():
                if devs is not None:
                    _capi_code(self).encode_batch_multi(ptr, sbs, sss, optr, obs, oss, nums, sz, ns, devs)
                else:
                    stream, flags = _batch_call_args(blocks)
                    _capi_code(self).encode_batch(ptr, sbs, sss, optr, obs, oss, nums, sz, ns, stream=stream,
                                                  flags=flags)
        return out

    def _encode_device(self, inblocks, desired):
        import torch

        inblocks = list(inblocks)
        k, m = self.k, self.m
        if desired is None:
            nums = list(range(m))
        else:
            try:
                nums = list(desired)
            except TypeError:
                raise TypeError("Second argument (optional) was not a sequence.")
            for x in nums:
                if not isinstance(x, int):
                    raise Error("Precondition violation: second argument is required to contain int.")
                if x < 0 or x >= m:
                    raise Error(
                        "Precondition violation: desired block nums are required to be in [0, m-1] = [0, %d], "
                        "but one was %d" % (m - 1, x)
                    )
        bl, sz, dev = _device_blocks(inblocks, k)
        sec = [x for x in nums if x >= k]
        outs = [torch.empty(sz, dtype=torch.uint8, device=dev) for _ in sec]
        if sec and sz:
            self.encode_into(
                [b.data_ptr() for b in bl], [o.data_ptr() for o in outs], sec, sz, stream=_stream_handle(dev)
            )
        it = iter(outs)
        return [inblocks[x] if x < k else next(it) for x in nums]


class Decoder(_fec.Decoder):
    """Decoder(k, m) -- see zfec/_fecmodule.c:321-325."""

    # decode(blocks, blocknums) is _fec.Decoder.decode; device tensors come
    # back to _decode_device (fecmodule.cpp route_device)

    def decode_batch(self, blocks, blocknums, devices=None):
        """Decode many independent stripes that all received the same block
        numbers, in one launch (fec_decode_batch).

        blocks: uint8 device tensor or host numpy array [nstripes, k, sz]
        (strides as in Encoder.encode_batch), or a list of device tensors (one
        per GPU), slot j of every stripe holding block blocknums[j];
        a primary block must sit at its own slot (primary i at slot i, as
        fec_decode requires, zfec/fec.c:549).  devices: as in
        Encoder.encode_batch (fec_decode_batch_multi).  Returns a new
        [nstripes, r, sz] tensor of the r missing primaries in ascending order."""
        from . import capi

        if isinstance(blocks, (list, tuple)):
            return [self.decode_batch(b, blocknums) for b in blocks]
        k, m = self.k, self.m
        try:
            nums = list(blocknums)
        except TypeError:
            raise TypeError("Second argument was not a sequence.")
        if len(nums) != k or len(set(nums)) != k:
            raise Error("Precondition violation: blocknums is required to hold k = %d distinct block nums" % k)
        for i, x in enumerate(nums):
            if not isinstance(x, int) or x < 0 or x >= m:
                raise Error("Precondition violation: block nums are required to be in [0, m-1] = [0, %d], but one "
                            "was %r" % (m - 1, x))
            if x < k and x != i:
                raise Error("Precondition violation: decode_batch requires primary block %d at slot %d" % (x, x))
        ns, sz, sbs, sss, ptr = _batch_view(blocks, k, "blocks")
        devs = _devices_arg(blocks, devices)
        r = sum(1 for x in nums if x >= k)
        out = _batch_out(blocks, sss < sbs, ns, r, sz)
        if r and ns and sz:
            optr, obs, oss = _batch_strides(out)
            with _as_error():
                if devs is not None:
                    _capi_code(self).decode_batch_multi(ptr, sbs, sss, optr, obs, oss, nums, sz, ns, devs)
                else:
                    stream, flags = _batch_call_args(blocks)
                    _capi_code(self).decode_batch(ptr, sbs, sss, optr, obs, oss, nums, sz, ns, stream=stream,
                                                  flags=flags)
        return out

    def _check_blocknums(self, blocknums):
        """Validated list of k block numbers (the reference's checks,
        zfec/_fecmodule.c:429-472, plus distinctness)."""
        k, m = self.k, self.m
        try:
            nums = list(blocknums)
        except TypeError:
            raise TypeError("Second argument was not a sequence.")
        if len(nums) != k:
            raise Error(
                "Precondition violation: Wrong length -- blocknums is required to contain exactly k blocks.  "
                "len(blocknums): %d, k: %d" % (len(nums), k)
            )
        for x in nums:
            if not isinstance(x, int):
                raise Error("Precondition violation: second argument is required to contain int.")
            if x < 0 or x > 255:
                raise Error("Precondition violation: block nums can't be less than zero or greater than 255.  %d\n" % x)
            if x >= m:
                raise Error(
                    "Precondition violation: block nums are required to be less than m = %d, but one was %d" % (m, x)
                )
        if len(set(nums)) != k:
            raise Error("Precondition violation: block nums are required to be distinct")
        return nums

    def _decode_device(self, blocks, blocknums):
        blocks = list(blocks)
        import torch

        k = self.k
        nums = self._check_blocknums(blocknums)
        bl, sz, dev = _device_blocks(blocks, k)
        objs = list(blocks)
        # primary i into slot i (zfec/_fecmodule.c:482-493)
        i = 0
        while i < k:
            c = nums[i]
            if c >= k or c == i:
                i += 1
            else:
                nums[i], nums[c] = nums[c], nums[i]
                bl[i], bl[c] = bl[c], bl[i]
                objs[i], objs[c] = objs[c], objs[i]
        missing = [i for i in range(k) if nums[i] >= k]
        outs = [torch.empty(sz, dtype=torch.uint8, device=dev) for _ in missing]
        if missing and sz:
            self.decode_into(
                [b.data_ptr() for b in bl], [o.data_ptr() for o in outs], nums, sz, stream=_stream_handle(dev)
            )
        it = iter(outs)
        return [objs[i] if nums[i] == i else next(it) for i in range(k)]


from . import easyfec  # noqa: E402  (needs Encoder/Decoder above)
from . import filefec, cmdline_zfec, cmdline_zunfec  # noqa: E402  (as zfec/__init__.py imports them)


def reuse_host_memory(keep_bytes=1 << 30, mmap_threshold=32 << 20):
    """Let this process's C allocator (glibc) keep freed blocks for reuse.

    Output ``bytes`` of large host-memory calls are new objects; by default glibc
    serves each one of more than a few MiB with fresh pages (mmap, or a heap it
    trims on free), so every call faults them in and every free returns them to
    the kernel.  On the MI355X host that is most of a K=3/M=10 64 MiB encode from
    ``bytes``: 3.0 GB/s per call with the freeing counted, 15.5 GB/s when blocks
    are reused (tools/e2e_host.py).  This sets
    M_MMAP_THRESHOLD (blocks under ``mmap_threshold`` come from the heap; glibc
    caps it at 32 MiB) and M_TRIM_THRESHOLD (up to ``keep_bytes`` of free heap is
    kept), the same as ``GLIBC_TUNABLES=glibc.malloc.mmap_threshold=...:
    glibc.malloc.trim_threshold=...`` at start-up.  It is process-wide, so it is
    opt-in.  Returns True if glibc accepted both settings.
    """
    import ctypes
    import ctypes.util

    try:
        libc = ctypes.CDLL(ctypes.util.find_library("c") or "libc.so.6")
        mallopt = libc.mallopt
    except (OSError, AttributeError):
        return False
    mallopt.argtypes = [ctypes.c_int, ctypes.c_int]
    mallopt.restype = ctypes.c_int
    M_TRIM_THRESHOLD, M_MMAP_THRESHOLD = -1, -3
    ok = mallopt(M_MMAP_THRESHOLD, int(min(mmap_threshold, 32 << 20))) == 1
    return mallopt(M_TRIM_THRESHOLD, int(min(keep_bytes, (1 << 31) - 1))) == 1 and ok
