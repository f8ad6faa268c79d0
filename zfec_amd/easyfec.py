"""easyfec -- one buffer in, m blocks out (mirrors /root/reference/zfec/easyfec.py:24-55).

The buffer is split into k blocks of ceil(len/k) bytes, the last one(s)
zero-padded; decoding joins the k primaries and strips ``padlen`` bytes.  The
coding itself runs on the GPU through zfec_amd.Encoder / Decoder.

Two kinds of buffer:

* bytes-like (bytes, bytearray, memoryview, numpy): as the reference, the
  blocks and the decoded data are ``bytes``;
* a torch tensor on a ROCm device (any dtype, contiguous; encoded as its
  bytes): split, pad, join and strip all stay on the device.  The primary
  blocks that lie wholly inside the data are zero-copy views of it; only a
  block that runs past the end is materialised (zero-filled, on the device).
  Decoding writes each recovered primary straight into its place in one
  output buffer, copies the present primaries there on the device, and
  returns a view with the padding stripped.
"""
import zfec_amd


def div_ceil(n, d):
    """The smallest integer q such that q*d >= n (zfec/easyfec.py:7-11)."""
    return (n // d) + (n % d != 0)


def _device_bytes(t):
    import torch

    if not t.is_contiguous():
        raise zfec_amd.Error("Precondition violation: the data tensor is required to be contiguous.")
    return t.reshape(-1) if t.dtype == torch.uint8 else t.reshape(-1).view(torch.uint8)


class Encoder(object):
    def __init__(self, k, m):
        self.fec = zfec_amd.Encoder(k, m)

    def encode(self, data):
        """@return: the m blocks, any k of which recover ``data``."""
        if zfec_amd._is_device_tensor(data):
            return self._encode_device(data)
        k = self.fec.k
        chunksize = div_ceil(len(data), k)
        mv = memoryview(data).cast("B") if not isinstance(data, (bytes, bytearray)) else data
        blocks = []
        for i in range(k):
            piece = bytes(mv[i * chunksize:(i + 1) * chunksize])
            if len(piece) < chunksize:
                piece += b"\x00" * (chunksize - len(piece))
            blocks.append(piece)
        return self.fec.encode(blocks)

    def _encode_device(self, data):
        import torch

        k = self.fec.k
        flat = _device_bytes(data)
        n = flat.numel()
        cs = div_ceil(n, k)
        blocks = []
        for i in range(k):
            lo, hi = i * cs, (i + 1) * cs
            if hi <= n:
                blocks.append(flat[lo:hi])  # a view: no copy
            else:  # runs past the end: zero-filled block with the tail (if any) copied in
                b = torch.zeros(cs, dtype=torch.uint8, device=flat.device)
                if lo < n:
                    b[:n - lo].copy_(flat[lo:n])
                blocks.append(b)
        if cs == 0:
            return [torch.empty(0, dtype=torch.uint8, device=flat.device) for _ in range(self.fec.m)]
        return self.fec.encode(blocks)


class Decoder(object):
    def __init__(self, k, m):
        self.fec = zfec_amd.Decoder(k, m)

    def decode(self, blocks, sharenums, padlen):
        """@param padlen: bytes of padding to strip (= k*blocksize - len(data))."""
        try:
            first = blocks[0]
        except Exception:
            first = None
        if first is not None and zfec_amd._is_device_tensor(first):
            return self._decode_device(list(blocks), sharenums, padlen)
        data = b"".join(self.fec.decode(blocks, sharenums))
        if padlen:
            return data[:-padlen]
        return data

    def _decode_device(self, blocks, sharenums, padlen):
        """The k primaries joined in one device buffer (recovered ones written in
        place by the kernel), padding stripped by a view with the same slicing
        as the bytes path."""
        import torch

        k = self.fec.k
        nums = self.fec._check_blocknums(sharenums)
        bl, sz, dev = zfec_amd._device_blocks(blocks, k)
        # primary i into slot i (zfec/_fecmodule.c:482-493)
        i = 0
        while i < k:
            c = nums[i]
            if c >= k or c == i:
                i += 1
            else:
                nums[i], nums[c] = nums[c], nums[i]
                bl[i], bl[c] = bl[c], bl[i]
        out = torch.empty(k * sz, dtype=torch.uint8, device=dev)
        missing = [i for i in range(k) if nums[i] >= k]
        for i in range(k):
            if nums[i] == i:
                out[i * sz:(i + 1) * sz].copy_(bl[i])
        if missing and sz:
            self.fec.decode_into([b.data_ptr() for b in bl], [out.data_ptr() + i * sz for i in missing], nums, sz,
                                 stream=zfec_amd._stream_handle(dev))
        # the reference's own slicing (zfec/easyfec.py:53-55): data[:-padlen],
        # so an oversized padlen gives an empty result rather than an error
        return out[:-padlen] if padlen else out
