"""easyfec -- one buffer in, m blocks out (mirrors /root/reference/zfec/easyfec.py:24-55).

The buffer is split into k blocks of ceil(len/k) bytes, the last one
zero-padded; decoding joins the k primaries and strips ``padlen`` bytes.  The
coding itself runs on the GPU through zfec_amd.Encoder / Decoder.
"""
import zfec_amd


def div_ceil(n, d):
    """The smallest integer q such that q*d >= n (zfec/easyfec.py:7-11)."""
    return (n // d) + (n % d != 0)


class Encoder(object):
    def __init__(self, k, m):
        self.fec = zfec_amd.Encoder(k, m)

    def encode(self, data):
        """@return: the m blocks, any k of which recover ``data``."""
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


class Decoder(object):
    def __init__(self, k, m):
        self.fec = zfec_amd.Decoder(k, m)

    def decode(self, blocks, sharenums, padlen):
        """@param padlen: bytes of padding to strip (= k*blocksize - len(data))."""
        data = b"".join(self.fec.decode(blocks, sharenums))
        if padlen:
            return data[:-padlen]
        return data
