"""filefec -- zfec's share-file format and file encode/decode, on the MI355X engine.

Mirrors /root/reference/zfec/filefec.py: the 1-4 byte bit-packed header
(`_build_header` :58-118, `_parse_header` :123-181), `encode_to_files`
(:185-256), `decode_from_files` (:264-316) and the segment callback API
(`encode_file` :318-375, `encode_file_not_really` :385-414,
`encode_file_not_really_and_hash` :416-448, `encode_file_stringy` :450-492,
`encode_file_stringy_easyfec` :494-522).  Share files are byte-identical to
the reference's (tests/test_filefec.py checks them against files written by
the reference itself).

The reference encodes a file segment by segment: each segment is k*4096
input bytes split easyfec-style into k blocks, and share i is the header
followed by block i of every segment.  Here a window of W whole segments is
one batched GPU call (stripe = segment): it reads the window as the file lays
it out and writes the m share bodies of the window block-major, so each share
file gets one contiguous write per window.  Decoding: W*4096 bytes of each
of k shares are the k blocks of one call, and the recovered rows are
regrouped segment-major for the output.  Window buffers are page-locked
(fec_host_alloc), so the kernel reads and writes them in place over PCIe.
Only the final, short segment takes the per-segment path.
"""
import itertools
import os
import struct

import numpy as np

import zfec_amd
from zfec_amd import capi, easyfec

CHUNKSIZE = 4096
WINDOW_BYTES = 64 << 20  # input bytes per GPU call (rounded down to whole segments)


def pad_size(n, k):
    """The smallest number that has to be added to n to equal a multiple of k (filefec.py:10-17)."""
    return k - n % k if n % k else 0


def log_ceil(n, b):
    """The smallest integer k such that b^k >= n (filefec.py:19-31)."""
    p, k = 1, 0
    while p < n:
        p *= b
        k += 1
    return k


class InsufficientShareFilesError(zfec_amd.Error):
    def __init__(self, k, kb, *args, **kwargs):
        zfec_amd.Error.__init__(self, *args, **kwargs)
        self.k = k
        self.kb = kb

    def __repr__(self):
        return ("Insufficient share files -- %d share files are required to recover this file, but only %d were "
                "given" % (self.k, self.kb))

    def __str__(self):
        return self.__repr__()


class CorruptedShareFilesError(zfec_amd.Error):
    pass


def _build_header(m, k, pad, sh):
    """Pack (m, k, pad, shnum) into 2-4 bytes (filefec.py:58-118): 8 bits of m-1,
    then log_ceil(m) bits of k-1, log_ceil(k) bits of pad, log_ceil(m) bits of
    shnum, left-aligned in the smallest of 2, 3 or 4 bytes."""
    assert 1 <= m <= 256 and 1 <= k <= m and 0 <= pad < k and 0 <= sh < m
    fields = [(m - 1, 8), (k - 1, log_ceil(m, 2)), (pad, log_ceil(k, 2)), (sh, log_ceil(m, 2))]
    val, used = 0, 0
    for v, bits in fields:
        val = (val << bits) | v
        used += bits
    assert 8 <= used <= 32, used
    nbytes = 2 if used <= 16 else 3 if used <= 24 else 4
    val <<= 8 * nbytes - used
    return struct.pack(">I", val)[4 - nbytes:]


def MASK(bits):
    return (1 << bits) - 1


def _truncated(inf):
    return CorruptedShareFilesError(
        "Share files were corrupted -- share file %r didn't have a complete metadata header at the front.  "
        "Perhaps the file was truncated." % (getattr(inf, "name", inf),))


def _parse_header(inf):
    """Read 1-4 header bytes from `inf` and return (m, k, pad, shnum) (filefec.py:123-181)."""
    ch = inf.read(1)
    if not ch:
        raise _truncated(inf)
    m = ord(ch) + 1
    kbits = log_ceil(m, 2)
    b2_bits_left = 8 - kbits
    kbitmask = MASK(kbits) << b2_bits_left
    ch = inf.read(1)
    if not ch:
        raise _truncated(inf)
    byte = ord(ch)
    k = ((byte & kbitmask) >> b2_bits_left) + 1
    shbits = log_ceil(m, 2)
    padbits = log_ceil(k, 2)
    val = byte & ~kbitmask
    needed_padbits = padbits - b2_bits_left
    if needed_padbits > 0:
        ch = inf.read(1)
        if not ch:
            raise _truncated(inf)
        val = (val << 8) | ord(ch)
        needed_padbits -= 8
    assert needed_padbits <= 0
    extrabits = -needed_padbits
    pad = val >> extrabits
    val &= MASK(extrabits)
    needed_shbits = shbits - extrabits
    if needed_shbits > 0:
        ch = inf.read(1)
        if not ch:
            raise _truncated(inf)
        val = (val << 8) | ord(ch)
        needed_shbits -= 8
    assert needed_shbits <= 0
    sh = val >> -needed_shbits
    return (m, k, pad, sh)


FORMAT_FORMAT = "%%s.%%0%dd_%%0%dd%%s"
RE_FORMAT = "%s.[0-9]+_[0-9]+%s"


class _PinnedArray(object):
    """A numpy view over pinned host memory from the engine (fec_host_alloc)."""

    def __init__(self, nbytes):
        self.nbytes = max(1, nbytes)
        self.ptr = capi.lib().fec_host_alloc(self.nbytes)
        if not self.ptr:
            raise MemoryError("fec_host_alloc(%d) failed: %s" % (self.nbytes, capi.lib().fec_last_error_message().decode()))
        import ctypes

        self.array = np.ctypeslib.as_array((ctypes.c_ubyte * self.nbytes).from_address(self.ptr))

    def free(self):
        if self.ptr:
            capi.lib().fec_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.free()


def _readinto_full(inf, view):
    """Read up to len(view) bytes into `view`; returns the count (short only at EOF)."""
    got = 0
    n = len(view)
    while got < n:
        if hasattr(inf, "readinto"):
            r = inf.readinto(view[got:])
        else:
            data = inf.read(n - got)
            r = len(data)
            view[got:got + r] = data
        if not r:
            break
        got += r
    return got


def encode_to_files(inf, fsize, dirname, prefix, k, m, suffix=".fec", overwrite=False, verbose=False):
    """Encode inf into m share files named prefix.<shnum>_<m><suffix> in dirname
    (filefec.py:185-256).  Returns 0, or 1 after removing the partial files if
    an EnvironmentError occurred."""
    mlen = len(str(m))
    fmt = FORMAT_FORMAT % (mlen, mlen)
    padbytes = pad_size(fsize, k)
    fns, fs = [], []
    got_error = False
    try:
        for shnum in range(m):
            hdr = _build_header(m, k, padbytes, shnum)
            fn = os.path.join(dirname, fmt % (prefix, shnum, m, suffix))
            if verbose:
                print("Creating share file %r..." % (fn,))
            if overwrite:
                f = open(fn, "wb")
            else:
                flags = os.O_WRONLY | os.O_CREAT | os.O_EXCL | (hasattr(os, "O_BINARY") and os.O_BINARY)
                f = os.fdopen(os.open(fn, flags), "wb")
            fs.append(f)
            fns.append(fn)
            f.write(hdr)
        _encode_stream(inf, fsize, k, m, fs, verbose)
    except EnvironmentError as le:
        print("Cannot complete because of exception: ")
        print(le)
        got_error = True
    finally:
        for f in fs:
            f.close()
        if got_error:
            print("Cleaning up...")
            for fn in fns:
                try:
                    os.remove(fn)
                except EnvironmentError:
                    pass
            return 1
    if verbose:
        print()
        print("Done!")
    return 0


def _encode_stream(inf, fsize, k, m, fs, verbose):
    """Whole segments go through the GPU a window at a time: ONE batched call
    per window reads the window as the file lays it out (segment-major, stripe
    = segment, block j of segment s at s*k*4096 + j*4096) and writes all m
    share rows block-major (row i = block i of every segment; rows i < k are
    copies of the primaries), so each share file gets one contiguous write.
    Both buffers are page-locked, so the kernel reads and writes them in place.
    Two window buffers alternate: while one window's m share writes run (a
    thread pool, one file per task), the next window is read and encoded; a
    window's writes start only after the previous window's have finished, so
    every file is written in order."""
    from concurrent.futures import ThreadPoolExecutor

    seg = k * CHUNKSIZE
    wseg = max(1, WINDOW_BYTES // seg)
    code = capi.Code(k, m)
    nums = list(range(m))
    bufs = [(_PinnedArray(wseg * seg), _PinnedArray(m * wseg * CHUNKSIZE)) for _ in range(2)]
    pool = ThreadPoolExecutor(max_workers=min(m, 8))
    pending = []  # the previous window's writes

    def drain():
        for fut in pending:
            fut.result()
        del pending[:]

    total = 0
    try:
        for it in itertools.count():
            win_in, rows = bufs[it % 2]  # its writes (two windows ago) were drained before the last submit
            got = _readinto_full(inf, memoryview(win_in.array)[:wseg * seg])
            if got == 0:
                break
            total += got
            if total > fsize:
                raise IOError("Wrong file size -- possibly the size of the file changed during encoding.  "
                              "Original size: %d, observed size at least: %s" % (fsize, total))
            nfull = got // seg
            if nfull:
                w = nfull * CHUNKSIZE  # bytes per share in this window
                code.encode_batch(win_in.ptr, CHUNKSIZE, seg, rows.ptr, w, CHUNKSIZE, nums, CHUNKSIZE, nfull,
                                  flags=capi.FEC_FLAG_LIBRARY_STREAM)
                drain()
                view = memoryview(rows.array)
                pending.extend(pool.submit(fs[i].write, view[i * w:(i + 1) * w]) for i in range(m))
            rest = got - nfull * seg
            if rest:  # the final, short segment: easyfec split/pad, as the reference does
                drain()
                tail = bytes(win_in.array[nfull * seg:got])
                for i, b in enumerate(easyfec.Encoder(k, m).encode(tail)):
                    fs[i].write(b)
            if verbose:
                print("%d%% ..." % (100 * total // max(1, fsize)), end=" ")
            if got < wseg * seg:
                break
        drain()
    finally:
        pool.shutdown(wait=True)
        for pair in bufs:
            for a in pair:
                a.free()


def decode_from_files(outf, infiles, verbose=False):
    """Decode from the first k files in infiles, writing the result to outf
    (filefec.py:264-316)."""
    assert len(infiles) >= 2
    infs, shnums = [], []
    m = k = padlen = None
    for f in infiles:
        (nm, nk, npadlen, shnum) = _parse_header(f)
        if not (m is None or m == nm):
            raise CorruptedShareFilesError(
                "Share files were corrupted -- share file %r said that m was %s but another share file previously "
                "said that m was %s" % (f.name, nm, m))
        m = nm
        if not (k is None or k == nk):
            raise CorruptedShareFilesError(
                "Share files were corrupted -- share file %r said that k was %s but another share file previously "
                "said that k was %s" % (f.name, nk, k))
        if not (k is None or k <= len(infiles)):
            raise InsufficientShareFilesError(k, len(infiles))
        k = nk
        if not (padlen is None or padlen == npadlen):
            raise CorruptedShareFilesError(
                "Share files were corrupted -- share file %r said that pad length was %s but another share file "
                "previously said that pad length was %s" % (f.name, npadlen, padlen))
        padlen = npadlen
        infs.append(f)
        shnums.append(shnum)
        if len(infs) == k:
            break
    if len(infs) < k:
        raise InsufficientShareFilesError(k, len(infs))

    # slot order: primary i at slot i (zfec/_fecmodule.c:482-493)
    order = sorted(range(k), key=lambda i: shnums[i])
    slots = [None] * k
    rest = [i for i in order if shnums[i] >= k]
    for i in order:
        if shnums[i] < k:
            slots[shnums[i]] = i
    it = iter(rest)
    slots = [s if s is not None else next(it) for s in slots]
    slot_nums = [shnums[i] for i in slots]

    # One batched call per window: stripe = segment, slot j of segment s at
    # ins + j*w_max + s*4096 (the window of share slots[j]); all k primaries
    # come out segment-major, i.e. in file order (FEC_FLAG_ALL_PRIMARIES: a
    # present primary's row is a copy).  Two window buffers alternate, so the
    # output write of one window overlaps the share reads (one thread per
    # share) and the decode of the next.
    from concurrent.futures import ThreadPoolExecutor

    wseg = max(1, WINDOW_BYTES // (k * CHUNKSIZE))
    code = capi.Code(k, m)
    w_max = wseg * CHUNKSIZE
    bufs = [(_PinnedArray(k * w_max), _PinnedArray(k * w_max)) for _ in range(2)]
    pool = ThreadPoolExecutor(max_workers=min(k, 8) + 1)
    pending = []  # the previous window's output write
    byteswritten = 0
    try:
        for it in itertools.count():
            ins, outbuf = bufs[it % 2]
            lens = list(pool.map(lambda j: _readinto_full(infs[slots[j]],
                                                          memoryview(ins.array)[j * w_max:(j + 1) * w_max]), range(k)))
            if any(n != lens[-1] for n in lens):
                raise CorruptedShareFilesError(
                    "Share files were corrupted -- all share files are required to be the same length, but they "
                    "weren't.")
            n = lens[-1]
            if n == 0:
                break
            nfull, tail = divmod(n, CHUNKSIZE)
            if nfull:
                code.decode_batch(ins.ptr, w_max, CHUNKSIZE, outbuf.ptr, CHUNKSIZE, k * CHUNKSIZE, slot_nums,
                                  CHUNKSIZE, nfull, flags=capi.FEC_FLAG_LIBRARY_STREAM | capi.FEC_FLAG_ALL_PRIMARIES)
                for fut in pending:
                    fut.result()
                pending = [pool.submit(outf.write, memoryview(outbuf.array)[:nfull * k * CHUNKSIZE])]
                byteswritten += nfull * k * CHUNKSIZE
            if tail:  # the final, short segment of each share
                for fut in pending:
                    fut.result()
                pending = []
                blocks = [bytes(ins.array[j * w_max + nfull * CHUNKSIZE:j * w_max + n]) for j in range(k)]
                data = b"".join(zfec_amd.Decoder(k, m).decode(blocks, slot_nums))
                outf.write(data)
                byteswritten += len(data)
            if verbose:
                print(str(byteswritten // 10 ** 6) + " MB ...", end=" ")
            if n < w_max:
                break
        for fut in pending:
            fut.result()
    finally:
        pool.shutdown(wait=True)
        for pair in bufs:
            for a in pair:
                a.free()
    if padlen:
        outf.truncate(byteswritten - padlen)
    if verbose:
        print()
        print("Done!")


def _segments(inf, k, m, chunksize):
    """Whole segments of k*chunksize input bytes, encoded a window at a time:
    the window is read into page-locked memory and ONE batched GPU call
    (fec_encode_batch, stripe = segment) computes the parity of all its full
    segments.  Yields (window bytes, offset of the segment, parity rows,
    offset of its parity) per full segment in file order, then
    (tail bytes, None, None, None) once for the final short segment -- empty
    when the file is a whole number of segments, as the reference's loops
    (filefec.py:352-375, :473-492) also end on a segment they pad entirely.
    The window starts at 4 segments and doubles up to WINDOW_BYTES, so a slow
    stream (a pipe, a socket) sees its first callbacks after a few segments,
    as with the reference's segment-at-a-time loop, not after 64 MiB."""
    seg = k * chunksize
    r = m - k
    wseg = max(1, WINDOW_BYTES // seg)
    code = capi.Code(k, m)
    win_in, rows = _PinnedArray(wseg * seg), _PinnedArray(max(1, r) * wseg * chunksize)
    cur = min(wseg, 4)
    try:
        while True:
            got = _readinto_full(inf, memoryview(win_in.array)[:cur * seg])
            nfull = got // seg
            if nfull and r:
                code.encode_batch(win_in.ptr, chunksize, seg, rows.ptr, chunksize, r * chunksize, list(range(k, m)),
                                  chunksize, nfull, flags=capi.FEC_FLAG_LIBRARY_STREAM)
            win = win_in.array[:nfull * seg].tobytes()
            par = rows.array[:nfull * r * chunksize].tobytes()
            for s in range(nfull):
                yield win, s * seg, par, s * r * chunksize
            if got < cur * seg:
                yield bytes(win_in.array[nfull * seg:got]), None, None, None
                return
            cur = min(wseg, 2 * cur)
    finally:
        win_in.free()
        rows.free()


def _segment_results(k, m, chunksize, win, off, par, poff, blocks):
    """cb's first argument: the k input blocks (`blocks`, filled from the
    segment) followed by the m - k parity blocks as bytes."""
    for j in range(k):
        blocks[j][:] = win[off + j * chunksize:off + (j + 1) * chunksize]
    return list(blocks) + [par[poff + i * chunksize:poff + (i + 1) * chunksize] for i in range(m - k)]


def encode_file(inf, cb, k, m, chunksize=4096):
    """Segment callback API (filefec.py:318-375): read k blocks of chunksize
    bytes at a time, encode them into m blocks, call cb(blocks, indatasize).
    The first k items of `blocks` are mutable arrays (bytearray) whose contents
    the next segment overwrites; the rest are new bytes.  indatasize is
    k*chunksize except for the final segment, which is zero-padded and carries
    the number of real bytes in it (0 when the file length is a multiple of
    k*chunksize).  The reference builds its arrays with the Python 2 typecode
    'c', which Python 3 rejects; this keeps the documented behaviour."""
    enc = zfec_amd.Encoder(k, m)
    blocks = tuple(bytearray(chunksize) for _ in range(k))
    for win, off, par, poff in _segments(inf, k, m, chunksize):
        if off is not None:
            cb(_segment_results(k, m, chunksize, win, off, par, poff, blocks), k * chunksize)
            continue
        padded = win + b"\x00" * (k * chunksize - len(win))
        for j in range(k):
            blocks[j][:] = padded[j * chunksize:(j + 1) * chunksize]
        res = enc.encode(list(blocks))
        cb(list(blocks) + list(res[k:]), len(win))


def encode_file_stringy(inf, cb, k, m, chunksize=4096):
    """Segment callback API with bytes blocks (filefec.py:450-492): as
    encode_file, with the k input blocks as bytes.  The final segment's
    indatasize is what the reference reports: i*chunksize + len(last read),
    with i counting the short read itself (one chunksize more than the real
    byte count; chunksize for an all-padding final segment); pinned against
    the reference's own callback sequences (tests/golden/segments.json)."""
    enc = zfec_amd.Encoder(k, m)
    for win, off, par, poff in _segments(inf, k, m, chunksize):
        if off is not None:
            blocks = [win[off + j * chunksize:off + (j + 1) * chunksize] for j in range(k)]
            cb(blocks + [par[poff + i * chunksize:poff + (i + 1) * chunksize] for i in range(m - k)], k * chunksize)
            continue
        i = len(win) // chunksize + 1  # the read that came back short, counted from 1
        padded = win + b"\x00" * (k * chunksize - len(win))
        blocks = [padded[j * chunksize:(j + 1) * chunksize] for j in range(k)]
        ind = i * chunksize + len(win) % chunksize
        cb(enc.encode(blocks), ind)
        if ind == k * chunksize and win:
            # (k-1)*chunksize bytes left: the reference's loop condition still
            # holds, so it reads once more and reports an all-padding segment
            # of "chunksize" bytes.  (With k == 1 and an empty tail its loop
            # never ends; here the stream ends.)
            blocks = [b"\x00" * chunksize] * k
            cb(enc.encode(blocks), chunksize)


def encode_file_not_really(inf, cb, k, m, chunksize=4096):
    """Benchmark control (filefec.py:385-414): read and pad segments as
    encode_file does, encode nothing, call cb(None, None) per segment."""
    for _ in _segments_read_only(inf, k, chunksize):
        cb(None, None)


def encode_file_not_really_and_hash(inf, cb, k, m, chunksize=4096):
    """Benchmark control (filefec.py:416-448): as encode_file_not_really, and
    SHA-1 every padded input block (the reference's `sha1.new()` is Python 2)."""
    import hashlib

    hasher = hashlib.sha1()
    for blocks in _segments_read_only(inf, k, chunksize):
        for b in blocks:
            hasher.update(b)
        cb(None, None)
    return hasher.hexdigest()


def _segments_read_only(inf, k, chunksize):
    """The padded k blocks of every segment, read without encoding (the final,
    possibly all-padding segment included)."""
    seg = k * chunksize
    while True:
        data = inf.read(seg)
        if len(data) < seg:
            data = data + b"\x00" * (seg - len(data))
            yield [data[j * chunksize:(j + 1) * chunksize] for j in range(k)]
            return
        yield [data[j * chunksize:(j + 1) * chunksize] for j in range(k)]


def encode_file_stringy_easyfec(inf, cb, k, m, chunksize=4096):
    """Segment callback API (filefec.py:494-522): read chunksize*k bytes at a
    time, encode with easyfec, call cb(blocks, length)."""
    enc = easyfec.Encoder(k, m)
    readsize = k * chunksize
    indata = inf.read(readsize)
    while indata:
        cb(enc.encode(indata), len(indata))
        indata = inf.read(readsize)
