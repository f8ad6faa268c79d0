"""`zfec` command line (mirrors /root/reference/zfec/cmdline_zfec.py:18-91):
encode a file into M share files, any K of which recover it.  The coding runs
on the GPU through zfec_amd.filefec."""
from __future__ import print_function

import argparse
import sys

import zfec_amd
from zfec_amd import filefec

__version__ = zfec_amd.__version__
DEFAULT_K = 3
DEFAULT_M = 8


def _parser():
    p = argparse.ArgumentParser(description="Encode a file into a set of share files, a subset of which can later "
                                            "be used to recover the original file.")
    p.add_argument("inputfile", type=argparse.FileType("rb"), metavar="INF", help='file to encode or "-" for stdin')
    p.add_argument("-d", "--output-dir", default=".", metavar="D",
                   help='directory in which share file names will be created (default ".")')
    p.add_argument("-p", "--prefix", metavar="P",
                   help="prefix for share file names; If omitted, the name of the input file will be used.")
    p.add_argument("-s", "--suffix", default=".fec", metavar="S", help='suffix for share file names (default ".fec")')
    p.add_argument("-m", "--totalshares", default=DEFAULT_M, type=int, metavar="M",
                   help="the total number of share files created (default %d)" % DEFAULT_M)
    p.add_argument("-k", "--requiredshares", default=DEFAULT_K, type=int, metavar="K",
                   help="the number of share files required to reconstruct (default %d)" % DEFAULT_K)
    p.add_argument("-f", "--force", action="store_true", help="overwrite any existing share file")
    p.add_argument("-v", "--verbose", action="store_true", help="print out messages about progress")
    p.add_argument("-q", "--quiet", action="store_true",
                   help="quiet progress indications and warnings about silly choices of K and M")
    p.add_argument("-V", "--version", action="store_true", help="print out version number and exit")
    return p


def main():
    if "-V" in sys.argv or "--version" in sys.argv:
        print("zfec library version: ", zfec_amd.__version__)
        print("zfec command-line tool version: ", __version__)
        sys.exit(0)
    args = _parser().parse_args()
    from_stdin = False
    if args.prefix is None:
        args.prefix = args.inputfile.name
        if args.prefix == "<stdin>":
            args.prefix, from_stdin = "", True
    if args.verbose and args.quiet:
        print("Please choose only one of --verbose and --quiet.")
        sys.exit(1)
    if not 1 <= args.totalshares <= 256:
        print("Invalid parameters, totalshares is required to be <= 256 and >= 1\n"
              "Please see the accompanying documentation.")
        sys.exit(1)
    if not 1 <= args.requiredshares <= args.totalshares:
        print("Invalid parameters, requiredshares is required to be <= totalshares and >= 1\n"
              "Please see the accompanying documentation.")
        sys.exit(1)
    if not args.quiet:
        if args.requiredshares == 1:
            print("warning: silly parameters: requiredshares == 1, which means that every share will be a complete "
                  "copy of the file.  You could use \"cp\" for the same effect.  But proceeding to do it anyway...")
        if args.requiredshares == args.totalshares:
            print("warning: silly parameters: requiredshares == totalshares, which means that all shares will be "
                  "required in order to reconstruct the file.  You could use \"split\" for the same effect.  But "
                  "proceeding to do it anyway...")
    inf = args.inputfile
    if from_stdin:  # a pipe cannot be measured up front: buffer it (the reference reads it whole too)
        import io

        raw = getattr(inf, "buffer", inf).read()
        inf = io.BytesIO(raw if isinstance(raw, bytes) else raw.encode())
        fsize = len(raw)
    else:
        inf.seek(0, 2)
        fsize = inf.tell()
        inf.seek(0, 0)
    try:
        return filefec.encode_to_files(inf, fsize, args.output_dir, args.prefix, args.requiredshares,
                                       args.totalshares, args.suffix, args.force, args.verbose)
    finally:
        args.inputfile.close()


if __name__ == "__main__":
    sys.exit(main())
