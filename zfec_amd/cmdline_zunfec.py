"""`zunfec` command line (mirrors /root/reference/zfec/cmdline_zunfec.py:15-62):
recover a file from any K of its share files, on the GPU."""
from __future__ import print_function

import argparse
import os
import sys

import zfec_amd
from zfec_amd import filefec

__version__ = zfec_amd.__version__


def main():
    if "-V" in sys.argv or "--version" in sys.argv:
        print("zfec library version: ", zfec_amd.__version__)
        print("zunfec command-line tool version: ", __version__)
        return 0
    p = argparse.ArgumentParser(description="Decode data from share files.")
    p.add_argument("-o", "--outputfile", required=True, type=str, metavar="OUTF",
                   help='file to write the resulting data to, or "-" for stdout')
    p.add_argument("sharefiles", nargs="*", type=str, metavar="SHAREFILE",
                   help="shares file to read the encoded data from")
    p.add_argument("-v", "--verbose", action="store_true", help="print out messages about progress")
    p.add_argument("-f", "--force", action="store_true", help="overwrite any existing output file")
    p.add_argument("-V", "--version", action="store_true", help="print out version number and exit")
    args = p.parse_args()
    if len(args.sharefiles) < 2:
        print("At least two sharefiles are required.")
        return 1
    if args.force:
        outf = open(args.outputfile, "wb")
    else:
        try:
            fd = os.open(args.outputfile, os.O_WRONLY | os.O_CREAT | os.O_EXCL | (hasattr(os, "O_BINARY") and os.O_BINARY))
        except OSError:
            print("There is already a file named %r -- aborting.  Use --force to overwrite." % (args.outputfile,))
            return 2
        outf = os.fdopen(fd, "wb")
    # sorted: primaries (share number < k) first, which need no arithmetic
    sharefs = [open(fn, "rb") for fn in sorted(args.sharefiles)]
    try:
        filefec.decode_from_files(outf, sharefs, args.verbose)
    except filefec.InsufficientShareFilesError as e:
        print(str(e))
        return 3
    finally:
        outf.close()
        for f in sharefs:
            f.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
