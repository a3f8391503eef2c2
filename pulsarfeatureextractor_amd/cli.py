"""ScoreGenerator-compatible command line (ScoreGenerator.py:99-292), batched on the GPU.

  python -m pulsarfeatureextractor_amd.cli -c <dir|file> -o <out> [--phcx|--superb]
         [--arff] [--profile] [--dmprof] [-v] [--device N] [--workers K]

Same flags, same output-file probing (:147-160), same mode dispatch (:219-290).  --pfd and
--label are recognised and rejected (PFD is a 'next' row, labelling is interactive).
"""
from __future__ import annotations

import os
import sys
from optparse import OptionParser

from . import processor


def main(argv=None):
    p = OptionParser()
    p.add_option("-c", action="store", dest="candDir", default="")
    p.add_option("-v", action="store_true", dest="verbose", default=False)
    p.add_option("-o", action="store", dest="outputPath", type="string", default="")
    p.add_option("--pfd", action="store_true", dest="pfd", default=False)
    p.add_option("--phcx", action="store_true", dest="phcx", default=False)
    p.add_option("--superb", action="store_true", dest="superb", default=False)
    p.add_option("--arff", action="store_true", dest="arff", default=False)
    p.add_option("--profile", action="store_true", dest="profile", default=False)
    p.add_option("--label", action="store_true", dest="label", default=False)
    p.add_option("--dmprof", action="store_true", dest="dmprof", default=False)
    p.add_option("--device", action="store", dest="device", type="int", default=0)
    p.add_option("--workers", action="store", dest="workers", type="int", default=None)
    args, _ = p.parse_args(argv)
    if args.pfd:
        print("PFD candidates are not supported by this build.", file=sys.stderr)
        return 2
    if args.label:
        print("--label (interactive labelling) is not supported by this build.", file=sys.stderr)
        return 2
    # output-file probing (:147-160)
    single_file = os.path.exists(args.outputPath)
    if not single_file:
        try:
            open(args.outputPath, "w").close()
        except (IOError, OSError):
            pass
        single_file = os.path.exists(args.outputPath)
    # candidate directory / single file (:165-182)
    single = False
    if os.path.isdir(args.candDir):
        search = args.candDir + "/"
    elif os.path.isfile(args.candDir):
        single, search = True, args.candDir
    else:
        search = ""
    from .candidate import get_engine

    get_engine(args.device)
    dp = processor.DataProcessor(args.verbose, workers=args.workers)
    if args.dmprof:
        if args.phcx and not args.superb:
            dp.dmprofPHCX(search, args.verbose, args.outputPath, args.arff, single)
        elif args.superb and not args.phcx:
            dp.dmprofSUPERB(search, args.verbose, args.outputPath, args.arff, single)
    elif args.phcx and not args.superb:
        if not single_file:
            dp.processPHCXSeparately(search, args.verbose, single)
        else:
            dp.processPHCXCollectively(search, args.verbose, args.outputPath, args.arff,
                                       args.profile, single)
    elif args.superb and not args.phcx:
        dp.processSUPERBCollectively(search, args.verbose, args.outputPath, args.arff,
                                     args.profile, single)
    else:
        print("Didn't know what to do with your input.")
    print("Done.")
    return 0


if __name__ == "__main__":
    sys.exit(main())
