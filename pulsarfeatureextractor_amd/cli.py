"""ScoreGenerator-compatible command line (ScoreGenerator.py:99-292), batched on the GPU.

  python -m pulsarfeatureextractor_amd.cli -c <dir|file> -o <out> [--phcx|--superb]
         [--arff] [--profile] [--dmprof] [-v] [--device N] [--workers K] [--start K]
         [--metrics FILE] [--gpus N [--devices D0,D1,...]]

Same flags, same output-file probing (:147-160), same mode dispatch (:215-290), for PHCX,
SUPERB and PFD files in every mode, --label included (its prompt is commented out in the
reference, DataProcessor.py:754-774: every candidate is labelled "0").
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
    # multi-GPU (not in the reference): N worker processes, one GPU each, over N contiguous
    # shards of the discovered candidates; outputs concatenated in discovery order
    p.add_option("--gpus", action="store", dest="gpus", type="int", default=1)
    # the GPU of each worker, e.g. "0,1,2,3" (default: worker r on GPU r % visible GPUs)
    p.add_option("--devices", action="store", dest="devices", type="string", default=None)
    # resume offset (not in the reference): skip the first K discovered candidates, e.g. the
    # ones a stopped collective run had already appended to its output file
    # (collective modes also keep <output>.progress = the --start value that resumes after
    # the last batch appended)
    p.add_option("--start", action="store", dest="start", type="int", default=0)
    # structured per-run metrics (not in the reference): one JSON object written to FILE at
    # the end of the run (candidates, successes, failures by reason, candidates/s, times)
    p.add_option("--metrics", action="store", dest="metrics", type="string", default=None)
    args, _ = p.parse_args(argv)
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
    devices = [int(d) for d in args.devices.split(",")] if args.devices else None
    if args.gpus <= 1:
        from .candidate import get_engine

        get_engine(devices[0] if devices else args.device)
    # else: the parent never initialises a GPU -- each shard worker is a spawned process that
    # opens its own device (processor.DataProcessor._run_shards)
    dp = processor.DataProcessor(args.verbose, workers=args.workers, start=args.start,
                                 metrics_path=args.metrics, gpus=args.gpus, devices=devices)
    phcx, pfd, superb = args.phcx, args.pfd, args.superb
    try:
        if args.label:  # :220-225 (labelPFD with the two arguments ScoreGenerator passes)
            if phcx and not pfd and not superb:
                dp.labelPHCX(search, args.verbose)
            elif not phcx and pfd:
                dp.labelPFD(search, args.verbose)
        elif args.dmprof:
            if phcx and not pfd and not superb:
                dp.dmprofPHCX(search, args.verbose, args.outputPath, args.arff, single)
            elif not phcx and pfd and not superb:
                dp.dmprofPFD(search, args.verbose, args.outputPath, args.arff, single)
            elif not phcx and not pfd and superb:
                dp.dmprofSUPERB(search, args.verbose, args.outputPath, args.arff, single)
        elif phcx and not pfd and not superb:
            if not single_file:
                dp.processPHCXSeparately(search, args.verbose, single)
            else:
                dp.processPHCXCollectively(search, args.verbose, args.outputPath, args.arff,
                                           args.profile, single)
        elif not phcx and pfd and not superb:
            if not single_file:
                dp.processPFDSeparately(search, args.verbose, single)
            else:
                dp.processPFDCollectively(search, args.verbose, args.outputPath, args.arff,
                                          args.profile, single)
        elif phcx and pfd and not superb:
            if not single_file:
                dp.processPFDAndPHCXSeparately(search, args.verbose, single)
            else:
                dp.processPFDAndPHCXCollectively(search, args.verbose, args.outputPath,
                                                 args.arff, args.profile, single)
        elif superb and not pfd and not phcx:
            dp.processSUPERBCollectively(search, args.verbose, args.outputPath, args.arff,
                                         args.profile, single)
        elif not phcx and not pfd:
            if not single_file:
                dp.processPFDAndPHCXSeparately(search, args.verbose, single)
            else:
                dp.processPFDAndPHCXCollectively(search, args.verbose, args.outputPath,
                                                 args.arff, args.profile, single)
        else:
            print("Didn't know what to do with your input.")
    except NotImplementedError as e:
        print(f"not supported by this build: {e}", file=sys.stderr)
        return 2
    print("Done.")
    return 0


if __name__ == "__main__":
    sys.exit(main())
