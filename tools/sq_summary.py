#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc SQ passes (one or more pmc_counter_collection.csv).

usage: sq_summary.py DIR [DIR ...] > summary.json
Sums each counter over dispatches of a kernel and reports per-wave values plus the derived
issue/occupancy ratios (SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_WAIT_* count quad-cycles on gfx950).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    # each pass (directory) is normalised by its own SQ_WAVES / SQ_WAVE_CYCLES
    out = {}
    for d in sys.argv[1:]:
        tot = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((f, r["Dispatch_Id"]))
        for k, c in tot.items():
            w = c.get("SQ_WAVES", 0.0)
            row = out.setdefault(k, {"dispatches": len(disp[k]), "waves": w})
            for n, v in sorted(c.items()):
                if n != "SQ_WAVES":
                    row.setdefault(n + "_per_wave", v / w if w else None)
            if w and c.get("SQ_WAVE_CYCLES"):
                wc = c["SQ_WAVE_CYCLES"]
                for n in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                          "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS"):
                    if n in c:
                        row.setdefault("frac_" + n, c[n] / wc)
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
