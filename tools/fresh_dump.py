#!/usr/bin/env python3
"""GPU scores of the fresh (non-golden) batches the parity tests draw, for the host-side
analysis of which (score, shape) pairs need the one-candidate allowance
(tools/fresh_report.py):

  python tools/fresh_dump.py gpurun_out/r03_fresh_gpu.npz     (on the GPU box)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from pulsarfeatureextractor_amd._native import Engine  # noqa: E402
from pulsarfeatureextractor_amd.synth import bates_batch  # noqa: E402

# (tag, lp, n, seed): tests/test_bates22_gpu.py's fresh batches
CASES = [("fresh128", 128, 160, 77), ("lp256", 256, 96, 1256), ("lp100", 100, 64, 1100),
         ("lp200", 200, 48, 1200), ("lp512", 512, 24, 1512), ("cfg3tile0", 128, 300, 20261018)]


def main():
    from test_bates22_gpu import wide_histogram_batch

    res = {}
    with Engine(0) as e:
        for tag, lp, n, seed in CASES:
            if tag == "cfg3tile0":
                b = bates_batch(16384, seed=seed)
                b = {k: v[:n] for k, v in b.items()}
            else:
                b = bates_batch(n, lp=lp, lsb=lp, seed=seed)
            out, st = e.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
            res[tag + "_out"], res[tag + "_st"] = out, st
        b = wide_histogram_batch(80, 5)
        out, st = e.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
        res["wide_out"], res["wide_st"] = out, st
    np.savez_compressed(sys.argv[1], **res)


if __name__ == "__main__":
    main()
