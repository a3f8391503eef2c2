#!/usr/bin/env python3
"""GPU scores of the golden Bates sets (current build, default solver) for host-side reports:

  python tools/golden_dump.py gpurun_out/r04_golden_gpu.npz          (on the GPU box)
  python tools/envelope_report.py gpurun_out/r04_golden_gpu.npz      (here)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from golden_util import bates_inputs, load  # noqa: E402
from pulsarfeatureextractor_amd._native import Engine  # noqa: E402

SETS = ("bates22_phcx128", "bates22_superb64", "all30_phcx128", "bates22_phcx128_wide",
        "bates22_phcx128_big", "bates22_superb64_big", "label_phcx")


def main():
    res = {}
    with Engine(0) as e:
        for name in SETS:
            prof, sub, curve, scal = bates_inputs(load(name))
            out, st = e.bates22(prof, sub, curve, scal)
            res[name + "_out"], res[name + "_st"] = out, st
    np.savez_compressed(sys.argv[1], **res)


if __name__ == "__main__":
    main()
