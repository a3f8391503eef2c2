#!/usr/bin/env python3
"""Row-by-row envelope report of the 22 scores (host only, from tools/golden_dump.py output):
for every golden set and LM score, the rows where the reference's K = 50 samples agree
(tight: the GPU must be inside on every one), the rows where they spread (wide), how many
wide rows the GPU value falls outside, and the binomial bound the test applies
(golden_util.envelope_check).

  python tools/envelope_report.py gpurun_out/r04_golden_gpu.npz > profiles/r04_envelope_rows.txt
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from golden_util import envelope_check  # noqa: E402

BITEXACT = (2, 3, 11, 12, 13, 14, 15, 19, 21)
SETS = ("bates22_phcx128", "bates22_superb64", "all30_phcx128", "bates22_phcx128_wide",
        "bates22_phcx128_big", "bates22_superb64_big", "label_phcx")


def main():
    g = np.load(sys.argv[1])
    print(f"GPU dump: {sys.argv[1]}")
    print("score  tight(inside)  wide  outside  bound   inside-fraction (all enveloped rows)")
    for name in SETS:
        st = envelope_check(g[name + "_out"], g[name + "_st"], name, skip=BITEXACT,
                            cols=slice(8, None) if name.startswith("all30") else slice(None))
        print(f"== {name}")
        for j, (t, w, o, b) in st.items():
            frac = 1.0 - o / max(1, t + w)
            print(f"s{j:<4d} {t:8d}       {w:5d}  {o:6d}  {b:6.1f}   {frac:.4f}")


if __name__ == "__main__":
    main()
