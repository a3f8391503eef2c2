#!/usr/bin/env python3
"""Per-column agreement of pfe_pfd_bates22 with the reference's golden rows and with the CPU
restatement on fresh folds (diagnostic; the bar is tests/test_pfd22_gpu.py)."""
import os
import sys
import tempfile
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
warnings.simplefilter("ignore")

from oracle import pfd as opfd  # noqa: E402
from pulsarfeatureextractor_amd import pfd  # noqa: E402
from pulsarfeatureextractor_amd._native import Engine  # noqa: E402
from test_oracle_pfd import SETS, build_files, load_set  # noqa: E402
from test_pfd22_gpu import oracle_rows, rel_err  # noqa: E402


def report(tag, out, st, ref, ok):
    gok = (st & 0xFF) == 0
    print(f"{tag}: n={len(ok)} fail-pattern-equal={np.array_equal(gok, ok)} "
          f"gpu-status={[int(x) for x in st]}")
    both = gok & ok
    r = rel_err(out[both], ref[both])
    for j in range(22):
        print(f"  s{j + 1:2d} max {r[:, j].max():9.3g}  >1e-12 {np.mean(r[:, j] > 1e-12):.2f}"
              f"  >1e-5 {np.mean(r[:, j] > 1e-5):.2f}")


def main():
    e = Engine(0)
    with tempfile.TemporaryDirectory() as tmp:
        for name in SETS:
            g = load_set(name)
            os.makedirs(os.path.join(tmp, name), exist_ok=True)
            files = build_files(os.path.join(tmp, name), g)
            datas = [pfd.read(f) for f in files]
            out, st = e.pfd_bates22(*pfd.batch_inputs(datas))
            report(name + " vs reference", out, st, g["bates22"], g["bates22_ok"])
            ref, ok = oracle_rows(datas)
            report(name + " vs oracle", out, st, ref, ok)


if __name__ == "__main__":
    main()
