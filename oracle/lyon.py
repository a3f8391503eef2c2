"""ORACLE (test infrastructure only) — CPU restatement of the 8 Lyon features.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker.  The product path (libpfe.so) never calls it.

Restates, per candidate, exactly what the reference computes:
  PHCXFile.computeProfileStatScores   PulsarFeatureExtractor/src/PHCXFile.py:320-349
  PHCXFile.computeDMCurveStatScores   PulsarFeatureExtractor/src/PHCXFile.py:351-379
    bins = [float(v) for v in row]                    (:334-335; DM: getDMCurveData :365)
    [numpy.mean(bins), numpy.std(bins), scipy.stats.skew(bins), scipy.stats.kurtosis(bins)]
  DataProcessor.dmprof concatenates profile stats then DM stats  DataProcessor.py:884-886

Pinned by tests/golden/lyon8_*.npz, produced by running the reference itself
(tools/make_golden.py) on synthetic PHCX/SUPERB files.
"""
from __future__ import annotations

import numpy as np
from scipy.stats import kurtosis, skew


def lyon_row(row) -> list:
    """[mean, std, skew, kurt] of one row, as PHCXFile.py:333-343 computes it."""
    bins = [float(v) for v in row]
    return [np.mean(bins), np.std(bins), skew(bins), kurtosis(bins)]


def lyon8(prof: np.ndarray, dm: np.ndarray) -> np.ndarray:
    """Reference-equivalent per-candidate loop: (n,Lp),(n,Ld) -> (n,8) float64.

    This is the scalar 'port' timed as bench.py's cpu_baseline (one scipy call per row, as
    the reference makes them)."""
    n = prof.shape[0]
    out = np.empty((n, 8), dtype=np.float64)
    for i in range(n):
        out[i, :4] = lyon_row(prof[i])
        out[i, 4:] = lyon_row(dm[i])
    return out


def lyon8_batched(prof: np.ndarray, dm: np.ndarray) -> np.ndarray:
    """Same statistics computed along axis 1 in one numpy/scipy call per array.

    numpy's pairwise sums along a contiguous axis run in the same order as on a 1-D row,
    so this agrees with :func:`lyon8` to the last bit on the fixtures (checked in tests);
    it exists so that large parity cases finish in seconds."""
    out = np.empty((prof.shape[0], 8), dtype=np.float64)
    for j, a in enumerate((prof, dm)):
        a = np.ascontiguousarray(a, dtype=np.float64)
        out[:, 4 * j + 0] = np.mean(a, axis=1)
        out[:, 4 * j + 1] = np.std(a, axis=1)
        out[:, 4 * j + 2] = skew(a, axis=1)
        out[:, 4 * j + 3] = kurtosis(a, axis=1)
    return out
