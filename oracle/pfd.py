"""CPU restatement of the reference's PFD preprocessing and PFD Lyon features.

TEST INFRASTRUCTURE ONLY (checker for tests/, smoke() and bench.py's cpu_baseline leg).

Follows (paths relative to PulsarFeatureExtractor/src/):
  PFDFile.dedisperse            PFDFile.py:330-374   (integer-bin rotation at the best DM)
  PFDFile.getprofile / scale    PFDFile.py:256-310   ((sumprof - min) / mean, then 0..255)
  PFDFile.plot_chi2_vs_DM       PFDFile.py:378-423   (100 DMs, rotations accumulate; float32)
  PFDFile.calc_redchi2          PFDFile.py:427-438
  PFDFile.computeProfileStatScores / computeDMCurveStatScores   PFDFile.py:522-583
  PFDOperations.delay_from_DM / span / rotate   PFDOperations.py:474-527
with numpy doing the same operations in the same order, so results are bit-identical to the
reference on these inputs (pinned by tests/golden/pfd_lyon8.npz, tools/make_golden.py).
"""
from __future__ import annotations

import numpy as np
from scipy.stats import kurtosis, skew


class PFDError(Exception):
    pass


def delay_from_dm(dm, freqs):
    """PFDOperations.delay_from_DM (:474-488), array branch."""
    return np.where(freqs > 0.0, dm / (0.000241 * freqs * freqs), 0.0)


def rotate(arr, bins):
    """PFDOperations.rotate (:517-527): left rotation by bins (Python modulo)."""
    bins = bins % len(arr)
    if bins == 0:
        return arr
    return np.concatenate((arr[bins:], arr[:bins]))


def span(lo, hi, number):
    """PFDOperations.span (:504-515) for float end points."""
    return lo + (hi - lo) * np.arange(number) / (number - 1)


class PFDState:
    """The mutable part of a PFD object the score path touches."""

    def __init__(self, d):
        self.d = d
        self.profs = d.profs.copy()
        self.subdelays_bins = np.zeros(d.nsub, dtype="d")
        self.sumprof = None

    def dedisperse(self, dm=None):
        d = self.d
        if dm is None:
            dm = d.bestdm
        subdelays = delay_from_dm(dm, d.subfreqs)
        hifreqdelay = subdelays[-1]
        subdelays = subdelays - hifreqdelay
        delaybins = subdelays * d.binspersec - self.subdelays_bins
        new = np.floor(delaybins + 0.5)
        for ii in range(d.nsub):
            rotbins = int(new[ii]) % d.proflen
            if rotbins:
                sub = self.profs[:, ii, :]
                self.profs[:, ii] = np.concatenate((sub[:, rotbins:], sub[:, :rotbins]), 1)
        self.subdelays_bins += new
        self.sumprof = self.profs.sum(0).sum(0)

    def profile(self):
        """getprofile + scale (:256-310): a float64 array in [0, 255]."""
        if self.sumprof is None:
            self.dedisperse()
        normprof = self.sumprof - min(self.sumprof)
        s = normprof / np.mean(normprof)
        mn, mx = min(s), max(s)
        out = []
        for v in s:
            out.append((0 * (1 - ((v - mn) / (mx - mn)))) + (255 * ((v - mn) / (mx - mn))))
        return np.array(out)

    def chi2_vs_dm(self, lo, hi, n=100):
        d = self.d
        profs = self.profs.sum(0)  # summed in time; rotated in place below (aliasing)
        dms = span(lo, hi, n)
        chis = np.zeros(n, dtype="f")
        sdb = self.subdelays_bins.copy()
        for ii, dm in enumerate(dms):
            subdelays = delay_from_dm(dm, d.subfreqs)
            hifreqdelay = subdelays[-1]
            subdelays = subdelays - hifreqdelay
            delaybins = subdelays * d.binspersec - sdb
            new = np.floor(delaybins + 0.5)
            for jj in range(d.nsub):
                profs[jj] = rotate(profs[jj], int(new[jj]))
            sdb += new
            sumprof = profs.sum(0)
            chis[ii] = ((sumprof - d.avgprof) ** 2.0 / d.varprof).sum() / (len(sumprof) - 1.0)
        return chis, dms


def dm_curve(d):
    """PFDOperations.getDMCurveData (:242-252) on a freshly loaded file."""
    if np.ndim(d.dms) == 0 or d.numdms == 1:
        raise PFDError("dms is a scalar (numdms == 1): indexing raises")
    st = PFDState(d)
    st.dedisperse()  # getprofile() in load (:246-252) dedisperses first
    return st.chi2_vs_dm(d.dms[0], d.dms[-1])[0]


def stats4(bins):
    return [np.mean(bins), np.std(bins), skew(bins), kurtosis(bins)]


def lyon8_one(d):
    """[profile mean, std, skew, kurt, DM-curve mean, std, skew, kurt] of one file
    (calculateProfileStatScores + calculateDMCurveStatScores, each on a fresh object)."""
    st = PFDState(d)
    prof = st.profile()
    a = stats4([float(v) for v in prof])
    b = stats4(dm_curve(d))
    return [float(v) for v in a + b]
