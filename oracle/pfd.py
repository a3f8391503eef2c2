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


# ---------------------------------------------------------------------------------------
# the PFD 22-score path   PFDFile.compute :587-613 (PFDOperations extends ProfileOperations)
# ---------------------------------------------------------------------------------------
KDM_PFD = 8.3 * 10 ** 6      # PFDOperations.getDMFittings :342-344
DF_PFD = 32
F_PFD = 135


def fft_rotate(arr, bins):
    """PFDOperations.fft_rotate (:490-500), with Py2 integer arr.size/2."""
    arr = np.asarray(arr)
    freqs = np.arange(arr.size // 2 + 1, dtype=float)
    phasor = np.exp(complex(0.0, (2.0 * np.pi)) * freqs * bins / float(arr.size))
    return np.fft.irfft(phasor * np.fft.rfft(arr))


def pfd_parameters(d, profile):
    """PFDOperations.getCandidateParameters (:93-233) -> (period, snr, dm, width).  The width
    rotates the profile with fft_rotate (round-off ~1e-13 of the exact integer rotation)."""
    period = d.bary_p1 * 1000
    avg = profile.mean()
    var = profile.var()
    sigma = np.sqrt(var)
    keep = []
    for v in profile:                                               # :141-144
        if v > avg - 3 * sigma and v < avg + 3 * sigma:
            keep.append(v)
    snr_profile = np.array(keep)
    avg = snr_profile.mean()
    var = snr_profile.var()
    snr = ((profile - avg) / np.sqrt(var)).sum()                    # :151
    if snr < 0:
        snr = 0.1
    peak = profile.argmax()
    shift = peak - len(profile) // 2                                # Py2 int '/' (:202)
    rot = fft_rotate(profile, shift) - min(profile)
    peak = rot.argmax()
    half = max(rot) / 2
    left = peak
    while left > 0:
        if rot[left] < half:
            break
        left -= 1
    right = peak
    while right < len(rot):
        if rot[right] < half:
            break
        right += 1
    width = (1.0 * (right - left - 1.0)) / len(rot)                # :231
    return period, snr, d.bestdm, width


def pfd_dm_scores(chis, dms, period, snr, dm, width):
    """PFDOperations.getDMFittings (:274-393): [s16, s17, s18 (before filterScore), s19].
    yData = 255./max(chis)*chis in float32 (numpy 2 scalar rules, as the fixtures were made)."""
    from oracle import bates as ob  # ob.leastsq (so the chaos-floor tools can nudge it)

    y = np.asarray(chis, dtype=np.float32)
    y = 255. / max(y) * y                                           # :332
    n = len(chis)
    dm_start, dm_end = float(dms[1]), float(dms[n - 1])             # :337
    step = abs(dm_start - dm_end) / n
    wint = (width * period) ** 2
    peak = snr / np.sqrt((period - np.sqrt(wint)) / np.sqrt(wint))
    x = np.array([dm_start + i * step for i in range(n)])
    help_ = []
    for i in range(n):
        weff = np.sqrt(wint + pow(KDM_PFD * abs(dm - x[i]) * DF_PFD / pow(F_PFD, 3), 2))
        if weff > period:
            weff = period
        help_.append(float(np.sqrt((period - weff) / weff)))
    hmax = max(help_)
    theo = (255. / hmax) * np.array(help_)                          # ZeroDivisionError at 0

    def model(p, x_):
        amp, prop, shift, up = p
        weff = np.sqrt(wint + pow(prop * KDM_PFD * abs((dm + shift) - x_) * DF_PFD / pow(F_PFD, 3), 2))
        weff = np.where(weff > period, period, weff)
        return up + amp * np.sqrt((period - weff) / weff)

    p = ob.leastsq(lambda p_, x_, y_: y_ - model(p_, x_), (255. / hmax, 1, 0, 0), args=(x, y))[0]
    fit = model(p, x)
    chi_theo, ndeg = 0, 0
    for i in range(n):
        if theo[i] > 0:
            chi_theo += (y[i] - theo[i]) ** 2 / theo[i]
            ndeg += 1
    chi_theo = chi_theo / ndeg                                      # ZeroDivisionError at 0
    del fit
    return [float(peak), float(abs(1 - p[1])), float(p[2]), float(chi_theo)]


def bates22_one(d):
    """22 scores of one .pfd (PFDFile.compute), or raise bates.CandidateFailure."""
    import warnings

    from oracle import bates as ob

    flags = {"dgf_indexerror": False}
    out = []
    st = PFDState(d)
    with warnings.catch_warnings(), np.errstate(all="ignore"):
        warnings.simplefilter("ignore")
        profile = st.profile()
        par = {}

        def params():
            period, snr, dm, width = pfd_parameters(d, profile)
            par.update(period=period, snr=snr, dm=dm, width=width)
            return [float(period), ob._filter_neg(float(snr)), ob._filter_neg(float(dm)),
                    float(width)]

        def dmfit():
            if np.ndim(d.dms) == 0 or d.numdms == 1:
                raise PFDError("dms is a scalar (numdms == 1): indexing raises")
            chis, dms = st.chi2_vs_dm(d.dms[0], d.dms[-1])
            r = pfd_dm_scores(chis, dms, par["period"], par["snr"], par["dm"], par["width"])
            r[2] = float(abs(r[2]))                                 # filterScore(18)
            return r

        def subband():
            sub = st.profs.sum(0)                                   # plot_subbands :442-456
            return ob.subband_scores(sub, profile, par["width"])

        for group, fn in (("sine", lambda: ob.sinusoid_scores(profile)),
                          ("gauss", lambda: ob.gaussian_scores(profile)),
                          ("params", params), ("dmfit", dmfit), ("subband", subband)):
            try:
                r = fn()
            except Exception as e:
                raise ob.CandidateFailure(group, e) from e
            if group == "gauss":
                r, flags["dgf_indexerror"] = r
            out.extend(r)
    return out, flags
