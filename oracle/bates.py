"""ORACLE (test infrastructure only) — CPU restatement of the 22 Bates scores.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker.  libpfe.so never calls it.

A Python-3 restatement of the reference's per-candidate score path with the reference's
Python-2.7 semantics (integer '/' floors; ``ndarray == []`` is False), operation for
operation on the same numpy/scipy primitives (numpy ufuncs, numpy.histogram,
scipy.stats.scoreatpercentile, numpy.corrcoef, scipy.optimize.leastsq -> MINPACK lmdif), so
that on identical inputs it reproduces the reference bit for bit.  It is pinned against
tests/golden/bates22_*.npz, which tools/make_golden.py produced by running the reference.

Each function cites the reference lines it restates (PulsarFeatureExtractor/src/...).
Candidate inputs (arrays, as the PHCX parser produces them):
  prof  (L,)        int profile of the scored section          PHCXFile.py:140,144-186
  sub   (nsub,Lsb)  int sub-bands of the scored section         PHCXOperations.py:334-338
  curve (ndm,)      reduced DM curve (max of 127 per 128)       PHCXOperations.py:165-167,237-259
  scal  (8,)        [period_ms, snr, dm, width, dm_start, dm_end, length_all, _]
"""
from __future__ import annotations

import math
import warnings

import numpy as np
from numpy import argmax, delete, exp, histogram, log, mean, pi, sin, sqrt, std
from scipy.optimize import leastsq
from scipy.stats import scoreatpercentile

FWHM_C = 2 * sqrt(2 * log(2))  # the reference's 2*sqrt(2*log(2)) (numpy scalars)


class CandidateFailure(Exception):
    """The reference would have raised (candidate logged to CandidateErrorLog.txt)."""

    def __init__(self, group: str, cause: BaseException):
        super().__init__(f"{group}: {type(cause).__name__}: {cause}")
        self.group = group
        self.cause = cause


def _pymax(seq):
    """Python builtin max() (first element wins unless a later one is strictly greater)."""
    return max(seq)


def _py2div(a, b):
    """Python-2 '/': floor division when both operands are integers."""
    if isinstance(a, (int, np.integer)) and isinstance(b, (int, np.integer)):
        return a // b
    return a / b


# ---------------------------------------------------------------------------------------
# helpers shared by several groups   ProfileOperationsInterface.py:138-207
# ---------------------------------------------------------------------------------------
def fd_bins(data) -> int:
    """Freedman-Diaconis bin count  (ProfileOperationsInterface.py:138-166)."""
    iqr = scoreatpercentile(data, 75) - scoreatpercentile(data, 25)
    bw = 2 * iqr * pow(len(data), -0.3333333)
    if bw <= 0:
        bw = 60
    rng = max(data) - min(data)
    return int(np.ceil(_py2div(rng, bw)))


def backward_diff(y):
    """dy[i] = y[i] - y[i+1]  (ProfileOperationsInterface.py:170-186)."""
    return [y[i] - y[i + 1] for i in range(len(y) - 1)]


def _rotate_half(y):
    """Py2 scale() is always 0 (integer '/'), so T1/T2 always swap the halves at L//2
    (ProfileOperations.py:1098-1110, 1158-1170)."""
    cut = len(y) // 2
    return list(y[cut:]) + list(y[:cut]), cut


# ---------------------------------------------------------------------------------------
# scores 1-4   ProfileOperations.getSinusoidFittings  :190-376
# ---------------------------------------------------------------------------------------
def count_peaks(profile) -> int:
    """Number of peak blocks in the clipped profile (:255-334).  The zero counter is never
    reset by a non-zero bin, so a block closes at every 5th zero (that zero is dropped);
    a block counts when its maximum is non-zero."""
    t = profile - profile.mean() - profile.std()
    t[t < 0] = 0
    blocks, cur_nonzero, zeros = 0, False, 0
    for v in t:
        if v != 0:
            cur_nonzero = True
        elif zeros < 4:
            zeros += 1
        else:
            blocks += cur_nonzero
            cur_nonzero, zeros = False, 0
    return blocks + cur_nonzero


def _chisq_mean(y, fit):
    """sum((y_i - fit_i)**2) in index order, divided by len(y)."""
    c = 0
    for i in range(len(y)):
        c += (y[i] - fit[i]) ** 2
    return c / len(y)


def fit_sine(y, maxima):
    """:380-491  amp = bg = |max-min|/2 fixed; LM over (f, phi)."""
    x = np.array(range(len(y)))
    amp = abs(max(y) - min(y)) / 2.
    f0 = float(maxima / (len(y) - 1.))
    bg = abs(max(y) - min(y)) / 2.

    def model(p, x_):
        return abs(amp) * sin(2 * pi * p[0] * x_ + p[1]) + abs(bg)

    if y[0] == bg:
        phi0 = 0
    elif y[0] < bg:
        phi0 = -1 / (4 * f0) if f0 != 0 else -1.0 / (4.0 * 0.00000000001)
    elif y[0] > bg:
        phi0 = +1 / (4 * f0) if f0 != 0 else +1.0 / (4.0 * 0.00000000001)
    else:  # NaN (a float PFD profile of a constant fold): phi0 never assigned (:427-441)
        raise UnboundLocalError("local variable 'phi0' referenced before assignment")
    p = leastsq(lambda p_, x_, y_: y_ - model(p_, x_), (f0, phi0), args=(x, y), full_output=True)[0]
    return _chisq_mean(y, model(p, x))


def fit_sine_sqr(y, maxima):
    """:495-587  the residual is  y - amp*sin^2(.) + bg  (sign bug kept), the evaluated
    model amp*sin^2(.) + bg."""
    x = np.array(range(len(y)))
    amp = abs(max(y) - min(y)) / 2.
    f0 = float(maxima / (len(y) - 1.) / 2.)
    bg = abs(max(y) - min(y)) / 2.

    def resid(p, x_, y_):
        return y_ - (abs(amp) * pow(sin(2 * pi * p[0] * x_ + p[1]), 2)) + abs(bg)

    def model(p, x_):
        return abs(amp) * pow(sin(2 * pi * p[0] * x_ + p[1]), 2) + abs(bg)

    if y[0] == 0:
        phi0 = 0
    else:
        phi0 = -1 / (4 * f0) if f0 != 0 else -1.0 / (4.0 * 0.00000000001)
    p = leastsq(resid, (f0, phi0), args=(x, y), full_output=True)[0]
    return _chisq_mean(y, model(p, x))


def sinusoid_scores(profile):
    """[s1, s2, s3, s4]  (:233-376; PHCXFile.py:454-459)."""
    pmax, pmin = profile.max(), profile.min()
    s4 = 0
    for v in profile:
        s4 += (abs(pmax - pmin) / 2.) - v
    maxima = count_peaks(profile)
    # np.float64 / 0 gives inf (nan for 0/0) with a warning, as in the reference (:373-374)
    s1 = fit_sine(profile, maxima) / maxima
    s2 = fit_sine_sqr(profile, maxima) / maxima
    return [float(s1), float(s2), float(max(maxima - 1, 0)), float(s4)]


# ---------------------------------------------------------------------------------------
# scores 5-11   ProfileOperations.getGaussianFittings  :595-770
# ---------------------------------------------------------------------------------------
def _gauss(x, s, mu, a):
    return abs(a) * exp((-((x - mu) / s) ** 2) / 2)


def fit_gaussian_hist(edges, counts):
    """:774-983  Gaussian to a histogram (x = left edges).  Pads to 3 points; retries (at
    most 6 times) while chi2 > mean(y)^2*len and sigma < 0.2*len, each time deleting the
    ORIGINAL argmax index from a shrinking copy and moving mu0 to x[argmax(copy)+retry]."""
    x, y = edges, counts
    idx = argmax(y)
    mu0 = x[idx]
    s0 = std(y)
    a0 = max(y)
    meansq = mean(y) ** 2
    temp = y
    if len(x) == len(y) + 1:
        x = x[0:-1]
    nx = len(x)
    retry = 0
    while True:
        p0 = [s0, mu0, a0]
        while len(p0) > len(x):
            x = np.append(x, 0)
            y = np.append(y, 0)
        p = leastsq(lambda p_, x_, y_: y_ - _gauss(x_, *p_), p0, args=(x, y))[0]
        fwhm = abs(FWHM_C * p[0])
        fit = _gauss(x, *p)
        chisq = 0
        for i in range(nx):
            chisq += (y[i] - fit[i]) ** 2
        chisq /= len(y)
        if (chisq > meansq * nx) & (p[0] < 0.2 * nx):
            retry += 1
            temp = delete(temp, idx)
            mu0 = x[argmax(temp) + retry]
            if retry > 5:
                break
        else:
            break
    return p, fwhm, chisq, fit


def fit_gaussian_fixed(edges, counts, bins):
    """:988-1057  mu fixed at the left edge of bin int(bins/2)-1; LM over (sigma, A)."""
    x, y = edges, counts
    if len(x) == len(y) + 1:
        x = x[0:-1]
    s0 = std(y)
    a0 = max(y)
    xmax = x[int(bins / 2) - 1]
    p = leastsq(lambda p_, x_, y_: y_ - _gauss(x_, p_[0], xmax, p_[1]), [s0, a0], args=(x, y))[0]
    fwhm = abs(FWHM_C * p[0])
    fit = _gauss(x, p[0], xmax, p[1])
    return p, fwhm, _chisq_mean(y, fit), fit, xmax


def _gbg(x, p):
    """:1226  |A| exp(-((x-mu)/|sigma|)^2/2) + bg"""
    s, mu, a, bg = p
    return abs(a) * exp((-((x - mu) / abs(s)) ** 2) / 2) + (bg)


def fit_gaussian_t1(y):
    """:1061-1132 -> fitGaussianWithBackground :1194-1264 (always rotated under Py2)."""
    y, _cut = _rotate_half(y)
    x = range(len(y))
    e = argmax(y)
    p0 = [std(y), e, y[e], 1.]
    p = leastsq(lambda p_, x_, y_: y_ - _gbg(x_, p_), p0, args=(x, y))[0]
    fwhm = abs(FWHM_C * p[0])
    fit = _gbg(x, p)
    chisq = 0
    for i in range(len(y)):
        chisq += (y[i] - fit[i]) ** 2
    chisq = chisq / len(y)
    return p, fwhm, chisq, fit


def _g_absbg(x, p):
    """fitDoubleGaussian's model (:1296): |A| exp(-((x-mu)/sigma)^2/2) + |bg|"""
    s, mu, a, bg = p
    return abs(a) * exp((-((x - mu) / s) ** 2) / 2) + abs(bg)


def _dg(x, p):
    """fitDoubleGaussianWithBackground's model (:1459-1460)."""
    s1, m1, a1, b1, s2, m2, a2, b2 = p
    return ((abs(a1) * exp((-((x - m1) / abs(s1)) ** 2) / 2)) +
            (abs(a2) * exp((-((x - m2) / abs(s2)) ** 2) / 2)) + (abs(b1) + abs(b2)) / 2)


def peel_peak(y):
    """The neighbour-deletion walk of fitDoubleGaussian (:1305-1354): returns (newx, newy)
    after deleting the peak and the symmetric/one-sided neighbours the descent rule
    (tolerance 5; operator precedence  A or (B & C)  at :1324) selects.  IndexError
    propagates (caught by getGaussianFittings)."""
    L = len(y)
    x = range(L)
    pos = argmax(y)
    nx, ny = delete(x, pos), delete(y, pos)
    tol, lim = 0, 5
    i = 1
    while i < L:
        if ((pos - i) > 0) & ((pos + i) < L):
            if (y[pos - i] < y[pos - i + 1]) & (y[pos + i] < y[pos + i - 1]):
                nx = delete(delete(nx, pos - i), pos - i)
                ny = delete(delete(ny, pos - i), pos - i)
            elif (y[pos - i] >= y[pos - i + 1]) or (y[pos + i] >= y[pos + i - 1]) & (tol < lim):
                nx = delete(delete(nx, pos - i), pos - i)
                ny = delete(delete(ny, pos - i), pos - i)
                tol += 1
            else:
                break
        elif (pos - i) < 0:
            if y[pos + i] < y[pos + i - 1]:
                nx, ny = delete(nx, pos - i + 1), delete(ny, pos - i + 1)
            elif (y[pos + i] >= y[pos + i - 1]) & (tol < lim):
                nx, ny = delete(nx, pos - i + 1), delete(ny, pos - i + 1)
                tol += 1
            else:
                break
        elif (pos + i) > L:
            if y[pos - i] < y[pos - i + 1]:
                nx, ny = delete(nx, pos - i + 1), delete(ny, pos - i + 1)
            elif (y[pos - i] >= y[pos - i + 1]) & (tol < lim):
                nx, ny = delete(nx, pos - i), delete(ny, pos - i)
                tol += 1
            else:
                break
        i += 1
    return nx, ny


def fit_double_gaussian(y):
    """:1268-1428  8 single-Gaussian passes with subtraction, then the 8-parameter fit."""
    L = len(y)
    x = range(L)
    nx, ny = peel_peak(y)
    store = {}
    for k in range(1, 9):
        npos = argmax(ny)
        p0 = [std(ny), nx[npos], max(ny), mean(ny)]
        while len(p0) > len(nx):
            nx = np.append(nx, 0)
            ny = np.append(ny, 0)
        p = leastsq(lambda p_, x_, y_: y_ - _g_absbg(x_, p_), p0, args=(nx, ny))[0]
        nfwhm = abs(FWHM_C * p[0])
        # subtraction  (:1389-1399; the window is centred on p[2], the amplitude)
        ny = []
        for i in range(L):
            ev = _g_absbg(x[i], p)
            if ev <= y[i]:
                ny.append(y[i] - ev + p[3])
            elif (ev > y[i]) & (x[i] > (p[2] - (1.5 * nfwhm) / 2)) & (x[i] < (p[2] + (1.5 * nfwhm) / 2)):
                ny.append(p[3])
            else:
                ny.append(y[i])
        nx = range(len(ny))
        if k == 7:
            store[2] = p
        elif k == 8:
            store[1] = p
    p1, p2 = store[1], store[2]
    pp = list(p1) + list(p2)
    # fitDoubleGaussianWithBackground  (:1432-1483)
    q = leastsq(lambda p_, x_, y_: y_ - _dg(x_, p_), np.array(pp), args=(x, y))[0]
    f_fwhm1, f_fwhm2 = abs(FWHM_C * q[0]), abs(FWHM_C * q[4])
    ffit = _dg(x, q)
    fchi = 0
    for i in range(L):
        if ffit[i] >= 1.:
            fchi += (y[i] - ffit[i]) ** 2 / L
    combi = _g_absbg(x, p1) + _g_absbg(x, p2) - p1[3] - p2[3] + (p1[3] + p2[3]) / 2
    cchi = 0
    for i in range(L):
        if combi[i] >= 1.:
            cchi += (y[i] - combi[i]) ** 2 / L
    c_fwhm1, c_fwhm2 = abs(FWHM_C * pp[0]), abs(FWHM_C * pp[4])
    if fchi <= cchi:
        return q, f_fwhm1, fchi, ffit, f_fwhm2
    return pp, c_fwhm2, cchi, combi, c_fwhm1


def gaussian_scores(profile):
    """[s5 .. s11]  (:654-770; PHCXFile.py:521-529)."""
    hbins = fd_bins(profile)
    dy = backward_diff(profile)
    dbins = fd_bins(dy)
    hd = histogram(dy, dbins)
    _s, d_mu, _a = fit_gaussian_hist(hd[1], hd[0])[0]
    hp = histogram(profile, hbins)
    _s, p_mu, p_a = fit_gaussian_hist(hp[1], hp[0])[0]
    fx = fit_gaussian_fixed(hp[1], hp[0], hbins)
    s5 = float(abs(fx[4] - p_mu))
    s6 = float(abs(fx[0][1] / p_a))
    s7 = float(abs(d_mu - p_mu))
    minbg = min(p_mu, profile.mean())
    if minbg > 0.:
        tp = []
        for v in profile:
            nv = v - minbg + profile.std()
            if nv < 0.:
                nv = 0.
            tp.append(nv)
    else:
        tp = profile
    gf = fit_gaussian_t1(tp)
    s8, s9 = float(gf[1]), float(gf[2])
    dgf_indexerror = False
    try:
        y2, _cut = _rotate_half(profile)
        dq, fw1, dchi, dfit, fw2 = fit_double_gaussian(y2)
        diff = dfit - (gf[3] + minbg - profile.std())
        dstd = float(abs(diff.std()))
        s10 = s8 if dstd < 3. else float(min(fw1, fw2))
        s11 = float(dchi)
    except IndexError:
        s10, s11 = 1000000.0, 1000000.0
        dgf_indexerror = True
    return [s5, s6, s7, s8, s9, s10, s11], dgf_indexerror


# ---------------------------------------------------------------------------------------
# scores 12-15, 16-19   PHCXOperations.getCandidateParameters :81-112, getDMFittings :121-233
# ---------------------------------------------------------------------------------------
def _filter_neg(v, eps=0.000005):
    """CandidateFileInterface.filterScore for scores 13/14 (:97-107, isEqual :116-149)."""
    return 0.0 if (abs(v - 0.0) > eps and v < 0.0) else v


def parameter_scores(scal):
    period, snr, dm, width = scal[0], scal[1], scal[2], scal[3]
    return [float(period), _filter_neg(float(snr)), _filter_neg(float(dm)), float(width)]


KDM = 8.3 * 10 ** 6
DF = 400
F = 1374


def dm_scores(curve, scal, signed_shift=False):
    """[s16..s19]  (PHCXOperations.py:150-233; filterScore(18) = abs).  signed_shift: the
    third value as getDMFittings returns it (plsq[0][2], :232), before PHCXFile's filter."""
    period, snr, dm, width = float(scal[0]), float(scal[1]), float(scal[2]), float(scal[3])
    dm_start, dm_end, length_all = float(scal[4]), float(scal[5]), int(scal[6])
    y = np.asarray(curve)
    n = len(y)
    xk = np.arange(n) * 128 - 1                 # dm_curve's x: i - 128 at i = 128k+127
    step = abs(dm_start - dm_end) / length_all
    wint = (width * period) ** 2
    peak = snr / sqrt((period - sqrt(wint)) / sqrt(wint))
    x = np.array([dm_start + xk[i] * step for i in range(n)])
    help_ = []
    for i in range(n):
        weff = sqrt(wint + pow(KDM * abs(dm - x[i]) * DF / pow(F, 3), 2))
        help_.append(float(sqrt((period - weff) / weff)))
    hmax = _pymax(help_)
    theo = (255. / hmax) * np.array(help_)

    def model(p, x_):
        a, prop, shift = p
        weff = sqrt(wint + pow(prop * KDM * abs((dm + shift) - x_) * DF / pow(F, 3), 2))
        return a * sqrt((period - weff) / weff)

    p = leastsq(lambda p_, x_, y_: y_ - model(p_, x_), (255. / hmax, 1, 0), args=(x, y))[0]
    fit = model(p, x)
    chi = 0
    for i in range(n):
        if fit[i] >= 1.:
            chi += (y[i] - theo[i]) ** 2
    chi = chi / n
    shift = float(p[2]) if signed_shift else float(abs(float(p[2])))
    return [float(peak), float(abs(1 - p[1])), shift, float(chi)]


# ---------------------------------------------------------------------------------------
# scores 20-22   ProfileOperations.getSubband_scores :1585-1686; PHCXOperations :305-415
# ---------------------------------------------------------------------------------------
def subband_scores(sub, profile, width):
    nsub, nb = sub.shape
    wb = int(np.ceil(width * nb))
    sums = []
    for i in range(nsub):
        row = []
        for j in range(nb - wb + 1):
            s = 0
            for b in range(wb):
                s += sub[i][j + b]
            row.append(s)
        sums.append(row)
    max_bins = []
    mb = None  # max_bin is one local across the bands: a band with no sum > -10000 repeats
    for i in range(len(sums)):  # the previous band's position (:1619-1628)
        best = -10000.0
        for j in range(len(sums[i])):
            if sums[i][j] > best:
                best = sums[i][j]
                mb = j + wb // 2
        if mb is None:
            raise UnboundLocalError("max_bin referenced before assignment")
        max_bins.append(float(mb))
    med = np.array(max_bins).mean()
    cnt, vm = 0, 0.0
    for v in max_bins:
        if abs(v - med) <= float(wb):
            cnt += 1
            vm += pow(v - med, 2)
    if cnt > 1:
        var = vm / float(cnt - 1)
    else:
        mu, var = 0, 0
        for v in max_bins:
            mu += v
        mu /= float(len(max_bins))
        for v in max_bins:
            var += pow(v - mu, 2)
        var /= float(len(max_bins) - 1)
    sd = sqrt(var)
    m, tot = 0, 0.0
    for i in range(len(sums)):
        for k in range(i + 1, len(sums)):
            cc = np.corrcoef(sums[i], sums[k])[0][1]
            if str(cc) != "nan":
                tot += cc
                m += 1
    mean_corr = tot / float(m)          # ZeroDivisionError when no pair is valid
    rms = sd / float(wb)
    corr = []
    for j in range(nsub):
        c = abs(np.corrcoef(sub[j], profile))
        if c[0][1] > 0.0055:
            corr.append(c[0][1])
    integ = 0
    for c in np.array(corr):
        integ += c
    return [float(rms), float(mean_corr), float(integ)]


# ---------------------------------------------------------------------------------------
# the whole candidate   PHCXFile.compute :383-409
# ---------------------------------------------------------------------------------------
def bates22_one(prof, sub, curve, scal):
    """22 scores for one candidate, or raise CandidateFailure like the reference."""
    profile = np.asarray(prof, dtype=np.int64)
    subb = np.asarray(sub, dtype=np.int64)
    flags = {"dgf_indexerror": False}
    out = []
    with warnings.catch_warnings(), np.errstate(all="ignore"):
        warnings.simplefilter("ignore")
        for group, fn in (
            ("sine", lambda: sinusoid_scores(profile)),
            ("gauss", lambda: gaussian_scores(profile)),
            ("params", lambda: parameter_scores(scal)),
            ("dmfit", lambda: dm_scores(curve, scal)),
            ("subband", lambda: subband_scores(subb, profile, float(scal[3]))),
        ):
            try:
                r = fn()
            except Exception as e:  # the reference re-raises a generic Exception per group
                raise CandidateFailure(group, e) from e
            if group == "gauss":
                r, flags["dgf_indexerror"] = r
            out.extend(r)
    return out, flags


GROUP_BITS = {"sine": 0x001, "gauss": 0x002, "params": 0x002, "dmfit": 0x004, "subband": 0x008}


def bates22(prof, sub, curve, scal):
    """Batch form: (n,22) float64 scores (NaN rows for failures) and (n,) uint32 status
    bits in the libpfe PFE_ST_* encoding."""
    n = len(prof)
    out = np.full((n, 22), np.nan)
    st = np.zeros(n, dtype=np.uint32)
    for i in range(n):
        try:
            v, fl = bates22_one(prof[i], sub[i], curve[i], scal[i])
            out[i] = v
            if fl["dgf_indexerror"]:
                st[i] |= 0x100
        except CandidateFailure as e:
            st[i] |= GROUP_BITS[e.group]
    return out, st


def math_isclose(a, b):  # pragma: no cover - debugging helper
    return math.isclose(a, b, rel_tol=1e-12)
