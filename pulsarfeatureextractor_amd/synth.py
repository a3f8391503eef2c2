"""Synthetic pulsar-candidate batches.

Per row: Gaussian noise N(40, 8); for half the rows ("pulsar-like") a Gaussian pulse of
amplitude A at a random phase with sigma ~ U(1, 8) bins; then min-max scaling to 0-255 and
rounding to uint8, the 02X byte range of PHCX data.  Seeds are numpy default_rng
(base 20261015 + config index).

Two generators produce the same recipe: ``numpy`` (host, for fixtures and parity tests) and
``torch`` (on-device, for the 10M-row bench batches, which would take minutes on the host).
"""
from __future__ import annotations

import numpy as np

BASE_SEED = 20261015


def _rows_numpy(rng: np.random.Generator, n: int, L: int, amp_lo: float, amp_hi: float,
                pulsar_frac: float = 0.5, centred: bool = False) -> np.ndarray:
    x = rng.normal(40.0, 8.0, size=(n, L))
    pulsar = rng.random(n) < pulsar_frac
    amp = rng.uniform(amp_lo, amp_hi, size=n)
    mu = np.full(n, L / 2.0) if centred else rng.uniform(0, L, size=n)
    sig = rng.uniform(1.0, 8.0, size=n)
    t = np.arange(L)[None, :]
    # periodic distance so pulses near the edges wrap like a folded profile
    d = np.abs(t - mu[:, None])
    d = np.minimum(d, L - d)
    x += np.where(pulsar[:, None], amp[:, None] * np.exp(-0.5 * (d / sig[:, None]) ** 2), 0.0)
    lo = x.min(axis=1, keepdims=True)
    hi = x.max(axis=1, keepdims=True)
    y = (x - lo) / np.where(hi > lo, hi - lo, 1.0) * 255.0
    return np.rint(y).astype(np.uint8)


def lyon_batch(n: int, lp: int = 128, ld: int = 128, seed: int = BASE_SEED + 2,
               adversarial: bool = True):
    """Profile + DM arrays for the 8-feature path: ((n,lp) uint8, (n,ld) uint8)."""
    rng = np.random.default_rng(seed)
    prof = _rows_numpy(rng, n, lp, 150.0, 150.0)
    dm = _rows_numpy(rng, n, ld, 150.0, 150.0)
    if adversarial and n >= 8:
        prof[0, :] = 0            # constant rows: std 0, skew/kurt NaN
        dm[0, :] = 255
        prof[1, :] = 7
        prof[2, :] = 0
        prof[2, 5] = 255          # single spike: extreme skew/kurt
        dm[3, :] = 255
        dm[3, ::2] = 0            # two-valued
        prof[4, :] = np.arange(lp) % 256  # ramp
    return prof, dm


def bates_batch(n: int, lp: int = 128, nsub: int = 16, lsb: int = 128, ndm: int = 128,
                seed: int = BASE_SEED + 3):
    """Inputs of the 22-score path: profile, sub-bands, reduced DM curve and scalars.

    Scalars follow §8(d): P ~ U(0.05, 1.0) s, dm ~ U(10, 150), snr ~ U(8, 30),
    width ~ U(0.02, 0.1); DmIndex spans 0..200.  Returns a dict of numpy arrays.
    """
    rng = np.random.default_rng(seed)
    prof = _rows_numpy(rng, n, lp, 150.0, 150.0)
    sub = _rows_numpy(rng, n * nsub, lsb, 20.0, 150.0).reshape(n, nsub, lsb)
    dmc = _rows_numpy(rng, n, ndm, 150.0, 150.0, pulsar_frac=1.0, centred=True).astype(np.float64)
    period_ms = rng.uniform(0.05, 1.0, size=n) * 1000.0
    dmv = rng.uniform(10.0, 150.0, size=n)
    snr = rng.uniform(8.0, 30.0, size=n)
    width = rng.uniform(0.02, 0.1, size=n)
    scal = np.zeros((n, 8), dtype=np.float64)
    scal[:, 0] = period_ms
    scal[:, 1] = snr
    scal[:, 2] = dmv
    scal[:, 3] = width
    scal[:, 4] = 0.0          # dm_start
    scal[:, 5] = 200.0        # dm_end
    scal[:, 6] = ndm * 128.0  # length_all (decoded DataBlock length)
    return {"prof": prof, "sub": sub, "dmcurve": dmc, "scal": scal}


def lyon_batch_torch(n: int, lp: int = 128, ld: int = 128, seed: int = BASE_SEED + 2,
                     device="cuda"):
    """Same recipe generated on the GPU with torch (bench-sized batches)."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)

    def rows(L):
        out = torch.empty((n, L), dtype=torch.uint8, device=device)
        chunk = 1 << 20 if L <= 1024 else max(1, (1 << 28) // L)  # float temporaries <= 1 GiB
        t = torch.arange(L, device=device, dtype=torch.float32)[None, :]
        for s in range(0, n, chunk):
            m = min(chunk, n - s)
            x = torch.randn((m, L), generator=g, device=device) * 8.0 + 40.0
            pulsar = torch.rand((m, 1), generator=g, device=device) < 0.5
            mu = torch.rand((m, 1), generator=g, device=device) * L
            sig = torch.rand((m, 1), generator=g, device=device) * 7.0 + 1.0
            d = (t - mu).abs()
            d = torch.minimum(d, L - d)
            x = x + pulsar * (150.0 * torch.exp(-0.5 * (d / sig) ** 2))
            lo = x.amin(dim=1, keepdim=True)
            hi = x.amax(dim=1, keepdim=True)
            y = (x - lo) / torch.where(hi > lo, hi - lo, torch.ones_like(hi)) * 255.0
            out[s:s + m] = torch.round(y).to(torch.uint8)
        return out

    return rows(lp), rows(ld)


def pfd_candidate(rng: np.random.Generator, npart: int = 8, nsub: int = 16, proflen: int = 64,
                  pulsar: bool = True, lofreq: float = 1200.0, chan_wid: float = 1.0,
                  chan_per_sub: int = 4):
    """Arrays of one synthetic PRESTO fold (pfd.write keywords): noise sub-integration
    profiles plus, for pulsar-like candidates, a pulse dispersed at the true DM, so that
    de-dispersion at the best DM lines the sub-bands up.  The DM grid spans the best DM."""
    f1 = rng.uniform(1.0, 20.0)  # fold frequency (Hz): bins per second = f1 * proflen
    dm_true = rng.uniform(10.0, 150.0)
    bestdm = dm_true + rng.normal(0.0, 0.5)
    numchan = nsub * chan_per_sub
    subdelta = chan_wid * chan_per_sub
    subfreqs = np.arange(nsub) * subdelta + lofreq + subdelta - chan_wid
    delays = dm_true / (0.000241 * subfreqs ** 2)
    shift = (delays - delays[-1]) * f1 * proflen  # bins the pulse lags in each sub-band
    t = np.arange(proflen)
    profs = rng.normal(100.0, 10.0, size=(npart, nsub, proflen))
    if pulsar:
        mu, sig, amp = rng.uniform(0, proflen), rng.uniform(1.0, 4.0), rng.uniform(5.0, 40.0)
        for j in range(nsub):
            d = np.abs(t - (mu + shift[j]) % proflen)
            d = np.minimum(d, proflen - d)
            profs[:, j, :] += amp * np.exp(-0.5 * (d / sig) ** 2)
    stats = np.zeros((npart, nsub, 7))
    stats[:, :, 0] = 1000.0
    stats[:, :, 5] = profs.var(axis=2) * rng.uniform(0.9, 1.1)
    ndms = int(rng.integers(20, 80))
    dms = np.linspace(bestdm - rng.uniform(5, 30), bestdm + rng.uniform(5, 30), ndms)
    return dict(profs=profs, stats=stats, dms=dms, bestdm=bestdm, fold_p1=f1,
                bary_p1=1.0 / f1, lofreq=lofreq, chan_wid=chan_wid, numchan=numchan)


def pfd_fold_block(n: int, shape, seed: int):
    """n synthetic PRESTO folds of one (npart, nsub, proflen) shape as pfd.PFDData records
    (what pfd.read returns for the files pfd.write would make of them): bench.py's PFD
    workload, fold i drawn from default_rng(seed + i)."""
    from . import pfd as _pfd

    npart, nsub, L = shape
    datas = []
    for i in range(n):
        c = pfd_candidate(np.random.default_rng(seed + i), npart, nsub, L)
        chanpersub = c["numchan"] // nsub
        sd = c["chan_wid"] * chanpersub
        stats = c["stats"]
        datas.append(_pfd.PFDData(
            npart=npart, nsub=nsub, proflen=L, profs=c["profs"], bestdm=c["bestdm"],
            binspersec=c["fold_p1"] * L, avgprof=(c["profs"] / L).sum(),
            varprof=float(stats[:, :, 5].sum()), dms=c["dms"], numdms=len(c["dms"]),
            bary_p1=c["fold_p1"],
            subfreqs=np.arange(nsub, dtype="d") * sd + (c["lofreq"] + sd - c["chan_wid"])))
    return datas
