#!/usr/bin/env python3
"""Golden vectors from the REAL reference (run only in the build container).

What it does:
  1. copies PulsarFeatureExtractor/src/*.py from /root/reference into a temporary directory
     (never into this repository), converts it with lib2to3 (fixers print, except, has_key,
     long, numliterals) and applies the minimal compatibility patches below, which restore
     the Python-2.7 semantics the reference was written for (.pydevproject:6);
  2. writes synthetic PHCX (gzip, 128-bin, section 1) and SUPERB PHCX (plain, 64-bin,
     section 0) candidate files with pulsarfeatureextractor_amd.phcx.write;
  3. runs, in a child process inside that temporary directory,
        Candidate(f, f).calculateProfileStatScores(False) + calculateDMCurveStatScores(False)
        (the dmprof path, DataProcessor.py:882-886)  and
        Candidate(f, f).calculateScores(False)       (the 22-score path, :505-510);
  4. stores inputs (as arrays) and outputs under tests/golden/*.npz plus a JSON manifest
     with numpy/scipy versions, seeds and the patch list.

Compatibility patches (each restores Py2 behaviour, none changes the algorithm):
  ProfileOperationsInterface.py  Py2 '/' on integers is floor division: nbins and scale()
                                  use _py2div (scale() therefore returns 0 for every index,
                                  so fitGaussianT1/fitDoubleGaussianT2 always rotate)
  ProfileOperations.py           'from scipy import std' -> numpy.std (removed from scipy);
                                  'xData == []' on an ndarray was False in 2014 numpy
                                  (raises on numpy 2) -> _py2_eq_empty; ceil(L/2) -> L//2;
                                  width_bins/2 -> width_bins//2 (Py2 int division)
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF_SRC = "/root/reference/PulsarFeatureExtractor/src"
GOLDEN = os.path.join(ROOT, "tests", "golden")

HELPERS = '''
import numpy as _np
def _py2div(a, b):
    """Python-2 '/' : floor division when both operands are integers."""
    if isinstance(a, (int, _np.integer)) and isinstance(b, (int, _np.integer)) \\
            and not isinstance(a, bool) and not isinstance(b, bool):
        return a // b
    return a / b
def _py2_eq_empty(x):
    """Python-2 era 'x == []': True only for an empty list."""
    return isinstance(x, list) and len(x) == 0
'''

PATCHES = {
    "ProfileOperationsInterface.py": [
        ("from Utilities import Utilities", "from Utilities import Utilities\n" + HELPERS),
        ("nbins = ceil( rnge / binwidth )", "nbins = ceil( _py2div(rnge, binwidth) )"),
        ("x = (newMin * (1-( (x-min_) /( max_-min_ )))) + (newMax * ( (x-min_) /( max_-min_ ) ))",
         "x = (newMin * (1-( _py2div((x-min_), ( max_-min_ ))))) + "
         "(newMax * ( _py2div((x-min_), ( max_-min_ )) ))"),
    ],
    "ProfileOperations.py": [
        ("from scipy import std", "from numpy import std"),
        ("from ProfileOperationsInterface import ProfileOperationsInterface",
         "from ProfileOperationsInterface import ProfileOperationsInterface, _py2div, _py2_eq_empty"),
        ("if xData == []:", "if _py2_eq_empty(xData):"),
        ("int(ceil(yDataLength/2))", "int(ceil(yDataLength//2))"),
        ("max_bin = j+width_bins/2", "max_bin = j+width_bins//2"),
    ],
}

# Python-3 compatibility of the PFD reader / operations (bytes vs str) plus the Py2 integer
# divisions the PFD path relies on
PFD_PATCHES = {
    "PFDFile.py": [
        ("if test[ii] not in '0123456789:.-\\0':", "if chr(test[ii]) not in '0123456789:.-\\0':"),
        ("self.rastr = test[:test.find('\\0')]", "self.rastr = test[:test.find(b'\\0')]"),
        ("self.decstr = test[:test.find('\\0')]", "self.decstr = test[:test.find(b'\\0')]"),
        ("self.chanpersub = self.numchan / self.nsub", "self.chanpersub = self.numchan // self.nsub"),
    ],
    "PFDOperations.py": [
        ("dtype=Num.float)", "dtype=float)"),
        ("shift = peak - len(profile.profile) / 2", "shift = peak - len(profile.profile) // 2"),
    ],
}

RUNNER = r'''
import json, sys, traceback, warnings
warnings.simplefilter("ignore")
import numpy as np
import Candidate
files = json.load(open(sys.argv[1]))
mode = sys.argv[2]
res = []
for f in files:
    try:
        c = Candidate.Candidate(f, f)
        if mode == "lyon8":
            a = list(c.calculateProfileStatScores(False))
            b = list(c.calculateDMCurveStatScores(False))
            v = [float(x) for x in a + b]
        elif mode == "profile":
            v = [float(x) for x in c.calculateProfileScores(False)]
        elif mode == "getters":
            v = {"subband": [float(x) for x in c.getSubbandData(False)],
                 "subint": [float(x) for x in c.getSubintData(False)],
                 "subband_types": sorted({type(x).__name__ for x in c.getSubbandData(False)})}
        elif mode == "all30":
            a = list(c.calculateProfileStatScores(False))
            b = list(c.calculateDMCurveStatScores(False))
            v = [float(x) for x in a + b]
            v += [float(x) for x in Candidate.Candidate(f, f).calculateScores(False)]
        else:
            v = [float(x) for x in c.calculateScores(False)]
        res.append({"ok": True, "v": v})
    except Exception as e:
        res.append({"ok": False, "err": "".join(traceback.format_exception_only(type(e), e)).strip()})
json.dump(res, open(sys.argv[3], "w"))
'''


def build_reference(tmp: str) -> str:
    dst = os.path.join(tmp, "ref")
    os.makedirs(dst)
    for fn in os.listdir(REF_SRC):
        if fn.endswith(".py"):
            shutil.copy(os.path.join(REF_SRC, fn), dst)
    subprocess.run([sys.executable, "-m", "lib2to3", "-f", "print", "-f", "except", "-f",
                    "has_key", "-f", "long", "-f", "numliterals", "-w", "-n", "."],
                   cwd=dst, check=True, capture_output=True)
    for fn, subs in list(PATCHES.items()) + list(PFD_PATCHES.items()):
        p = os.path.join(dst, fn)
        s = open(p).read()
        for a, b in subs:
            if a not in s:
                raise RuntimeError(f"patch anchor not found in {fn}: {a!r}")
            s = s.replace(a, b)
        open(p, "w").write(s)
    with open(os.path.join(dst, "_runner.py"), "w") as f:
        f.write(RUNNER)
    return dst


def run_reference(refdir: str, files: list[str], mode: str, tmp: str):
    fl = os.path.join(tmp, f"files_{mode}.json")
    out = os.path.join(tmp, f"out_{mode}.json")
    json.dump(files, open(fl, "w"))
    env = dict(os.environ, MPLBACKEND="Agg", PYTHONHASHSEED="0")
    subprocess.run([sys.executable, "_runner.py", fl, mode, out], cwd=refdir, check=True, env=env)
    return json.load(open(out))


# ------------------------------------------------------------------------------------------
# synthetic candidate sets
# ------------------------------------------------------------------------------------------
def lyon_set(rng, n, lp, l0, superb):
    from pulsarfeatureextractor_amd.synth import _rows_numpy

    prof = _rows_numpy(rng, n, lp, 150.0, 150.0)
    dm0 = _rows_numpy(rng, n, l0, 150.0, 150.0)
    # adversarial rows
    prof[0] = 0
    dm0[0] = 255
    prof[1] = 77
    prof[2] = 0
    prof[2, 5] = 255
    dm0[3] = 255
    dm0[3, ::2] = 0
    prof[4] = np.arange(lp) % 256
    return prof, dm0


def bates_set(rng, n, lp, nsub, lsb, ndm, superb):
    from pulsarfeatureextractor_amd.phcx import make_datablock
    from pulsarfeatureextractor_amd.synth import _rows_numpy

    prof = _rows_numpy(rng, n, lp, 150.0, 150.0)
    sub = _rows_numpy(rng, n * nsub, lsb, 20.0, 150.0).reshape(n, nsub, lsb)
    curve = _rows_numpy(rng, n, ndm, 150.0, 150.0, pulsar_frac=1.0, centred=True)
    period = rng.uniform(0.05, 1.0, size=n)
    dmv = rng.uniform(10.0, 150.0, size=n)
    snr = rng.uniform(8.0, 30.0, size=n)
    width = rng.uniform(0.02, 0.1, size=n)
    # adversarial rows
    prof[0] = 50                 # constant profile: maxima=0 -> s1,s2 inf; histogram fallback
    prof[1] = 0
    prof[1, ::3] = 200           # comb: many peaks
    prof[2] = 0
    prof[2, lp // 2] = 255       # single spike
    sub[3] = 0                   # all-zero sub-bands: corrcoef NaN everywhere -> m=0 -> fail
    width[4] = 0.0               # width*Lsb = 0 -> boxcar width 0
    width[5] = 1.0 / lsb * 3.0   # odd boxcar width 3
    prof[6] = np.roll(prof[6], -int(np.argmax(prof[6])))  # peak at bin 0
    prof[7] = np.roll(prof[7], lp - 1 - int(np.argmax(prof[7])))  # peak at the last bin
    blocks = np.stack([make_datablock(curve[i], rng) for i in range(n)])
    return prof, sub, curve, blocks, period, dmv, snr, width


def write_files(d, kind, arrays, superb):
    from pulsarfeatureextractor_amd import phcx

    os.makedirs(d, exist_ok=True)
    files = []
    ext = ".phcx" if superb else ".phcx.gz"
    for i in range(arrays["n"]):
        p = os.path.join(d, f"{kind}_{i:05d}{ext}")
        phcx.write(p, profile=arrays["prof"][i], subbands=arrays["sub"][i],
                   datablocks=(arrays["block0"][i], arrays["block1"][i]),
                   dm_start=arrays["dm_start"], dm_end=arrays["dm_end"],
                   n_dm_index=arrays["n_dm_index"], period_s=float(arrays["period"][i]),
                   snr=float(arrays["snr"][i]), dm=float(arrays["dm"][i]),
                   width=float(arrays["width"][i]), superb=superb)
        files.append(p)
    return files


def collect(res, nout):
    n = len(res)
    out = np.full((n, nout), np.nan)
    ok = np.zeros(n, dtype=bool)
    errs = []
    for i, r in enumerate(res):
        ok[i] = r["ok"]
        if r["ok"]:
            out[i] = r["v"]
            errs.append("")
        else:
            errs.append(r["err"])
    return out, ok, np.array(errs)


SPECS = [
    # name, mode, superb, n, lp, l0 (Lyon DM length), nsub, lsb, ndm, seed
    ("lyon8_superb64", "lyon8", True, 400, 64, 64, 16, 64, 2, 1),
    ("lyon8_phcx128", "lyon8", False, 400, 128, 128, 16, 128, 2, 2),
    ("lyon8_phcx128_dmplane", "lyon8", False, 60, 128, 120 * 128, 16, 128, 2, 3),
    ("bates22_phcx128", "bates22", False, 300, 128, 128, 16, 128, 128, 4),
    ("bates22_superb64", "bates22", True, 150, 64, 64, 16, 64, 120, 5),
    # config 4 as BASELINE.json words it (256-bin profile, 16 x 128 sub-bands): the
    # reference's corrcoef of a 128-bin band with the 256-bin profile raises ValueError
    ("bates22_cfg4_256x128", "bates22", False, 40, 256, 128, 16, 128, 128, 6),
    # 32 sub-bands (nSub is read from the file, PHCXOperations.py:330-338)
    ("bates22_phcx128_nsub32", "bates22", False, 60, 128, 128, 32, 128, 128, 7),
    # config 5's 30-column matrix: 8 Lyon features then the 22 scores of the same files
    ("all30_phcx128", "all30", False, 80, 128, 128, 16, 128, 128, 8),
    # near-flat profiles quantised from sigma ~ 0.5 noise under a narrow pulse: tiny
    # interquartile ranges, so Freedman-Diaconis histograms of 1000-1600 bins (rows 8..39)
    ("bates22_phcx128_wide", "bates22", False, 48, 128, 128, 16, 128, 128, 9),
    # round 4: larger sets for the per-row envelope pins of the chaotic LM scores (more tight
    # rows for s10/s11/s17/s18); stored with the reduced DM curves instead of the DataBlocks
    ("bates22_phcx128_big", "bates22", False, 1000, 128, 128, 16, 128, 128, 11),
    ("bates22_superb64_big", "bates22", True, 500, 64, 64, 16, 64, 120, 12),
]
COMPACT = ("bates22_phcx128_big", "bates22_superb64_big")


def lownoise_wide_rows(rng, n, lp):
    """Profiles whose profile or derivative histogram has more than 1024 FD bins."""
    from oracle.bates import backward_diff, fd_bins

    x = np.arange(lp)
    rows = []
    while len(rows) < n:
        base = rng.normal(100, 0.5, lp)
        mu, w = rng.uniform(10, lp - 10), rng.uniform(1.0, 3.0)
        p = np.clip(np.rint(base + 150 * np.exp(-0.5 * ((x - mu) / w) ** 2)), 0, 255)
        p = p.astype(np.int64)
        if max(fd_bins(p), fd_bins(backward_diff(p))) > 1024:
            rows.append(p.astype(np.uint8))
    return np.stack(rows)


def main(only=None):
    import scipy

    os.makedirs(GOLDEN, exist_ok=True)
    mpath = os.path.join(GOLDEN, "manifest.json")
    if only and os.path.exists(mpath):
        manifest = json.load(open(mpath))
    else:
        manifest = {"numpy": np.__version__, "scipy": scipy.__version__,
                    "python": sys.version.split()[0], "reference": REF_SRC,
                    "patches": {k: [a for a, _ in v] for k, v in PATCHES.items()},
                    "lib2to3_fixers": ["print", "except", "has_key", "long", "numliterals"],
                    "sets": {}}
    with tempfile.TemporaryDirectory(prefix="pfe_golden_") as tmp:
        refdir = build_reference(tmp)
        for name, mode, superb, n, lp, l0, nsub, lsb, ndm, seed in SPECS:
            if only and name not in only:
                continue
            rng = np.random.default_rng(20261015 + 100 * seed)
            if mode == "lyon8":
                prof, dm0 = lyon_set(rng, n, lp, l0, superb)
                from pulsarfeatureextractor_amd.phcx import make_datablock
                from pulsarfeatureextractor_amd.synth import _rows_numpy
                sub = _rows_numpy(rng, n * nsub, lsb, 20.0, 150.0).reshape(n, nsub, lsb)
                curve = _rows_numpy(rng, n, ndm, 150.0, 150.0, pulsar_frac=1.0, centred=True)
                block1 = np.stack([make_datablock(curve[i], rng) for i in range(n)])
                arrays = dict(n=n, prof=prof, sub=sub, block0=dm0,
                              block1=dm0 if superb else block1,
                              period=rng.uniform(0.05, 1.0, n), dm=rng.uniform(10, 150, n),
                              snr=rng.uniform(8, 30, n), width=rng.uniform(0.02, 0.1, n),
                              dm_start=0.0, dm_end=200.0, n_dm_index=101)
            else:
                prof, sub, curve, blocks, period, dmv, snr, width = bates_set(
                    rng, n, lp, nsub, lsb, ndm, superb)
                if name.endswith("_wide"):
                    prof[8:] = lownoise_wide_rows(rng, n - 8, lp)
                b0 = blocks if superb else _rows_lyon(rng, n, 128)
                arrays = dict(n=n, prof=prof, sub=sub, block0=b0, block1=blocks,
                              period=period, dm=dmv, snr=snr, width=width,
                              dm_start=0.0, dm_end=200.0, n_dm_index=101)
            files = write_files(os.path.join(tmp, name), name, arrays, superb)
            res = run_reference(refdir, files, mode, tmp)
            nout = {"lyon8": 8, "bates22": 22, "all30": 30}[mode]
            out, ok, errs = collect(res, nout)
            blocks_kw = dict(block0=np.asarray(arrays["block0"]).astype(np.uint8),
                             block1=np.asarray(arrays["block1"]).astype(np.uint8))
            if name in COMPACT:  # the scored section's reduced DM curve instead of the blocks
                from pulsarfeatureextractor_amd.phcx import reduce_dm_curve

                fit_blk = np.asarray(arrays["block0"] if superb else arrays["block1"])
                blocks_kw = dict(dmcurve=np.stack([reduce_dm_curve(b)[0] for b in fit_blk]),
                                 block_len=int(fit_blk.shape[1]))
            np.savez_compressed(
                os.path.join(GOLDEN, name + ".npz"),
                prof=arrays["prof"].astype(np.uint8), sub=arrays["sub"].astype(np.uint8),
                **blocks_kw,
                period=arrays["period"], dm=arrays["dm"], snr=arrays["snr"],
                width=arrays["width"], dm_start=arrays["dm_start"], dm_end=arrays["dm_end"],
                n_dm_index=arrays["n_dm_index"], superb=superb, out=out, ok=ok, err=errs)
            manifest["sets"][name] = {"mode": mode, "superb": superb, "n": n, "lp": lp,
                                      "lyon_dm_len": l0, "nsub": nsub, "lsb": lsb, "ndm": ndm,
                                      "seed": 20261015 + 100 * seed,
                                      "failures": int((~ok).sum())}
            print(f"{name}: {n} candidates, {int((~ok).sum())} reference failures", flush=True)
    with open(mpath, "w") as f:
        json.dump(manifest, f, indent=1)


PFD_SETS = [
    # name, n, npart, nsub, proflen, base seed
    ("pfd_64x16", 40, 8, 16, 64, 20261715),
    ("pfd_128x32", 16, 12, 32, 128, 20261815),
]


def pfd_candidates(n, npart, nsub, proflen, seed):
    """Deterministic synthetic PFD sets (regenerated from the seeds by the tests): candidate
    i uses default_rng(seed + i); rows 0-3 are adversarial."""
    from pulsarfeatureextractor_amd.synth import pfd_candidate

    out = []
    for i in range(n):
        c = pfd_candidate(np.random.default_rng(seed + i), npart, nsub, proflen,
                          pulsar=(i % 4 != 1))
        kw = {}
        if i == 0:
            c["profs"][:] = 100.0          # constant: normalised profile 0/0 -> NaN
        if i == 2:
            kw["big_endian"] = True
        if i == 3:
            kw["with_posn"] = False
        if i == 5:
            c["dms"] = c["dms"][:1]        # numdms == 1: dms becomes a scalar, indexing raises
        out.append((c, kw))
    return out


def make_pfd_golden(manifest):
    from pulsarfeatureextractor_amd import pfd

    with tempfile.TemporaryDirectory(prefix="pfe_golden_pfd_") as tmp:
        refdir = build_reference(tmp)
        for name, n, npart, nsub, proflen, seed in PFD_SETS:
            d = os.path.join(tmp, name)
            os.makedirs(d)
            files = []
            checks = []
            for i, (c, kw) in enumerate(pfd_candidates(n, npart, nsub, proflen, seed)):
                p = os.path.join(d, f"{name}_{i:04d}.pfd")
                pfd.write(p, **c, **kw)
                files.append(p)
                checks.append(float(np.asarray(c["profs"]).sum()))
            arrs = {}
            for mode, nout in (("lyon8", 8), ("profile", proflen), ("bates22", 22)):
                res = run_reference(refdir, files, mode, tmp)
                out, ok, errs = collect(res, nout)
                arrs[mode] = (out, ok, errs)
                print(f"{name} {mode}: {int((~ok).sum())} reference failures", flush=True)
            np.savez_compressed(
                os.path.join(GOLDEN, name + ".npz"), n=n, npart=npart, nsub=nsub,
                proflen=proflen, seed=seed, profs_sum=np.array(checks),
                lyon8=arrs["lyon8"][0], lyon8_ok=arrs["lyon8"][1], lyon8_err=arrs["lyon8"][2],
                profile=arrs["profile"][0], profile_ok=arrs["profile"][1],
                bates22=arrs["bates22"][0], bates22_ok=arrs["bates22"][1],
                bates22_err=arrs["bates22"][2])
            manifest["sets"][name] = {"mode": "pfd lyon8 + profile + bates22", "n": n,
                                      "npart": npart, "nsub": nsub, "proflen": proflen,
                                      "seed": seed, "generator": "synth.pfd_candidate",
                                      "patches": {k: [a for a, _ in v] for k, v in PFD_PATCHES.items()}}


LABEL_RUNNER = r'''
import sys, warnings
warnings.simplefilter("ignore")
import DataProcessor
dp = DataProcessor.DataProcessor(False)
# DataProcessor.label (:691-826) with the regexes labelPHCX / labelPFD pass (labelPFD itself
# cannot be called with the two arguments ScoreGenerator.py:225 gives it)
regex = [dp.phcxRegex] if sys.argv[2] == "phcx" else [dp.pfdRegex, dp.pfdScrunchedRegex]
dp.label(sys.argv[1], False, regex)
'''


def make_label_golden(manifest):
    """--label mode: the four files DataProcessor.label writes for a directory of PHCX files
    and one of PFD files (text, with the directory prefix replaced by '<DIR>')."""
    from pulsarfeatureextractor_amd import pfd

    with tempfile.TemporaryDirectory(prefix="pfe_golden_label_") as tmp:
        refdir = build_reference(tmp)
        with open(os.path.join(refdir, "_label_runner.py"), "w") as f:
            f.write(LABEL_RUNNER)
        out = {}
        # PHCX: 20 candidates of the 22-score recipe (rows 0, 3, 4 fail)
        rng = np.random.default_rng(20261015 + 100 * 10)
        prof, sub, curve, blocks, period, dmv, snr, width = bates_set(rng, 20, 128, 16, 128, 128, False)
        arrays = dict(n=20, prof=prof, sub=sub, block0=_rows_lyon(rng, 20, 128), block1=blocks,
                      period=period, dm=dmv, snr=snr, width=width, dm_start=0.0, dm_end=200.0,
                      n_dm_index=101)
        d = os.path.join(tmp, "label_phcx")
        write_files(d, "label", arrays, False)
        subprocess.run([sys.executable, "_label_runner.py", d, "phcx"], cwd=refdir, check=True,
                       env=dict(os.environ, MPLBACKEND="Agg"), capture_output=True)
        for k in ("Scores.csv", "Profile.csv", "DMCurve.csv", "Cands.meta"):
            out["phcx_" + k] = open(os.path.join(d, k)).read().replace(d, "<DIR>")
        for k, v in arrays.items():
            out["phcx_in_" + k] = np.asarray(v)
        # PFD: the first 12 folds of the pfd_64x16 recipe
        d = os.path.join(tmp, "label_pfd")
        os.makedirs(d)
        for i, (c, kw) in enumerate(pfd_candidates(12, 8, 16, 64, 20261915)):
            pfd.write(os.path.join(d, f"label_{i:04d}.pfd"), **c, **kw)
        subprocess.run([sys.executable, "_label_runner.py", d, "pfd"], cwd=refdir, check=True,
                       env=dict(os.environ, MPLBACKEND="Agg"), capture_output=True)
        for k in ("Scores.csv", "Profile.csv", "DMCurve.csv", "Cands.meta"):
            out["pfd_" + k] = open(os.path.join(d, k)).read().replace(d, "<DIR>")
        np.savez_compressed(os.path.join(GOLDEN, "label.npz"), **out)
        manifest["sets"]["label"] = {"mode": "DataProcessor.label", "phcx_seed": 20261015 + 1000,
                                     "phcx_n": 20, "pfd_seed": 20261915, "pfd_n": 12,
                                     "pfd_shape": [8, 16, 64]}


def make_getters_golden(manifest):
    """Candidate.getSubbandData / getSubintData (Candidate.py:290-340 ->
    PHCXOperations.py:422-505) on PHCX files that carry <SubIntegrations>; rows 0-1
    adversarial (constant / all-zero sub-integrations)."""
    from pulsarfeatureextractor_amd.synth import _rows_numpy

    n, seed = 12, 20262015
    rng = np.random.default_rng(seed)
    prof, sub, curve, blocks, period, dmv, snr, width = bates_set(rng, n, 128, 16, 128, 128, False)
    subints = _rows_numpy(rng, n * 32, 128, 20.0, 150.0).reshape(n, 32, 128)
    subints[0] = 77
    subints[1] = 0
    arrays = dict(n=n, prof=prof, sub=sub, block0=_rows_lyon(rng, n, 128), block1=blocks,
                  period=period, dm=dmv, snr=snr, width=width, dm_start=0.0, dm_end=200.0,
                  n_dm_index=101)
    from pulsarfeatureextractor_amd import phcx

    with tempfile.TemporaryDirectory(prefix="pfe_golden_getters_") as tmp:
        refdir = build_reference(tmp)
        d = os.path.join(tmp, "getters")
        os.makedirs(d)
        files = []
        for i in range(n):
            p = os.path.join(d, f"getters_{i:05d}.phcx.gz")
            phcx.write(p, profile=prof[i], subbands=sub[i], datablocks=(arrays["block0"][i], blocks[i]),
                       dm_start=0.0, dm_end=200.0, n_dm_index=101, period_s=float(period[i]),
                       snr=float(snr[i]), dm=float(dmv[i]), width=float(width[i]),
                       subints=subints[i])
            files.append(p)
        res = run_reference(refdir, files, "getters", tmp)
    assert all(r["ok"] for r in res), res
    np.savez_compressed(
        os.path.join(GOLDEN, "getters_phcx128.npz"), prof=prof.astype(np.uint8),
        sub=sub.astype(np.uint8), subints=subints.astype(np.uint8),
        block0=np.asarray(arrays["block0"]).astype(np.uint8), block1=blocks.astype(np.uint8),
        period=period, dm=dmv, snr=snr, width=width,
        subband=np.array([r["v"]["subband"] for r in res]),
        subint=np.array([r["v"]["subint"] for r in res]),
        subband_types=np.array([",".join(r["v"]["subband_types"]) for r in res]))
    manifest["sets"]["getters_phcx128"] = {"mode": "Candidate.getSubbandData/getSubintData",
                                           "seed": seed, "n": n, "subints": [32, 128]}


def _rows_lyon(rng, n, L):
    from pulsarfeatureextractor_amd.synth import _rows_numpy

    return _rows_numpy(rng, n, L, 150.0, 150.0)


if __name__ == "__main__":
    if "--pfd" in sys.argv:  # only the PFD sets (the PHCX sets are unchanged)
        mpath = os.path.join(GOLDEN, "manifest.json")
        man = json.load(open(mpath))
        make_pfd_golden(man)
        with open(mpath, "w") as f:
            json.dump(man, f, indent=1)
    elif "--getters" in sys.argv:  # the Candidate getters golden only
        mpath = os.path.join(GOLDEN, "manifest.json")
        man = json.load(open(mpath))
        make_getters_golden(man)
        with open(mpath, "w") as f:
            json.dump(man, f, indent=1)
    elif "--label" in sys.argv:  # the --label golden only
        mpath = os.path.join(GOLDEN, "manifest.json")
        man = json.load(open(mpath))
        make_label_golden(man)
        with open(mpath, "w") as f:
            json.dump(man, f, indent=1)
    elif "--only" in sys.argv:  # regenerate the named PHCX sets only, keep the others
        main(set(sys.argv[sys.argv.index("--only") + 1].split(",")))
    else:
        main()
