"""The PFD restatement (oracle/pfd.py) and the host .pfd reader against the reference's own
outputs on synthetic PRESTO folds (tests/golden/pfd_*.npz, tools/make_golden.py --pfd).

The fixtures hold generator seeds (files are rebuilt here with synth.pfd_candidate and
checked against the stored sums) and the reference's results for the dmprof path
(calculateProfileStatScores + calculateDMCurveStatScores), the profile-bins path
(calculateProfileScores) and the 22-score path."""
import os
import warnings

import numpy as np
import pytest

from golden_util import GOLDEN
from oracle import pfd as opfd
from pulsarfeatureextractor_amd import pfd

SETS = ["pfd_64x16", "pfd_128x32"]


def load_set(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def build_files(tmp_path, g):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(GOLDEN), "..", "tools"))
    from make_golden import pfd_candidates

    files = []
    for i, (c, kw) in enumerate(pfd_candidates(int(g["n"]), int(g["npart"]), int(g["nsub"]),
                                               int(g["proflen"]), int(g["seed"]))):
        assert float(np.asarray(c["profs"]).sum()) == g["profs_sum"][i], "generator drift"
        p = os.path.join(tmp_path, f"c{i:04d}.pfd")
        pfd.write(p, **c, **kw)
        files.append(p)
    return files


def same(a, b):
    return np.array_equal(a, b) or np.array_equal(np.nan_to_num(a, nan=7.25), np.nan_to_num(b, nan=7.25))


@pytest.mark.parametrize("name", SETS)
def test_oracle_matches_reference(tmp_path, name):
    g = load_set(name)
    files = build_files(tmp_path, g)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for i, f in enumerate(files):
            d = pfd.read(f)
            prof = opfd.PFDState(d).profile()
            assert g["profile_ok"][i]
            assert same(prof, g["profile"][i]), f"profile row {i}"
            if g["lyon8_ok"][i]:
                assert same(np.array(opfd.lyon8_one(d)), g["lyon8"][i]), f"lyon8 row {i}"
            else:
                with pytest.raises(opfd.PFDError):
                    opfd.lyon8_one(d)


def test_reader_layout_variants(tmp_path):
    from pulsarfeatureextractor_amd.synth import pfd_candidate

    c = pfd_candidate(np.random.default_rng(3), 4, 8, 32)
    ref = None
    for kw in ({}, {"big_endian": True}, {"with_posn": False}):
        p = os.path.join(tmp_path, "v.pfd")
        pfd.write(p, **c, **kw)
        d = pfd.read(p)
        assert d.profs.shape == (4, 8, 32) and d.chanpersub == c["numchan"] // 8
        got = (d.profs, d.subfreqs, d.avgprof, d.varprof, d.binspersec)
        if ref is None:
            ref = got
        for a, b in zip(got, ref):
            assert np.array_equal(a, b)


# the reference's s10 / s11 on these folds move between runs of the reference itself (last-ulp
# numpy SIMD differences feed the 8-pass double-Gaussian peel); s17 / s18 are the PFD DM fit,
# which a 1-ulp nudge of its start point moves in most folds (tests/golden/chaos_floor.json)
NOISY = (9, 10, 16, 17)


@pytest.mark.parametrize("name", SETS)
def test_oracle_22_matches_reference(tmp_path, name):
    """PFDFile.compute restated (oracle/pfd.bates22_one) against the reference's 22 scores:
    same failing folds and failing group, every other column bit-exact, the noisy columns
    within 1e-3 on all but a tenth of the folds."""
    from oracle import bates as ob

    g = load_set(name)
    files = build_files(tmp_path, g)
    rows, oks = [], []
    for i, f in enumerate(files):
        d = pfd.read(f)
        try:
            rows.append(np.array(opfd.bates22_one(d)[0]))
            oks.append(True)
        except ob.CandidateFailure as e:
            rows.append(np.full(22, np.nan))
            oks.append(False)
            group = {"sine": "Sinusoid", "gauss": "Gaussian", "params": "Candidate parameters",
                     "dmfit": "DM curve", "subband": "Subband"}[e.group]
            assert group in str(g["bates22_err"][i]), (i, e, g["bates22_err"][i])
    got, ok = np.array(rows), np.array(oks)
    assert np.array_equal(ok, g["bates22_ok"])
    ref = g["bates22"][ok]
    got = got[ok]
    for j in range(22):
        same = (got[:, j] == ref[:, j]) | (np.isnan(got[:, j]) & np.isnan(ref[:, j]))
        if j not in NOISY:
            assert same.all(), f"s{j + 1} rows {np.where(~same)[0]}"
        else:
            with np.errstate(all="ignore"):
                rel = np.abs(got[:, j] - ref[:, j]) / np.abs(ref[:, j])
            # the reference disagrees with itself between runs on 4-18 % of rows (s10/s11), and
            # the oracle's own last-ulp numpy SIMD drift depends on heap state in the same way
            allowed = max(2, int(0.1 * len(rel)))
            assert (rel[~same] > 1e-3).sum() <= allowed, f"s{j + 1}: {np.sort(rel[~same])[-3:]}"
