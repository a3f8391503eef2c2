"""The per-candidate plug-in API (candidate.Candidate / PHCXFile / SUPERBPHCXFile / PFDFile,
the drop-in for Candidate.py:116-286 and CandidateFileInterface.py) on the GPU, against the
reference's own outputs for the same files (tests/golden).

Same bar as the batched paths: Lyon features mean/std bit-exact, skew/kurt within 1e-12
(relative, or absolute below 1); the bit-exact 22-score columns bit-exact; a candidate the
reference fails raises Exception with the reference's text for that score group."""
import numpy as np
import pytest

from golden_util import load
from pulsarfeatureextractor_amd.candidate import Candidate
from test_phcx_native import _write_golden

pytestmark = pytest.mark.gpu

BITEXACT = (2, 3, 11, 12, 13, 14, 15, 19, 21)


def close_lyon(got, ref):
    got, ref = np.asarray(got, dtype=float), np.asarray(ref, dtype=float)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    m = ~np.isnan(ref)
    assert (np.abs(got - ref)[m] <= 1e-12 * np.maximum(1.0, np.abs(ref[m]))).all(), (got, ref)
    for c in (0, 1):
        assert got[c] == ref[c] or (np.isnan(got[c]) and np.isnan(ref[c]))


@pytest.mark.parametrize("name", ["lyon8_phcx128", "lyon8_superb64", "lyon8_phcx128_dmplane"])
def test_stat_scores(tmp_path, name):
    d = load(name)
    rows = range(0, len(d["ok"]), max(1, len(d["ok"]) // 10))
    paths = _write_golden(str(tmp_path), name, rows)
    for i, p in zip(rows, paths):
        c = Candidate(p.rsplit("/", 1)[-1], p)
        c.candidateName = p
        prof = c.calculateProfileStatScores(False)
        dm = c.calculateDMCurveStatScores(False)
        assert len(prof) == 4 and len(dm) == 4
        close_lyon(prof, d["out"][i][:4])
        close_lyon(dm, d["out"][i][4:])


def test_scores_and_failures(tmp_path):
    d = load("bates22_phcx128")
    ok = d["ok"].astype(bool)
    rows = list(np.where(ok)[0][:12]) + list(np.where(~ok)[0][:3])
    paths = _write_golden(str(tmp_path), "bates22_phcx128", rows)
    for i, p in zip(rows, paths):
        c = Candidate(p, p)
        if ok[i]:
            s = c.calculateScores(False)
            assert len(s) == 22
            for j in BITEXACT:
                assert s[j] == d["out"][i][j], (i, j, s[j], d["out"][i][j])
            assert c.getScore(3) == s[2]
        else:
            with pytest.raises(Exception) as e:
                c.calculateScores(False)
            assert "exception" in str(e.value)
    # profile bins (--profile) and the DM-curve data (label mode) of the same candidate
    c = Candidate(paths[0], paths[0])
    assert c.calculateProfileScores(False) == [float(v) for v in d["prof"][rows[0]]]
    assert list(c.getDMCurveData(False)) == [int(v) for v in d["block0"][rows[0]]]


def test_pfd_candidate(tmp_path):
    from test_oracle_pfd import build_files, load_set

    g = load_set("pfd_64x16")
    files = build_files(str(tmp_path), g)
    for i, f in enumerate(files[:8]):
        c = Candidate(f, f)
        if g["lyon8_ok"][i]:
            prof = c.calculateProfileStatScores(False)
            dm = c.calculateDMCurveStatScores(False)
            ref = g["lyon8"][i]
            # bit-exact, NaN where the reference's is (a flat fold: 0/0 in the 0..255 scaling)
            assert np.array_equal(np.array(prof[:2]), ref[:2], equal_nan=True), (i, prof, ref[:4])
            assert (abs(dm[0] - ref[4]) <= 1e-6 * abs(ref[4])
                    or (np.isnan(dm[0]) and np.isnan(ref[4]))), (i, dm[0], ref[4])
        if g["bates22_ok"][i]:
            s = c.calculateScores(False)
            for j in (2, 3, 11, 12, 13, 14, 15, 18, 19):
                assert s[j] == g["bates22"][i][j] or (np.isnan(s[j]) and np.isnan(g["bates22"][i][j])), (i, j)
