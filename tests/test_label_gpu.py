"""--label on the GPU (DataProcessor.label, DataProcessor.py:691-826): the four files the
reference wrote for the same PHCX and PFD candidates (tests/golden/label.npz, made by
tools/make_golden.py --label running the reference's own DataProcessor.label).

Compared per candidate (os.walk order is the filesystem's): the same candidates in
Cands.meta with label "0" and in every CSV with ",0,%<candidate>"; the same failures in
CandidateErrorLog.txt; profile bins and PHCX DM-curve data exactly (the reference writes
them with Python 3's shortest repr here and this build with Python 2's str(), so values are
compared after parsing: float64 to 1e-11, the float32 PFD curve to the 6 significant digits Python 2 prints).  The
PHCX scores are the engine's own scores of the same candidates written as Python 2 writes
them, and the columns that are bit-exact against the reference equal the reference's; the
PFD scores are held to the PFD 22-score bar (tests/test_pfd22_gpu.py)."""
import json
import os
import sys

import numpy as np
import pytest

from golden_util import GOLDEN, envelope_check, load
from pulsarfeatureextractor_amd import cli, pfd, phcx
from pulsarfeatureextractor_amd._native import Engine
from test_pfd22_gpu import check as pfd_check

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse_csv(text, base):
    rows = {}
    for ln in text.splitlines():
        if not ln:
            continue
        vals, name = ln.rsplit(",%", 1)
        parts = vals.split(",")
        assert parts[-1] == "0", ln[:80]
        rows[name.replace(base, "<DIR>")] = [float(v) for v in parts[:-1]]
    return rows


def run_label(tmp_path, monkeypatch, d, flag):
    monkeypatch.chdir(tmp_path)
    assert cli.main(["-c", d, "-o", str(tmp_path / "unused.csv"), flag, "--label",
                     "--workers", "1"]) == 0
    base = d.rstrip("/")
    got = {k: open(os.path.join(d, k)).read() for k in ("Scores.csv", "Profile.csv", "DMCurve.csv",
                                                      "Cands.meta")}
    errlog = open(tmp_path / "CandidateErrorLog.txt").read()
    return base, got, errlog


def test_label_phcx(tmp_path, monkeypatch):
    g = np.load(os.path.join(GOLDEN, "label.npz"))
    d = str(tmp_path / "label_phcx")
    os.makedirs(d)
    n = int(g["phcx_in_n"])
    for i in range(n):
        phcx.write(os.path.join(d, f"label_{i:05d}.phcx.gz"), profile=g["phcx_in_prof"][i],
                   subbands=g["phcx_in_sub"][i],
                   datablocks=(g["phcx_in_block0"][i], g["phcx_in_block1"][i]),
                   dm_start=float(g["phcx_in_dm_start"]), dm_end=float(g["phcx_in_dm_end"]),
                   n_dm_index=int(g["phcx_in_n_dm_index"]), period_s=float(g["phcx_in_period"][i]),
                   snr=float(g["phcx_in_snr"][i]), dm=float(g["phcx_in_dm"][i]),
                   width=float(g["phcx_in_width"][i]), superb=False)
    base, got, errlog = run_label(tmp_path, monkeypatch, d + "/", "--phcx")
    ref_meta = sorted(str(g["phcx_Cands.meta"]).splitlines())
    got_meta = sorted(got["Cands.meta"].replace(base, "<DIR>").splitlines())
    assert [m.replace("//", "/") for m in got_meta] == [m.replace("//", "/") for m in ref_meta]
    names = [m.rsplit(",", 1)[0].replace("//", "/") for m in ref_meta]
    failed = sorted(set(f"<DIR>/label_{i:05d}.phcx.gz" for i in range(n)) - set(names))
    assert sorted(ln.replace(base, "<DIR>").replace("//", "/") for ln in errlog.split()) == failed

    def norm(rows):
        return {k.replace("//", "/"): v for k, v in rows.items()}

    for f in ("Profile.csv", "DMCurve.csv"):
        r, o = norm(parse_csv(str(g["phcx_" + f]), "<DIR>")), norm(parse_csv(got[f], base))
        assert r.keys() == o.keys()
        for k in r:
            assert r[k] == o[k], (f, k)
    r, o = norm(parse_csv(str(g["phcx_Scores.csv"]), "<DIR>")), norm(parse_csv(got["Scores.csv"], base))
    assert r.keys() == o.keys()
    # the label writer's numbers are the engine's scores of the same candidates, written with
    # Python 2's str() (12 significant digits) ...
    from golden_util import bates_inputs
    from pulsarfeatureextractor_amd.writers import py2_str

    arr = {k[len("phcx_in_"):]: g[k] for k in g.files if k.startswith("phcx_in_")}
    arr["superb"] = np.bool_(False)
    arr["ok"] = np.ones(n, dtype=bool)
    with Engine(0) as e:
        sc, st = e.bates22(*bates_inputs(arr))
    for i in range(n):
        k = f"<DIR>/label_{i:05d}.phcx.gz"
        if k in o:
            assert [py2_str(v) for v in sc[i]] == [py2_str(v) for v in o[k]], k
    # ... the columns that are bit-exact against the reference agree with its file
    for k in r:
        for j in (2, 3, 11, 12, 13, 14, 15, 19, 21):
            assert float("%.12g" % r[k][j]) == o[k][j], (k, j)
    # ... and the LM columns of the file lie in the reference's own per-row envelope of the
    # same candidates (tools/chaos_envelope.py set "label_phcx")
    text = np.full((n, 22), np.nan)
    tst = np.ones(n, dtype=np.uint32)
    for i in range(n):
        k = f"<DIR>/label_{i:05d}.phcx.gz"
        if k in o:
            text[i], tst[i] = o[k], 0
    envelope_check(text, tst, "label_phcx", skip=(2, 3, 11, 12, 13, 14, 15, 19, 21))


def test_label_pfd(tmp_path, monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from make_golden import pfd_candidates

    g = np.load(os.path.join(GOLDEN, "label.npz"))
    d = str(tmp_path / "label_pfd")
    os.makedirs(d)
    for i, (c, kw) in enumerate(pfd_candidates(12, 8, 16, 64, 20261915)):
        pfd.write(os.path.join(d, f"label_{i:04d}.pfd"), **c, **kw)
    base, got, errlog = run_label(tmp_path, monkeypatch, d + "/", "--pfd")
    norm = lambda rows: {k.replace("//", "/"): v for k, v in rows.items()}  # noqa: E731
    ref_meta = sorted(m.replace("//", "/") for m in str(g["pfd_Cands.meta"]).splitlines())
    got_meta = sorted(m.replace("//", "/") for m in got["Cands.meta"].replace(base, "<DIR>").splitlines())
    assert got_meta == ref_meta
    r, o = norm(parse_csv(str(g["pfd_Profile.csv"]), "<DIR>")), norm(parse_csv(got["Profile.csv"], base))
    assert r.keys() == o.keys()
    for k in r:
        a, b = np.array(r[k]), np.array(o[k])
        assert np.allclose(a, b, rtol=1e-11, atol=1e-11), k
    r, o = norm(parse_csv(str(g["pfd_DMCurve.csv"]), "<DIR>")), norm(parse_csv(got["DMCurve.csv"], base))
    for k in r:
        a, b = np.array(r[k], dtype=np.float32), np.array(o[k], dtype=np.float32)
        # Python 2's str() of a float32 keeps 6 significant digits (writers.py2_scalar_str)
        assert np.allclose(a, b, rtol=6e-6, atol=0), k
    r, o = norm(parse_csv(str(g["pfd_Scores.csv"]), "<DIR>")), norm(parse_csv(got["Scores.csv"], base))
    keys = sorted(r)
    ref = np.array([r[k] for k in keys])
    out = np.array([o[k] for k in keys])
    same12 = np.array([[float("%.12g" % a) == b for a, b in zip(rr, oo)] for rr, oo in zip(ref, out)])
    ref[same12] = out[same12]
    floor = json.load(open(os.path.join(GOLDEN, "chaos_floor.json")))["pfd_64x16"]
    pfd_check(out, np.zeros(len(keys), dtype=np.uint32), ref, np.ones(len(keys), dtype=bool),
              "label pfd", floor)
