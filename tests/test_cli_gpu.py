"""End to end on the GPU: synthetic PHCX/SUPERB files -> ScoreGenerator-compatible CLI ->
output text, compared with what the reference wrote for the same files (golden vectors).

Checks the discovery order, the file-type dispatch, the error log, the ARFF/CSV text and
the values (Lyon moments within 1e-11 relative or 1e-12 absolute -- the kurtosis is m4/m2^2 - 3; 22-score rows
for the bit-exact score columns)."""
import os

import numpy as np
import pytest

from golden_util import envelope_check, load
from pulsarfeatureextractor_amd import cli, phcx

pytestmark = pytest.mark.gpu


def write_set(d, dirname):
    superb = bool(d["superb"])
    os.makedirs(dirname, exist_ok=True)
    names = []
    for i in range(len(d["ok"])):
        p = os.path.join(dirname, f"cand_{i:05d}" + (".phcx" if superb else ".phcx.gz"))
        phcx.write(p, profile=d["prof"][i], subbands=d["sub"][i],
                   datablocks=(d["block0"][i], d["block1"][i]), dm_start=float(d["dm_start"]),
                   dm_end=float(d["dm_end"]), n_dm_index=int(d["n_dm_index"]),
                   period_s=float(d["period"][i]), snr=float(d["snr"][i]), dm=float(d["dm"][i]),
                   width=float(d["width"][i]), superb=superb)
        names.append(p)
    return names


def read_rows(path):
    rows = {}
    for ln in open(path).read().splitlines():
        if not ln or ln.startswith("@"):
            continue
        if "?%" in ln:
            vals, name = ln.split(",?%")
            rows[name] = [float(v) for v in vals.split(",")]
        else:
            parts = ln.split(",")
            rows[parts[0]] = [float(v) for v in parts[1:]]
    return rows


@pytest.mark.parametrize("name,flag", [("lyon8_phcx128", "--phcx"), ("lyon8_superb64", "--superb")])
def test_dmprof_cli(tmp_path, monkeypatch, name, flag):
    monkeypatch.chdir(tmp_path)
    d = load(name)
    names = write_set(d, str(tmp_path / "cands"))
    out = str(tmp_path / "out.arff")
    assert cli.main(["-c", str(tmp_path / "cands"), "-o", out, flag, "--dmprof", "--arff",
                     "--workers", "1"]) == 0
    rows = read_rows(out)
    assert len(rows) == len(names)
    ref = np.nan_to_num(d["out"], nan=0.0)  # the writer turns nan into 0
    base = str(tmp_path / "cands") + "/"
    for i, p in enumerate(names):
        got = np.array(rows[os.path.join(base, os.path.basename(p))])
        r = np.array([float(x) for x in ",".join("%.12g" % v for v in ref[i]).split(",")])
        assert np.allclose(got, r, rtol=1e-11, atol=1e-12), (i, got, r)


def test_bates_cli_and_error_log(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    d = load("bates22_phcx128")
    write_set(d, str(tmp_path / "cands"))
    out = str(tmp_path / "scores.csv")
    assert cli.main(["-c", str(tmp_path / "cands"), "-o", out, "--phcx", "--workers", "1"]) == 0
    rows = read_rows(out)
    assert len(rows) == int(d["ok"].sum())
    logged = [ln for ln in open("CandidateErrorLog.txt").read().splitlines() if ln]
    assert len(logged) == int((~d["ok"]).sum())
    base = str(tmp_path / "cands") + "/"
    n = len(d["ok"])
    text = np.full((n, 22), np.nan)
    st = np.ones(n, dtype=np.uint32)  # absent from the output = failed
    for i in np.where(d["ok"])[0]:
        got = rows[os.path.join(base, f"cand_{i:05d}.phcx.gz")]
        ref = np.nan_to_num(d["out"][i], nan=0.0, posinf=0.0)
        for j in (2, 3, 11, 12, 13, 14, 15, 19, 21):   # bit-exact score columns
            assert got[j] == float("%.12g" % ref[j]), (i, j, got[j], ref[j])
        text[i], st[i] = got, 0
    # the LM columns of the text against the reference's own per-row envelope (the writer
    # prints nan / inf as 0: there the reference's non-finite value is taken as written)
    gold = d["out"]
    text = np.where((text == 0.0) & ~np.isfinite(gold), gold, text)
    envelope_check(text, st, "bates22_phcx128", skip=(2, 3, 11, 12, 13, 14, 15, 19, 21))


def test_pfd_dmprof_and_profile_cli(tmp_path, monkeypatch):
    """--pfd --dmprof and --pfd --profile against the reference's PFD outputs."""
    from test_oracle_pfd import build_files, load_set

    monkeypatch.chdir(tmp_path)
    g = load_set("pfd_64x16")
    cand = tmp_path / "pfds"
    cand.mkdir()
    files = build_files(str(cand), g)
    out = str(tmp_path / "dmprof.csv")
    assert cli.main(["-c", str(cand), "-o", out, "--pfd", "--dmprof"]) == 0
    rows = read_rows(out)
    assert len(rows) == int(g["lyon8_ok"].sum())
    logged = [ln for ln in open("CandidateErrorLog.txt").read().splitlines() if ln]
    assert len(logged) == int((~g["lyon8_ok"]).sum())
    base = str(cand) + "/"
    for i, f in enumerate(files):
        key = os.path.join(base, os.path.basename(f))
        if not g["lyon8_ok"][i]:
            assert key not in rows
            continue
        ref = np.nan_to_num(g["lyon8"][i], nan=0.0)
        r = np.array([float("%.12g" % v) for v in ref])
        # the float32 DM-curve skew goes through powf: within 1e-6 (test_pfd_gpu.py)
        rtol = np.array([1e-11] * 6 + [1e-6, 1e-11])
        assert (np.abs(np.array(rows[key]) - r) <= rtol * np.abs(r) + 1e-12).all(), (i, rows[key], r)
    out2 = str(tmp_path / "prof.csv")
    assert cli.main(["-c", str(cand), "-o", out2, "--pfd", "--profile"]) == 0
    rows = read_rows(out2)
    for i, f in enumerate(files):
        ref = np.nan_to_num(g["profile"][i], nan=0.0)
        got = rows[os.path.join(base, os.path.basename(f))]
        assert got == [float("%.12g" % v) for v in ref], i
    # the 22-score mode (processPFDCollectively): same failing files, the bit-exact columns
    out3 = str(tmp_path / "s.csv")
    assert cli.main(["-c", str(cand), "-o", out3, "--pfd"]) == 0
    rows = read_rows(out3)
    assert len(rows) == int(g["bates22_ok"].sum())
    for i, f in enumerate(files):
        key = os.path.join(base, os.path.basename(f))
        if not g["bates22_ok"][i]:
            assert key not in rows
            continue
        for j in (2, 3, 11, 12, 13, 14, 15, 18, 19):  # tests/test_pfd22_gpu.py EXACT
            assert rows[key][j] == float("%.12g" % g["bates22"][i][j]), (i, j)
    # separately: one <file>.dat per scored fold (outputScores, DataProcessor.py:429-447)
    assert cli.main(["-c", str(cand), "-o", str(tmp_path / "absent" / "x.csv"), "--pfd"]) == 0
    dats = sorted(p for p in os.listdir(cand) if p.endswith(".dat"))
    assert len(dats) == int(g["bates22_ok"].sum())


def test_pipeline_slots_follow_the_callers_engine_options(tmp_path, monkeypatch):
    """gpu_depth = 2 scores odd batches on a second libpfe handle: every option set on the
    engine the caller passed (solver, pool size, ...) must reach that handle too, so one output
    file never mixes two configurations (round-4 advisor finding)."""
    from pulsarfeatureextractor_amd import processor
    from pulsarfeatureextractor_amd._native import OPTIONS, Engine

    monkeypatch.chdir(tmp_path)
    d = load("bates22_phcx128")
    write_set(d, str(tmp_path / "cands"))
    outs = {}
    with Engine(0) as e:
        e.set_option("solver", "batched")
        e.set_option("gslots", 7)
        for depth in (1, 2):
            p = processor.DataProcessor(engine=e, batch=64, gpu_depth=depth, ramp=False,
                                        log=lambda *a: None)
            out = str(tmp_path / f"d{depth}.csv")
            p.processPHCXCollectively(str(tmp_path / "cands"), False, out, False, False, False)
            outs[depth] = open(out).read()
            if depth == 2:
                slot = p._eng(1)
                assert slot is not e
                for name in OPTIONS:
                    assert slot.get_option(name) == e.get_option(name), name
        # both slots computed with the batched solver: the same text as one slot
        assert outs[1] == outs[2]


@pytest.mark.parametrize("extra", [[], ["--dmprof", "--arff"]])
def test_cli_two_gpu_shards_match_one(tmp_path, monkeypatch, extra):
    """--gpus 2 with both shard workers on cuda:0 (--devices 0,0; the box has one GPU): two
    spawned processes, each with its own engine, reader threads and pinned slabs, over the two
    contiguous halves of the discovery.  Output text, error log and <out>.progress are
    byte-identical to the one-process run (ARFF: but for the header's timestamp)."""
    d = load("bates22_phcx128")
    cands = str(tmp_path / "cands")
    write_set(d, cands)
    with open(os.path.join(cands, "zz_broken.phcx.gz"), "wb") as f:
        f.write(b"not gzip")
    got = {}
    for g in ("1", "2"):
        wd = tmp_path / f"w{g}"
        wd.mkdir()
        monkeypatch.chdir(wd)
        out = str(wd / "out.txt")
        open(out, "w").close()
        args = ["-c", cands, "-o", out, "--phcx", "--workers", "2", "--gpus", g, *extra]
        if g == "2":
            args += ["--devices", "0,0"]
        assert cli.main(args) == 0
        got[g] = [open(p, "rb").read() for p in (out, "CandidateErrorLog.txt", out + ".progress")]
        assert not [p for p in os.listdir(wd) if ".shard" in p]
    a, b = got["1"], got["2"]
    if extra:
        a[0], b[0] = a[0].split(b"\n", 1)[1], b[0].split(b"\n", 1)[1]
    assert a == b
    assert a[1].count(b"\n") >= 1 and int(a[2]) == len(d["ok"]) + 1
