"""Host plumbing of the streamed product path (processor.DataProcessor) on the CPU.

The GPU is replaced by a stub engine with a deterministic score function and the pinned slabs
by plain numpy buffers, so what is checked here is everything around the kernels: native
parse -> bulk infos -> shape groups -> pfe_phcx_pack -> engine -> pfe_format_rows text, in
discovery order over several streamed batches; files the native reader flags going through
the Python parser; failing candidates in CandidateErrorLog.txt; a group the library refuses
failing its rows only; the resume offset.  The expected text is built independently from the
Python parser (phcx.parse) and the Python writers (writers.score_line / arff_line)."""
import gzip
import os

import numpy as np
import pytest

from pulsarfeatureextractor_amd import _native, phcx, processor, writers
from test_phcx_native import _doc, _write_golden


class PlainSlabs:
    def view(self, key, shape, dtype):
        return np.empty(shape, dtype=dtype)


def stub22(prof, sub, dmc, scal):
    """A deterministic stand-in for the 22 scores of a batch of one shape."""
    n = prof.shape[0]
    out = np.empty((n, 22))
    out[:, 0] = prof.astype(np.float64).sum(1) / 7.0
    out[:, 1] = sub.reshape(n, -1).astype(np.float64).mean(1)
    out[:, 2] = dmc.max(1)
    out[:, 3:11] = scal
    out[:, 11:] = np.arange(11) * 0.1 + prof[:, :1]
    out[prof[:, 1] == 7, 4] = np.nan          # writer turns these into "0"
    st = np.where(prof[:, 0] % 13 == 0, _native.PFE_ST_GAUSS_FAIL, 0).astype(np.uint32)
    return out, st


def stub8(prof, dm):
    p, d = prof.astype(np.float64), dm.astype(np.float64)
    return np.stack([p.mean(1), p.std(1), p.max(1), p.min(1),
                     d.mean(1), d.std(1), d.max(1), d[:, -1]], 1)


class StubEngine:
    def __init__(self):
        self.calls = []

    def bates22(self, prof, sub, dmc, scal, out=None, status=None):
        self.calls.append(("bates22", prof.shape, sub.shape))
        if sub.shape[1] > 256:
            raise _native.PfeError("bates22: sub-band shape")
        o, st = stub22(prof, sub, dmc, scal)
        out[:] = o
        status[:] = st
        return out, status

    def lyon8(self, prof, dm, out=None, status=None):
        self.calls.append(("lyon8", prof.shape, dm.shape))
        o = stub8(prof, dm)
        if out is None:
            return o
        out[:] = o
        return out


def expected(paths, kind):
    ok_lines, failed = [], []
    for p in paths:
        try:
            c = phcx.parse(p)
        except Exception:
            failed.append(p)
            continue
        if kind == "lyon8":
            ok_lines.append((p, stub8(c.profile[None].astype(np.uint8), c.lyon_dm[None].astype(np.uint8))[0]))
            continue
        if len(c.dm_curve) < 3 or c.subbands.shape[0] > 256:
            failed.append(p)
            continue
        o, st = stub22(c.profile[None].astype(np.uint8), c.subbands[None].astype(np.uint8),
                       c.dm_curve[None], c.scal[None])
        if st[0]:
            failed.append(p)
        else:
            ok_lines.append((p, o[0]))
    return ok_lines, failed


def make_dir(tmp_path):
    d = tmp_path / "cands"
    d.mkdir()
    paths = _write_golden(str(d), "bates22_phcx128", range(40))
    # flagged by the native reader -> Python parser (same outcome as the reference)
    for k, case in enumerate(({"profile_text": "\nA\nBC0\nD\n"}, {"profile_text": "\n0A0B0C0D0E0F1011\n"})):
        p = str(d / f"flag_{k}.phcx.gz")
        with gzip.open(p, "wb") as f:
            f.write(_doc(**case).encode())
    # unreadable
    with open(d / "broken.phcx.gz", "wb") as f:
        f.write(b"not a gzip file")
    # a sub-band shape the library refuses (stub raises for nsub > 256): its rows fail alone
    p = str(d / "wide_sub.phcx.gz")
    with gzip.open(p, "wb") as f:
        f.write(_doc(sub_text="\n" + "01" * 300 + "\n", nbins=1, nsub=300).encode())
    # SUPERB-style name in the same walk is not matched by the PHCX pattern
    return str(d)


@pytest.mark.parametrize("arff", [False, True])
def test_stream_scores_text_and_error_log(tmp_path, monkeypatch, arff):
    monkeypatch.chdir(tmp_path)
    d = make_dir(tmp_path)
    eng = StubEngine()
    dp = processor.DataProcessor(engine=eng, workers=3, log=lambda *a: None, batch=16)
    dp._slabs = PlainSlabs()
    out = str(tmp_path / ("o.arff" if arff else "o.csv"))
    dp.processPHCXCollectively(d + "/", False, out, arff, False, False)
    paths = processor.discover(d + "/", [processor.PHCX_RE])
    ok_lines, failed = expected(paths, "bates22")
    fmt = writers.arff_line if arff else writers.score_line
    text = open(out).read()
    if arff:
        text = text[text.index("@data\n") + 6:]
    assert text == "".join(fmt(p, v) + "\n" for p, v in ok_lines)
    assert open("CandidateErrorLog.txt").read() == "".join(p + "\n" for p in failed)
    assert any(p.endswith("wide_sub.phcx.gz") for p in failed)
    assert len(ok_lines) > 20 and len(failed) >= 3
    # batches of 16 files: several streamed batches, shape groups packed per batch
    assert sum(1 for c in eng.calls if c[0] == "bates22") >= 3


def test_resume_offset(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    d = make_dir(tmp_path)
    full = str(tmp_path / "full.csv")
    part = str(tmp_path / "part.csv")
    for path, start in ((full, 0), (part, 17)):
        dp = processor.DataProcessor(engine=StubEngine(), workers=2, log=lambda *a: None,
                                     batch=8, start=start)
        dp._slabs = PlainSlabs()
        dp.processPHCXCollectively(d + "/", False, path, False, False, False)
    paths = processor.discover(d + "/", [processor.PHCX_RE])
    done = set(paths[:17])
    want = [ln for ln in open(full).read().splitlines() if ln.split(",")[0] not in done]
    assert open(part).read().splitlines() == want


def test_resume_offset_arff_single_header(tmp_path, monkeypatch):
    """Resuming an --arff run appends rows to the stopped run's file without a second
    '@relation ... @data' header; the .progress marker holds the --start value to resume."""
    monkeypatch.chdir(tmp_path)
    d = make_dir(tmp_path)
    full = str(tmp_path / "full.arff")
    part = str(tmp_path / "part.arff")
    paths = processor.discover(d + "/", [processor.PHCX_RE])

    def run(path, start):
        dp = processor.DataProcessor(engine=StubEngine(), workers=2, log=lambda *a: None,
                                     batch=8, start=start)
        dp._slabs = PlainSlabs()
        dp.processPHCXCollectively(d + "/", False, path, True, False, False)

    run(full, 0)
    assert int(open(full + ".progress").read()) == len(paths)
    # a "stopped" run: the header and the lines of the first 16 candidates
    text = open(full).read()
    head, body = text.split("@data\n")
    done = set(paths[:16])
    first = [ln for ln in body.splitlines() if ln.split(",?%")[-1] in done]
    with open(part, "w") as f:
        f.write(head + "@data\n" + "".join(ln + "\n" for ln in first))
    run(part, 16)
    got = open(part).read()
    assert got.count("@relation") == 1 and got.count("@data") == 1
    assert got == text
    assert int(open(part + ".progress").read()) == len(paths)


def test_run_metrics_json(tmp_path, monkeypatch):
    """--metrics: one JSON object per run with the reference's counts (DataProcessor.py:596-599)
    and failures by reason (PFE_ST_* names for the score groups)."""
    import json

    monkeypatch.chdir(tmp_path)
    d = make_dir(tmp_path)
    out = str(tmp_path / "s.csv")
    mpath = str(tmp_path / "m.json")
    dp = processor.DataProcessor(engine=StubEngine(), workers=2, log=lambda *a: None, batch=8,
                                 metrics_path=mpath)
    dp._slabs = PlainSlabs()
    dp.processPHCXCollectively(d + "/", False, out, False, False, False)
    m = json.load(open(mpath))
    assert m == dp.metrics
    paths = processor.discover(d + "/", [processor.PHCX_RE])
    ok_lines, failed = expected(paths, "scores")
    assert m["mode"] == "scores" and m["candidates"] == len(paths)
    assert m["successes"] == len(ok_lines) and m["failures"] == len(failed)
    assert sum(m["failures_by_reason"].values()) == len(failed)
    assert m["failures_by_reason"].get("PFE_ST_GAUSS_FAIL", 0) >= 1
    assert m["batches"] == -(-len(paths) // 8)
    for k in ("wall_s", "candidates_per_s", "parse_s", "score_s"):
        assert m[k] is not None and m[k] >= 0


def test_stream_dmprof_lyon8(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    d = make_dir(tmp_path)
    dp = processor.DataProcessor(engine=StubEngine(), workers=2, log=lambda *a: None, batch=32)
    dp._slabs = PlainSlabs()
    out = str(tmp_path / "l.csv")
    dp.dmprofPHCX(d + "/", False, out, False, False)
    paths = processor.discover(d + "/", [processor.PHCX_RE])
    ok_lines, failed = expected(paths, "lyon8")
    assert open(out).read() == "".join(writers.score_line(p, v) + "\n" for p, v in ok_lines)


def test_default_workers_respects_omp(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert processor.default_workers() <= 3
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert processor.default_workers() >= 1


def test_stream_cuts_ramp():
    """Long streamed runs ramp the batch size at both ends; every file is in exactly one
    batch, in order; short runs keep plain batches."""
    from pulsarfeatureextractor_amd.processor import _cuts

    c = _cuts(50000, 8192)
    sizes = np.diff(c)
    assert c[0] == 0 and c[-1] == 50000 and (sizes > 0).all()
    assert sizes[:3].tolist() == [1024, 2048, 4096] and sizes[-3:].tolist() == [4096, 2048, 1024]
    assert sizes.max() == 8192
    assert _cuts(100, 8192) == [0, 100]
    assert _cuts(20, 8) == [0, 8, 16, 20]


def test_verbose_runs_the_reference_validity_checks(tmp_path, monkeypatch):
    """-v (debug): PHCXFile.load runs isValid (PHCXFile.py:190-287) on each file.  The golden
    files are valid; a file with 64-bin sub-bands is not, and an invalid file leaves an empty
    profile, so the 22-score modes fail it in the sine group while the Lyon mode writes NaN
    profile moments (-> "0") and its unchanged DM-curve moments.  Without -v nothing changes."""
    monkeypatch.chdir(tmp_path)
    d = tmp_path / "cands"
    d.mkdir()
    good = _write_golden(str(d), "bates22_phcx128", range(6))
    assert all(phcx.is_valid(p) for p in good)
    c = phcx.parse(good[0])
    bad = str(d / "zz_bad.phcx.gz")
    phcx.write(bad, profile=c.profile, subbands=np.zeros((16, 64), np.uint8),
               datablocks=(np.zeros(128 * 120, np.uint8), np.zeros(128 * 120, np.uint8)),
               dm_start=0.0, dm_end=100.0, n_dm_index=120, period_s=0.5, snr=10.0, dm=12.0,
               width=0.05)
    assert not phcx.is_valid(bad)
    # section 0's SubBands empty: scored normally (section 1 is read), but isValid's
    # childNodes[0] of that element raises
    with gzip.open(good[0], "rb") as f:
        text = f.read().decode()
    i = text.index("<SubBands")
    i = text.index(">", i) + 1
    broken = str(d / "zz_raise.phcx.gz")
    with gzip.open(broken, "wb") as f:
        f.write((text[:i] + text[text.index("</SubBands>", i):]).encode())
    with pytest.raises(IndexError):
        phcx.is_valid(broken)
    assert len(phcx.parse(broken).profile) == 128
    logs = []
    for verbose in (False, True):
        dp = processor.DataProcessor(engine=StubEngine(), workers=2, log=logs.append, batch=4)
        dp._slabs = PlainSlabs()
        out = str(tmp_path / f"s{int(verbose)}.csv")
        dp.processPHCXCollectively(str(d) + "/", verbose, out, False, False, False)
        names = [ln.split(",")[0] for ln in open(out).read().splitlines()]
        assert (bad in names) != verbose and (broken in names) != verbose
        ok_good = [p for p, _v in expected(good, "bates22")[0]]
        assert [g for g in good if g in names] == ok_good
        dp = processor.DataProcessor(engine=StubEngine(), workers=2, log=logs.append, batch=4)
        dp._slabs = PlainSlabs()
        out8 = str(tmp_path / f"l{int(verbose)}.csv")
        dp.dmprofPHCX(str(d) + "/", verbose, out8, False, False)
        rows = {ln.split(",")[0]: ln.split(",")[1:] for ln in open(out8).read().splitlines()}
        assert (broken in rows) != verbose
        if verbose:
            assert rows[bad][:4] == ["0"] * 4 and rows[bad][4:] != ["0"] * 4
        else:
            assert rows[bad][:4] != ["0"] * 4
        # profile mode: load()'s 22 NaN scores plus the empty profile (PHCXFile.py:115-118,
        # :301-304), i.e. 22 NaNs written as "0" (DataProcessor.py:423) for the invalid file,
        # its 128 profile bins without -v
        dp = processor.DataProcessor(engine=StubEngine(), workers=2, log=logs.append, batch=4)
        dp._slabs = PlainSlabs()
        outp = str(tmp_path / f"p{int(verbose)}.csv")
        dp.processPHCXCollectively(str(d) + "/", verbose, outp, False, True, False)
        rows = {ln.split(",")[0]: ln.split(",")[1:] for ln in open(outp).read().splitlines()}
        if verbose:
            assert rows[bad] == ["0"] * 22, rows[bad]
        else:
            assert len(rows[bad]) == 128
        assert all(len(rows[g]) == 128 for g in good)
    assert any("Invalid PHCX candidate" in str(m) for m in logs)


def test_discover_matches_os_walk_fnmatch(tmp_path):
    """processor.discover builds os.path.join(root, fn) by concatenation: the same strings in
    the reference's os.walk / fnmatch order, with and without a trailing slash, nested."""
    import fnmatch

    (tmp_path / "a" / "b").mkdir(parents=True)
    for p in ("x.phcx.gz", "a/y.phcx.gz", "a/b/z.phcx.gz", "a/b/w.pfd", "v.pfd", "q.txt"):
        (tmp_path / p).write_text("")

    def ref(directory, regexes):
        out = []
        for ft in regexes:
            for root, _s, fns in os.walk(directory):
                out.extend(os.path.join(root, fn) for fn in fnmatch.filter(fns, ft))
        return out

    for d in (str(tmp_path), str(tmp_path) + "/", str(tmp_path / "a")):
        for pats in ([processor.PHCX_RE], [processor.PHCX_RE] + list(processor.PFD_RES)):
            assert processor.discover(d, pats) == ref(d, pats)


def test_stream_over_a_path_feed_still_being_walked():
    """A directory's paths come from a PathFeed whose walk runs beside the first batches:
    every path is emitted once, in order, with the same offsets as over the finished list;
    the batches open with batch/8, /4, /2 while the walk is still listing and close with
    /2, /4, /8 once it has ended; `skip` drops the first paths; a walk error reaches the
    reader."""
    import time as _time

    from pulsarfeatureextractor_amd.processor import PathFeed, _stream

    names = [f"d{i // 97}/f{i}.phcx.gz" for i in range(3000)]

    def slow_walk():
        for i in range(0, len(names), 97):
            _time.sleep(0.001)
            yield names[i:i + 97]

    def parse(part):  # slower than the walk, as parsing a file is than listing it
        _time.sleep(0.01)
        return list(part)

    for skip in (0, 250):
        got, sizes = [], []

        def emit(off, part, res, got=got, sizes=sizes):
            assert res == ("scored", len(part)) and off == len(got)
            got.extend(part)
            sizes.append(len(part))

        feed = PathFeed(slow_walk(), skip=skip)
        _stream(feed, parse, lambda parsed, slot: ("scored", len(parsed)), emit, batch=128, depth=2)
        assert got == names[skip:] and len(feed) == len(names) - skip
        assert sizes[:3] == [16, 32, 64] and sizes[-3:] == [64, 32, 16] and max(sizes) == 128

    done = []
    feed = PathFeed(iter([names[:10], names[10:20]]), skip=15, on_done=lambda t, s: done.append((t, s)))
    assert feed[:] == names[15:20] and done == [(20, 15)]

    def broken():
        yield names[:5]
        raise OSError("walk failed")

    with pytest.raises(OSError):
        len(PathFeed(broken()))
    assert len(PathFeed(iter([]))) == 0
    _stream(PathFeed(iter([])), None, None, None)  # nothing listed: no batch, no call


def test_discover_streams_large_directories_in_os_walk_order(tmp_path):
    """The streamed walk (listing chunks of 2048 entries) gives exactly os.walk + fnmatch's
    paths and order: a 5000-entry directory with non-matching names mixed in, nested
    subdirectories, a symlinked directory (listed by os.walk, not entered) and a symlinked
    file (matched as a file)."""
    import fnmatch

    big = tmp_path / "big"
    (big / "sub" / "deeper").mkdir(parents=True)
    for i in range(5000):
        (big / (f"c{i}.phcx.gz" if i % 3 else f"c{i}.txt")).write_text("")
    for p in ("sub/a.phcx.gz", "sub/deeper/b.phcx.gz", "sub/c.pfd"):
        (big / p).write_text("")
    os.symlink(big / "sub", big / "linked_dir")
    os.symlink(big / "c1.phcx.gz", big / "zz_link.phcx.gz")

    def ref(directory, regexes):
        out = []
        for ft in regexes:
            for root, _s, fns in os.walk(directory):
                out.extend(os.path.join(root, fn) for fn in fnmatch.filter(fns, ft))
        return out

    for d in (str(big), str(big) + "/"):
        for pats in ([processor.PHCX_RE], [processor.PHCX_RE] + list(processor.PFD_RES)):
            got = processor.discover(d, pats)
            assert got == ref(d, pats) and len(got) > 3000
    chunks = list(processor.iter_discover(str(big), [processor.PHCX_RE]))
    assert len(chunks) >= 3  # streamed while the big directory is listed


@pytest.mark.parametrize("mode", ["scores", "arff", "lyon8", "separately", "label"])
def test_sharded_run_matches_one_process(tmp_path, monkeypatch, mode):
    """--gpus N (DataProcessor(gpus=N)): the discovered paths in N contiguous shards, one
    spawned worker process each, outputs appended in rank order.  The output text, the error
    log, the .progress marker (and the label files / .dat files) are byte-identical to a
    one-process run, with a resume offset too.  Workers build the stub engine and plain slabs
    (shard_engine / shard_slabs) instead of libpfe's."""
    import shutil

    d0 = make_dir(tmp_path)
    results = {}
    wd = tmp_path / "run"
    for g in (1, 3):   # the same paths for both runs: a fresh copy of the tree in one place
        shutil.rmtree(wd, ignore_errors=True)
        shutil.copytree(d0, wd / "cands")
        monkeypatch.chdir(wd)
        d = str(wd / "cands")
        kw = dict(workers=2, log=lambda *a: None, batch=8, start=5)
        if g > 1:
            kw.update(gpus=g, shard_engine="test_processor_host:StubEngine",
                      shard_slabs="test_processor_host:PlainSlabs")
        dp = processor.DataProcessor(engine=StubEngine(), **kw)
        dp._slabs = PlainSlabs()
        out = str(wd / ("o.arff" if mode == "arff" else "o.csv"))
        if mode in ("scores", "arff"):
            dp.processPHCXCollectively(d + "/", False, out, mode == "arff", False, False)
        elif mode == "lyon8":
            dp.dmprofPHCX(d + "/", False, out, False, False)
        elif mode == "separately":
            dp.processPHCXSeparately(d + "/", False, False)
        else:
            dp.labelPHCX(d, False)
        files = {}
        for root, _dirs, names in os.walk(wd):
            for nm in names:
                p = os.path.join(root, nm)
                files[os.path.relpath(p, wd)] = open(p, "rb").read()
        assert not any(".shard" in k for k in files), sorted(files)
        results[g] = (files, dp.metrics)
    f1, m1 = results[1]
    f3, m3 = results[3]
    assert sorted(f1) == sorted(f3)
    for k in f1:
        a, b = f1[k], f3[k]
        if k.endswith(".arff"):  # "@relation PulsarCandidates_<now>": the run's timestamp
            assert a.split(b"\n", 1)[0][:27] == b.split(b"\n", 1)[0][:27]
            a, b = a.split(b"\n", 1)[1], b.split(b"\n", 1)[1]
        assert a == b, k
    assert len(f1["CandidateErrorLog.txt"]) > 0
    for key in ("candidates", "successes", "failures", "failures_by_reason"):
        assert m1[key] == m3[key], key
    assert [s["rank"] for s in m3["shards"]] == [0, 1, 2]
    assert sum(s["candidates"] for s in m3["shards"]) == m1["candidates"]


def test_cli_gpus_flag_parses_devices(tmp_path, monkeypatch):
    """The CLI's --gpus / --devices reach the DataProcessor, and with --gpus > 1 the parent
    does not open an engine (the workers do)."""
    from pulsarfeatureextractor_amd import candidate, cli

    seen = {}

    class Probe(processor.DataProcessor):
        def __init__(self, *a, **k):
            seen.update(k)
            super().__init__(*a, **k)

        def processPHCXCollectively(self, *a):
            seen["called"] = True

    monkeypatch.setattr(processor, "DataProcessor", Probe)
    monkeypatch.setattr(candidate, "get_engine", lambda *a: (_ for _ in ()).throw(AssertionError("engine opened")))
    monkeypatch.chdir(tmp_path)
    (tmp_path / "c").mkdir()
    out = str(tmp_path / "o.csv")
    open(out, "w").close()
    assert cli.main(["-c", str(tmp_path / "c"), "-o", out, "--phcx", "--gpus", "2",
                     "--devices", "0,0"]) == 0
    assert seen["gpus"] == 2 and seen["devices"] == [0, 0] and seen["called"]


class BrokenEngine(StubEngine):
    def bates22(self, *a, **k):
        raise RuntimeError("device lost")


def test_sharded_run_reports_a_failing_worker(tmp_path, monkeypatch):
    """A shard worker that raises fails the whole --gpus run with the worker's traceback and
    merges nothing (the shard files stay for inspection; the progress marker is not moved)."""
    monkeypatch.chdir(tmp_path)
    d = make_dir(tmp_path)
    out = str(tmp_path / "o.csv")
    dp = processor.DataProcessor(engine=StubEngine(), workers=2, log=lambda *a: None, batch=8,
                                 gpus=2, shard_engine="test_processor_host:BrokenEngine",
                                 shard_slabs="test_processor_host:PlainSlabs")
    with pytest.raises(RuntimeError, match="device lost"):
        dp.processPHCXCollectively(d + "/", False, out, False, False, False)
    assert not os.path.exists(out + ".progress")
