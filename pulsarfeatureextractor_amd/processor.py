"""Batched equivalent of the reference's DataProcessor (DataProcessor.py:51-995).

The reference walks a directory and scores one candidate at a time (parse -> score ->
buffer a text line), catching every exception per candidate
(DataProcessor.py:491-525, 867-901).  Here the same discovery order, file-type dispatch,
error log and output text are kept, but candidates are parsed on host worker processes,
packed into dense arrays and scored in large batches on the GPU through libpfe.

  processPHCXCollectively / processSUPERBCollectively  (:109-146, :451-599)
  processPHCXSeparately                                (:91-105, :603-687)
  dmprofPHCX / dmprofSUPERB                            (:255-301, :830-994)
  label                                                (:691-826)
PFD files (".pfd" in the name, Candidate.py:136) are read by pfd.read and go through
pfe_pfd_dmprof (dmprof, profile-bin and label modes) and pfe_pfd_bates22 (22 scores).

Streaming: the paths are taken in batches of BATCH files; batch k+1 is parsed on the host
(native reader threads; the ctypes call releases the GIL) while batch k is scored on the
GPU, and each batch's output lines are appended as soon as it is scored -- memory is bounded
by the batch, not the directory.  The reference buffers every line and appends once at the
end (DataProcessor.py:590-594); the final file content is the same, in discovery order.
"""
from __future__ import annotations

import datetime
import fnmatch
import os
from concurrent.futures import ProcessPoolExecutor, ThreadPoolExecutor

import numpy as np

from . import pfd as _pfd
from . import phcx as _phcx
from . import writers
from .candidate import get_engine, status_error

BATCH = 8192  # files per streamed batch

PHCX_RE = "*.phcx.gz"
SUPERB_RE = "*.phcx"
PFD_RES = ("*.pfd", "*.pfd.36scrunch")


def discover(directory: str, regexes) -> list[str]:
    """os.walk + fnmatch in the reference's order (:491-497)."""
    out = []
    for ft in regexes:
        for root, _subs, filenames in os.walk(directory):
            for fn in fnmatch.filter(filenames, ft):
                out.append(os.path.join(root, fn))
    return out


def _parse_one(path):
    try:
        return _phcx.parse(path), None
    except Exception as e:  # the reference logs and skips unreadable candidates
        return None, f"{type(e).__name__}: {e}"


def _from_native(b, i, inf, path):
    """PHCXCandidate from a file the native reader parsed (include/pfe_io.h)."""
    from ._native import (PFE_PHCX_DM_CURVE, PFE_PHCX_LYON_DM, PFE_PHCX_PROFILE,
                          PFE_PHCX_SUBBANDS)

    scal = np.array(inf.scal[:], dtype=np.float64)
    return _phcx.PHCXCandidate(
        path=path, superb=bool(inf.superb), section=inf.section,
        profile=b.fetch(i, PFE_PHCX_PROFILE, inf.lp).astype(np.int64),
        lyon_dm=b.fetch(i, PFE_PHCX_LYON_DM, inf.ld).astype(np.int64),
        subbands=b.fetch(i, PFE_PHCX_SUBBANDS, inf.nsub * inf.lsb).astype(np.int64)
        .reshape(inf.nsub, inf.lsb),
        dm_curve=b.fetch(i, PFE_PHCX_DM_CURVE, inf.ndm, np.float64),
        scal=scal, period_ms=scal[0], snr=scal[1], dm=scal[2], width=scal[3])


def parse_all(paths, workers: int | None = None, native: bool = True):
    """Parse candidate files in discovery order -> [(PHCXCandidate | None, error | None)].

    native: the threaded C++ reader of libpfe.so (pfe_phcx_parse); files it flags (malformed
    text, decoded values outside a byte, ...) are re-parsed by the Python parser so their
    outcome, including the exception, is the reference's.  native=False: Python parser on a
    process pool."""
    if native and len(paths):
        from ._native import PhcxBatch

        b = PhcxBatch(paths, threads=workers or 0)
        res = []
        for i, p in enumerate(paths):
            inf = b.info(i)
            res.append((_from_native(b, i, inf, p), None) if inf.status == 0 else _parse_one(p))
        b.close()
        return res
    if workers is None:
        workers = min(16, os.cpu_count() or 1)
    if workers <= 1 or len(paths) < 64:
        return [_parse_one(p) for p in paths]
    with ProcessPoolExecutor(max_workers=workers) as ex:
        return list(ex.map(_parse_one, paths, chunksize=64))


def is_pfd(path: str) -> bool:
    return ".pfd" in path  # Candidate.py:136-138


def _read_pfd(path):
    try:
        return _pfd.read(path), None
    except Exception as e:  # the reference logs and skips unreadable candidates
        return None, f"{type(e).__name__}: {e}"


def score_pfd(datas, engine=None, batch: int = 1 << 14):
    """PFD preprocessing + Lyon features on the GPU for parsed folds:
    returns (lyon8 (n,8), profiles [n arrays], errors [n])."""
    engine = engine or get_engine()
    n = len(datas)
    out = np.full((n, 8), np.nan)
    profiles = [None] * n
    err = [None] * n
    groups: dict = {}
    for i, d in enumerate(datas):
        groups.setdefault((d.npart, d.nsub, d.proflen), []).append(i)
    for _shape, idx in groups.items():
        for s0 in range(0, len(idx), batch):
            part = idx[s0:s0 + batch]
            profs, subfreqs, scal = _pfd.batch_inputs([datas[i] for i in part])
            r = engine.pfd_dmprof(profs, subfreqs, scal, chis=False)
            for j, i in enumerate(part):
                profiles[i] = r["profile"][j]
                if int(r["status"][j]) & 0x20:
                    err[i] = "Exception: DM curve stat score extraction exception"
                else:
                    out[i] = r["lyon8"][j]
    return out, profiles, err


def score_pfd22(datas, engine=None, batch: int = 1 << 16):
    """22 scores of parsed PFD folds on the GPU (pfe_pfd_bates22, PFDFile.compute):
    returns (scores (n,22), error message or None per fold)."""
    engine = engine or get_engine()
    n = len(datas)
    out = np.full((n, 22), np.nan)
    err = [None] * n
    groups: dict = {}
    for i, d in enumerate(datas):
        groups.setdefault((d.npart, d.nsub, d.proflen), []).append(i)
    for _shape, idx in groups.items():
        for s0 in range(0, len(idx), batch):
            part = idx[s0:s0 + batch]
            o, st = engine.pfd_bates22(*_pfd.batch_inputs([datas[i] for i in part]))
            for j, i in enumerate(part):
                msg = status_error(int(st[j]))
                if msg:
                    err[i] = msg
                else:
                    out[i] = o[j]
    return out, err


def pfd_profile_and_curve(datas, engine=None, batch: int = 1 << 14):
    """The 0..255 profile and the float32 chi^2-vs-DM curve of parsed PFD folds
    (PFDFile.computeProfileScores :479-492, getDMCurveData :494-520):
    -> (profiles [n arrays], curves [n float32 arrays], error or None per fold)."""
    engine = engine or get_engine()
    n = len(datas)
    profiles, curves, err = [None] * n, [None] * n, [None] * n
    groups: dict = {}
    for i, d in enumerate(datas):
        groups.setdefault((d.npart, d.nsub, d.proflen), []).append(i)
    for _shape, idx in groups.items():
        for s0 in range(0, len(idx), batch):
            part = idx[s0:s0 + batch]
            r = engine.pfd_dmprof(*_pfd.batch_inputs([datas[i] for i in part]), lyon8=False)
            for j, i in enumerate(part):
                profiles[i] = r["profile"][j]
                curves[i] = r["chis"][j]
                if int(r["status"][j]) & 0x20:
                    err[i] = "Exception: DM curve extraction exception"
    return profiles, curves, err


def _shape_key(c):
    return (len(c.profile), c.subbands.shape[0], c.subbands.shape[1], len(c.dm_curve))


def score_bates(cands, engine=None, batch: int = 1 << 18):
    """22 scores for parsed candidates: returns (scores (n,22), error message or None)."""
    engine = engine or get_engine()
    n = len(cands)
    out = np.full((n, 22), np.nan)
    err = [None] * n
    groups: dict = {}
    for i, c in enumerate(cands):
        groups.setdefault(_shape_key(c), []).append(i)
    for (lp, nsub, lsb, ndm), idx in groups.items():
        if ndm < 3:  # max() of an empty DM curve / leastsq m < n: the DM fit raises
            for i in idx:
                err[i] = "DM curve fitting exception"
            continue
        for s in range(0, len(idx), batch):
            part = idx[s:s + batch]
            prof = np.stack([cands[i].profile for i in part]).astype(np.uint8)
            sub = np.stack([cands[i].subbands for i in part]).astype(np.uint8)
            dmc = np.stack([cands[i].dm_curve for i in part]).astype(np.float64)
            scal = np.stack([cands[i].scal for i in part]).astype(np.float64)
            o, st = engine.bates22(prof, sub, dmc, scal)
            for j, i in enumerate(part):
                msg = status_error(int(st[j]))
                if msg:
                    err[i] = msg
                else:
                    out[i] = o[j]
    return out, err


def score_lyon8(cands, engine=None):
    """8 Lyon features (profile stats + section-0 DataBlock stats) for parsed candidates."""
    engine = engine or get_engine()
    n = len(cands)
    out = np.full((n, 8), np.nan)
    groups: dict = {}
    for i, c in enumerate(cands):
        groups.setdefault((len(c.profile), len(c.lyon_dm)), []).append(i)
    for (lp, ld), idx in groups.items():
        prof = np.stack([cands[i].profile for i in idx]).astype(np.uint8)
        dm = np.stack([cands[i].lyon_dm for i in idx]).astype(np.uint8)
        out[idx] = engine.lyon8(prof, dm)
    return out


def _stream(paths, parse, score, emit, batch=BATCH):
    """parse(batch paths) on a helper thread one batch ahead of score(parsed) on the calling
    thread; emit(batch offset, batch paths, results) in discovery order."""
    if not paths:
        return
    cuts = list(range(0, len(paths), batch)) + [len(paths)]
    with ThreadPoolExecutor(max_workers=1) as ex:
        fut = ex.submit(parse, paths[cuts[0]:cuts[1]])
        for k in range(len(cuts) - 1):
            parsed = fut.result()
            if k + 2 < len(cuts):
                fut = ex.submit(parse, paths[cuts[k + 1]:cuts[k + 2]])
            emit(cuts[k], paths[cuts[k]:cuts[k + 1]], score(parsed))


class DataProcessor:
    """Same entry points and output semantics as DataProcessor.py, batched on the GPU."""

    def __init__(self, debugFlag=False, engine=None, workers=None, log=print, batch=BATCH):
        self.debug = debugFlag
        self.engine = engine
        self.workers = workers
        self.log = log
        self.batch = batch
        self.scoreStore = []
        self.candidateErrorLog = "CandidateErrorLog.txt"
        self.superb = False
        self.phcx = False
        self.pfd = False
        self.positive = 0
        self.negative = 0
        if not os.path.exists(self.candidateErrorLog):       # :86-87
            writers.append_text(self.candidateErrorLog, "")

    # ---- discovery ---------------------------------------------------------------
    def _candidates(self, directory, regexes, single):
        if directory == "":
            directory = os.path.dirname(os.path.realpath(__file__))
        if not single:
            return discover(directory, regexes)
        if ".txt" in directory:  # a list of candidate paths (the reference reads self.path)
            with open(directory) as f:
                return [ln.strip() for ln in f if ln.strip()]
        return [directory]

    def _fail(self, cand, why):
        self.log(f"Error reading profile data :\n\t{why}\n{cand}  did not have scores generated.")
        writers.append_text(self.candidateErrorLog, cand + "\n")

    def _summary(self, processed, ok, failed, start, extra=""):
        end = datetime.datetime.now()
        self.log(f"\nCandidates processed:\t{processed}\nSuccesses:\t{ok}\nFailures:\t{failed}\n"
                 f"{extra}Execution time:  {end - start}")

    # ---- parse / score stages ---------------------------------------------------------
    def _parse(self, paths):
        """Host stage: PHCX / SUPERB files through the native reader (Python parser for the
        files it flags), PFD files through pfd.read.  -> (px, parsed, pf, read)."""
        px = [i for i, p in enumerate(paths) if not is_pfd(p)]
        pf = [i for i, p in enumerate(paths) if is_pfd(p)]
        parsed = parse_all([paths[i] for i in px], self.workers) if px else []
        rd = [_read_pfd(paths[i]) for i in pf]
        return px, parsed, pf, rd

    def _score(self, pre, mode):
        """GPU stage.  mode: "scores" (22 scores), "profile" (profile bins), "lyon8" (the 8
        Lyon features) or "label" ((scores, profile, DM-curve data)).
        -> {batch index: (row, None) | (None, error)}"""
        px, parsed, pf, rd = pre
        res = {}
        if px:
            good = [k for k, (c, e) in enumerate(parsed) if c is not None]
            cands = [parsed[k][0] for k in good]
            errs = [None] * len(cands)
            if mode == "profile":
                rows = [[float(v) for v in c.profile] for c in cands]
            elif mode == "lyon8":
                f = score_lyon8(cands, self.engine) if cands else np.zeros((0, 8))
                rows = [f[j] for j in range(len(cands))]
            else:
                sc, errs = score_bates(cands, self.engine)
                if mode == "label":  # Candidate.calculateProfileScores / getDMCurveData
                    rows = [(sc[j], [float(v) for v in c.profile],
                             list(c.lyon_dm) if not c.superb else [])
                            for j, c in enumerate(cands)]
                else:
                    rows = [sc[j] for j in range(len(cands))]
            for j, k in enumerate(good):
                res[px[k]] = (None, errs[j]) if errs[j] else (rows[j], None)
            for k, (c, e) in enumerate(parsed):
                if c is None:
                    res[px[k]] = (None, e)
        if pf:
            good = [k for k, (d, e) in enumerate(rd) if d is not None]
            datas = [rd[k][0] for k in good]
            if mode == "profile":       # PFDFile.computeProfileScores (:479-492)
                _f, profiles, _e = score_pfd(datas, self.engine)
                rows = [[float(v) for v in pr] for pr in profiles]
                errs = [None] * len(datas)
            elif mode == "lyon8":
                feats, _prof, errs = score_pfd(datas, self.engine)
                rows = [feats[j] for j in range(len(datas))]
            else:
                sc, errs = score_pfd22(datas, self.engine)
                if mode == "label":
                    prof, chis, derr = pfd_profile_and_curve(datas, self.engine)
                    rows = [(sc[j], [float(v) for v in prof[j]], list(chis[j]))
                            for j in range(len(datas))]
                    errs = [e or de for e, de in zip(errs, derr)]
                else:
                    rows = [sc[j] for j in range(len(datas))]
            for j, k in enumerate(good):
                res[pf[k]] = (None, errs[j]) if errs[j] else (rows[j], None)
            for k, (d, e) in enumerate(rd):
                if d is None:
                    res[pf[k]] = (None, e)
        return res

    def _run(self, paths, mode, on_row):
        """Stream the paths through parse -> score; on_row(path, row) for every scored
        candidate (in discovery order), the reference's failure handling for the rest."""
        counts = {"ok": 0, "failed": 0}

        def emit(_off, batch_paths, res):
            for i, p in enumerate(batch_paths):
                row, err = res[i]
                if row is None:
                    self._fail(p, err)
                    counts["failed"] += 1
                else:
                    on_row(p, row)
                    counts["ok"] += 1

        _stream(paths, self._parse, lambda pre: self._score(pre, mode), emit, self.batch)
        return counts["ok"], counts["failed"]

    # ---- 22 scores / profile bins ---------------------------------------------------
    def processCollectively(self, directory, verbose, regexes, outPath, arff, genProfileData,
                            single):
        if arff:                                              # prepareARFFFile (:329-367)
            nattr = 22
            if genProfileData and self.superb:
                nattr = 64
            elif genProfileData and self.phcx:
                nattr = 128
            writers.write_arff_header(outPath, writers.arff_header("scores", nattr))
        start = datetime.datetime.now()
        paths = self._candidates(directory, regexes, single)
        pending = []

        def on_row(p, s):
            pending.append(writers.arff_line(p, s) if arff else writers.score_line(p, s))

        def flush():
            if pending:
                writers.append_text(outPath, "".join(x + "\n" for x in pending))
                pending.clear()

        counts = {"ok": 0, "failed": 0}

        def emit(_off, batch_paths, res):
            for i, p in enumerate(batch_paths):
                row, err = res[i]
                if row is None:
                    self._fail(p, err)
                    counts["failed"] += 1
                else:
                    on_row(p, row)
                    counts["ok"] += 1
            flush()  # append this batch's lines now (bounded memory, partial output survives)

        mode = "profile" if genProfileData else "scores"
        _stream(paths, self._parse, lambda pre: self._score(pre, mode), emit, self.batch)
        self._summary(len(paths), counts["ok"], counts["failed"], start)

    def processPFDCollectively(self, directory, verbose, outPath, arff, genProfileData,
                               processSingleCandidate):
        self.pfd = True
        self.processCollectively(directory, verbose, list(PFD_RES), outPath, arff, genProfileData,
                                 processSingleCandidate)

    def processPHCXCollectively(self, directory, verbose, outPath, arff, genProfileData,
                                processSingleCandidate):
        self.phcx = True
        self.processCollectively(directory, verbose, [PHCX_RE], outPath, arff, genProfileData,
                                 processSingleCandidate)

    def processSUPERBCollectively(self, directory, verbose, outPath, arff, genProfileData,
                                  processSingleCandidate):
        self.superb = True
        self.processCollectively(directory, verbose, [SUPERB_RE], outPath, arff, genProfileData,
                                 processSingleCandidate)

    def processSeparately(self, directory, verbose, regexes, single):
        """:603-687 — each candidate's 22 scores into <candidate>.dat."""
        start = datetime.datetime.now()
        paths = self._candidates(directory, regexes, single)

        def on_row(p, s):
            with open(p + ".dat", "w") as f:                   # outputScores :429-447
                f.write(writers.dat_text(s))

        ok, failed = self._run(paths, "scores", on_row)
        self._summary(len(paths), ok, failed, start)

    def processPHCXSeparately(self, directory, verbose, processSingleCandidate):
        self.phcx = True
        self.processSeparately(directory, verbose, [PHCX_RE], processSingleCandidate)

    # ---- 8 Lyon features -------------------------------------------------------------
    def dmprof(self, directory, verbose, regexes, outPath, arff, single):
        if arff:
            writers.write_arff_header(outPath, writers.arff_header("dmprof"))
        start = datetime.datetime.now()
        paths = self._candidates(directory, regexes, single)
        pending = []
        counts = {"ok": 0, "failed": 0}

        def emit(_off, batch_paths, res):
            for i, p in enumerate(batch_paths):
                row, err = res[i]
                if row is None:
                    self._fail(p, err)
                    counts["failed"] += 1
                    continue
                pending.append(writers.arff_line(p, row) if arff else writers.score_line(p, row))
                counts["ok"] += 1
            if pending:
                writers.append_text(outPath, "".join(x + "\n" for x in pending))
                pending.clear()

        _stream(paths, self._parse, lambda pre: self._score(pre, "lyon8"), emit, self.batch)
        self._summary(len(paths), counts["ok"], counts["failed"], start)

    def dmprofPFD(self, directory, verbose, outPath, arff, processSingleCandidate):
        self.pfd = True
        self.dmprof(directory, verbose, list(PFD_RES), outPath, arff, processSingleCandidate)

    def dmprofPHCX(self, directory, verbose, outPath, arff, processSingleCandidate):
        self.phcx = True
        self.dmprof(directory, verbose, [PHCX_RE], outPath, arff, processSingleCandidate)

    def dmprofSUPERB(self, directory, verbose, outPath, arff, processSingleCandidate):
        self.superb = True
        self.dmprof(directory, verbose, [SUPERB_RE], outPath, arff, processSingleCandidate)

    def processPFDSeparately(self, directory, verbose, processSingleCandidate):
        self.pfd = True
        self.processSeparately(directory, verbose, list(PFD_RES), processSingleCandidate)

    def processPFDAndPHCXSeparately(self, directory, verbose, processSingleCandidate):
        self.pfd = self.phcx = True
        self.processSeparately(directory, verbose, [PHCX_RE] + list(PFD_RES),
                               processSingleCandidate)

    def processPFDAndPHCXCollectively(self, directory, verbose, outPath, arff, genProfileData,
                                      processSingleCandidate):
        self.pfd = self.phcx = True
        self.processCollectively(directory, verbose, [PHCX_RE] + list(PFD_RES), outPath, arff,
                                 genProfileData, processSingleCandidate)

    # ---- label mode (:691-826) --------------------------------------------------------
    def label(self, directory, verbose, regexes):
        """Scores.csv, Profile.csv, DMCurve.csv and Cands.meta in the candidate directory:
        per candidate the 22 scores, the profile bins and the DM-curve data, each row ending
        in the label and ",%<candidate>".  The reference's interactive prompt is commented
        out (:754-774), so every label is "0" and the positive/negative counts stay 0.
        Values are written as the reference's Python-2 str() writes them (no nan/inf
        replacement here, unlike storeScore)."""
        if directory == "":
            directory = os.path.dirname(os.path.realpath(__file__))
        meta = directory + "/Cands.meta"
        files = {"scores": directory + "/Scores.csv", "profile": directory + "/Profile.csv",
                 "dm": directory + "/DMCurve.csv"}
        start = datetime.datetime.now()
        paths = discover(directory, regexes)
        lab = "0"
        out = {k: [] for k in ("scores", "profile", "dm", "meta")}

        def on_row(p, row):
            sc, prof, dmc = row
            out["scores"].append("".join(writers.py2_str(v) + "," for v in sc) + lab + ",%" + p + "\n")
            out["profile"].append("".join(writers.py2_str(v) + "," for v in prof) + lab + ",%" + p + "\n")
            out["dm"].append("".join(writers.py2_scalar_str(v) + "," for v in dmc) + lab + ",%" + p + "\n")
            out["meta"].append(p + "," + lab + "\n")

        counts = {"ok": 0, "failed": 0}

        def emit(_off, batch_paths, res):
            for i, p in enumerate(batch_paths):
                row, err = res[i]
                if row is None:
                    self._fail(p, err)
                    counts["failed"] += 1
                else:
                    on_row(p, row)
                    counts["ok"] += 1
            for k, path in (("scores", files["scores"]), ("profile", files["profile"]),
                            ("dm", files["dm"]), ("meta", meta)):
                if out[k]:
                    writers.append_text(path, "".join(out[k]))
                    out[k].clear()

        _stream(paths, self._parse, lambda pre: self._score(pre, "label"), emit, self.batch)
        self._summary(len(paths), counts["ok"], counts["failed"], start,
                      f"Positive:\t{self.positive}\nNegative:\t{self.negative}\n")

    def labelPHCX(self, directory, verbose):
        self.phcx = True
        self.label(directory, verbose, [PHCX_RE])

    def labelPFD(self, directory, verbose, outPath=None, arff=None, genProfileData=None,
                 processSingleCandidate=None):
        """The reference declares six parameters but ScoreGenerator.py:225 passes two (a
        TypeError); the extra ones are optional here and unused, as in the reference."""
        self.pfd = True
        self.label(directory, verbose, list(PFD_RES))
