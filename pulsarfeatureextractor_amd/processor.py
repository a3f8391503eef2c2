"""Batched equivalent of the reference's DataProcessor (DataProcessor.py:51-995).

The reference walks a directory and scores one candidate at a time (parse -> score ->
buffer a text line), catching every exception per candidate
(DataProcessor.py:491-525, 867-901).  Here the same discovery order, file-type dispatch,
error log and output text are kept, but candidates are parsed on host worker processes,
packed into dense arrays and scored in large batches on the GPU through libpfe.

  processPHCXCollectively / processSUPERBCollectively  (:109-146, :451-599)
  processPHCXSeparately                                (:91-105, :603-687)
  dmprofPHCX / dmprofSUPERB                            (:255-301, :830-994)
PFD files (".pfd" in the name, Candidate.py:136) are read by pfd.read and go through
pfe_pfd_dmprof (dmprof and profile-bin modes); the PFD 22-score path is not in this build
yet and raises.  --label is interactive and out of scope.
"""
from __future__ import annotations

import datetime
import fnmatch
import os
from concurrent.futures import ProcessPoolExecutor

import numpy as np

from . import pfd as _pfd
from . import phcx as _phcx
from . import writers
from .candidate import get_engine, status_error

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


class DataProcessor:
    """Same entry points and output semantics as DataProcessor.py, batched on the GPU."""

    def __init__(self, debugFlag=False, engine=None, workers=None, log=print):
        self.debug = debugFlag
        self.engine = engine
        self.workers = workers
        self.log = log
        self.scoreStore = []
        self.candidateErrorLog = "CandidateErrorLog.txt"
        self.superb = False
        self.phcx = False
        self.pfd = False
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

    def _finish(self, outPath, processed, ok, failed, start):
        end = datetime.datetime.now()
        writers.append_text(outPath, "".join(s + "\n" for s in self.scoreStore))
        self.log(f"\nCandidates processed:\t{processed}\nSuccesses:\t{ok}\nFailures:\t{failed}\n"
                 f"Execution time:  {end - start}")

    # ---- 22 scores / profile bins ---------------------------------------------------
    def _rows(self, paths, genProfileData):
        """{index: (row, None)} or {index: (None, error)} in discovery order: PHCX / SUPERB
        files through the native reader and pfe_bates22, PFD files through the host reader
        and pfe_pfd_bates22 (or the profile bins, --profile)."""
        res = {}
        px = [i for i, p in enumerate(paths) if not is_pfd(p)]
        pf = [i for i, p in enumerate(paths) if is_pfd(p)]
        if px:
            parsed = parse_all([paths[i] for i in px], self.workers)
            good = [k for k, (c, e) in enumerate(parsed) if c is not None]
            cands = [parsed[k][0] for k in good]
            if genProfileData:
                rows = [[float(v) for v in c.profile] for c in cands]
                errs = [None] * len(cands)
            else:
                sc, errs = score_bates(cands, self.engine)
                rows = [sc[j] for j in range(len(cands))]
            for j, k in enumerate(good):
                res[px[k]] = (None, errs[j]) if errs[j] else (rows[j], None)
            for k, (c, e) in enumerate(parsed):
                if c is None:
                    res[px[k]] = (None, e)
        if pf:
            rd = [_read_pfd(paths[i]) for i in pf]
            good = [k for k, (d, e) in enumerate(rd) if d is not None]
            datas = [rd[k][0] for k in good]
            if genProfileData:       # PFDFile.computeProfileScores (:479-492)
                _f, profiles, _e = score_pfd(datas, self.engine)
                rows = [[float(v) for v in pr] for pr in profiles]
                errs = [None] * len(datas)
            else:
                sc, errs = score_pfd22(datas, self.engine)
                rows = [sc[j] for j in range(len(datas))]
            for j, k in enumerate(good):
                res[pf[k]] = (None, errs[j]) if errs[j] else (rows[j], None)
            for k, (d, e) in enumerate(rd):
                if d is None:
                    res[pf[k]] = (None, e)
        return res

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
        res = self._rows(paths, genProfileData)
        ok = failed = 0
        for i, p in enumerate(paths):
            s, e = res[i]
            if s is None:
                self._fail(p, e)
                failed += 1
                continue
            self.scoreStore.append(writers.arff_line(p, s) if arff else writers.score_line(p, s))
            ok += 1
        self._finish(outPath, len(paths), ok, failed, start)

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
        paths = self._candidates(directory, regexes, single)
        res = self._rows(paths, False)
        for i, p in enumerate(paths):
            s, e = res[i]
            if s is None:
                self._fail(p, e)
            else:
                with open(p + ".dat", "w") as f:                   # outputScores :429-447
                    f.write(writers.dat_text(s))

    def processPHCXSeparately(self, directory, verbose, processSingleCandidate):
        self.phcx = True
        self.processSeparately(directory, verbose, [PHCX_RE], processSingleCandidate)

    # ---- 8 Lyon features -------------------------------------------------------------
    def dmprof(self, directory, verbose, regexes, outPath, arff, single):
        if arff:
            writers.write_arff_header(outPath, writers.arff_header("dmprof"))
        start = datetime.datetime.now()
        paths = self._candidates(directory, regexes, single)
        row, why = self._lyon_rows(paths)
        ok = failed = 0
        for i, p in enumerate(paths):
            if i not in row:
                self._fail(p, why.get(i))
                failed += 1
                continue
            s = row[i]
            self.scoreStore.append(writers.arff_line(p, s) if arff else writers.score_line(p, s))
            ok += 1
        self._finish(outPath, len(paths), ok, failed, start)

    def _lyon_rows(self, paths):
        """{index: 8 features} for the files that score, {index: error} for the rest; PHCX /
        SUPERB files through pfe_lyon8_u8, PFD files through pfe_pfd_dmprof."""
        row, why = {}, {}
        px = [i for i, p in enumerate(paths) if not is_pfd(p)]
        pf = [i for i, p in enumerate(paths) if is_pfd(p)]
        if px:
            parsed = parse_all([paths[i] for i in px], self.workers)
            good = [k for k, (c, e) in enumerate(parsed) if c is not None]
            feats = score_lyon8([parsed[k][0] for k in good], self.engine)
            for j, k in enumerate(good):
                row[px[k]] = feats[j]
            for k, (c, e) in enumerate(parsed):
                if c is None:
                    why[px[k]] = e
        if pf:
            rd = [_read_pfd(paths[i]) for i in pf]
            good = [k for k, (d, e) in enumerate(rd) if d is not None]
            feats, _prof, errs = score_pfd([rd[k][0] for k in good], self.engine)
            for j, k in enumerate(good):
                if errs[j]:
                    why[pf[k]] = errs[j]
                else:
                    row[pf[k]] = feats[j]
            for k, (d, e) in enumerate(rd):
                if d is None:
                    why[pf[k]] = e
        return row, why

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

    # ---- not in this build -------------------------------------------------------------
    def _label(self, *a, **k):
        raise NotImplementedError("--label (interactive labelling, DataProcessor.py:691-826) "
                                  "is not in this build")

    labelPHCX = labelPFD = _label
