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
import json
import os
import re
import threading
import time
from concurrent.futures import ProcessPoolExecutor, ThreadPoolExecutor

import numpy as np

from . import pfd as _pfd
from . import phcx as _phcx
from . import writers
from .candidate import GROUP_ERRORS, get_engine, status_error

BATCH = 8192  # files per streamed batch

PHCX_RE = "*.phcx.gz"
SUPERB_RE = "*.phcx"
PFD_RES = ("*.pfd", "*.pfd.36scrunch")


def _walk_matches(top: str, ft: str, chunk: int = 2048):
    """os.walk(top) + fnmatch.filter(files, ft) in os.walk's order -- top-down, a directory's
    files in listing order, then its subdirectories depth-first in listing order, symlinked
    directories listed but not entered, unreadable directories skipped -- yielding the matches
    as lists of at most `chunk` listed entries, so the paths of one huge directory stream out
    while it is still being listed (os.walk hands over a directory only once it is fully
    listed).  os.path.join(root, fn) is root + "/" + fn (root + fn when root ends in "/"): the
    same strings without a call per file."""
    match = re.compile(fnmatch.translate(ft)).match
    stack = [top]
    while stack:
        root = stack.pop()
        pre = root if root.endswith("/") or not root else root + "/"
        subs = []
        try:
            it = os.scandir(root)
        except OSError:
            continue
        with it:
            names = []
            failed = False
            while True:
                try:
                    e = next(it)
                except StopIteration:
                    break
                except OSError:
                    # os.walk drops the whole directory (its files and subdirectories) when
                    # listing fails partway; chunks already yielded from it cannot be taken
                    # back (a documented divergence: only a directory of > `chunk` entries
                    # that fails after its first chunk differs)
                    failed = True
                    break
                try:
                    is_dir = e.is_dir()
                except OSError:
                    is_dir = False
                if is_dir:
                    subs.append(e.name)
                else:
                    names.append(e.name)
                    if len(names) >= chunk:
                        hit = [pre + n for n in names if match(n)]
                        names = []
                        if hit:
                            yield hit
            if failed:
                continue
            hit = [pre + n for n in names if match(n)]
            if hit:
                yield hit
        # os.walk enters a listed directory unless it is a symlink (followlinks=False)
        for d in reversed(subs):
            path = os.path.join(root, d)
            if not os.path.islink(path):
                stack.append(path)


def iter_discover(directory: str, regexes):
    """os.walk + fnmatch in the reference's order (:491-497), in chunks of paths (see
    _walk_matches)."""
    for ft in regexes:
        yield from _walk_matches(directory, ft)


def discover(directory: str, regexes) -> list[str]:
    out = []
    for hit in iter_discover(directory, regexes):
        out.extend(hit)
    return out


class PathFeed:
    """The discovered candidate paths of a run, filled by a background walk (iter_discover's
    order, the first `skip` dropped) while the first batches are already parsed: _stream
    takes a batch as soon as its paths are listed, so the walk of a large directory overlaps
    the parsing instead of preceding it.  Reads block until the paths they need are listed;
    len() waits for the whole walk.  on_done(total, skipped) runs on the walk thread, before
    the walk is marked done."""

    def __init__(self, gen=None, skip=0, on_done=None, paths=None):
        self._paths = list(paths) if paths is not None else []
        self._done = gen is None
        self._err = None
        self._cv = threading.Condition()
        if gen is not None:
            threading.Thread(target=self._walk, args=(gen, int(skip), on_done), daemon=True).start()

    def _walk(self, gen, skip, on_done):
        seen = 0
        try:
            for hit in gen:
                if seen + len(hit) <= skip:
                    seen += len(hit)
                    continue
                hit = hit[max(0, skip - seen):]
                seen = max(seen, skip) + len(hit)
                with self._cv:
                    self._paths.extend(hit)
                    self._cv.notify_all()
            # before the walk reports done: a reader waiting on len() (the run summary) sees
            # on_done's metric and log line first
            if on_done is not None:
                on_done(seen, min(seen, skip))
        except BaseException as e:  # re-raised to the reader
            self._err = e
        finally:
            with self._cv:
                self._done = True
                self._cv.notify_all()

    def wait(self, n):
        """Block until n paths are listed or the walk is over; -> the number listed (<= n)."""
        with self._cv:
            self._cv.wait_for(lambda: self._done or len(self._paths) >= n)
            if self._err is not None:
                raise self._err
            return min(n, len(self._paths))

    def known_total(self):
        with self._cv:
            return len(self._paths) if self._done else None

    def __len__(self):
        with self._cv:
            self._cv.wait_for(lambda: self._done)
        if self._err is not None:
            raise self._err
        return len(self._paths)

    def __getitem__(self, k):
        if isinstance(k, slice):
            stop = len(self) if k.stop is None else k.stop
            self.wait(stop)
        else:
            self.wait(k + 1)
        return self._paths[k]

    def __iter__(self):
        return iter(self[:])


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


def _cuts(n, batch, ramp=True):
    """Batch boundaries of a streamed run: full batches, except that a long run starts and
    ends with batch/8, batch/4, batch/2 so the GPU stage starts after a short first parse and
    the last batch's scoring and output trail the last parse by little."""
    steps = [batch // 8, batch // 4, batch // 2]
    if not ramp or batch < 64 or n < 2 * sum(steps) + batch:
        return list(range(0, n, batch)) + [n]
    sizes = list(steps)
    rem = n - 2 * sum(steps)
    while rem > 0:
        sizes.append(min(batch, rem))
        rem -= sizes[-1]
    sizes += steps[::-1]
    return [0] + np.cumsum(sizes).tolist()


def _tail_cuts(lo, n, batch, ramp=True):
    """The rest of _cuts once the total n is known at offset lo: full batches, then the
    closing batch/2, batch/4, batch/8 when the remainder is long enough."""
    steps = [batch // 8, batch // 4, batch // 2]
    rem = n - lo
    if rem <= 0:
        return []
    if not ramp or batch < 64 or rem < sum(steps) + batch:
        return list(range(lo + batch, n, batch)) + [n]
    sizes = []
    r = rem - sum(steps)
    while r > 0:
        sizes.append(min(batch, r))
        r -= sizes[-1]
    sizes += steps[::-1]
    return (lo + np.cumsum(sizes)).tolist()


class _Cuts:
    """Batch boundaries over a PathFeed: _cuts(n) when the total is known up front; while the
    walk is still listing, the opening batch/8, batch/4, batch/2 and then full batches, each
    taken once its paths are listed, and _tail_cuts from wherever the walk ends."""

    def __init__(self, feed, batch, ramp):
        self.feed, self.batch, self.ramp = feed, batch, ramp
        n = feed.known_total()
        self.cuts = _cuts(n, batch, ramp) if n else [0]
        self.final = n is not None

    def has(self, k):
        """Is there a batch k (cuts[k]..cuts[k + 1])?  Blocks until that is known."""
        while len(self.cuts) <= k + 1 and not self.final:
            lo = self.cuts[-1]
            nb = len(self.cuts) - 1
            steps = [self.batch // 8, self.batch // 4, self.batch // 2]
            size = steps[nb] if self.ramp and self.batch >= 64 and nb < 3 else self.batch
            got = self.feed.wait(lo + size + 1)  # one more: is this the last batch?
            n = self.feed.known_total()
            if n is not None:
                self.cuts += _tail_cuts(lo, n, self.batch, self.ramp)
                self.final = True
            elif got > lo + size:
                self.cuts.append(lo + size)
        return len(self.cuts) > k + 1


def _stream(paths, parse, score, emit, batch=BATCH, depth=1, ahead=3, ramp=True):
    """parse(batch paths) on a helper thread, up to `ahead` batches beyond those being scored
    (the parser never waits for a GPU step unless it is that far ahead); score(parsed, slot)
    of batch k on slot k % depth (one thread per slot, so up to `depth` batches are scored at
    once, each on its own engine handle and pinned slabs); emit(batch offset, batch paths,
    results) on the calling thread in discovery order, overlapping the next batches'
    scoring.  `paths` is a list or a PathFeed still being filled by its walk."""
    feed = paths if isinstance(paths, PathFeed) else PathFeed(paths=paths)
    cut = _Cuts(feed, batch, ramp)
    if not cut.has(0):
        return
    cuts = cut.cuts

    def part(k):
        return feed[cuts[k]:cuts[k + 1]]

    slots = [ThreadPoolExecutor(max_workers=1) for _ in range(depth)]
    try:
        with ThreadPoolExecutor(max_workers=1) as px:
            parsed, scored = {}, {}

            def submit_parse(k):
                if k not in parsed and k not in scored and cut.has(k):
                    parsed[k] = px.submit(parse, part(k))

            def submit_score(k):
                if k not in scored and cut.has(k):
                    submit_parse(k)
                    f = parsed.pop(k)
                    scored[k] = slots[k % depth].submit(lambda f=f, k=k: score(f.result(), k % depth))

            for k in range(depth + ahead):
                submit_parse(k)
            for k in range(depth):
                submit_score(k)
            k = 0
            while cut.has(k):
                res = scored.pop(k).result()
                submit_score(k + depth)
                submit_parse(k + depth + ahead)
                emit(cuts[k], part(k), res)
                k += 1
    finally:
        for ex in slots:
            ex.shutdown(wait=True)


class PinnedSlabs:
    """Pinned host buffers (pfe_host_alloc) reused across batches and grown on demand: the
    native packer writes each shape group's rows straight into them and libpfe DMAs them in
    place.  view(key, shape, dtype) -> a numpy view of the slab `key` (valid until the next
    view of the same key).  rows: the batch size; a slab is first sized for that many rows
    of its shape (shape[0] is the row count), so the ramped first batches of a run do not
    regrow it (a pinned free synchronises the device)."""

    def __init__(self, rows=0):
        self._slabs = {}
        self.rows = int(rows)

    def view(self, key, shape, dtype):
        from ._native import host_empty

        dt = np.dtype(dtype)
        shape = tuple(int(v) for v in shape)
        need = max(1, int(np.prod(shape, dtype=np.int64)) * dt.itemsize)
        s = self._slabs.get(key)
        if s is None or s.nbytes < need:
            want = need
            if shape and 0 < shape[0] < self.rows:
                want = need // shape[0] * self.rows
            s = host_empty((want + want // 4 + 4096,), np.uint8)
            self._slabs[key] = s
        return s[:need].view(dt)[: int(np.prod(shape, dtype=np.int64))].reshape(shape)


class ParsedBatch:
    """One streamed batch after the host stage.  PHCX / SUPERB files stay inside the native
    reader (`nb`, pfe_phcx_parse) with their infos as one structured array; only the files it
    flags are parsed by the Python parser (`fallback`: {k: (PHCXCandidate | None, error)}, k
    indexing `px`).  PFD files are read by pfd.read (`rd`)."""

    __slots__ = ("paths", "px", "pf", "nb", "info", "fallback", "rd")

    def close(self):
        if self.nb is not None:
            self.nb.close()
            self.nb = None


class BatchScores:
    """GPU stage output for a batch: `mat` (n, width) float64 when every row of the mode has
    one width (scores, Lyon features, uniform profiles), else `rows` (a list); `err[i]` is
    None or the failure text of file i."""

    __slots__ = ("mat", "rows", "err")

    def __init__(self, n, width=None):
        self.mat = np.full((n, width), np.nan) if width else None
        self.rows = None if width else [None] * n
        self.err = [None] * n

    def row(self, i):
        return self.mat[i] if self.mat is not None else self.rows[i]


def _groups(keys: np.ndarray, idx: np.ndarray):
    """Rows `idx` grouped by equal key rows (first-seen order of np.unique)."""
    if len(idx) == 0:
        return []
    uniq, inv = np.unique(keys, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    order = np.argsort(inv, kind="stable")
    bounds = np.searchsorted(inv[order], np.arange(len(uniq) + 1))
    return [(tuple(int(v) for v in uniq[g]), idx[order[bounds[g]:bounds[g + 1]]])
            for g in range(len(uniq))]


def default_workers() -> int:
    """Host threads for the reader: the CPUs this process may run on, capped by
    OMP_NUM_THREADS when set (the GPU box's per-job CPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS", "")
    if cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def _write_progress(out_path, done):
    """<out_path>.progress: the number of discovered candidates whose lines (or failures) are
    in the outputs -- the --start value that resumes after the last completed batch."""
    tmp = out_path + ".progress.tmp"
    with open(tmp, "w") as f:
        f.write(f"{done}\n")
    os.replace(tmp, out_path + ".progress")


class RunMetrics:
    """Structured per-run metrics: candidates, successes, failures by
    reason (the reference's messages; the score-group ones are the PFE_ST_* bits of
    pfe_bates22), candidates/s, and the host time spent parsing (helper thread) and scoring
    (GPU stage: pack, DMA, kernels).  The counts mirror DataProcessor.py:596-599."""

    _BITS = {msg: name for (_bit, msg), name in zip(
        GROUP_ERRORS, ("PFE_ST_SINE_FAIL", "PFE_ST_GAUSS_FAIL", "PFE_ST_DMFIT_FAIL",
                       "PFE_ST_SUBBAND_FAIL", "PFE_ST_UNSUPPORTED"))}

    def __init__(self, mode, start_offset=0):
        self.mode = mode
        self.start_offset = int(start_offset)
        self.t0 = time.perf_counter()
        self.parse_s = 0.0
        self.parse_span = None  # (first parse start, last parse end), seconds after t0
        self.score_s = 0.0
        self.stage = {}  # finer host timers of the GPU stage (pack, gpu), summed over slots
        self.batches = 0
        self.reasons = {}
        self.shards = []  # --gpus N: one entry per worker (merge)
        # the pipeline's slot threads add to the same timers concurrently
        self._lock = threading.Lock()

    def add(self, key, dt):
        with self._lock:
            self.stage[key] = self.stage.get(key, 0.0) + dt

    def timed_parse(self, fn):
        def wrapped(paths):
            t = time.perf_counter()
            try:
                return fn(paths)
            finally:
                e = time.perf_counter()
                self.parse_s += e - t
                first = self.parse_span[0] if self.parse_span else t - self.t0
                self.parse_span = (first, e - self.t0)
        return wrapped

    def timed_score(self, fn):
        def wrapped(pre, slot=0):
            t = time.perf_counter()
            try:
                return fn(pre, slot)
            finally:
                dt = time.perf_counter() - t
                with self._lock:
                    self.score_s += dt
        return wrapped

    def merge(self, m, rank, n, device, engine_start_s=None):
        """Fold one --gpus shard's metrics (its worker's finish()) into this run's: batches,
        failures by reason, the parser / GPU-stage timers summed over the workers (host
        seconds, as over the slots of one process), plus a per-shard entry."""
        if not m:
            return
        with self._lock:
            self.batches += m.get("batches", 0)
            for k, v in m.get("failures_by_reason", {}).items():
                self.reasons[k] = self.reasons.get(k, 0) + v
            self.parse_s += m.get("parse_s", 0.0)
            self.score_s += m.get("score_s", 0.0)
            for k, v in m.items():
                if k.endswith("_s") and k[:-2] in ("pack", "gpu", "emit", "discover"):
                    self.stage[k[:-2]] = self.stage.get(k[:-2], 0.0) + v
            self.shards.append({"rank": rank, "device": int(device), "candidates": int(n),
                                "engine_start_s": engine_start_s, "wall_s": m.get("wall_s"),
                                "candidates_per_s": m.get("candidates_per_s")})

    def batch(self, res):
        self.batches += 1
        for e in res.err:
            if e:
                key = self._BITS.get(e) or str(e).strip().split("\n")[0][:120]
                self.reasons[key] = self.reasons.get(key, 0) + 1

    def finish(self, processed, ok, failed):
        wall = time.perf_counter() - self.t0
        return {"mode": self.mode, "start_offset": self.start_offset,
                "candidates": int(processed), "successes": int(ok), "failures": int(failed),
                "failures_by_reason": dict(sorted(self.reasons.items())),
                "batches": self.batches, "wall_s": round(wall, 6),
                "candidates_per_s": round(processed / wall, 3) if wall > 0 else None,
                "parse_s": round(self.parse_s, 6), "score_s": round(self.score_s, 6),
                # where the parser was not busy: before its first batch, between batches
                # (waiting for the pipeline), after its last
                **({"parse_head_s": round(self.parse_span[0], 6),
                    "parse_idle_s": round(self.parse_span[1] - self.parse_span[0] - self.parse_s, 6),
                    "parse_tail_s": round(wall - self.parse_span[1], 6)} if self.parse_span else {}),
                **{k + "_s": round(v, 6) for k, v in sorted(self.stage.items())},
                **({"shards": self.shards} if self.shards else {})}


class DataProcessor:
    """Same entry points and output semantics as DataProcessor.py, batched on the GPU.

    start: resume offset -- skip the first `start` discovered candidates (a run that stopped
    after appending k batches resumes with start = the number of candidates already
    processed; the reference has no resume and loses the whole run, DataProcessor.py:590-594).
    """

    def __init__(self, debugFlag=False, engine=None, workers=None, log=print, batch=BATCH,
                 start=0, gpu_batch=1 << 18, metrics_path=None, gpu_depth=2, ramp=True,
                 gpus=1, devices=None, shard_engine=None, shard_slabs=None):
        self.debug = debugFlag
        # --gpus N: the discovered paths are cut into N contiguous shards, each scored by its
        # own worker process on its own GPU (own reader threads, pinned slabs, engine handles);
        # the parent never touches a GPU and concatenates the shards' outputs in discovery
        # order (_run_shards).  devices: the GPU of each worker (default rank % GPUs);
        # shard_engine / shard_slabs: "module:callable" factories a worker builds its engine /
        # slabs from instead of libpfe's (host tests)
        self.gpus = max(1, int(gpus))
        self.devices = list(devices) if devices else None
        self.shard_engine, self.shard_slabs = shard_engine, shard_slabs
        self._shard = None    # in a worker: (rank, suffix, its paths)
        self.verbose = False  # the entry point's verbose flag (-v): isValid per PHCX file
        self._run = None      # RunMetrics of the mode being run (stage timers)
        self.metrics_path = metrics_path
        self.metrics = None   # RunMetrics.as_dict() of the last mode run
        self.engine = engine
        self.workers = workers or default_workers()
        self.log = log
        self.batch = batch
        self.start = int(start)
        self.gpu_batch = int(gpu_batch)
        self.scoreStore = []
        self.candidateErrorLog = "CandidateErrorLog.txt"
        self.superb = False
        self.phcx = False
        self.pfd = False
        self.positive = 0
        self.negative = 0
        # gpu_depth batches are scored at once (processor._stream), each slot with its own
        # engine handle (stream + workspace) and pinned slabs
        self.depth = max(1, int(gpu_depth))
        # ramped batch sizes at both ends of a streamed run (_cuts): the first GPU step starts
        # after a short parse, the last one trails the last parse by little; with the slabs
        # sized for the batch and the handle's workspace grown geometrically, faster in every
        # alternating pair measured (profiles/r04_ab_e2e_ramp.txt)
        self.ramp = bool(ramp)
        self._slabs = [PinnedSlabs(self.batch) for _ in range(self.depth)]
        self._engines = {}
        if not os.path.exists(self.candidateErrorLog):       # :86-87
            writers.append_text(self.candidateErrorLog, "")

    # ---- discovery ---------------------------------------------------------------
    def _candidates(self, directory, regexes, single):
        """The run's candidate paths: a PathFeed whose walk runs beside the first batches'
        parsing for a directory, a list otherwise.  Run metrics "discover": the walk's time."""
        if self._shard is not None:  # a worker: its shard of the parent's discovery
            return list(self._shard[2])
        t0 = time.perf_counter()
        if directory == "":
            directory = os.path.dirname(os.path.realpath(__file__))
        if not single:
            run = self._run

            def done(total, skipped):
                if run is not None:
                    run.add("discover", time.perf_counter() - t0)
                if self.start:
                    self.log(f"Resuming after the first {skipped} of {total} candidates")

            return PathFeed(iter_discover(directory, regexes), skip=self.start, on_done=done)
        try:
            return self._candidates_(directory, regexes)
        finally:
            if self._run is not None:
                self._run.add("discover", time.perf_counter() - t0)

    def _candidates_(self, directory, regexes):
        if ".txt" in directory:  # a list of candidate paths (the reference reads self.path)
            with open(directory) as f:
                paths = [ln.strip() for ln in f if ln.strip()]
        else:
            paths = [directory]
        if self.start:
            self.log(f"Resuming after the first {min(self.start, len(paths))} of "
                     f"{len(paths)} candidates")
            paths = paths[self.start:]
        return paths

    def _resuming(self, out_path):
        """A resumed run (start > 0) appends to the output the stopped run wrote: its ARFF
        header is already there, so a second one would break the file."""
        return self._shard is not None or (self.start > 0 and os.path.exists(out_path))

    def _fail(self, cand, why):
        self.log(f"Error reading profile data :\n\t{why}\n{cand}  did not have scores generated.")
        writers.append_text(self.candidateErrorLog, cand + "\n")

    def _fail_batch(self, batch_paths, res):
        """The reference's per-candidate failure handling (:517-523) for a batch: one log
        message per failed candidate, one append of their names to the error log."""
        failed = [i for i, e in enumerate(res.err) if e]
        for i in failed:
            self.log(f"Error reading profile data :\n\t{res.err[i]}\n{batch_paths[i]}  "
                     "did not have scores generated.")
        if failed:
            writers.append_text(self.candidateErrorLog,
                                "".join(batch_paths[i] + "\n" for i in failed))
        return failed

    def _summary(self, processed, ok, failed, start, extra="", run=None):
        if self._shard is not None:  # a worker: the parent reports the run
            self.metrics = run.finish(processed, ok, failed) if run is not None else None
            return
        end = datetime.datetime.now()
        self.log(f"\nCandidates processed:\t{processed}\nSuccesses:\t{ok}\nFailures:\t{failed}\n"
                 f"{extra}Execution time:  {end - start}")
        if run is not None:
            self.metrics = run.finish(processed, ok, failed)
            if self.metrics_path:
                with open(self.metrics_path, "w") as f:
                    json.dump(self.metrics, f, indent=1)
                    f.write("\n")

    # ---- parse / score stages ---------------------------------------------------------
    def _parse(self, paths):
        """Host stage (helper thread): PHCX / SUPERB files through the native reader's
        threads (the ctypes call releases the GIL), the Python parser only for files the
        reader flags; PFD files through pfd.read."""
        from ._native import PhcxBatch

        pre = ParsedBatch()
        pre.paths = paths
        pre.px = np.array([i for i, p in enumerate(paths) if not is_pfd(p)], dtype=np.int64)
        pre.pf = [i for i, p in enumerate(paths) if is_pfd(p)]
        pre.nb, pre.info, pre.fallback = None, None, {}
        if len(pre.px):
            pre.nb = PhcxBatch([paths[i] for i in pre.px], threads=self.workers)
            pre.info = pre.nb.infos()
            for k in np.flatnonzero(pre.info["status"] != 0):
                pre.fallback[int(k)] = _parse_one(paths[pre.px[k]])
        pre.rd = [_read_pfd(paths[i]) for i in pre.pf]
        return pre

    def _eng(self, slot=0):
        """Slot 0: the caller's engine (or the process default); slot k > 0: a second libpfe
        handle on the same device (a handle's stream and workspace serve one call at a
        time).  A non-libpfe engine (a test stub) serves every slot."""
        from ._native import Engine

        from ._native import OPTIONS

        base = self.engine or get_engine()
        if slot == 0 or not isinstance(base, Engine):
            return base
        e = self._engines.get(slot)
        if e is None:
            e = self._engines[slot] = Engine(base.device)
        # every handle option of the caller's engine (solver, kernels, pools ...), read again
        # at each batch: the slots of one run compute exactly what the caller's engine would
        for name in OPTIONS:
            v = base.get_option(name)
            if e.get_option(name) != v:
                e.set_option(name, v)
        return e

    def _slab(self, slot):
        s = self._slabs
        return s[slot % len(s)] if isinstance(s, list) else s

    def _bates_native(self, pre, mat, err, slot=0):
        """22 scores of the reader's good files: one pfe_phcx_pack per (shape, chunk) into
        pinned slabs, pfe_bates22 on them (DataProcessor.py:491-525 batched)."""
        from ._native import PfeError

        info, px, sl = pre.info, pre.px, self._slab(slot)
        ok = np.flatnonzero(info["status"] == 0)
        keys = np.stack([info["lp"], info["nsub"], info["lsb"], info["ndm"]], 1)[ok]
        for (lp, nsub, lsb, ndm), rows in _groups(keys, ok):
            if ndm < 3:  # max() of an empty DM curve / leastsq m < n: the DM fit raises
                for k in rows:
                    err[px[k]] = "DM curve fitting exception"
                continue
            for s0 in range(0, len(rows), self.gpu_batch):
                r = rows[s0:s0 + self.gpu_batch]
                m, dst = len(r), px[r]
                t0 = time.perf_counter()
                a = pre.nb.pack(r, lp=lp, nsub_lsb=(nsub, lsb), ndm=ndm, alloc=sl.view,
                                threads=self.workers)
                o = sl.view("out22", (m, 22), np.float64)
                st = sl.view("status", (m,), np.uint32)
                t1 = time.perf_counter()
                try:
                    self._eng(slot).bates22(a["prof"], a["sub"], a["dmcurve"], a["scal"], out=o,
                                        status=st)
                except PfeError as e:  # a shape the library refuses fails its rows, not the run
                    for d in dst:
                        err[d] = f"Exception: {e}"
                    continue
                finally:
                    if self._run is not None:
                        self._run.add("pack", t1 - t0)
                        self._run.add("gpu", time.perf_counter() - t1)
                mat[dst] = o
                for j in np.flatnonzero(st & 0xFF):
                    err[dst[j]] = status_error(int(st[j]))

    def _fallback_cands(self, pre, res):
        """Files the native reader flagged, parsed by the Python parser: (batch indices,
        PHCXCandidates); their parse errors go straight into res.err."""
        idx, cands = [], []
        for k, (c, e) in pre.fallback.items():
            if c is None:
                res.err[pre.px[k]] = e
            else:
                idx.append(int(pre.px[k]))
                cands.append(c)
        return idx, cands

    def _score_phcx(self, pre, mode, res, slot=0):
        info, px, sl = pre.info, pre.px, self._slab(slot)
        eng = self._eng(slot)
        ok = np.flatnonzero(info["status"] == 0)
        fidx, fcands = self._fallback_cands(pre, res)
        if mode in ("scores", "label"):
            mat = res.mat if mode == "scores" else np.full((len(pre.paths), 22), np.nan)
            self._bates_native(pre, mat, res.err, slot)
            if fcands:
                sc, errs = score_bates(fcands, eng)
                for j, i in enumerate(fidx):
                    mat[i], res.err[i] = sc[j], errs[j]
            if mode == "label":  # Candidate.calculateProfileScores / getDMCurveData
                from ._native import PFE_PHCX_LYON_DM, PFE_PHCX_PROFILE

                for k in ok:
                    i = int(px[k])
                    if res.err[i]:
                        continue
                    prof = pre.nb.fetch(int(k), PFE_PHCX_PROFILE, int(info["lp"][k]))
                    dm = ([] if info["superb"][k] else
                          list(pre.nb.fetch(int(k), PFE_PHCX_LYON_DM, int(info["ld"][k]))))
                    res.rows[i] = (mat[i], [float(v) for v in prof], dm)
                for j, i in enumerate(fidx):
                    if not res.err[i]:
                        c = fcands[j]
                        res.rows[i] = (mat[i], [float(v) for v in c.profile],
                                       list(c.lyon_dm) if not c.superb else [])
        elif mode == "lyon8":
            keys = np.stack([info["lp"], info["ld"]], 1)[ok]
            for (lp, ld), rows in _groups(keys, ok):
                for s0 in range(0, len(rows), self.gpu_batch):
                    r = rows[s0:s0 + self.gpu_batch]
                    a = pre.nb.pack(r, lp=lp, ld=ld, alloc=sl.view, threads=self.workers)
                    o = sl.view("out8", (len(r), 8), np.float64)
                    eng.lyon8(a["prof"], a["lyon_dm"], out=o)
                    res.mat[px[r]] = o
            if fcands:
                f = score_lyon8(fcands, eng)
                res.mat[fidx] = f
        else:  # "profile": the profile bins as float scores (PHCXFile.computeProfileScores)
            keys = info["lp"][ok][:, None]
            for (lp,), rows in _groups(keys, ok):
                a = pre.nb.pack(rows, lp=lp, alloc=sl.view, threads=self.workers)
                for j, k in enumerate(rows):
                    res.rows[px[k]] = a["prof"][j].astype(np.float64)
            for j, i in enumerate(fidx):
                res.rows[i] = np.asarray(fcands[j].profile, dtype=np.float64)

    def _score_pfd(self, pre, mode, res, slot=0):
        pf, rd = pre.pf, pre.rd
        eng = self._eng(slot)
        good = [k for k, (d, e) in enumerate(rd) if d is not None]
        for k, (d, e) in enumerate(rd):
            if d is None:
                res.err[pf[k]] = e
        datas = [rd[k][0] for k in good]
        if not datas:
            return
        if mode == "profile":       # PFDFile.computeProfileScores (:479-492)
            _f, profiles, _e = score_pfd(datas, eng)
            for j, k in enumerate(good):
                res.rows[pf[k]] = np.asarray(profiles[j], dtype=np.float64)
        elif mode == "lyon8":
            feats, _prof, errs = score_pfd(datas, eng)
            for j, k in enumerate(good):
                res.mat[pf[k]], res.err[pf[k]] = feats[j], errs[j]
        else:
            sc, errs = score_pfd22(datas, eng)
            if mode == "label":
                prof, chis, derr = pfd_profile_and_curve(datas, eng)
                for j, k in enumerate(good):
                    res.err[pf[k]] = errs[j] or derr[j]
                    res.rows[pf[k]] = (sc[j], [float(v) for v in prof[j]], list(chis[j]))
            else:
                for j, k in enumerate(good):
                    res.mat[pf[k]], res.err[pf[k]] = sc[j], errs[j]

    def _score(self, pre, mode, slot=0):
        """GPU stage on pipeline slot `slot`.  mode: "scores" (22 scores), "profile" (profile
        bins), "lyon8" (the 8 Lyon features) or "label" ((scores, profile, DM-curve data))
        -> BatchScores."""
        width = {"scores": 22, "lyon8": 8}.get(mode)
        res = BatchScores(len(pre.paths), width)
        try:
            if len(pre.px):
                self._score_phcx(pre, mode, res, slot)
            if pre.pf:
                self._score_pfd(pre, mode, res, slot)
        finally:
            pre.close()
        if self.verbose and len(pre.px):
            self._debug_validity(pre, mode, res)
        return res

    def _debug_validity(self, pre, mode, res):
        """Debug (-v) mode: PHCXFile.load (PHCXFile.py:108-134) runs isValid on every PHCX /
        SUPERB file first.  An invalid file keeps 22 NaN scores and an EMPTY profile list, so
        compute()'s sine group then fails (profile.mean() of a list: "Sinusoid fitting
        exception", :470) and the 22-score modes drop the file; the Lyon mode's profile
        moments of [] are NaN (numpy mean / std of an empty list) while the DM-curve moments,
        read from the XML, are unchanged.  An exception inside isValid fails the file.  The
        reference's debug prints and matplotlib windows are not reproduced."""
        for k in range(len(pre.px)):
            i = int(pre.px[k])
            if res.err[i]:
                continue
            path = pre.paths[i]
            try:
                valid = _phcx.is_valid(path)
            except Exception as e:  # noqa: BLE001 -- the reference's load() raises it
                res.err[i] = f"{type(e).__name__}: {e}"
                continue
            if valid:
                continue
            self.log(f"Invalid {'SUPERB ' if '.gz' not in path else ''}PHCX candidate:  {path}")
            if mode in ("scores", "label"):
                res.err[i] = GROUP_ERRORS[0][1]
            elif mode == "lyon8":
                res.mat[i, :4] = np.nan
            else:  # profile mode: load() already filled scores with numberOfScores (22) NaNs
                # (PHCXFile.py:115-118, SUPERBPHCXFile.py:114-117) and computeProfileScores
                # (:301-304) appends the empty profile to that list
                res.rows[i] = np.full(22, np.nan)

    def _stream_text(self, paths, mode, out_path, style, run):
        """Collective modes: stream parse -> score, append each batch's lines (pfe_format_rows,
        storeScore / storeScoreARFF text) in discovery order, then log the batch's failures and
        rewrite <out_path>.progress with the number of discovered candidates done (the --start
        value that resumes after this batch)."""
        from ._native import format_rows

        counts = {"ok": 0, "failed": 0}
        self._run = run

        def emit(off, batch_paths, res):
            t0 = time.perf_counter()
            try:
                _emit(off, batch_paths, res)
            finally:
                run.add("emit", time.perf_counter() - t0)

        def _emit(off, batch_paths, res):
            nfail = sum(1 for e in res.err if e)
            counts["failed"] += nfail
            counts["ok"] += len(batch_paths) - nfail
            run.batch(res)
            mat, skip = _as_matrix(res)
            if mat is not None:
                text = format_rows(batch_paths, mat, style, skip, threads=self.workers)
            else:  # rows of different widths (profile mode over mixed shapes)
                fmt = writers.arff_line if style == 1 else writers.score_line
                text = "".join(fmt(p, res.rows[i]) + "\n" for i, p in enumerate(batch_paths)
                               if not res.err[i]).encode()
            if text:
                with open(out_path, "ab") as f:
                    f.write(text)
            self._fail_batch(batch_paths, res)
            _write_progress(out_path, self.start + off + len(batch_paths))

        _stream(paths, run.timed_parse(self._parse),
                run.timed_score(lambda pre, slot: self._score(pre, mode, slot)), emit, self.batch,
                self.depth, ramp=self.ramp)
        return counts["ok"], counts["failed"]

    # ---- 22 scores / profile bins ---------------------------------------------------
    def processCollectively(self, directory, verbose, regexes, outPath, arff, genProfileData,
                            single):
        self.verbose = bool(verbose)
        if arff and not self._resuming(outPath):              # prepareARFFFile (:329-367)
            nattr = 22
            if genProfileData and self.superb:
                nattr = 64
            elif genProfileData and self.phcx:
                nattr = 128
            writers.write_arff_header(outPath, writers.arff_header("scores", nattr))
        start = datetime.datetime.now()
        mode = "profile" if genProfileData else "scores"
        run = RunMetrics(mode, self.start)
        self._run = run
        paths = self._candidates(directory, regexes, single)
        if self._sharding(single):
            ok, failed = self._run_shards(
                "processCollectively", (directory, verbose, regexes, outPath, arff,
                                        genProfileData, single), paths, run, outs=[outPath],
                out_arg=3)
        else:
            ok, failed = self._stream_text(paths, mode, outPath, 1 if arff else 0, run)
        self._summary(len(paths), ok, failed, start, run=run)

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
        self.verbose = bool(verbose)
        start = datetime.datetime.now()
        run = RunMetrics("separately", self.start)
        self._run = run
        paths = self._candidates(directory, regexes, single)
        if self._sharding(single):
            ok, failed = self._run_shards("processSeparately", (directory, verbose, regexes, single),
                                          paths, run, outs=[])
            self._summary(len(paths), ok, failed, start, run=run)
            return

        from ._native import format_rows

        counts = {"ok": 0, "failed": 0}

        def emit(_off, batch_paths, res):
            failed = self._fail_batch(batch_paths, res)
            counts["failed"] += len(failed)
            counts["ok"] += len(batch_paths) - len(failed)
            run.batch(res)
            mat, skip = _as_matrix(res)
            keep = [i for i in range(len(batch_paths)) if not res.err[i]]
            if mat is not None:
                texts = format_rows(batch_paths, mat, 2, skip).decode().split("\n")
            else:
                texts = [writers.dat_text(res.rows[i]) for i in keep]
            for i, t in zip(keep, texts):
                with open(batch_paths[i] + ".dat", "w") as f:   # outputScores :429-447
                    f.write(t)

        _stream(paths, run.timed_parse(self._parse),
                run.timed_score(lambda pre, slot: self._score(pre, "scores", slot)), emit,
                self.batch, self.depth, ramp=self.ramp)
        self._summary(len(paths), counts["ok"], counts["failed"], start, run=run)

    def processPHCXSeparately(self, directory, verbose, processSingleCandidate):
        self.phcx = True
        self.processSeparately(directory, verbose, [PHCX_RE], processSingleCandidate)

    # ---- 8 Lyon features -------------------------------------------------------------
    def dmprof(self, directory, verbose, regexes, outPath, arff, single):
        self.verbose = bool(verbose)
        if arff and not self._resuming(outPath):
            writers.write_arff_header(outPath, writers.arff_header("dmprof"))
        start = datetime.datetime.now()
        run = RunMetrics("lyon8", self.start)
        self._run = run
        paths = self._candidates(directory, regexes, single)
        if self._sharding(single):
            ok, failed = self._run_shards("dmprof", (directory, verbose, regexes, outPath, arff,
                                                     single), paths, run, outs=[outPath],
                                          out_arg=3)
        else:
            ok, failed = self._stream_text(paths, "lyon8", outPath, 1 if arff else 0, run)
        self._summary(len(paths), ok, failed, start, run=run)

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

    # ---- --gpus N: contiguous shards over worker processes ---------------------------
    def _sharding(self, single):
        return self.gpus > 1 and self._shard is None and not single

    def _run_shards(self, entry, args, paths, run, outs, out_arg=None, progress=True):
        """Score `paths` (the whole discovery, resume offset applied) as self.gpus contiguous
        shards, one spawned worker process per shard (_shard_worker): worker r runs the same
        entry point of a single-GPU DataProcessor on device devices[r] over its shard, writing
        every output file, the error log and the progress marker with the suffix ".shard<r>".
        The parent (which never initialises a GPU, so spawning is safe) then appends the
        shards' files to the real ones in rank order -- the discovery order of a one-process
        run, byte for byte -- removes them, and writes <out>.progress = start + len(paths).
        Only a finished run is merged: a stopped run leaves its shard files and the previous
        progress marker, so it resumes from --start as before."""
        import multiprocessing as mp

        g = self.gpus
        devices = self.devices or _default_devices(g)
        threads = max(1, self.workers // g)
        ctx = mp.get_context("spawn")
        procs, pipes = [], []
        kw = {"debugFlag": self.debug, "workers": threads, "batch": self.batch,
              "gpu_batch": self.gpu_batch, "gpu_depth": self.depth, "ramp": self.ramp}
        flags = {"phcx": self.phcx, "pfd": self.pfd, "superb": self.superb}
        # the workers start (interpreter, engine, GPU) while the walk is still listing; each
        # gets its shard of paths once the walk is done
        for r in range(g):
            sfx = f".shard{r}"
            a = list(args)
            if out_arg is not None:
                a[out_arg] = a[out_arg] + sfx
            mine, theirs = ctx.Pipe(duplex=True)
            p = ctx.Process(target=_shard_worker, name=f"pfe-shard{r}",
                            args=(theirs, kw, flags, entry, tuple(a), r, sfx,
                                  int(devices[r % len(devices)]), self.shard_engine,
                                  self.shard_slabs))
            p.start()
            theirs.close()
            procs.append(p)
            pipes.append(mine)
        paths = list(paths)
        n = len(paths)
        cuts = [n * r // g for r in range(g + 1)]
        for r, c in enumerate(pipes):
            try:
                c.send(paths[cuts[r]:cuts[r + 1]])
            except (BrokenPipeError, OSError):
                pass  # the worker failed while starting: its error is read below
        results, errors = [], []
        for r, (p, c) in enumerate(zip(procs, pipes)):
            try:
                res = c.recv()
            except EOFError:
                res = {"error": f"shard {r}: worker exited with code {p.exitcode}"}
            p.join()
            if res.get("error"):
                errors.append(res["error"])
            results.append(res)
        if errors:
            raise RuntimeError("sharded run failed:\n" + "\n".join(errors))
        t0 = time.perf_counter()
        for out in list(outs) + [self.candidateErrorLog]:
            with open(out, "ab") as dst:
                for r in range(g):
                    part = out + f".shard{r}"
                    if os.path.exists(part):
                        with open(part, "rb") as src:
                            while True:
                                b = src.read(1 << 24)
                                if not b:
                                    break
                                dst.write(b)
                        os.remove(part)
        for out in outs:
            for r in range(g):
                q = out + f".shard{r}.progress"
                if os.path.exists(q):
                    os.remove(q)
        if progress and outs:
            _write_progress(outs[0], self.start + n)
        run.add("merge", time.perf_counter() - t0)
        ok = failed = 0
        for r, res in enumerate(results):
            ok += res["ok"]
            failed += res["failed"]
            run.merge(res.get("metrics"), r, cuts[r + 1] - cuts[r], devices[r % len(devices)],
                      res.get("engine_start_s"))
        return ok, failed

    # ---- label mode (:691-826) --------------------------------------------------------
    def label(self, directory, verbose, regexes):
        """Scores.csv, Profile.csv, DMCurve.csv and Cands.meta in the candidate directory:
        per candidate the 22 scores, the profile bins and the DM-curve data, each row ending
        in the label and ",%<candidate>".  The reference's interactive prompt is commented
        out (:754-774), so every label is "0" and the positive/negative counts stay 0.
        Values are written as the reference's Python-2 str() writes them (no nan/inf
        replacement here, unlike storeScore)."""
        self.verbose = bool(verbose)
        if directory == "":
            directory = os.path.dirname(os.path.realpath(__file__))
        sfx = self._shard[1] if self._shard is not None else ""
        meta = directory + "/Cands.meta" + sfx
        files = {"scores": directory + "/Scores.csv" + sfx,
                 "profile": directory + "/Profile.csv" + sfx, "dm": directory + "/DMCurve.csv" + sfx}
        start = datetime.datetime.now()
        run = RunMetrics("label", self.start)
        self._run = run
        paths = self._candidates(directory, regexes, False)
        if self._sharding(False):
            ok, failed = self._run_shards("label", (directory, verbose, regexes), paths, run,
                                          outs=[files["scores"], files["profile"], files["dm"],
                                                meta], progress=False)
            self._summary(len(paths), ok, failed, start,
                          f"Positive:\t{self.positive}\nNegative:\t{self.negative}\n", run=run)
            return
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
            run.batch(res)
            failed = [i for i, e in enumerate(res.err) if e]
            counts["failed"] += len(failed)
            for i, p in enumerate(batch_paths):
                if not res.err[i]:
                    on_row(p, res.rows[i])
                    counts["ok"] += 1
            for k, path in (("scores", files["scores"]), ("profile", files["profile"]),
                            ("dm", files["dm"]), ("meta", meta)):
                if out[k]:
                    writers.append_text(path, "".join(out[k]))
                    out[k].clear()
            self._fail_batch(batch_paths, res)

        _stream(paths, run.timed_parse(self._parse),
                run.timed_score(lambda pre, slot: self._score(pre, "label", slot)), emit,
                self.batch, self.depth, ramp=self.ramp)
        self._summary(len(paths), counts["ok"], counts["failed"], start,
                      f"Positive:\t{self.positive}\nNegative:\t{self.negative}\n", run=run)

    def labelPHCX(self, directory, verbose):
        self.phcx = True
        self.label(directory, verbose, [PHCX_RE])

    def labelPFD(self, directory, verbose, outPath=None, arff=None, genProfileData=None,
                 processSingleCandidate=None):
        """The reference declares six parameters but ScoreGenerator.py:225 passes two (a
        TypeError); the extra ones are optional here and unused, as in the reference."""
        self.pfd = True
        self.label(directory, verbose, list(PFD_RES))


def _as_matrix(res):
    """(matrix, skip mask) for pfe_format_rows, or (None, None) when the rows differ in width."""
    skip = np.array([1 if e else 0 for e in res.err], dtype=np.uint8)
    if res.mat is not None:
        return res.mat, skip
    rows = [r for r, e in zip(res.rows, res.err) if not e]
    widths = {len(r) for r in rows}
    if len(widths) > 1:
        return None, None
    w = widths.pop() if widths else 0
    mat = np.zeros((len(res.rows), w))
    for i, (r, e) in enumerate(zip(res.rows, res.err)):
        if not e:
            mat[i] = r
    return mat, skip


def _visible_gpus():
    """GPUs this process may use, without initialising one (and without importing torch,
    whose first import costs seconds): the HIP / ROCr / CUDA visibility list when one is
    set, else the GPU nodes of the KFD topology (nodes with SIMDs)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None and v.strip():
            return len([x for x in v.split(",") if x.strip()])
    n = 0
    try:
        base = "/sys/class/kfd/kfd/topology/nodes"
        for node in os.listdir(base):
            with open(os.path.join(base, node, "properties")) as f:
                for ln in f:
                    k, _, v = ln.partition(" ")
                    if k == "simd_count" and int(v) > 0:
                        n += 1
                        break
    except (OSError, ValueError):
        return 0
    return n


def _default_devices(g):
    """rank r -> GPU r % (visible GPUs)."""
    nd = _visible_gpus()
    return list(range(max(1, min(g, nd)))) if nd else [0]


def _load_factory(spec):
    import importlib

    mod, _, fn = spec.partition(":")
    return getattr(importlib.import_module(mod), fn)


def _bind_numa(device):
    """Best effort: run this worker on the host CPUs of its GPU's NUMA node (sysfs), so its
    reader threads and the first touch of its pinned slabs are node-local.  The PCI address
    comes from the HIP runtime libpfe already loaded (no torch in a worker: its import and
    device setup cost seconds per process)."""
    try:
        import ctypes

        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, int(device)) != 0:
            return None
        bus = buf.value.decode().lower()
        with open(f"/sys/bus/pci/devices/{bus}/numa_node") as f:
            node = int(f.read().strip())
        if node < 0:
            return None
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            spec = f.read().strip()
        cpus = set()
        for part in spec.split(","):
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
        mine = cpus & os.sched_getaffinity(0)
        if mine:
            os.sched_setaffinity(0, mine)
            return node
    except Exception:  # noqa: BLE001
        return None
    return None


def _shard_worker(conn, kw, flags, entry, args, rank, suffix, device, engine_spec,
                  slabs_spec):
    """One shard of a --gpus N run (a spawned process): opens its engine on `device`, then
    receives its paths from the parent and runs a single-GPU DataProcessor over them, its files
    suffixed; sends {"ok", "failed", "metrics"} back."""
    import traceback

    t0 = time.perf_counter()
    try:
        if engine_spec:
            engine = _load_factory(engine_spec)()
        else:
            from .candidate import set_engine
            from ._native import Engine

            engine = Engine(device)
            _bind_numa(device)
            set_engine(engine)
        init_s = time.perf_counter() - t0  # interpreter imports done: the engine's start
        paths = conn.recv()
        dp = DataProcessor(engine=engine, log=lambda *a: print(f"[shard {rank}]", *a), **kw)
        if slabs_spec:
            dp._slabs = _load_factory(slabs_spec)()
        dp.candidateErrorLog = "CandidateErrorLog.txt" + suffix
        for k, v in flags.items():
            setattr(dp, k, v)
        dp._shard = (rank, suffix, paths)
        counts = {}
        real = dp._summary

        def capture(processed, ok, failed, start, extra="", run=None):
            counts["ok"], counts["failed"] = ok, failed
            real(processed, ok, failed, start, extra, run)

        dp._summary = capture
        getattr(dp, entry)(*args)
        conn.send({"ok": counts.get("ok", 0), "failed": counts.get("failed", 0),
                   "metrics": dp.metrics, "engine_start_s": init_s})
    except BaseException:  # noqa: BLE001 -- reported to the parent
        conn.send({"error": f"shard {rank}:\n" + traceback.format_exc()})
    finally:
        conn.close()
