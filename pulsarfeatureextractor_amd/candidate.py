"""Drop-in mirrors of the reference's per-candidate plug-in API, backed by libpfe.

Reference classes (PulsarFeatureExtractor/src/) and what replaces them here:
  Candidate               Candidate.py:42-547        -> Candidate (same methods, same dispatch)
  CandidateFileInterface  CandidateFileInterface.py  -> CandidateFileInterface (filterScore,
                                                        isEqual, numberOfScores, epsilon)
  PHCX / SUPERBPHCX       PHCXFile.py, SUPERBPHCXFile.py -> PHCXFile / SUPERBPHCXFile
  PFD                     PFDFile.py                 -> PFDFile (pfe_pfd_dmprof, pfe_pfd_bates22)

Score values come from the gfx950 kernels through the C-ABI (a batch of one candidate
here; pulsarfeatureextractor_amd.processor batches whole directories).  As in the reference,
a candidate whose scoring would have raised raises ``Exception`` with the reference's
message for that score group.
"""
from __future__ import annotations

import threading

import numpy as np

from . import pfd as _pfd
from . import phcx as _phcx
from ._native import (PFE_ST_DMFIT_FAIL, PFE_ST_GAUSS_FAIL, PFE_ST_SINE_FAIL,
                      PFE_ST_SUBBAND_FAIL, Engine)

_engine = None
_engine_lock = threading.Lock()


def get_engine(device: int = 0) -> Engine:
    """Process-wide default engine (lazily created on `device`)."""
    global _engine
    with _engine_lock:
        if _engine is None:
            _engine = Engine(device)
        return _engine


def set_engine(engine: Engine) -> None:
    global _engine
    with _engine_lock:
        _engine = engine


# status bit -> the exception text the reference raises for that score group
GROUP_ERRORS = (
    (PFE_ST_SINE_FAIL, "Sinusoid fitting exception"),          # PHCXFile.py:470
    (PFE_ST_GAUSS_FAIL, "Gaussian fitting exception"),         # :543
    (PFE_ST_DMFIT_FAIL, "DM curve fitting exception"),         # :629
    (PFE_ST_SUBBAND_FAIL, "Subband scoring exception"),        # :668
    (0x010, "Unsupported candidate shape"),
)


def status_error(st: int) -> str | None:
    for bit, msg in GROUP_ERRORS:
        if st & bit:
            return msg
    return None


def band_sum(rows):
    """PHCXOperations.getSubbandData / getSubintData post-processing (:440-464), with the
    reference's statements kept: ``sum_ = [0] * 128`` then ``sum_ += row - mean(row)`` per
    row.  Python tries the number protocol before list concatenation, so the first ``+=``
    turns the list into ndarray.__radd__'s float64 array and the rows are summed element by
    element in order (a row of another length raises, as in the reference); then negatives
    become 0.0.  Pinned by tests/golden/getters_phcx128.npz.  Host data getter (no score is
    computed from it; the reference's callers are commented out, DataProcessor.py:749-750)."""
    out = [0] * 128
    for r in np.asarray(rows):
        r = np.asarray(r)
        out += r - np.mean(r)
    for i in range(len(out)):
        if out[i] < 0:
            out[i] = 0.0
    return out


class CandidateFileInterface:
    """CandidateFileInterface.py:38-194 — per-format scorer interface."""

    def __init__(self, debugFlag=False):
        self.debug = debugFlag
        self.numberOfScores = 22          # :63
        self.epsilon = 0.000005           # :64

    def setNumberOfScores(self, n):
        self.numberOfScores = int(n)

    def filterScore(self, s, value):
        """:84-112 — scores 13/14 below -epsilon become 0.0; score 18 is made absolute."""
        if s == 13 or s == 14:
            return 0.0 if self.isEqual(value, 0.0, self.epsilon) == -1 else value
        if s == 18:
            return float(abs(value))
        return value

    def isEqual(self, a, b, epsln):
        """:116-149"""
        if abs(a - b) > epsln:
            return -1 if a < b else 1
        return 0

    # abstract API (:153-194)
    def compute(self):
        raise NotImplementedError("Please Implement this method")

    def load(self):
        raise NotImplementedError("Please Implement this method")

    def getProfile(self):
        raise NotImplementedError("Please Implement this method")

    def isValid(self):
        raise NotImplementedError("Please Implement this method")


class PHCXFile(CandidateFileInterface):
    """PHCXFile.PHCX (gzip, section 1); SUPERBPHCXFile subclasses with superb=True."""

    SUPERB = False

    def __init__(self, debugFlag, candidateName, engine: Engine | None = None):
        super().__init__(debugFlag)
        self.cand = candidateName
        self.profileIndex = 0 if self.SUPERB else 1
        self.scores = []
        self._engine = engine
        self.setNumberOfScores(22)
        self.load()

    def load(self):
        self.data = _phcx.parse(self.cand, superb=self.SUPERB)
        self.profile = np.asarray(self.data.profile)

    def getprofile(self):
        return [int(v) for v in self.data.profile]

    def isValid(self):
        """PHCXFile.isValid (:190-287) on the parsed arrays."""
        d = self.data
        nb = 64 if self.SUPERB else 128
        return (len(d.profile) > 50 and d.subbands.shape == (16, nb) and len(d.dm_curve) > 0)

    @property
    def engine(self):
        return self._engine or get_engine()

    def _bates(self):
        d = self.data
        out, st = self.engine.bates22(d.profile[None, :].astype(np.uint8),
                                      d.subbands[None, :, :].astype(np.uint8),
                                      d.dm_curve[None, :], d.scal[None, :])
        msg = status_error(int(st[0]))
        if msg:
            raise Exception(msg)
        return [float(v) for v in out[0]]

    def compute(self):
        """PHCXFile.compute (:383-409): the 22 scores."""
        self.scores = self._bates()
        return self.scores

    def computeProfileScores(self):
        """:291-304 — the profile bins as float scores (--profile)."""
        self.scores = [float(v) for v in self.data.profile]
        return self.scores

    def _lyon8(self):
        """The 8 Lyon features of this candidate -- profile and section-0 DataBlock -- from
        one pfe_lyon8_u8 call, kept for the second of the two stat-score calls."""
        if getattr(self, "_l8", None) is None:
            p = np.ascontiguousarray(np.asarray(self.data.profile, dtype=np.uint8)[None, :])
            d = np.ascontiguousarray(np.asarray(self.data.lyon_dm, dtype=np.uint8)[None, :])
            self._l8 = [float(v) for v in self.engine.lyon8(p, d)[0]]
        return self._l8

    def computeProfileStatScores(self):
        """:320-349 — [mean, std, skew, kurtosis] of the profile."""
        return self._lyon8()[:4]

    def computeDMCurveStatScores(self):
        """:351-379 — the same statistics of the section-0 DataBlock."""
        return self._lyon8()[4:]

    def getDMCurveData(self):
        """:306-318 — the decoded section-0 DataBlock."""
        return np.asarray(self.data.lyon_dm)

    def getSubbandData(self):
        """:704-716 -> PHCXOperations.getSubbandData (:422-464)."""
        return band_sum(_phcx.band_rows(self.cand, "SubBands", self.SUPERB))

    def getSubintData(self):
        """:688-700 -> PHCXOperations.getSubintData (:468-505)."""
        return band_sum(_phcx.band_rows(self.cand, "SubIntegrations", self.SUPERB))


class SUPERBPHCXFile(PHCXFile):
    """SUPERBPHCXFile.SUPERBPHCX: plain XML, section 0, 64-bin (SUPERBPHCXFile.py:80,103)."""

    SUPERB = True


class PFDFile(CandidateFileInterface):
    """PFDFile.PFD (PFDFile.py:64-875): a PRESTO fold read on the host (pfd.read, :96-252),
    scored through pfe_pfd_bates22 / pfe_pfd_dmprof."""

    def __init__(self, debugFlag, candidateName, engine=None):
        super().__init__(debugFlag)
        self.cand = candidateName
        self.engine = engine or get_engine()
        self.data = _pfd.read(candidateName)
        self.scores = []

    def _batch(self):
        return _pfd.batch_inputs([self.data])

    def _dmprof(self):
        """pfe_pfd_dmprof of this fold (profile, chi^2 curve, Lyon features), launched once
        and shared by the profile / DM-curve / stat-score calls."""
        if getattr(self, "_dmp", None) is None:
            profs, subfreqs, scal = self._batch()
            self._dmp = self.engine.pfd_dmprof(profs, subfreqs, scal)
        return self._dmp

    def isValid(self):
        return self.data.proflen > 0 and self.data.numchan > 0          # :460-475

    def getProfile(self):
        return self._dmprof()["profile"][0]

    def compute(self):
        """PFDFile.compute (:587-613): the 22 scores."""
        out, st = self.engine.pfd_bates22(*self._batch())
        msg = status_error(int(st[0]))
        if msg:
            raise Exception(msg)
        self.scores = [float(v) for v in out[0]]
        return self.scores

    def computeProfileScores(self):
        """:479-492 — the 0..255 profile bins."""
        self.scores = [float(v) for v in self.getProfile()]
        return self.scores

    def computeProfileStatScores(self):
        """:522-551"""
        return [float(v) for v in self._dmprof()["lyon8"][0, :4]]

    def computeDMCurveStatScores(self):
        """:553-583"""
        r = self._dmprof()
        if int(r["status"][0]) & 0x20:
            raise Exception("DM curve stat score extraction exception")
        return [float(v) for v in r["lyon8"][0, 4:]]

    def getDMCurveData(self):
        """:494-520 — the float32 chi^2-vs-DM curve."""
        r = self._dmprof()
        if int(r["status"][0]) & 0x20:
            raise Exception("DM curve extraction exception")
        return r["chis"][0]


class Candidate:
    """Candidate.py:42-547 with the same methods and file-name dispatch (:136-150)."""

    def __init__(self, name="Unknown", path=""):
        self.candidateName = name
        self.candidatePath = path
        self.scores = []
        self.label = "Unknown"
        self.specialScore = -1
        self.special = "None"

    def _file(self, verbose):
        """The candidate's file object (Candidate.py:136-150 dispatch), parsed once and kept:
        the reference re-reads the file for every calculate* call (:218, :278); here
        calculateProfileStatScores and calculateDMCurveStatScores share one parse and one
        Lyon-8 launch."""
        f = getattr(self, "_cand_file", None)
        if f is None:
            if ".pfd" in self.candidateName:
                f = PFDFile(verbose, self.candidateName)
            elif ".gz" in self.candidateName:
                f = PHCXFile(verbose, self.candidateName)
            else:
                f = SUPERBPHCXFile(verbose, self.candidateName)
            self._cand_file = f
        return f

    def addScores(self, lineFromFile):
        for s in lineFromFile.split(","):
            if s != "" or len(s) != 0:
                self.scores.append(float(s))

    def calculateScores(self, verbose):
        self.scores = self._file(verbose).compute()
        return self.scores

    def calculateProfileScores(self, verbose):
        self.scores = self._file(verbose).computeProfileScores()
        return self.scores

    def calculateProfileStatScores(self, verbose):
        self.scores = self._file(verbose).computeProfileStatScores()
        return self.scores

    def calculateDMCurveStatScores(self, verbose):
        self.scores = self._file(verbose).computeDMCurveStatScores()
        return self.scores

    def getDMCurveData(self, verbose):
        """Candidate.py:231-255: PFD and gzipped PHCX files; [] for SUPERB PHCX."""
        if ".pfd" not in self.candidateName and ".gz" not in self.candidateName:
            return []
        self.scores = self._file(verbose).getDMCurveData()
        return self.scores

    def getSubbandData(self, verbose):
        """Candidate.py:290-313: gzipped PHCX files only; [] for PFD and SUPERB PHCX."""
        if ".pfd" in self.candidateName or ".gz" not in self.candidateName:
            return []
        self.scores = self._file(verbose).getSubbandData()
        return self.scores

    def getSubintData(self, verbose):
        """Candidate.py:317-340: gzipped PHCX files only; [] for PFD and SUPERB PHCX."""
        if ".pfd" in self.candidateName or ".gz" not in self.candidateName:
            return []
        self.scores = self._file(verbose).getSubintData()
        return self.scores

    def getScore(self, index):
        return float(self.scores[index - 1])

    def getName(self):
        return self.candidateName

    def getPath(self):
        return self.candidatePath

    def setLabel(self, l):
        self.label = l

    def getLabel(self):
        return self.label

    def isPulsar(self):
        return self.label == "POSITIVE"

    def setSpecialScore(self, special):
        try:
            self.specialScore = int(special)
        except Exception:
            self.specialScore = -1

    def getSpecialScore(self):
        return int(self.specialScore)

    def setScores(self, data):
        self.scores = [float(i) for i in data]

    def setSpecial(self, s):
        self.special = str(s)

    def getSpecial(self):
        return str(self.special)

    def __str__(self):
        return self.candidateName + "," + self.candidatePath
