"""Score writers with the reference's exact text semantics.

Reference (PulsarFeatureExtractor/src/DataProcessor.py):
  storeScore          :305-325  "<candidate>,v1,...,vn" then "nan"->"0", "inf"->"0"
  storeScoreARFF      :405-425  "v1,...,vn,?%<candidate>" then the same replacements
  outputScores        :429-447  "<candidate>.dat" holding "v1,...,vn"
  prepareARFFFile     :329-367  22 / 64 / 128 score attributes + class {0,1}
  prepareDMProfileARFFFile :369-401  the 8 Lyon attributes + class {0,1}
  processCollectively :590-594  one append of all buffered lines at the end

Values are formatted like Python 2.7's ``str(float)`` (the reference's interpreter,
.pydevproject:6): ``'%.12g'`` with ".0" appended to integral results; nan/inf/-inf as
'nan'/'inf'/'-inf', which the replacements turn into '0' (and '-0').
"""
from __future__ import annotations

import datetime
import math
import os


def py2_str(x) -> str:
    """Python 2.7 str() of a float (12 significant digits).

    Pinned by CPython 2.7's definition rather than by Python-2-written files (none ship with
    the reference, and no Python 2 is available here): float_str is
    PyOS_double_to_string(v, 'g', 12, Py_DTSF_ADD_DOT_0) -- correctly rounded '%.12g' with
    ".0" appended when the text has neither a point nor an exponent; tests/test_writers.py
    holds the edge cases (integral values, -0.0, 12/13-digit integers, 1e-05, subnormals)."""
    x = float(x)
    if math.isnan(x):
        return "nan"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    s = "%.12g" % x
    if "." not in s and "e" not in s and "n" not in s:
        s += ".0"
    return s


def py2_scalar_str(x) -> str:
    """Python-2 str() of a numpy scalar as the label writer meets them: integers as
    integers (the PHCX DM-curve data, PHCXOperations.getDM_FFT :279-293), float64 as
    py2_str, float32 (the PFD chi^2 curve, PFDFile.py:393) as the numpy of the reference's
    Python 2 era formats a float32 scalar's str(): '%.6g' (its FLOATPREC_STR; repr used 8
    digits) with ".0" appended to integral text.  Parity unpinned: the golden label files
    were written under Python 3, whose str() of a float32 is the shortest repr, so
    tests/test_label_gpu.py compares that column to 6 significant digits."""
    import numpy as np

    if isinstance(x, (int, np.integer)):
        return str(int(x))
    if isinstance(x, np.float32):
        v = float(x)
        if math.isnan(v):
            return "nan"
        if math.isinf(v):
            return "inf" if v > 0 else "-inf"
        s = "%.6g" % v
        if "." not in s and "e" not in s:
            s += ".0"
        return s
    return py2_str(x)


def _clean(s: str) -> str:
    return s.replace("nan", "0").replace("inf", "0")


def score_line(candidate: str, scores) -> str:
    """DataProcessor.storeScore (:321-325)."""
    return _clean(candidate + "," + ",".join(py2_str(v) for v in scores))


def arff_line(candidate: str, scores) -> str:
    """DataProcessor.storeScoreARFF (:421-425)."""
    return _clean(",".join(py2_str(v) for v in scores) + ",?%" + candidate)


def dat_text(scores) -> str:
    """DataProcessor.outputScores (:443-446)."""
    return _clean(",".join(py2_str(v) for v in scores))


def arff_header(kind: str = "scores", n_attributes: int = 22, now=None) -> str:
    """prepareARFFFile (:342-360) / prepareDMProfileARFFFile (:382-394)."""
    dt = (now or datetime.datetime.now()).isoformat()
    h = "@relation PulsarCandidates_" + dt + "\n"
    if kind == "dmprof":
        for a in ("Profile_mean", "Profile_stdev", "Profile_skewness", "Profile_kurtosis",
                  "DM_mean", "DM_stdev", "DM_skewness", "DM_kurtosis"):
            h += "@attribute " + a + " numeric\n"
    else:
        for n in range(1, n_attributes + 1):
            h += "@attribute Score" + str(n) + " numeric\n"
    h += "@attribute class {0,1}\n@data\n"
    return h


def append_text(path: str, text: str) -> None:
    """Utilities.appendToFile: append (create if missing)."""
    with open(path, "a") as f:
        f.write(text)


def write_arff_header(path: str, header: str) -> None:
    """The reference writes the header to a new file, or appends it to an existing one."""
    if not os.path.exists(path):
        with open(path, "w+") as f:
            f.write(header)
    else:
        append_text(path, header)
