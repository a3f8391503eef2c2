"""ORACLE (test infrastructure only) — ctypes binding of oracle/c/lyon8_omp.c, the C
restatement of the 8 Lyon features with OpenMP over candidates (the
multi-core CPU baseline).  Only tests/ and bench.py's cpu_baseline leg use it; built by
`make -C oracle` (called from __graft_entry__.build())."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_c", "liblyon8_omp.so")
_lib = None


def available() -> bool:
    return os.path.exists(_LIB)


def _load():
    global _lib
    if _lib is None:
        _lib = C.CDLL(_LIB)
        f = _lib.pfe_oracle_lyon8_u8
        f.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_longlong, C.c_void_p, C.c_int]
        f.restype = C.c_int
    return _lib


def lyon8_omp(prof: np.ndarray, dm: np.ndarray, threads: int = 1) -> np.ndarray:
    """(n, lp) and (n, ld) uint8 rows -> (n, 8) float64 [mean, std, skew, kurt] x 2."""
    prof = np.ascontiguousarray(prof, dtype=np.uint8)
    dm = np.ascontiguousarray(dm, dtype=np.uint8)
    n = prof.shape[0]
    out = np.empty((n, 8), dtype=np.float64)
    rc = _load().pfe_oracle_lyon8_u8(prof.ctypes.data, prof.shape[1], dm.ctypes.data, dm.shape[1],
                                     n, out.ctypes.data, threads)
    if rc != 0:
        raise ValueError("pfe_oracle_lyon8_u8 rejected its arguments")
    return out
