"""ctypes binding of libpfe.so (the C-ABI declared in include/pfe.h).

This is the reference-side binding a maintainer would add to PulsarFeatureExtractor: a thin
ctypes layer over the extern "C" entry points.  It never falls back to a CPU
implementation: if the library is missing or no GPU is visible, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PFE_LIBRARY", os.path.join(_HERE, "lib", "libpfe.so"))

PFE_OK = 0
PFE_FLAG_DEVICE_PTRS = 0x1
PFE_NSCAL = 8
PFE_ST_FAIL_MASK = 0x0FF
PFE_ST_SINE_FAIL = 0x001
PFE_ST_GAUSS_FAIL = 0x002
PFE_ST_DMFIT_FAIL = 0x004
PFE_ST_SUBBAND_FAIL = 0x008
PFE_ST_UNSUPPORTED = 0x010
PFE_ST_DGF_INDEXERROR = 0x100

# every symbol include/pfe.h declares (checked by tests/test_capi_symbols.py)
EXPORTED_SYMBOLS = (
    "pfe_abi_version",
    "pfe_device_count",
    "pfe_create",
    "pfe_destroy",
    "pfe_last_error",
    "pfe_set_stream",
    "pfe_synchronize",
    "pfe_set_option",
    "pfe_get_option",
    "pfe_host_alloc",
    "pfe_host_free",
    "pfe_lyon8_u8",
    "pfe_lyon8_f64",
    "pfe_bates22",
    "pfe_subband3",
    "pfe_sinusoid4",
    "pfe_gauss7",
    "pfe_params4",
    "pfe_dmfit4",
    "pfe_pfd_dmprof",
    "pfe_pfd_bates22",
)
PFE_PFD_NSCAL = 8
PFE_PFD_NDM = 100
PFE_ST_PFD_DMCURVE_FAIL = 0x020
# every symbol include/pfe_io.h declares
EXPORTED_IO_SYMBOLS = (
    "pfe_phcx_parse",
    "pfe_phcx_count",
    "pfe_phcx_info_get",
    "pfe_phcx_fetch",
    "pfe_phcx_pack",
    "pfe_phcx_free",
    "pfe_phcx_info_all",
    "pfe_format_rows",
)
PFE_PHCX_PROFILE, PFE_PHCX_LYON_DM, PFE_PHCX_SUBBANDS, PFE_PHCX_DM_CURVE, PFE_PHCX_FIT_BLOCK = range(5)
PFE_IO_STATUS = {0: "ok", 1: "open", 2: "gzip", 3: "xml", 4: "value", 5: "range", 6: "shape"}


# handle options (include/pfe.h PFE_OPT_*): name -> (id, default)
OPTIONS = {
    "solver": 1,        # 0 pooled (default), 1 batched, 2 wave per fit
    "serial": 2,
    "handover": 3,
    "gslots": 4,
    "lyon8_blocks": 5,
    "lyon8_burst": 6,
    "pfd_waves": 7,
    "lyon8_dm": 8,      # DataBlock kernels: 0 default, 1 round 3, 2 exact power sums (pfe.h)
    "pfd_split": 9,     # 0 fused kernel (default), 1 part sums streamed beside the sweep
    "lyon8_dm_split": 10,  # 1 (default) chain splits + paired one-chunk rows, 2 splits only, 0 off
}
SOLVERS = {"pooled": 0, "batched": 1, "wave": 2}


class PfeError(RuntimeError):
    """Raised when a libpfe call fails (the message is pfe_last_error())."""


class BatesIn(C.Structure):
    _fields_ = [
        ("prof", C.c_void_p),
        ("lp", C.c_int32),
        ("sub", C.c_void_p),
        ("nsub", C.c_int32),
        ("lsb", C.c_int32),
        ("dmcurve", C.c_void_p),
        ("ndm", C.c_int32),
        ("scal", C.c_void_p),
        ("n", C.c_int64),
    ]


class PfdIn(C.Structure):
    _fields_ = [
        ("profs", C.c_void_p),
        ("subfreqs", C.c_void_p),
        ("scal", C.c_void_p),
        ("npart", C.c_int32),
        ("nsub", C.c_int32),
        ("proflen", C.c_int32),
        ("n", C.c_int64),
    ]


class PhcxInfo(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("superb", C.c_int32),
        ("section", C.c_int32),
        ("lp", C.c_int32),
        ("nsub", C.c_int32),
        ("lsb", C.c_int32),
        ("ndm", C.c_int32),
        ("reserved", C.c_int32),
        ("ld", C.c_int64),
        ("lfit", C.c_int64),
        ("scal", C.c_double * 8),
    ]


# numpy view of pfe_phcx_info (include/pfe_io.h), for pfe_phcx_info_all
PHCX_INFO_DTYPE = np.dtype([
    ("status", "<i4"), ("superb", "<i4"), ("section", "<i4"), ("lp", "<i4"),
    ("nsub", "<i4"), ("lsb", "<i4"), ("ndm", "<i4"), ("reserved", "<i4"),
    ("ld", "<i8"), ("lfit", "<i8"), ("scal", "<f8", (8,)),
])
assert PHCX_INFO_DTYPE.itemsize == C.sizeof(PhcxInfo)

_lib = None
_lock = threading.Lock()


def _preload_torch_hip_runtime():
    """Share ONE HIP runtime with PyTorch.

    torch ships its own libamdhip64.so (soname libamdhip64.so.7).  If libpfe.so resolved
    /opt/rocm's copy first, the process would hold two HIP runtimes and whichever initialises
    second sees no GPU.  Loading torch's copy globally first makes libpfe's NEEDED entry bind
    to it, and torch later recognises the same file (same inode) -- without importing torch.
    """
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return None
    for loc in spec.submodule_search_locations:
        p = os.path.join(loc, "lib", "libamdhip64.so")
        if os.path.exists(p):
            return C.CDLL(p, mode=C.RTLD_GLOBAL)
    return None


def load_library(path: str | None = None) -> C.CDLL:
    """Load libpfe.so and declare its signatures.  Raises OSError when it is missing."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise OSError(
                f"libpfe.so not found at {p}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` "
                "(there is no CPU fallback)"
            )
        if os.environ.get("PFE_SYSTEM_HIP", "0") != "1":
            _preload_torch_hip_runtime()
        lib = C.CDLL(p)
        vp, i32, i64, u32 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32
        lib.pfe_abi_version.restype = C.c_int
        lib.pfe_abi_version.argtypes = []
        lib.pfe_device_count.restype = C.c_int
        lib.pfe_device_count.argtypes = []
        lib.pfe_create.restype = C.c_int
        lib.pfe_create.argtypes = [C.c_int, C.POINTER(vp)]
        lib.pfe_destroy.restype = None
        lib.pfe_destroy.argtypes = [vp]
        lib.pfe_last_error.restype = C.c_char_p
        lib.pfe_last_error.argtypes = [vp]
        lib.pfe_set_stream.restype = C.c_int
        lib.pfe_set_stream.argtypes = [vp, vp]
        lib.pfe_synchronize.restype = C.c_int
        lib.pfe_synchronize.argtypes = [vp]
        lib.pfe_set_option.restype = C.c_int
        lib.pfe_set_option.argtypes = [vp, i32, i64]
        lib.pfe_get_option.restype = C.c_int
        lib.pfe_get_option.argtypes = [vp, i32, C.POINTER(i64)]
        lib.pfe_host_alloc.restype = C.c_int
        lib.pfe_host_alloc.argtypes = [C.c_size_t, C.POINTER(vp)]
        lib.pfe_host_free.restype = None
        lib.pfe_host_free.argtypes = [vp]
        lib.pfe_lyon8_u8.restype = C.c_int
        lib.pfe_lyon8_u8.argtypes = [vp, vp, i64, i32, vp, i64, i32, i64, vp, vp, u32]
        lib.pfe_lyon8_f64.restype = C.c_int
        lib.pfe_lyon8_f64.argtypes = [vp, vp, i64, i32, vp, i64, i32, i64, vp, vp, u32]
        lib.pfe_bates22.restype = C.c_int
        lib.pfe_bates22.argtypes = [vp, C.POINTER(BatesIn), vp, vp, u32]
        lib.pfe_subband3.restype = C.c_int
        lib.pfe_subband3.argtypes = [vp, C.POINTER(BatesIn), vp, vp, u32]
        for g in ("pfe_sinusoid4", "pfe_gauss7", "pfe_params4", "pfe_dmfit4"):
            getattr(lib, g).restype = C.c_int
            getattr(lib, g).argtypes = [vp, C.POINTER(BatesIn), vp, vp, u32]
        lib.pfe_pfd_dmprof.restype = C.c_int
        lib.pfe_pfd_dmprof.argtypes = [vp, C.POINTER(PfdIn), vp, vp, vp, vp, u32]
        lib.pfe_pfd_bates22.restype = C.c_int
        lib.pfe_pfd_bates22.argtypes = [vp, C.POINTER(PfdIn), vp, vp, u32]
        pp = C.POINTER(C.c_char_p)
        lib.pfe_phcx_parse.restype = C.c_int
        lib.pfe_phcx_parse.argtypes = [pp, i64, i32, i32, C.POINTER(vp)]
        lib.pfe_phcx_count.restype = i64
        lib.pfe_phcx_count.argtypes = [vp]
        lib.pfe_phcx_info_get.restype = C.c_int
        lib.pfe_phcx_info_get.argtypes = [vp, i64, C.POINTER(PhcxInfo)]
        lib.pfe_phcx_fetch.restype = C.c_int
        lib.pfe_phcx_fetch.argtypes = [vp, i64, i32, vp, i64]
        lib.pfe_phcx_pack.restype = C.c_int
        lib.pfe_phcx_pack.argtypes = [vp, vp, i64, i32, vp, i64, vp, i64, vp, i64, vp, i64, vp]
        lib.pfe_phcx_free.restype = None
        lib.pfe_phcx_free.argtypes = [vp]
        lib.pfe_phcx_info_all.restype = C.c_int
        lib.pfe_phcx_info_all.argtypes = [vp, vp, i64]
        lib.pfe_format_rows.restype = C.c_int
        lib.pfe_format_rows.argtypes = [vp, vp, vp, i64, i32, i64, i32, vp, i32, vp, i64,
                                        C.POINTER(i64)]
        if path is None:
            _lib = lib
        return lib


def _row_stride(stride, a):
    """Row stride in elements; a single-row array may carry any stride on its row axis
    (numpy's and torch's relaxed strides, e.g. x[None, :] has stride 0): use the row length."""
    return a.shape[1] if a.shape[0] <= 1 else stride


def _ptr(a) -> int:
    """Raw address of a numpy array or a torch tensor (host or device)."""
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return int(a.data_ptr())  # torch.Tensor


def _is_device(a) -> bool:
    if isinstance(a, np.ndarray):
        return False
    return bool(getattr(a, "is_cuda", False))


class _Pinned:
    """Owner of one pfe_host_alloc block; numpy arrays made by Engine.host_empty keep it
    alive as their base and it is freed with the last of them."""

    def __init__(self, lib, nbytes: int):
        self.lib = lib
        p = C.c_void_p()
        if lib.pfe_host_alloc(max(1, int(nbytes)), C.byref(p)) != PFE_OK or not p.value:
            raise MemoryError(f"pfe_host_alloc({nbytes}) failed")
        self.ptr = p.value
        self.nbytes = int(nbytes)
        self.__array_interface__ = {"shape": (self.nbytes,), "typestr": "|u1",
                                    "data": (self.ptr, False), "version": 3}

    def __del__(self):
        if getattr(self, "ptr", None):
            self.lib.pfe_host_free(self.ptr)
            self.ptr = None


def host_empty(shape, dtype=np.uint8) -> np.ndarray:
    """An uninitialised numpy array in pinned host memory (pfe_host_alloc): host-pointer
    engine calls DMA such buffers in place instead of staging them."""
    lib = load_library()
    dt = np.dtype(dtype)
    shape = tuple(int(v) for v in np.atleast_1d(shape))
    nbytes = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
    raw = np.asarray(_Pinned(lib, nbytes))
    return raw.view(dt).reshape(shape) if nbytes else np.empty(shape, dtype=dt)


class Engine:
    """One libpfe handle: a GPU ordinal plus a HIP stream.

    Arguments may be numpy arrays (host; the call stages and synchronises) or torch CUDA
    tensors (device; the call is asynchronous on torch's current stream).  Mixed placements
    are rejected, and device tensors are checked for dtype, shape, contiguity and device
    before any pointer reaches the library.
    """

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = C.c_void_p()
        rc = self.lib.pfe_create(int(device), C.byref(h))
        if rc != PFE_OK:
            raise PfeError(self.lib.pfe_last_error(None).decode())
        self._h = h
        self.device = device

    # -- lifecycle -----------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self.lib.pfe_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int):
        if rc != PFE_OK:
            raise PfeError(self.lib.pfe_last_error(self._h).decode())

    def set_stream(self, stream_handle: int | None):
        """Launch on an external hipStream_t (e.g. a torch.cuda.Stream's ``cuda_stream``;
        0/None is the HIP default stream)."""
        self._check(self.lib.pfe_set_stream(self._h, stream_handle or None))

    def _follow_torch(self):
        """Device-tensor calls run on torch's current stream, so they are ordered after the
        kernels that produced their inputs and before the ones that consume the outputs."""
        import torch

        self.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def synchronize(self):
        self._check(self.lib.pfe_synchronize(self._h))

    # -- options -------------------------------------------------------------------------
    def set_option(self, name: str, value):
        """pfe_set_option: name in OPTIONS ('solver' also takes 'pooled'/'batched'/'wave')."""
        if name == "solver" and isinstance(value, str):
            value = SOLVERS[value]
        self._check(self.lib.pfe_set_option(self._h, OPTIONS[name], int(value)))

    def get_option(self, name: str) -> int:
        v = C.c_int64()
        self._check(self.lib.pfe_get_option(self._h, OPTIONS[name], C.byref(v)))
        return int(v.value)

    def options(self, **kw):
        """Context manager: set options for a block, restore the previous values after."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            old = {k: self.get_option(k) for k in kw}
            try:
                for k, v in kw.items():
                    self.set_option(k, v)
                yield self
            finally:
                for k, v in old.items():
                    self.set_option(k, v)

        return cm()

    # -- argument checks of the device path ----------------------------------------------
    def _dev(self, t, name, dtypes, shape=None, rows_contig=False):
        import torch

        if not isinstance(t, torch.Tensor) or not t.is_cuda:
            raise TypeError(f"{name}: expected a CUDA tensor (all arguments device or all host)")
        if t.dtype not in dtypes:
            raise TypeError(f"{name}: dtype {t.dtype}, expected one of {tuple(dtypes)}")
        if t.device.index != self.device:
            raise ValueError(f"{name}: on cuda:{t.device.index}, engine is on cuda:{self.device}")
        if shape is not None and tuple(t.shape) != tuple(shape):
            raise ValueError(f"{name}: shape {tuple(t.shape)}, expected {tuple(shape)}")
        if rows_contig:
            if t.dim() != 2 or t.stride(1) != 1 or t.stride(0) < t.shape[1]:
                raise ValueError(f"{name}: rows must be contiguous (stride(1) == 1)")
        elif not t.is_contiguous():
            raise ValueError(f"{name}: device tensors must be contiguous")
        return t

    def _status_dev(self, status, n):
        import torch

        if status is None:
            return torch.empty((n,), dtype=torch.int32, device=f"cuda:{self.device}")
        return self._dev(status, "status", (torch.int32,), (n,))

    @staticmethod
    def _status_host(status, n):
        if status is None:
            return np.empty((n,), dtype=np.uint32)
        if not isinstance(status, np.ndarray) or status.dtype.itemsize != 4 or \
                status.dtype.kind not in "iu" or status.shape != (n,) or not status.flags.c_contiguous:
            raise ValueError("status must be a contiguous (n,) 4-byte integer array")
        return status

    @staticmethod
    def _out_host(out, n, width):
        if out is None:
            return np.empty((n, width), dtype=np.float64)
        if not isinstance(out, np.ndarray) or out.dtype != np.float64 or out.shape != (n, width) \
                or not out.flags.c_contiguous:
            raise ValueError(f"out must be a contiguous ({n}, {width}) float64 array")
        return out

    # -- 8 Lyon features -----------------------------------------------------------------
    def lyon8(self, prof, dm, out=None, status=None):
        """[mean,std,skew,kurt] of each profile row then each DM row -> (n, 8) float64."""
        if prof.ndim != 2 or dm.ndim != 2 or prof.shape[0] != dm.shape[0]:
            raise ValueError("prof and dm must be 2-D with the same number of rows")
        n = prof.shape[0]
        dev = _is_device(prof)
        if dev != _is_device(dm):
            raise ValueError("prof and dm must both be host arrays or both device tensors")
        if dev:
            import torch

            self._dev(prof, "prof", (torch.uint8, torch.float64), rows_contig=True)
            self._dev(dm, "dm", (prof.dtype,), rows_contig=True)
            kind = "u8" if prof.dtype == torch.uint8 else "f64"
            self._follow_torch()
            if out is None:
                out = torch.empty((n, 8), dtype=torch.float64, device=prof.device)
            self._dev(out, "out", (torch.float64,), (n, 8))
            if status is not None:
                self._status_dev(status, n)
            ps, ds = _row_stride(prof.stride(0), prof), _row_stride(dm.stride(0), dm)
            flags = PFE_FLAG_DEVICE_PTRS
        else:
            if prof.dtype == np.uint8 and dm.dtype == np.uint8:
                kind = "u8"
            elif prof.dtype == np.float64 and dm.dtype == np.float64:
                kind = "f64"
            else:
                raise TypeError("lyon8: rows must be uint8 or float64 (same dtype)")
            prof = prof if prof.strides[1] == prof.itemsize else np.ascontiguousarray(prof)
            dm = dm if dm.strides[1] == dm.itemsize else np.ascontiguousarray(dm)
            ps = _row_stride(prof.strides[0] // prof.itemsize, prof)
            ds = _row_stride(dm.strides[0] // dm.itemsize, dm)
            out = self._out_host(out, n, 8)
            if status is not None:
                self._status_host(status, n)
            flags = 0
        fn = self.lib.pfe_lyon8_u8 if kind == "u8" else self.lib.pfe_lyon8_f64
        st = None if status is None else _ptr(status)
        self._check(
            fn(self._h, _ptr(prof), ps, prof.shape[1], _ptr(dm), ds, dm.shape[1], n,
               _ptr(out), st, flags)
        )
        return out

    # -- 22 Bates scores / sub-band scores -----------------------------------------------
    def _bates_args(self, prof, sub, dmcurve, scal, with_dm):
        n = prof.shape[0]
        if prof.ndim != 2 or sub.ndim != 3 or scal.ndim != 2 or scal.shape[1] != PFE_NSCAL:
            raise ValueError("prof must be (n,lp), sub (n,nsub,lsb), scal (n,%d)" % PFE_NSCAL)
        if sub.shape[0] != n or scal.shape[0] != n or (with_dm and dmcurve.shape[0] != n):
            raise ValueError("inputs must have the same number of rows")
        if with_dm and dmcurve.ndim != 2:
            raise ValueError("dmcurve must be (n, ndm)")
        dev = _is_device(prof)
        if dev:
            import torch

            self._dev(prof, "prof", (torch.uint8,))
            self._dev(sub, "sub", (torch.uint8,))
            self._dev(scal, "scal", (torch.float64,))
            if with_dm:
                self._dev(dmcurve, "dmcurve", (torch.float64,))
            self._follow_torch()
        else:
            prof = np.ascontiguousarray(prof, dtype=np.uint8)
            sub = np.ascontiguousarray(sub, dtype=np.uint8)
            scal = np.ascontiguousarray(scal, dtype=np.float64)
            if with_dm:
                dmcurve = np.ascontiguousarray(dmcurve, dtype=np.float64)
        bi = BatesIn(
            _ptr(prof), prof.shape[1], _ptr(sub), sub.shape[1], sub.shape[2],
            _ptr(dmcurve) if with_dm else None, dmcurve.shape[1] if with_dm else 0,
            _ptr(scal), n,
        )
        return bi, dev, (prof, sub, dmcurve, scal)

    def bates22(self, prof, sub, dmcurve, scal, out=None, status=None):
        """22 scores per candidate -> ((n, 22) float64, (n,) status)."""
        bi, dev, keep = self._bates_args(prof, sub, dmcurve, scal, True)
        n = bi.n
        if dev:
            import torch

            if out is None:
                out = torch.empty((n, 22), dtype=torch.float64, device=prof.device)
            self._dev(out, "out", (torch.float64,), (n, 22))
            status = self._status_dev(status, n)
            flags = PFE_FLAG_DEVICE_PTRS
        else:
            out = self._out_host(out, n, 22)
            status = self._status_host(status, n)
            flags = 0
        self._check(self.lib.pfe_bates22(self._h, C.byref(bi), _ptr(out), _ptr(status), flags))
        del keep
        return out, status

    def subband3(self, prof, sub, scal, out=None, status=None):
        """Scores 20-22 alone (pfe_subband3, PHCXOperations.getSubbandParameters):
        -> ((n, 3) float64, (n,) status)."""
        bi, dev, keep = self._bates_args(prof, sub, None, scal, False)
        n = bi.n
        if dev:
            import torch

            if out is None:
                out = torch.empty((n, 3), dtype=torch.float64, device=prof.device)
            self._dev(out, "out", (torch.float64,), (n, 3))
            status = self._status_dev(status, n)
            flags = PFE_FLAG_DEVICE_PTRS
        else:
            out = self._out_host(out, n, 3)
            status = self._status_host(status, n)
            flags = 0
        self._check(self.lib.pfe_subband3(self._h, C.byref(bi), _ptr(out), _ptr(status), flags))
        del keep
        return out, status

    # ---- one score group (ProfileOperationsInterface.py:69-130; pfe.h per-group block) ----
    def _group(self, fn, k, prof, dmcurve, scal, out, status):
        n = scal.shape[0]
        dev = _is_device(scal)
        if dev:
            import torch

            for a, nm in ((prof, "prof"), (dmcurve, "dmcurve")):
                if a is not None:
                    self._dev(a, nm, (torch.uint8,) if nm == "prof" else (torch.float64,))
            self._dev(scal, "scal", (torch.float64,))
            self._follow_torch()
            if out is None:
                out = torch.empty((n, k), dtype=torch.float64, device=scal.device)
            self._dev(out, "out", (torch.float64,), (n, k))
            status = self._status_dev(status, n)
            flags = PFE_FLAG_DEVICE_PTRS
        else:
            prof = None if prof is None else np.ascontiguousarray(prof, dtype=np.uint8)
            dmcurve = None if dmcurve is None else np.ascontiguousarray(dmcurve, dtype=np.float64)
            scal = np.ascontiguousarray(scal, dtype=np.float64)
            out = self._out_host(out, n, k)
            status = self._status_host(status, n)
            flags = 0
        for a in (prof, dmcurve):
            if a is not None and a.shape[0] != n:
                raise ValueError("inputs must have the same number of rows")
        bi = BatesIn(_ptr(prof) if prof is not None else None, prof.shape[1] if prof is not None else 0,
                     None, 0, 0, _ptr(dmcurve) if dmcurve is not None else None,
                     dmcurve.shape[1] if dmcurve is not None else 0, _ptr(scal), n)
        self._check(getattr(self.lib, fn)(self._h, C.byref(bi), _ptr(out), _ptr(status), flags))
        return out, status

    def sinusoid4(self, prof, scal, out=None, status=None):
        """getSinusoidFittings (pfe_sinusoid4): s1-s4 -> ((n, 4), (n,) status)."""
        return self._group("pfe_sinusoid4", 4, prof, None, scal, out, status)

    def gauss7(self, prof, scal, out=None, status=None):
        """getGaussianFittings (pfe_gauss7): s5-s11 -> ((n, 7), (n,) status)."""
        return self._group("pfe_gauss7", 7, prof, None, scal, out, status)

    def params4(self, scal, out=None, status=None):
        """getCandidateParameters (pfe_params4): [period_ms, snr, dm, width], unfiltered."""
        return self._group("pfe_params4", 4, None, None, scal, out, status)

    def dmfit4(self, dmcurve, scal, out=None, status=None):
        """getDMFittings (pfe_dmfit4): [peak, |1 - Prop|, Shift (signed), chi_theo]."""
        return self._group("pfe_dmfit4", 4, None, dmcurve, scal, out, status)

    def features30(self, prof, lyon_dm, sub, dmcurve, scal, out=None):
        """Config 5's feature matrix: the 8 Lyon features (profile + Lyon DM rows) then the
        22 Bates scores of each candidate -> ((n, 30) float64, (n,) status)."""
        n = prof.shape[0]
        dev = _is_device(prof)
        if dev:
            import torch

            if out is None:
                out = torch.empty((n, 30), dtype=torch.float64, device=prof.device)
            self._dev(out, "out", (torch.float64,), (n, 30))
            o8 = self.lyon8(prof, lyon_dm)
            o22, st = self.bates22(prof, sub, dmcurve, scal)
            out[:, :8].copy_(o8)
            out[:, 8:].copy_(o22)
        else:
            out = self._out_host(out, n, 30)
            out[:, :8] = self.lyon8(prof, lyon_dm)
            o22, st = self.bates22(prof, sub, dmcurve, scal)
            out[:, 8:] = o22
        return out, st

    # -- PFD -----------------------------------------------------------------------------
    def _pfd_args(self, profs, subfreqs, scal, fn):
        if profs.ndim != 4:
            raise ValueError(f"{fn}: profs must be (n,npart,nsub,L)")
        n, npart, nsub, L = profs.shape
        if tuple(subfreqs.shape) != (n, nsub) or tuple(scal.shape) != (n, PFE_PFD_NSCAL):
            raise ValueError(f"{fn}: subfreqs must be (n,nsub), scal (n,{PFE_PFD_NSCAL})")
        dev = _is_device(profs)
        if dev:
            import torch

            self._dev(profs, "profs", (torch.float64,))
            self._dev(subfreqs, "subfreqs", (torch.float64,))
            self._dev(scal, "scal", (torch.float64,))
            self._follow_torch()
        else:
            profs = np.ascontiguousarray(profs, dtype=np.float64)
            subfreqs = np.ascontiguousarray(subfreqs, dtype=np.float64)
            scal = np.ascontiguousarray(scal, dtype=np.float64)
        pin = PfdIn(_ptr(profs), _ptr(subfreqs), _ptr(scal), npart, nsub, L, n)
        return pin, dev, (profs, subfreqs, scal)

    def pfd_dmprof(self, profs, subfreqs, scal, profile=True, chis=True, lyon8=True):
        """PFD preprocessing + Lyon features (pfe_pfd_dmprof) for a batch of folds of one
        shape: profs (n,npart,nsub,L) f64, subfreqs (n,nsub), scal (n,PFE_PFD_NSCAL).
        Returns dict(profile (n,L) f64, chis (n,100) f32, lyon8 (n,8) f64, status (n,))."""
        pin, dev, keep = self._pfd_args(profs, subfreqs, scal, "pfd_dmprof")
        n, L = pin.n, pin.proflen
        out = {}
        if dev:
            import torch

            mk = lambda shape, dt: torch.empty(shape, dtype=dt, device=profs.device)  # noqa: E731
            f64, f32, i32 = torch.float64, torch.float32, torch.int32
            flags = PFE_FLAG_DEVICE_PTRS
        else:
            mk = lambda shape, dt: np.empty(shape, dtype=dt)  # noqa: E731
            f64, f32, i32 = np.float64, np.float32, np.uint32
            flags = 0
        out["profile"] = mk((n, L), f64) if profile else None
        out["chis"] = mk((n, PFE_PFD_NDM), f32) if chis else None
        out["lyon8"] = mk((n, 8), f64) if lyon8 else None
        out["status"] = mk((n,), i32)
        self._check(self.lib.pfe_pfd_dmprof(
            self._h, C.byref(pin), _ptr(out["profile"]) if profile else None,
            _ptr(out["chis"]) if chis else None, _ptr(out["lyon8"]) if lyon8 else None,
            _ptr(out["status"]), flags))
        del keep
        return out

    def pfd_bates22(self, profs, subfreqs, scal, out=None, status=None):
        """The 22 scores of PFD folds (pfe_pfd_bates22, PFDFile.compute) for a batch of one
        shape: profs (n,npart,nsub,L) f64, subfreqs (n,nsub), scal (n,PFE_PFD_NSCAL) with
        scal[:, 7] = bary_p1.  Returns (out (n,22) f64, status (n,))."""
        pin, dev, keep = self._pfd_args(profs, subfreqs, scal, "pfd_bates22")
        n = pin.n
        if dev:
            import torch

            if out is None:
                out = torch.empty((n, 22), dtype=torch.float64, device=profs.device)
            self._dev(out, "out", (torch.float64,), (n, 22))
            status = self._status_dev(status, n)
            flags = PFE_FLAG_DEVICE_PTRS
        else:
            out = self._out_host(out, n, 22)
            status = self._status_host(status, n)
            flags = 0
        self._check(self.lib.pfe_pfd_bates22(self._h, C.byref(pin), _ptr(out), _ptr(status), flags))
        del keep
        return out, status


class PhcxBatch:
    """Files parsed by the native reader (pfe_phcx_parse): per-file info and decoded fields."""

    def __init__(self, paths, mode: int = -1, threads: int = 0):
        self.lib = load_library()
        self.paths = [os.fsencode(p) for p in paths]
        arr = (C.c_char_p * max(1, len(self.paths)))(*self.paths)
        h = C.c_void_p()
        rc = self.lib.pfe_phcx_parse(arr, len(self.paths), int(mode), int(threads), C.byref(h))
        if rc != PFE_OK:
            raise PfeError(f"pfe_phcx_parse failed ({rc})")
        self._h = h

    def __len__(self):
        return len(self.paths)

    def close(self):
        if getattr(self, "_h", None):
            self.lib.pfe_phcx_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self, i: int) -> PhcxInfo:
        inf = PhcxInfo()
        if self.lib.pfe_phcx_info_get(self._h, i, C.byref(inf)) != PFE_OK:
            raise IndexError(i)
        return inf

    def infos(self) -> np.ndarray:
        """Every file's pfe_phcx_info as one structured array (PHCX_INFO_DTYPE)."""
        out = np.empty(len(self.paths), dtype=PHCX_INFO_DTYPE)
        if self.lib.pfe_phcx_info_all(self._h, out.ctypes.data if len(out) else None,
                                      len(out)) != PFE_OK:
            raise PfeError("pfe_phcx_info_all failed")
        return out

    def fetch(self, i: int, field: int, count: int, dtype=np.uint8) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        if self.lib.pfe_phcx_fetch(self._h, i, field, out.ctypes.data, count) != PFE_OK:
            raise PfeError(f"pfe_phcx_fetch({i}, {field}) failed")
        return out

    def pack(self, rows, lp=None, ld=None, nsub_lsb=None, ndm=None, threads: int = 0,
             alloc=None):
        """Dense arrays of the given rows (all of one shape): dict of numpy arrays.
        alloc(name, shape, dtype) -> array supplies the destination buffers (e.g. views of
        reused pinned slabs); default np.empty."""
        alloc = alloc or (lambda _k, shape, dt: np.empty(shape, dtype=dt))
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        n = len(rows)
        out = {"scal": alloc("scal", (n, 8), np.float64)}
        ptr = {}
        if lp is not None:
            out["prof"] = alloc("prof", (n, lp), np.uint8)
        if ld is not None:
            out["lyon_dm"] = alloc("lyon_dm", (n, ld), np.uint8)
        if nsub_lsb is not None:
            out["sub"] = alloc("sub", (n,) + tuple(nsub_lsb), np.uint8)
        if ndm is not None:
            out["dmcurve"] = alloc("dmcurve", (n, ndm), np.float64)
        for k in ("prof", "lyon_dm", "sub", "dmcurve"):
            ptr[k] = out[k].ctypes.data if k in out else None
        rc = self.lib.pfe_phcx_pack(
            self._h, rows.ctypes.data, n, int(threads),
            ptr["prof"], lp or 0, ptr["lyon_dm"], ld or 0,
            ptr["sub"], (nsub_lsb[0] * nsub_lsb[1]) if nsub_lsb else 0,
            ptr["dmcurve"], ndm or 0, out["scal"].ctypes.data)
        if rc != PFE_OK:
            raise PfeError("pfe_phcx_pack: rows of another shape or failed files")
        return out


def format_rows(names, vals: np.ndarray, style: int = 0, skip=None, threads: int = 0) -> bytes:
    """pfe_format_rows: the text DataProcessor writes for score rows (storeScore style 0,
    storeScoreARFF style 1, outputScores style 2) -- see include/pfe_io.h.  names: str or
    bytes per row; vals (n, width) float64 with contiguous rows; skip: rows to leave out."""
    lib = load_library()
    vals = np.asarray(vals, dtype=np.float64)
    if vals.ndim != 2 or (vals.shape[0] and vals.strides[1] != 8):
        vals = np.ascontiguousarray(vals.reshape(len(vals), -1))
    n, width = vals.shape
    if n == 0:
        return b""
    enc = [os.fsencode(x) if isinstance(x, str) else bytes(x) for x in names]
    if len(enc) != n:
        raise ValueError("one name per row")
    blob = b"".join(enc)
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum([len(e) for e in enc], out=off[1:])
    sk = None
    if skip is not None:
        sk = np.ascontiguousarray(skip, dtype=np.uint8)
        if sk.shape != (n,):
            raise ValueError("skip must have one entry per row")
    cap = len(blob) + n * (24 * width + 8) + 16
    buf = C.create_string_buffer(cap)
    used = C.c_int64()
    rc = lib.pfe_format_rows(blob, off.ctypes.data, vals.ctypes.data, n, width,
                             _row_stride(vals.strides[0] // 8, vals), int(style),
                             None if sk is None else sk.ctypes.data, int(threads), buf, cap,
                             C.byref(used))
    if rc != PFE_OK:
        raise PfeError("pfe_format_rows failed")
    return buf.raw[:used.value]
