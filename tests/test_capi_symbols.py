"""libpfe.so loads on a CPU-only host, exports every symbol include/pfe.h declares, and
refuses to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import pytest

from pulsarfeatureextractor_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(name="pfe.h"):
    src = open(os.path.join(ROOT, "include", name)).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*|int64_t)\s+(pfe_\w+)\s*\(",
                                 src, re.M)))


def test_header_and_binding_agree():
    assert header_functions() == sorted(_native.EXPORTED_SYMBOLS)
    assert header_functions("pfe_io.h") == sorted(_native.EXPORTED_IO_SYMBOLS)


def test_library_exports_all_symbols():
    lib = _native.load_library()
    for s in header_functions() + header_functions("pfe_io.h"):
        assert hasattr(lib, s), s
    assert lib.pfe_abi_version() == 1


def test_no_cpu_backend():
    lib = _native.load_library()
    h = ctypes.c_void_p()
    assert lib.pfe_create(-1, ctypes.byref(h)) != 0
    assert b"no CPU backend" in lib.pfe_last_error(None)


def test_cpu_host_has_no_device():
    lib = _native.load_library()
    if lib.pfe_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_native.PfeError):
        _native.Engine(0)
