"""ASan + UBSan build of the native PHCX reader (csrc/phcx_io.cpp, SURVEY.md §5 "sanitizer
build of the host C++").  g++ compiles phcx_io.cpp with tests/native/phcx_io_driver.cpp into
one sanitized executable (-fsanitize=address,undefined, no recovery: the first report aborts
it), which is run over the inputs of tests/test_phcx_native.py: golden files, every edge
case gzipped and plain, missing / not-gzip / truncated files, a multi-member gzip file, with
libdeflate and with zlib, one and four threads.  The driver fetches every field (and checks
that one element too few is refused), packs, and prints per-file status, shape and an FNV
hash of the fields; those must equal what the product library (libpfe.so, not sanitized)
gives for the same files.  CPU only; skipped when g++ or the sanitizer runtimes are absent."""
import gzip
import os
import shutil
import subprocess

import numpy as np
import pytest

from pulsarfeatureextractor_amd import _native
from test_phcx_native import CASES, _doc, _write_golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "pulsarfeatureextractor_amd", "csrc", "phcx_io.cpp")
DRIVER = os.path.join(ROOT, "tests", "native", "phcx_io_driver.cpp")
SAN_ENV = {"ASAN_OPTIONS": "abort_on_error=0:halt_on_error=1:detect_leaks=1:exitcode=66",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1:exitcode=67"}


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("san") / "phcx_io_san")
    cmd = [cxx, "-std=c++17", "-g", "-O1", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-I" + os.path.join(ROOT, "include"), SRC, DRIVER, "-o", exe, "-lz", "-ldl", "-pthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        if "asan" in r.stderr or "ubsan" in r.stderr:
            pytest.skip("sanitizer runtimes not available: " + r.stderr[-200:])
        raise AssertionError(r.stderr)
    probe = subprocess.run([exe, "1", os.devnull], capture_output=True, text=True,
                           env={**os.environ, **SAN_ENV})
    if "LeakSanitizer does not work" in probe.stderr:   # ptrace-less sandboxes
        SAN_ENV["ASAN_OPTIONS"] = SAN_ENV["ASAN_OPTIONS"].replace("detect_leaks=1", "detect_leaks=0")
    return exe


def fnv(h, b):
    for c in b:
        h = ((h ^ c) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def expected(paths, threads):
    """The driver's lines, computed from the product library."""
    b = _native.PhcxBatch(paths, threads=threads)
    lines = []
    for i in range(len(paths)):
        inf = b.info(i)
        h = 1469598103934665603
        if inf.status == 0:
            for f, cnt, dt in ((0, inf.lp, np.uint8), (1, inf.ld, np.uint8),
                               (2, inf.nsub * inf.lsb, np.uint8), (3, inf.ndm, np.float64),
                               (4, inf.lfit, np.uint8)):
                h = fnv(h, b.fetch(i, f, cnt, dt).tobytes())
            h = fnv(h, np.array(inf.scal[:8], dtype=np.float64).tobytes())
        lines.append(f"{i} {inf.status} {inf.lp} {inf.nsub} {inf.lsb} {inf.ndm} {inf.ld} "
                     f"{inf.lfit} {h:016x}")
    return lines


def run_driver(exe, paths, threads, libdeflate):
    env = {**os.environ, **SAN_ENV, "PFE_NO_LIBDEFLATE": "0" if libdeflate else "1"}
    r = subprocess.run([exe, str(threads), *paths], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, f"sanitized reader failed ({r.returncode}):\n{r.stderr[-4000:]}"
    assert "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, r.stderr[-4000:]
    return r.stdout.splitlines()


def edge_files(tmp_path):
    paths = []
    for case in sorted(CASES):
        text = _doc(**CASES[case])
        for gz in (True, False):
            p = os.path.join(tmp_path, f"{case}.phcx" + (".gz" if gz else ""))
            if gz:
                with gzip.open(p, "wb") as f:
                    f.write(text.encode())
            else:
                with open(p, "w", newline="") as f:
                    f.write(text)
            paths.append(p)
    notgz = os.path.join(tmp_path, "plain_text.phcx.gz")
    with open(notgz, "w") as f:
        f.write(_doc())
    data = gzip.compress(_doc().encode())
    trunc = os.path.join(tmp_path, "trunc.phcx.gz")
    with open(trunc, "wb") as f:
        f.write(data[: len(data) // 2])
    empty = os.path.join(tmp_path, "empty.phcx.gz")
    open(empty, "wb").close()
    empty_xml = os.path.join(tmp_path, "empty.phcx")
    open(empty_xml, "wb").close()
    return paths + [os.path.join(tmp_path, "missing.phcx.gz"), notgz, trunc, empty, empty_xml]


@pytest.mark.parametrize("libdeflate", [True, False])
@pytest.mark.parametrize("threads", [1, 4])
def test_sanitized_reader_edge_cases(driver, tmp_path, threads, libdeflate):
    paths = edge_files(tmp_path)
    got = run_driver(driver, paths, threads, libdeflate)
    want = expected(paths, threads)
    assert [ln for ln in got if not ln.startswith("pack")] == want


@pytest.mark.parametrize("libdeflate", [True, False])
def test_sanitized_reader_golden_files(driver, tmp_path, libdeflate):
    paths = _write_golden(tmp_path, "bates22_phcx128", range(0, 128, 9))
    paths += _write_golden(tmp_path, "bates22_superb64", range(0, 64, 11))
    raw = gzip.decompress(open(paths[0], "rb").read())
    multi = os.path.join(tmp_path, "multi.phcx.gz")
    with open(multi, "wb") as f:
        f.write(gzip.compress(raw[: len(raw) // 3]) + gzip.compress(raw[len(raw) // 3:]) + b"\0" * 8)
    paths.append(multi)
    got = run_driver(driver, paths, 4, libdeflate)
    want = expected(paths, 4)
    assert [ln for ln in got if not ln.startswith("pack")] == want
    pack = [ln for ln in got if ln.startswith("pack")]
    assert len(pack) == 1 and int(pack[0].split()[1]) == 15 + 1   # the HTRU files + multi
