"""Native PHCX reader (include/pfe_io.h, csrc/phcx_io.cpp) vs the host Python parser, which
follows the reference's decoding rules (PHCXFile.py:144-186, PHCXOperations.py:81-383).

Every field of every file must be identical; files the native reader flags must be the
ones whose text it cannot reproduce exactly, and parse_all must then give the Python
parser's outcome (including its exception).  CPU only: no GPU call is made."""
import gzip
import os
import re

import numpy as np
import pytest

from golden_util import load
from pulsarfeatureextractor_amd import _native, phcx, processor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "pfe_io.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|void)\s+(pfe_\w+)\s*\(", src, re.M)))


def test_io_header_and_binding_agree():
    assert header_functions() == sorted(_native.EXPORTED_IO_SYMBOLS)
    lib = _native.load_library()
    for s in header_functions():
        assert hasattr(lib, s), s


def _same(a, b):
    assert a.superb == b.superb and a.section == b.section
    for f in ("profile", "lyon_dm", "subbands", "dm_curve"):
        x, y = getattr(a, f), getattr(b, f)
        assert x.shape == y.shape and np.array_equal(x, y), f
    assert np.array_equal(a.scal, b.scal)


def _write_golden(tmp_path, name, rows):
    d = load(name)
    superb = bool(d["superb"])
    paths = []
    for i in rows:
        p = os.path.join(tmp_path, f"{name}_{i}" + (".phcx" if superb else ".phcx.gz"))
        phcx.write(p, profile=d["prof"][i], subbands=d["sub"][i],
                   datablocks=(d["block0"][i], d["block1"][i]), dm_start=float(d["dm_start"]),
                   dm_end=float(d["dm_end"]), n_dm_index=int(d["n_dm_index"]),
                   period_s=float(d["period"][i]), snr=float(d["snr"][i]), dm=float(d["dm"][i]),
                   width=float(d["width"][i]), superb=superb)
        paths.append(p)
    return paths


@pytest.mark.parametrize("name", ["bates22_phcx128", "bates22_superb64", "lyon8_phcx128_dmplane"])
def test_native_matches_python_on_golden_files(tmp_path, name):
    n = len(load(name)["ok"])
    paths = _write_golden(tmp_path, name, range(0, n, max(1, n // 12)))
    nat = processor.parse_all(paths, workers=4, native=True)
    py = processor.parse_all(paths, workers=1, native=False)
    b = _native.PhcxBatch(paths, threads=3)
    for (a, ea), (c, ec), i in zip(nat, py, range(len(paths))):
        assert ea is None and ec is None
        assert b.info(i).status == 0
        _same(a, c)


def _doc(profile_text="\n0A0B0C0D\n", block_text=None, sub_text=None, dmindex="\n0.0\n100.0\n200.0\n",
         scal=("0.5", "25.5", "12.0", "0.05"), nbins=2, nsub=2):
    if block_text is None:
        block_text = "\n" + "".join("%02X" % (k % 251) for k in range(256)) + "\n"
    if sub_text is None:
        sub_text = "\n01020304\n"
    sec = []
    for _ in range(2):
        sec.append(
            "<Section><BestValues>"
            f"<BaryPeriod>{scal[0]}</BaryPeriod><Dm>{scal[2]}</Dm><Snr>{scal[1]}</Snr>"
            f"<Width>{scal[3]}</Width></BestValues>"
            f"<SubBands nBins='{nbins}' nSub=\"{nsub}\" format='02X'>{sub_text}</SubBands>"
            f"<Profile nBins='4'>{profile_text}</Profile>"
            f"<DmCurve><DmIndex>{dmindex}</DmIndex></DmCurve>"
            f"<DataBlock format='02X'>{block_text}</DataBlock></Section>")
    return "<?xml version='1.0'?>\n<!-- synthetic -->\n<phcf>" + "".join(sec) + "</phcf>\n"


CASES = {
    "plain": dict(),
    "odd_lines": dict(profile_text="\nA\nBC0\nD\n"),
    "whitespace_pair": dict(profile_text="\n0A 0B\t0C\n"),
    "bad_pair_stops": dict(profile_text="\n0A0BZZ0C\n"),
    "crlf": dict(profile_text="\r\n0A0B\r\n0C0D\r\n", dmindex="\r\n0.0\r\n5.0\r\n7.5\r\n"),
    "entity": dict(profile_text="\n0A&#48;B0C\n"),
    "signed_pair": dict(profile_text="\n0A-10C\n"),          # native: range -> Python
    "empty_profile": dict(profile_text=""),
    "dmindex_unterminated": dict(dmindex="\n0.0\n100.0\n200.0"),
    "dmindex_short": dict(dmindex="\n0.0"),                  # IndexError in the reference
    "bad_scalar": dict(scal=("0.5", "abc", "12.0", "0.05")),  # ValueError
    "inf_scalar": dict(scal=("0.5", "inf", "12.0", "0.05")),  # native defers to Python
    "shape_mismatch": dict(nbins=3),                         # reshape error
    "partial_chunk": dict(block_text="\n" + "01" * 300 + "\n"),
    "no_dm_chunk": dict(block_text="\n0102\n"),
    # runs of >= 16 hex digits (the reader's SSE2 path) with the quirks inside or at the edge
    # of a 16-character chunk
    "long_lower": dict(profile_text="\n" + "0a1b2c3d4e5f6a7b8c9d" * 4 + "\n"),
    "long_bad_mid": dict(profile_text="\n" + "0A" * 10 + "G1" + "0B" * 10 + "\n"),
    "long_odd_line": dict(profile_text="\n" + "0123456789ABCDEF0" + "\n" + "123456789ABCDEF" * 3 + "\n"),
    "long_space_mid": dict(profile_text="\n" + "AB" * 12 + " C" + "DE" * 12 + "\n"),
    "long_sign_mid": dict(profile_text="\n" + "AB" * 9 + "+C" + "DE" * 12 + "\n"),
    "long_block_64": dict(block_text="\n" + "\n".join("%02X" * 32 % tuple((k * 7 + j) % 256 for j in range(32)) for k in range(64)) + "\n"),
}


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("gz", [True, False])
def test_edge_cases_match_python(tmp_path, case, gz):
    text = _doc(**CASES[case])
    p = os.path.join(tmp_path, "e.phcx" + (".gz" if gz else ""))
    if gz:
        with gzip.open(p, "wb") as f:
            f.write(text.encode())
    else:
        with open(p, "w", newline="") as f:
            f.write(text)
    (nat, en), = processor.parse_all([p], native=True)
    (py, ep), = processor.parse_all([p], native=False)
    assert (en is None) == (ep is None), (en, ep)
    if ep is None:
        _same(nat, py)
    else:
        assert en == ep


def test_status_codes(tmp_path):
    missing = os.path.join(tmp_path, "nope.phcx.gz")
    notgz = os.path.join(tmp_path, "plain.phcx.gz")
    with open(notgz, "w") as f:
        f.write(_doc())
    trunc = os.path.join(tmp_path, "trunc.phcx.gz")
    data = gzip.compress(_doc().encode())
    with open(trunc, "wb") as f:
        f.write(data[: len(data) // 2])
    b = _native.PhcxBatch([missing, notgz, trunc])
    assert [b.info(i).status for i in range(3)] == [1, 2, 2]
    res = processor.parse_all([missing, notgz, trunc], native=True)
    assert all(c is None and e for c, e in res)


def test_pack_matches_fetch(tmp_path):
    paths = _write_golden(tmp_path, "bates22_phcx128", range(6))
    b = _native.PhcxBatch(paths, threads=2)
    inf = b.info(0)
    rows = np.arange(len(paths))
    out = b.pack(rows, lp=inf.lp, ld=inf.ld, nsub_lsb=(inf.nsub, inf.lsb), ndm=inf.ndm)
    for i in rows:
        c = phcx.parse(paths[i])
        assert np.array_equal(out["prof"][i], c.profile)
        assert np.array_equal(out["lyon_dm"][i], c.lyon_dm)
        assert np.array_equal(out["sub"][i], c.subbands)
        assert np.array_equal(out["dmcurve"][i], c.dm_curve)
        assert np.array_equal(out["scal"][i], c.scal)
    with pytest.raises(_native.PfeError):
        b.pack(rows, lp=inf.lp - 1)


def test_libdeflate_and_zlib_paths_agree(tmp_path, monkeypatch):
    """The reader inflates with libdeflate when the system has it and falls back to zlib
    (PFE_NO_LIBDEFLATE=1, or any libdeflate error): both give identical documents, also for
    multi-member gzip files with trailing zero padding."""
    paths = _write_golden(tmp_path, "bates22_phcx128", range(0, 40, 7))
    # a two-member file with zero padding (Python's gzip module reads it)
    raw = gzip.decompress(open(paths[0], "rb").read())
    half = len(raw) // 2
    multi = os.path.join(tmp_path, "multi.phcx.gz")
    with open(multi, "wb") as f:
        f.write(gzip.compress(raw[:half]) + gzip.compress(raw[half:]) + b"\0" * 16)
    paths.append(multi)
    monkeypatch.setenv("PFE_NO_LIBDEFLATE", "1")
    z = processor.parse_all(paths, workers=2, native=True)
    monkeypatch.setenv("PFE_NO_LIBDEFLATE", "0")
    d = processor.parse_all(paths, workers=2, native=True)
    for (a, ea), (c, ec) in zip(z, d):
        assert ea is None and ec is None
        _same(a, c)
    _same(d[-1][0], d[0][0])
