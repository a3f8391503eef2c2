"""Host PHCX/SUPERB parser vs the reference's decoding rules (PHCXFile.py:144-186,
PHCXOperations.py:172-183, 237-297, 353-383)."""
import os

import numpy as np
import pytest

from golden_util import load
from pulsarfeatureextractor_amd import phcx


def ref_hex_loop(points):
    """The reference's decode loop, restated literally (PHCXOperations.py:284-297)."""
    out, x = [], 0
    while x < len(points):
        if points[x] != "\n":
            try:
                out.append(int(points[x:x + 2], 16))
                x += 2
            except ValueError:
                break
        else:
            x += 1
    return out


@pytest.mark.parametrize("text", [
    "\n0A0B\nFF00\n", "0a0b", "\nAB\nC", "\nA\nBC\n", "0102ZZ03", "01 02", "\n\n\n", "",
    "0\n102", "FF\t", "1234\n56 7\n",
])
def test_hex_decode_quirks(text):
    assert list(phcx.hex_decode(text)) == ref_hex_loop(text)


def test_dm_index_parse():
    assert phcx.parse_dm_index("\n0.0\n1.5\n3.0\n") == (0.0, 3.0)
    assert phcx.parse_dm_index("\n0.0\n1.5\n3.0") == (0.0, 1.5)  # last token not terminated


def test_reduce_dm_curve():
    rng = np.random.default_rng(0)
    blk = rng.integers(0, 256, 128 * 5 + 17)
    y, x = phcx.reduce_dm_curve(blk)
    ry, rx, tmp = [], [], []
    for i in range(len(blk)):  # PHCXOperations.dm_curve restated literally
        if (i + 1) % 128 == 0:
            ry.append(max(tmp))
            rx.append(i - 128)
            tmp = []
        else:
            tmp.append(blk[i])
    assert list(y) == ry and list(x) == rx


@pytest.mark.parametrize("name", ["bates22_phcx128", "bates22_superb64", "lyon8_phcx128_dmplane"])
def test_roundtrip_golden_files(tmp_path, name):
    d = load(name)
    superb = bool(d["superb"])
    for i in range(0, len(d["ok"]), max(1, len(d["ok"]) // 7)):
        p = os.path.join(tmp_path, f"c{i}" + (".phcx" if superb else ".phcx.gz"))
        phcx.write(p, profile=d["prof"][i], subbands=d["sub"][i],
                   datablocks=(d["block0"][i], d["block1"][i]), dm_start=float(d["dm_start"]),
                   dm_end=float(d["dm_end"]), n_dm_index=int(d["n_dm_index"]),
                   period_s=float(d["period"][i]), snr=float(d["snr"][i]), dm=float(d["dm"][i]),
                   width=float(d["width"][i]), superb=superb)
        c = phcx.parse(p)
        assert c.superb == superb
        assert np.array_equal(c.profile, d["prof"][i])
        assert np.array_equal(c.subbands, d["sub"][i])
        assert np.array_equal(c.lyon_dm, d["block0"][i])
        blk = d["block0"][i] if superb else d["block1"][i]
        assert np.array_equal(c.dm_curve, phcx.reduce_dm_curve(blk)[0])
        assert c.scal[0] == float(d["period"][i]) * 1000
        assert c.scal[6] == len(blk)
