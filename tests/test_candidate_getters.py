"""Candidate.getSubbandData / getSubintData (Candidate.py:290-340 -> PHCXOperations.py:422-505)
against the reference's own outputs for PHCX files with <SubIntegrations>
(tests/golden/getters_phcx128.npz, made by tools/make_golden.py --getters).  Host data getters:
no GPU involved."""
import numpy as np

from golden_util import load
from pulsarfeatureextractor_amd import candidate, phcx


def _write(tmp_path, d, i):
    p = str(tmp_path / f"g_{i:03d}.phcx.gz")
    phcx.write(p, profile=d["prof"][i], subbands=d["sub"][i],
               datablocks=(d["block0"][i], d["block1"][i]), dm_start=0.0, dm_end=200.0,
               n_dm_index=101, period_s=float(d["period"][i]), snr=float(d["snr"][i]),
               dm=float(d["dm"][i]), width=float(d["width"][i]), subints=d["subints"][i])
    return p


def test_getters_vs_reference(tmp_path):
    d = load("getters_phcx128")
    for i in range(len(d["prof"])):
        c = candidate.Candidate(_write(tmp_path, d, i), "")
        sb = np.asarray(c.getSubbandData(False), dtype=np.float64)
        si = np.asarray(c.getSubintData(False), dtype=np.float64)
        assert np.array_equal(sb, d["subband"][i]), i
        assert np.array_equal(si, d["subint"][i]), i


def test_getters_empty_for_superb_and_pfd():
    for name in ("x.phcx", "x.pfd", "cand_x.pfd"):
        c = candidate.Candidate(name, "")
        assert c.getSubbandData(False) == [] and c.getSubintData(False) == []
