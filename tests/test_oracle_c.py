"""The C restatement of the Lyon features (oracle/c/lyon8_omp.c, the multi-core CPU
baseline) against the Python oracle and the reference's golden vectors: mean bit-exact, std
bit-exact for power-of-two row lengths, everything else within 1e-12 relative (absolute below
1), NaN exactly on zero-variance rows, and thread count independence."""
import os
import subprocess
import warnings

import numpy as np
import pytest

from golden_util import GOLDEN
from oracle import lyon as L
from oracle import lyon_c

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def built():
    if not lyon_c.available():
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                       capture_output=True)
    assert lyon_c.available()


def close(got, ref, lens):
    """lens: the profile and DM row lengths.  The mean is bit-exact; so is the std when the
    row length is a power of two (every squared deviation and partial sum is then an exact
    dyadic number, whatever the summation order); otherwise numpy's pairwise order and the
    sequential C sum differ in the last bits."""
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    m = ~np.isnan(ref)
    for j in range(8):
        g, r = got[:, j][m[:, j]], ref[:, j][m[:, j]]
        n = lens[j // 4]
        if j % 4 == 0 or (j % 4 == 1 and n & (n - 1) == 0):
            assert np.array_equal(g, r), f"feature {j} not bit-exact"
        else:
            err = np.abs(g - r) / np.maximum(1.0, np.abs(r))
            assert err.max(initial=0.0) <= 1e-12, f"feature {j}: {err.max():.3g}"


@pytest.mark.parametrize("name", ["lyon8_superb64", "lyon8_phcx128", "lyon8_phcx128_dmplane"])
def test_vs_golden(name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    close(lyon_c.lyon8_omp(g["prof"], g["block0"]), g["out"],
          (g["prof"].shape[1], g["block0"].shape[1]))


def test_vs_oracle_and_threads():
    rng = np.random.default_rng(7)
    prof = rng.integers(0, 256, (3000, 128), dtype=np.uint8)
    dm = rng.integers(0, 256, (3000, 64), dtype=np.uint8)
    prof[5] = 17  # zero variance -> NaN skew/kurt
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        ref = L.lyon8_batched(prof, dm)
    one = lyon_c.lyon8_omp(prof, dm, threads=1)
    close(one, ref, (128, 64))
    many = lyon_c.lyon8_omp(prof, dm, threads=4)
    assert np.array_equal(np.nan_to_num(one, nan=9.0), np.nan_to_num(many, nan=9.0))
