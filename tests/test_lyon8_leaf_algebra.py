"""CPU check of the arithmetic lyon8_u8_pow2 relies on (csrc/lyon8.hip): for a DM row of
n = 2^k bytes, numpy.std's leaf sums (128-value leaves of its pairwise tree) are the exact
rationals (2^2k B - 2^(k+1) S1 A + 128 S1^2) * 2^-2k, so only numpy's tree above the leaves
rounds.  The emulation below builds the std that way (integer leaf sums, the perfect tree
over the leaves, (0 + c0) + c1 for the two 8192-value chunks of a 16 KiB row) and must equal
numpy.std bit for bit; the GPU kernel is held to the same values by test_lyon8_gpu.py."""
import numpy as np
import pytest


def tree(v):
    if len(v) == 1:
        return v[0]
    h = len(v) // 2
    return tree(v[:h]) + tree(v[h:])


def std_exact_leaves(row):
    n = row.size
    k = n.bit_length() - 1
    assert n == 1 << k
    x = row.astype(np.int64)
    s1 = int(x.sum())
    leaves = x.reshape(-1, 128)
    a, b = leaves.sum(1), (leaves * leaves).sum(1)
    v2k = (b << (2 * k)) - ((2 * s1 * a) << k) + 128 * s1 * s1
    assert int(v2k.max()) < 2 ** 53 and int(v2k.min()) >= 0
    lv = [float(v) * 2.0 ** (-2 * k) for v in v2k]
    if n > 8192:  # numpy's buffered chunks of 8192, each a pairwise tree, added in order
        ssq = 0.0
        for c in range(0, len(lv), 64):
            ssq = ssq + tree(lv[c:c + 64])
    else:
        ssq = tree(lv)
    return np.sqrt(ssq / n)


@pytest.mark.parametrize("n", [8192, 16384])
def test_exact_leaf_std_matches_numpy(n):
    rng = np.random.default_rng(n)
    rows = [rng.integers(0, 256, n, dtype=np.uint8),
            np.clip(rng.normal(128, 3, n), 0, 255).astype(np.uint8),
            np.where(rng.random(n) < 0.5, 0, 255).astype(np.uint8),
            np.full(n, 255, dtype=np.uint8),
            np.zeros(n, dtype=np.uint8)]
    near = np.full(n, 77, dtype=np.uint8)
    near[rng.integers(0, n)] = 78
    rows.append(near)
    for _ in range(40):
        lo = int(rng.integers(0, 200))
        rows.append(rng.integers(lo, lo + int(rng.integers(1, 56)), n).astype(np.uint8))
    for r in rows:
        assert std_exact_leaves(r) == np.std(r)
