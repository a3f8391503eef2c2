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


@pytest.mark.parametrize("seed", range(8))
def test_paired_tri_rows_layout_matches_numpy(seed):
    """lyon8_u8_dm<1, true, 32> (two one-chunk tri rows per wave, nDM = 33): the staging
    table's image layout (block b's 128-byte leaf in slot 2b, its 64- and 72-byte leaves back
    to back in slot 2b + 1, stride DM_S_T = 140), dm_leaf_tri_pair's 17-word chain loop with
    the odd lane's restart at word 8, and half_sum_f64's butterfly (lane ^ 1, ^ 2, half-row and
    row mirrors, ^ 16) give numpy's sum of squared deviations of the 4224-byte row bit for bit
    (the kernel works in a power-of-two scaled domain, which is exact; adversarial rows too)."""
    S = 140
    rng = np.random.default_rng(100 + seed)
    x = rng.integers(0, 256, 4224).astype(np.uint8)
    if seed == 1:
        x[:] = 255
        x[::7] = 0
    if seed == 2:
        x = np.sort(x)
    mean = x.astype(np.float64).sum() / 4224
    ref = np.sum((x.astype(np.float64) - mean) ** 2)
    img = np.zeros(32 * S, np.uint8)
    for ln in range(32):
        for j in range(9):
            for h in range(2):
                o = 16 * ln + 512 * j + 8 * h
                if o < 4224:
                    b, w = divmod(o, 264)
                    a = (2 * b + (w >= 128)) * S + (w if w < 128 else w - 128)
                    img[a:a + 8] = x[o:o + 8]
    vals = []
    for ln in range(32):
        odd = ln & 1
        vb = img[ln * S:ln * S + 136].astype(np.float64)
        r, sv = [0.0] * 8, [0.0] * 8
        for k in range(17):
            if k == 8:
                sv = list(r)
                if odd:
                    r = [0.0] * 8
            for j in range(8):
                d = vb[8 * k + j] - mean if 8 * k + j < 136 else 0.0
                sq = d * d if (k < 16 or odd) else 0.0
                r[j] = sq if k == 0 else r[j] + sq
        tr = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        ts = ((sv[0] + sv[1]) + (sv[2] + sv[3])) + ((sv[4] + sv[5]) + (sv[6] + sv[7]))
        vals.append(ts + tr if odd else tr)
    v = np.array(vals)
    for perm in (lambda i: i ^ 1, lambda i: i ^ 2, lambda i: (i & ~7) | (7 - (i & 7)),
                 lambda i: (i & ~15) | (15 - (i & 15)), lambda i: i ^ 16):
        v = np.array([v[i] + v[perm(i)] for i in range(32)])
    assert (v == ref).all()
