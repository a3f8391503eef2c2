"""Diagnostic: lyon8_u8_dm rows processed several per wave (lyon8_blocks cap) vs one per wave
and vs the oracle; prints the rows / columns that differ."""
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle.lyon import lyon8_batched  # noqa: E402
from pulsarfeatureextractor_amd._native import Engine  # noqa: E402
from pulsarfeatureextractor_amd.synth import lyon_batch  # noqa: E402


def diff(tag, a, b):
    ne = ~((a == b) | (np.isnan(a) & np.isnan(b)))
    rows = np.where(ne.any(1))[0]
    print(f"{tag}: {len(rows)} rows differ; cols {np.where(ne.any(0))[0].tolist()}; rows {rows[:20].tolist()}")
    for r in rows[:4]:
        print("   row", r, "a", a[r].tolist(), "\n          b", b[r].tolist())


with Engine(0) as e:
    for ld, n, adv in ((15360, 8, False), (15360, 8, True), (15360, 600, True), (7680, 600, True)):
        prof, dm = lyon_batch(n, 128, ld, seed=3 + ld, adversarial=adv)
        ref = lyon8_batched(prof, dm)
        d = e.lyon8(prof, dm)
        print(f"== ld {ld} n {n} adv {adv}")
        diff("default vs oracle", d, ref)
        for b in (1, 2):
            with e.options(lyon8_blocks=b):
                g = e.lyon8(prof, dm)
            diff(f"blocks={b} vs default", g, d)
