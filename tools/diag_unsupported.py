"""Which score columns differ between pfe_bates22 on the same candidates with a supported
and an unsupported sub-band shape, and between two identical calls."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from pulsarfeatureextractor_amd._native import Engine
from pulsarfeatureextractor_amd.synth import bates_batch

eng = Engine(0)
b = bates_batch(64, lp=128, nsub=16, lsb=128, seed=77)
rng = np.random.default_rng(3)
big = rng.integers(0, 256, (64, 32, 1024), dtype=np.uint8)
o1, s1 = eng.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
o2, s2 = eng.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
o3, s3 = eng.bates22(b["prof"], big, b["dmcurve"], b["scal"])
def diff(a, c):
    d = ~((a == c) | (np.isnan(a) & np.isnan(c)))
    return {int(j): int(d[:, j].sum()) for j in range(a.shape[1]) if d[:, j].any()}
print("repeat:", diff(o1, o2), (s1 != s2).sum())
print("unsupported vs supported:", diff(o1[:, :19], o3[:, :19]))
with eng.options(serial=1):
    o4, s4 = eng.bates22(b["prof"], b["sub"], b["dmcurve"], b["scal"])
    o5, s5 = eng.bates22(b["prof"], big, b["dmcurve"], b["scal"])
print("serial vs concurrent:", diff(o1, o4))
print("serial unsupported vs serial supported:", diff(o4[:, :19], o5[:, :19]))
