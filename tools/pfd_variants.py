#!/usr/bin/env python3
"""Times pfe_pfd_dmprof with different outputs requested (which parts of the kernel run)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import pfd_block  # noqa: E402
from pulsarfeatureextractor_amd import pfd as _pfd  # noqa: E402
from pulsarfeatureextractor_amd._native import Engine  # noqa: E402

n, blk = 32768, 1024
profs, subfreqs, pscal = _pfd.batch_inputs(pfd_block(blk, (16, 32, 128), 7))
reps = n // blk
t = [torch.from_numpy(np.ascontiguousarray(a)).cuda().repeat((reps,) + (1,) * (a.ndim - 1))
     for a in (profs, subfreqs, pscal)]
eng = Engine(0)
for name, kw in (("lyon8", dict(profile=False, chis=False, lyon8=True)),
                 ("chis", dict(profile=False, chis=True, lyon8=False)),
                 ("profile", dict(profile=True, chis=False, lyon8=False))):
    for _ in range(2):
        eng.pfd_dmprof(*t, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        eng.pfd_dmprof(*t, **kw)
    torch.cuda.synchronize()
    print(name, f"{(time.perf_counter() - t0) / 5 * 1e3:.2f} ms", flush=True)
