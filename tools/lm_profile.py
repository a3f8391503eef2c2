#!/usr/bin/env python3
"""Phase-cycle breakdown of the wave-parallel MINPACK lmdif inside the 22-score kernels.

Needs the instrumented library (python pulsarfeatureextractor_amd/build.py --lm-profile).
Counters are per translation unit and per parameter count N (see lm_wave.h).
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["calls", "iters", "lmpar", "qrsolv", "nfev", "cyc_fdjac2", "cyc_qrfac", "cyc_qtf_r_gnorm",
         "cyc_lmpar", "cyc_trial", "cyc_total"]
SLOTS = {0: 2, 1: 3, 2: 4, 3: 8}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    args = ap.parse_args()
    import torch

    from pulsarfeatureextractor_amd import _native
    from pulsarfeatureextractor_amd.synth import bates_batch

    lib = _native.load_library(os.path.join(ROOT, "pulsarfeatureextractor_amd", "lib", "libpfe_lmprof.so"))
    _native._lib = lib  # route the Engine through the instrumented build
    base = bates_batch(args.n, lp=128, lsb=128, seed=31)
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in base.items()}
    eng = _native.Engine(0)
    out = torch.empty((args.n, 22), dtype=torch.float64, device="cuda")
    st = torch.empty((args.n,), dtype=torch.int32, device="cuda")
    buf = (C.c_ulonglong * 64)()
    for tag in ("gauss", "sine_dm_sub"):
        getattr(lib, f"pfe_lmprof_{tag}")(buf, 1)
    eng.bates22(t["prof"], t["sub"], t["dmcurve"], t["scal"], out, st)
    torch.cuda.synchronize()
    res = {}
    for tag in ("gauss", "sine_dm_sub"):
        fn = getattr(lib, f"pfe_lmprof_{tag}")
        fn.argtypes = [C.c_void_p, C.c_int]
        assert fn(buf, 0) == 0
        a = np.array(buf[:], dtype=np.float64).reshape(4, 16)
        for s, npar in SLOTS.items():
            row = a[s]
            if row[0] == 0:
                continue
            d = {nm: row[i] for i, nm in enumerate(NAMES)}
            calls = d["calls"]
            per = {
                "calls": int(calls),
                "iters_per_call": d["iters"] / calls,
                "lmpar_per_iter": d["lmpar"] / max(d["iters"], 1),
                "qrsolv_per_lmpar": d["qrsolv"] / max(d["lmpar"], 1),
                "nfev_per_call": d["nfev"] / calls,
                "kcycles_per_call": d["cyc_total"] / calls / 1e3,
            }
            tot = d["cyc_total"]
            for nm in NAMES[5:10]:
                per["frac_" + nm[4:]] = d[nm] / tot
            per["cycles_per_iter"] = {nm[4:]: d[nm] / max(d["iters"], 1) for nm in NAMES[5:9]}
            per["cycles_per_iter"]["trial"] = d["cyc_trial"] / max(d["lmpar"], 1)
            per["cycles_per_qrsolv_call_lmpar"] = d["cyc_lmpar"] / max(d["lmpar"], 1)
            res[f"{tag}/N={npar}"] = per
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
