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
    ap.add_argument("--path", choices=["bates22", "pfd22"], default="bates22",
                    help="pfd22: PRESTO folds (bench.py's 16x32x128 block) through "
                         "pfe_pfd_bates22, the DM fit counted in the pfd22 unit")
    ap.add_argument("--solver", default=None,
                    help="handle solver option (batched: per-solve statistics are counted)")
    args = ap.parse_args()
    import torch

    from pulsarfeatureextractor_amd import _native
    from pulsarfeatureextractor_amd.synth import bates_batch

    lib = _native.load_library(os.path.join(ROOT, "pulsarfeatureextractor_amd", "lib", "libpfe_lmprof.so"))
    _native._lib = lib  # route the Engine through the instrumented build
    eng = _native.Engine(0)
    if args.solver:
        eng.set_option("solver", args.solver)
    # one counter set per translation unit
    tags = ("gauss", "gauss_peel", "gauss_dg8", "sine_dm_sub") + (("pfd22",) if args.path == "pfd22" else ())
    buf = (C.c_ulonglong * 64)()
    import time
    if args.path == "bates22":
        blk = min(args.n, 16384)  # a synthetic block tiled to n rows (as bench.py --path bates22)
        base = bates_batch(blk, lp=128, lsb=128, seed=31)
        reps = (args.n + blk - 1) // blk
        t = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in base.items()}
        t = {k: v.repeat((reps,) + (1,) * (v.dim() - 1))[:args.n].contiguous() for k, v in t.items()}
        out = torch.empty((args.n, 22), dtype=torch.float64, device="cuda")
        st = torch.empty((args.n,), dtype=torch.int32, device="cuda")
        run = lambda: eng.bates22(t["prof"], t["sub"], t["dmcurve"], t["scal"], out, st)  # noqa: E731
    else:
        sys.path.insert(0, ROOT)
        from bench import pfd_block
        from pulsarfeatureextractor_amd import pfd as _pfd

        profs, subfreqs, pscal = _pfd.batch_inputs(pfd_block(min(args.n, 1024), (16, 32, 128), 20261019))
        tp, tf, ts = (torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (profs, subfreqs, pscal))
        out = torch.empty((tp.shape[0], 22), dtype=torch.float64, device="cuda")
        st = torch.empty((tp.shape[0],), dtype=torch.int32, device="cuda")
        run = lambda: eng.pfd_bates22(tp, tf, ts, out=out, status=st)  # noqa: E731
    for tag in tags:
        getattr(lib, f"pfe_lmprof_{tag}")(buf, 1)
    torch.cuda.synchronize()
    print(f"lm_profile: inputs ready, n={args.n}", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    print(f"lm_profile: {args.path} done in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    res = {"_elapsed_s_instrumented": time.perf_counter() - t0, "_n": int(out.shape[0]),
           "_path": args.path, "_solver": args.solver or "default"}
    for tag in tags:
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
            if row[13] > 0:  # pooled group engine (lm_group.h): per-wave phase cycles
                tot = row[10]
                res[f"{tag}/N={npar}/pooled"] = {
                    "waves": int(row[0]),
                    "frac_refill": row[11] / tot, "frac_O_phase": row[13] / tot,
                    "frac_SIMT": row[12] / tot, "frac_T_phase": row[9] / tot,
                    "mean_fits_per_O_round": row[14] / 1000.0 / max(row[0], 1),
                    "mean_fits_per_T_round": row[15] / 1000.0 / max(row[0], 1),
                    "mcycles_per_wave": tot / max(row[0], 1) / 1e6,
                }
                continue
            if row[14] > 0:  # batched solver (lm_batch.h): per-wave phase cycles
                per["batched"] = {
                    "simt_phases": int(row[14]),
                    "fits_per_simt_phase": row[15] / row[14],
                    "trial_visits": int(row[2]),
                    "outer_iters": int(row[1]),
                    "kcyc_init": row[11] / 1e3,
                    "kcyc_simt": row[12] / 1e3,
                    "kcyc_trial_visits_incl_outer": row[9] / 1e3,
                    "kcyc_outer_fdjac": row[5] / 1e3,
                    "kcyc_outer_qrfac": row[6] / 1e3,
                    "kcyc_outer_qtf": row[7] / 1e3,
                    "kcyc_total": row[10] / 1e3,
                    "cyc_per_simt_phase": row[12] / row[14],
                    "cyc_per_outer": (row[5] + row[6] + row[7]) / max(row[1], 1),
                }
            res[f"{tag}/N={npar}"] = per
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
