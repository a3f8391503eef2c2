#!/usr/bin/env python3
"""Dump / compare the 22-score outputs of one libpfe build (GPU), for bit-identity checks of
kernel changes that must not move any result (e.g. a cheaper but exact division).

  PFE_LIBRARY=libA.so python tools/lib_outputs.py dump out_a.npz
  PFE_LIBRARY=libB.so python tools/lib_outputs.py dump out_b.npz
  python tools/lib_outputs.py compare out_a.npz out_b.npz

Inputs: the golden PHCX sets and synthetic batches (pulsarfeatureextractor_amd.synth) of
64- and 128-bin candidates, the default (pooled) solver and the batched one.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def dump(path):
    from golden_util import bates_inputs, load
    from pulsarfeatureextractor_amd._native import Engine
    from pulsarfeatureextractor_amd.synth import bates_batch

    res = {}
    with Engine(0) as e:
        sets = {}
        for name in ("bates22_phcx128", "bates22_superb64", "bates22_phcx128_nsub32"):
            sets[name] = bates_inputs(load(name))
        for lp, n, seed in ((128, 20000, 77), (64, 20000, 78)):
            b = bates_batch(n, lp=lp, lsb=lp, seed=seed)
            sets[f"synth{lp}"] = (b["prof"], b["sub"], b["dmcurve"], b["scal"])
        # pfe_subband3 (fast kernel: power-of-two nBins <= 256; nsub 20 = a partial block)
        for nsub, lsb, n, seed in ((16, 256, 20000, 80), (20, 128, 8000, 81), (16, 64, 8000, 82),
                                   (3, 32, 4000, 83), (40, 16, 4000, 84)):
            b = bates_batch(n, lp=lsb, nsub=nsub, lsb=lsb, seed=seed)
            out, st = e.subband3(b["prof"], b["sub"], b["scal"])
            res[f"sub{nsub}x{lsb}_out"] = np.asarray(out)
            res[f"sub{nsub}x{lsb}_st"] = np.asarray(st)
            # the same bands with wide windows (wb up to 60 % of the band) and bright rows
            rng = np.random.default_rng(seed)
            b["scal"][:, 3] = rng.uniform(0.5 / lsb, 0.6, size=n)
            b["sub"][: n // 4] = np.maximum(b["sub"][: n // 4], 200)
            out, st = e.subband3(b["prof"], b["sub"], b["scal"])
            res[f"sub{nsub}x{lsb}w_out"] = np.asarray(out)
            res[f"sub{nsub}x{lsb}w_st"] = np.asarray(st)
        # pfe_pfd_dmprof (fast sweep: L = 64/128 with nsub % 8 == 0; the others general) and
        # pfe_pfd_bates22
        from bench import pfd_block
        from pulsarfeatureextractor_amd import pfd as _pfd

        for shape in ((16, 32, 128), (8, 16, 64), (4, 8, 96), (4, 12, 128), (2, 40, 64)):
            profs, subfreqs, pscal = _pfd.batch_inputs(pfd_block(64, shape, 9100 + shape[1]))
            r = e.pfd_dmprof(profs, subfreqs, pscal)
            tag = "pfd%dx%dx%d" % shape
            res[f"{tag}_chis_out"] = np.asarray(r["chis"]).astype(np.float64)
            res[f"{tag}_profile_out"] = np.asarray(r["profile"])
            res[f"{tag}_lyon8_out"] = np.asarray(r["lyon8"])
            res[f"{tag}_st"] = np.asarray(r["status"])
            out, st = e.pfd_bates22(profs, subfreqs, pscal)
            res[f"{tag}_b22_out"] = np.asarray(out)
            res[f"{tag}_b22_st"] = np.asarray(st)
        for solver in ("pooled", "batched"):
            e.set_option("solver", solver)
            for name, args in sets.items():
                out, st = e.bates22(*args)
                res[f"{name}_{solver}_out"] = np.asarray(out)
                res[f"{name}_{solver}_st"] = np.asarray(st)
    np.savez(path, **res)
    print("dumped", path, len(res))


def compare(pa, pb):
    a, b = np.load(pa), np.load(pb)
    total = 0
    for k in sorted(a.files):
        x, y = a[k], b[k]
        if k.endswith("_st"):
            d = int((x != y).sum())
            print(f"{k:40s} status differs in {d} rows")
            total += d
            continue
        same = (x.view(np.uint64) == y.view(np.uint64))
        cols = [(j + 1, int((~same[:, j]).sum())) for j in range(x.shape[1]) if not same[:, j].all()]
        total += sum(c for _, c in cols)
        print(f"{k:40s} {x.shape[0]} rows, columns differing (score: rows): {cols}")
    print("IDENTICAL" if total == 0 else f"DIFFER: {total}")
    return total


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
