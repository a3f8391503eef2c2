"""Build libpfe.so (all HIP kernels + the C-ABI) in-tree for gfx950.

The shared library lands in ``pulsarfeatureextractor_amd/lib/libpfe.so`` so that it travels
with the repository snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
BUILDDIR = os.path.join(HERE, "lib", "obj")
LIB = os.path.join(LIBDIR, "libpfe.so")
SOURCES = ["capi.hip", "lyon8.hip", "bates22.hip", "bates_sine_dm_sub.hip", "bates_gauss.hip", "bates_gauss_peel.hip",
           "bates_gauss_dg8.hip", "subband.hip",
           "pfd.hip", "pfd22.hip"]
# The Levenberg-Marquardt translation units are compiled without the two-address v_fmac_f64:
# with it the register allocator copies the accumulator (a v_mov_b64 per fma whose addend
# stays live -- every polynomial coefficient of exp, every Householder update), ~600 extra
# VALU per k_gdgg; the three-address v_fma_f64 needs none.  Same operations, same bits
# (tools/ab.sh exact), k_gdgg / k_gdg8g 3-4 % faster (profiles/r06_ab_no_fmac.txt).  The
# host half of hipcc ignores the feature with a warning.
NO_FMAC = ["-Xclang", "-target-feature", "-Xclang", "-fmacf64-inst"]
NO_FMAC_SOURCES = {"bates_sine_dm_sub.hip", "bates_gauss.hip", "bates_gauss_peel.hip",
                   "bates_gauss_dg8.hip", "pfd22.hip"}
HOST_SOURCES = ["phcx_io.cpp"]  # host-only C++ (PHCX reader / batch packer), built with g++
HOST_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-pthread"]
ARCH = os.environ.get("PFE_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (set HIPCC or install ROCm)")


COMMON = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    # Keep every fp64 operation individually rounded, as numpy evaluates it: no FMA
    # contraction and no fast-math in any kernel (parity with the reference's arithmetic).
    "-ffp-contract=off",
    "-fno-fast-math",
    "-Wall",
    "-Wno-unused-function",
]


def _needs(obj: str, deps: list[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, force: bool = False, variant: str = "",
          defines: tuple[str, ...] = (), csrc: str | None = None,
          flags: tuple[str, ...] = ()) -> str:
    """Compile every source and link lib/libpfe.so.  A non-empty ``variant`` builds an
    instrumented copy (lib/libpfe_<variant>.so, objects under lib/obj_<variant>/) with the
    extra -D ``defines`` (e.g. the LM phase-cycle profiler, -DPFE_LM_PROFILE); the product
    library is never built with them.  ``csrc``: another source tree for a variant (an A/B
    against an earlier revision: tools/build_variant.py); ``flags``: extra compiler arguments of
    a variant's kernels."""
    CSRC = csrc or globals()["CSRC"]
    builddir = BUILDDIR + (f"_{variant}" if variant else "")
    lib = os.path.join(LIBDIR, f"libpfe_{variant}.so") if variant else LIB
    extra = [f"-D{d}" for d in defines]
    kflags = list(flags)
    os.makedirs(builddir, exist_ok=True)
    cc = hipcc()
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers.append(os.path.join(HERE, "..", "include", "pfe.h"))
    objs = []
    jobs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(builddir, src.replace(".hip", ".o"))
        objs.append(o)
        if force or _needs(o, [s] + headers):
            tu = NO_FMAC if src in NO_FMAC_SOURCES else []
            jobs.append([cc, *COMMON, *tu, *extra, *kflags, "-c", s, "-o", o])

    cxx = shutil.which("g++") or "g++"
    for src in HOST_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(builddir, src.replace(".cpp", ".o"))
        objs.append(o)
        if force or _needs(o, [s] + headers + [os.path.join(HERE, "..", "include", "pfe_io.h")]):
            jobs.append([cxx, *HOST_FLAGS, *extra, "-c", s, "-o", o])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    if force or jobs or not os.path.exists(lib):
        tmp = lib + ".tmp"
        run([cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs, "-lz", "-ldl", "-pthread"])
        os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    if "--lm-profile" in sys.argv:
        print(build(verbose=True, force="--force" in sys.argv, variant="lmprof",
                    defines=("PFE_LM_PROFILE",)))
    else:
        print(build(verbose=True, force="--force" in sys.argv))
