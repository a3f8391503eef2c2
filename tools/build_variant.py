#!/usr/bin/env python3
"""Build an A/B variant of libpfe.so (host side, in the build container).

  tools/build_variant.py NAME [--rev REV] [-D DEF ...] [--flag=ARG ...]

-> pulsarfeatureextractor_amd/lib/libpfe_NAME.so, from the kernel sources (csrc/ and
include/) of git revision REV (default: the working tree) with the extra -D definitions and
compiler arguments (--flag=-Xclang, one argument each).
The variant's objects go to lib/obj_NAME/; the product library is not touched.  Run the A/B
on the GPU box with tools/ab.sh.
"""
import argparse
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def export(rev: str, dst: str) -> str:
    """csrc/ and include/ of `rev` under dst (the relative ../../include paths kept)."""
    csrc = os.path.join(dst, "p", "csrc")
    os.makedirs(csrc)
    os.makedirs(os.path.join(dst, "include"))
    for sub, out in (("pulsarfeatureextractor_amd/csrc", csrc), ("include", os.path.join(dst, "include"))):
        names = subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", f"{rev}:{sub}"],
                               check=True, capture_output=True, text=True).stdout.split()
        for n in names:
            data = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:{sub}/{n}"], check=True,
                                  capture_output=True).stdout
            with open(os.path.join(out, n), "wb") as f:
                f.write(data)
    return csrc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--rev", default=None)
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--flag", dest="flags", action="append", default=[])
    a = ap.parse_args()
    from pulsarfeatureextractor_amd import build as b

    tmp = None
    csrc = None
    if a.rev:
        tmp = tempfile.mkdtemp(prefix=f"pfe_variant_{a.name}_")
        csrc = export(a.rev, tmp)
    try:
        print(b.build(verbose=False, force=True, variant=a.name, defines=tuple(a.defines),
                      csrc=csrc, flags=tuple(a.flags)))
    finally:
        if tmp:
            shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
