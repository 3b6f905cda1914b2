"""Build libertdiff_hip.so (gfx950 only) in-tree with hipcc.

    python ert-conditional-diffusion-model_amd/build.py [--force] [--verbose] [--diag]

The shared library lands next to the Python drop-in module
(ertdiff/libertdiff_hip.so) so it travels with the repo snapshot to the GPU
box.  Sources are compiled in parallel into objects under build/ and linked
once; a source is rebuilt when it or any header is newer than its object.

--diag builds the diagnostic variant instead (-DERTD_DIAG, objects under
build/diag/, ertdiff/libertdiff_hip_diag.so): the only build that reads the
ERTD_* schedule knobs and has the ablation kernels (csrc/unet.h ERTD_KNOB).
Tools load it through ERTD_LIB_PATH for same-box A/B; nothing else does.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
BUILD = os.path.join(PKG, "build")
OUT = os.path.join(PKG, "ertdiff", "libertdiff_hip.so")
OUT_DIAG = os.path.join(PKG, "ertdiff", "libertdiff_hip_diag.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CFLAGS = [
    "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
    # exact fp32 op sequences (no implicit contraction): the update and the
    # dot-product chains must round exactly as written
    "-ffp-contract=off",
    "-Wall", "-Wno-unused-function",
    "-I", INCLUDE, "-I", CSRC,
]


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    return hs


def _stale(obj, src, newest_header):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or newest_header > t


def build(force: bool = False, verbose: bool = False, diag: bool = False) -> str:
    bdir = os.path.join(BUILD, "diag") if diag else BUILD
    out = OUT_DIAG if diag else OUT
    flags = CFLAGS + (["-DERTD_DIAG"] if diag else [])
    os.makedirs(bdir, exist_ok=True)
    srcs = _sources()
    newest_h = max([os.path.getmtime(h) for h in _headers()] + [0.0])
    objs, jobs = [], []
    for s in srcs:
        o = os.path.join(bdir, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if force or _stale(o, s, newest_h):
            jobs.append([HIPCC, *flags, "-c", s, "-o", o])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {cmd[-3]}:\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr.strip():
            print(r.stderr, flush=True)

    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            list(ex.map(run, jobs))
    if jobs or force or not os.path.exists(out) or any(
            os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", out])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--diag", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, verbose=a.verbose, diag=a.diag))


if __name__ == "__main__":
    sys.exit(main())
