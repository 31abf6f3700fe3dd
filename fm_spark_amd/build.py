"""Build libfm_hip.so (HIP for gfx950) in-tree with hipcc.  No JIT cache, no setuptools:
the .so lands in fm_spark_amd/lib/ so it travels with the repo snapshot to the GPU box."""

from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIB_DIR = PKG / "lib"
LIB = LIB_DIR / "libfm_hip.so"
INCLUDE = PKG.parent / "include"
ARCH = os.environ.get("FM_HIP_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = ["fm_kernels.hip", "fm_sort.hip", "fm_capi.hip", "fm_shard.hip", "fm_group.hip", "fm_sampler.cpp",
           "fm_libsvm.cpp"]
HEADERS = ["fm_internal.h", "fm_device.h", "fm_context.h", "fm_hostpool.h"]

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


def _newer(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def build(verbose: bool = False, force: bool = False, out: Path | None = None, defines=()) -> Path:
    """Build the library (incrementally).  ``out``/``defines``: an experiment variant with
    extra -D flags, built into its own object directory (tools/variants.sh)."""
    lib = Path(out) if out else LIB
    lib.parent.mkdir(parents=True, exist_ok=True)
    objdir = (LIB_DIR / "obj") if out is None else lib.parent / (lib.stem + "_obj")
    objdir.mkdir(exist_ok=True)
    dflags = [f"-D{d}" for d in defines]
    headers = [CSRC / h for h in HEADERS] + [INCLUDE / "fm_hip.h"]
    objs = []
    for src in SOURCES:
        s = CSRC / src
        o = objdir / (src + ".o")
        objs.append(o)
        if force or _newer(o, [s, *headers]):
            if src.endswith(".hip"):
                cmd = [HIPCC, f"--offload-arch={ARCH}", *CXXFLAGS, *dflags, "-c", str(s), "-o", str(o)]
            else:
                cmd = [HIPCC, *CXXFLAGS, "-x", "c++", "-c", str(s), "-o", str(o)]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)
    if force or _newer(lib, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(lib),
               "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    return lib


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("-D", dest="defines", action="append", default=[])
    args = ap.parse_args()
    print(build(verbose=True, force=args.force, out=args.out, defines=args.defines))
