"""Build libpandasim.so in-tree with hipcc for gfx950 (no JIT, no torch extension)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
OUT = os.path.join(HERE, "libpandasim.so")
SOURCES = ["pandasim.hip"]


def deps() -> list:
    """Every source the library is built from: all of csrc/ (the kernels
    include each header there) and the two public headers."""
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".h")))

HEADERS = [os.path.join(ROOT, "include", h) for h in ("pandasim.h", "panda_model.h")]


# diagnostic variants (never loaded by the product unless PANDASIM_LIB names them)
VARIANTS = {"": [], "prof": ["-DPS_PROFILE_PHASES"]}


def out_path(variant: str = "") -> str:
    return OUT if not variant else os.path.join(HERE, f"libpandasim_{variant}.so")


def needs_build(variant: str = "") -> bool:
    out = out_path(variant)
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(p) > t for p in deps() + HEADERS)


def build(force: bool = False, verbose: bool = True, variant: str = "", extra=()) -> str:
    out = out_path(variant)
    if not force and not extra and not needs_build(variant):
        return out
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    # -fno-slp-vectorize: SLP packing into v_pk_fma_f32 pairs made the register
    # allocator spill 590 VGPRs of the step kernel to scratch
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize", "-fPIC", "-shared", "-I", os.path.join(ROOT, "include"),
           *VARIANTS[variant], *extra, "-o", out + ".tmp"] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, variant="prof" if "--prof" in sys.argv else "")
