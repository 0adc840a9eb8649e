#!/usr/bin/env python
"""Register, scratch and LDS use of every step kernel of a built object or
library, from the code objects' AMDGPU metadata (no GPU needed).

usage: python scripts/kernel_resources.py [lib or .o ...] [--json out.json]
(default: the product library's objects under pandasim/build/libpandasim/)
"""
from __future__ import annotations

import glob
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
FIELDS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
          ".private_segment_fixed_size", ".group_segment_fixed_size")


def code_objects(path: str, tmp: str) -> list:
    """Device code objects of a host object/library (clang-offload-bundler)."""
    out = os.path.join(tmp, os.path.basename(path) + ".gfx950")
    r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={path}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={out}"], capture_output=True)
    if r.returncode == 0 and os.path.getsize(out) > 0:
        return [out]
    # a linked library: extract the fat binary's bundles
    r = subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={out}.fatbin", path, os.devnull],
                       capture_output=True)
    if r.returncode != 0:
        return []
    r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={out}.fatbin",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={out}"], capture_output=True)
    return [out] if r.returncode == 0 else []


def kernels(co: str) -> dict:
    txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    res, cur = {}, None
    for line in txt.splitlines():
        m = re.match(r"\s*-?\s*\.name:\s+(\S+)", line)
        if m and "k_" in m.group(1):
            cur = m.group(1)
            res[cur] = {}
            continue
        for f in FIELDS:
            m = re.match(r"\s*" + re.escape(f) + r":\s+(\d+)", line)
            if m and cur:
                res[cur][f[1:]] = int(m.group(1))
    return res


def demangle(name: str) -> str:
    r = subprocess.run(["c++filt", name], capture_output=True, text=True)
    return r.stdout.strip().replace("(anonymous namespace)::", "").split("(")[0]


def main(argv):
    out_json = None
    if "--json" in argv:
        i = argv.index("--json")
        out_json = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    paths = argv or sorted(glob.glob(os.path.join(ROOT, "panda-lang-manip_amd", "pandasim", "build", "libpandasim",
                                                  "step_*.o")))
    table = {}
    with tempfile.TemporaryDirectory() as tmp:
        for p in paths:
            for co in code_objects(p, tmp):
                for k, v in kernels(co).items():
                    if "k_step" in k or "k_sim_step" in k:
                        table[demangle(k)] = v
    for k, v in sorted(table.items()):
        print(f"{k:40s} vgpr {v.get('vgpr_count', 0):3d} agpr {v.get('agpr_count', 0):3d} "
              f"scratch {v.get('private_segment_fixed_size', 0):4d} B  spill v {v.get('vgpr_spill_count', 0):3d} "
              f"s {v.get('sgpr_spill_count', 0):3d}  lds {v.get('group_segment_fixed_size', 0)}")
    if out_json:
        json.dump(table, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
