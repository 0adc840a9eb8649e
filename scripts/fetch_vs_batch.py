#!/usr/bin/env python
"""FETCH_SIZE / WRITE_SIZE of the step kernel against the batch size (the
passes of scripts/passes/gpu_r06m.sh): per-launch bytes (FETCH x 2, the gfx950
correction of summarize_profiles.py) for each run directory
gpurun_out/<prefix>_<tag>_{fetch,write}/ (prefix: argv[1], default fvb), and a least-squares line bytes = a + b B
per kernel, to split the per-launch traffic into a part that grows with the
envs and a fixed part."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def per_launch(path, counter):
    vals = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter and "k_step" in r["Kernel_Name"]:
                vals[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return {k: float(np.mean(v[2:] if len(v) > 4 else v)) for k, v in vals.items()}


def main():
    pre = sys.argv[1] if len(sys.argv) > 1 else "fvb"
    rows = []
    for d in sorted(glob.glob(os.path.join(OUT, f"{pre}_*_fetch"))):
        tag = os.path.basename(d)[len(pre) + 1:-6]  # <env>_<batch>_<lanes>
        m = re.match(r"(.+)_(\d+)_(\d+)$", tag)
        env, B, lanes = m.group(1), int(m.group(2)), int(m.group(3))
        fp = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        wp = glob.glob(os.path.join(OUT, f"{pre}_{tag}_write", "**", "*counter_collection.csv"), recursive=True)
        f = per_launch(fp[0], "FETCH_SIZE")
        w = per_launch(wp[0], "WRITE_SIZE")
        for k in f:
            rows.append((env, lanes, k, B, 2.0 * f[k] * 1024, w.get(k, 0.0) * 1024))
    print(f"{'env':22s} {'lanes':>5s} {'envs':>7s} {'fetch MB':>9s} {'write MB':>9s}  kernel")
    for env, lanes, k, B, fb, wb in sorted(rows):
        print(f"{env:22s} {lanes:5d} {B:7d} {fb / 1e6:9.3f} {wb / 1e6:9.3f}  {k}")
    fits = defaultdict(list)
    for env, lanes, k, B, fb, wb in rows:
        fits[(env, lanes)].append((B, fb, wb))
    for (env, lanes), pts in sorted(fits.items()):
        if len(pts) < 2:
            continue
        B = np.array([p[0] for p in pts], float)
        for name, col in (("fetch", 1), ("write", 2)):
            y = np.array([p[col] for p in pts])
            b, a = np.polyfit(B, y, 1)
            print(f"{env} lanes {lanes} {name}: {a / 1e6:.3f} MB per launch + {b:.1f} B per env")


if __name__ == "__main__":
    sys.exit(main())
