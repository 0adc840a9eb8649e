"""Bit-for-bit comparison of two libpandasim builds: every task (ee and
joints control) at B envs for K steps with the same seeded resets and
actions, each library in its own process (PANDASIM_LIB); prints per task the
number of state floats that differ and the largest difference.  For changes
meant to keep the arithmetic (instruction selection, data placement).
Usage: python scripts/compare_libs.py LIB_A LIB_B [B] [K]"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, numpy as np, torch
sys.path.insert(0, os.path.join(os.environ["ROOT"], "panda-lang-manip_amd"))
from pandasim.envs import PandaVecEnv
B, K = int(os.environ["B"]), int(os.environ["K"])
out = {}
LANES = int(os.environ.get("LANES", "0"))
for task in ("reach", "push", "pick_and_place", "slide", "flip") + (("stack",) if LANES <= 1 else ()):
    for control in ("ee", "joints"):
        env = PandaVecEnv(task, "sparse", control, B, "cuda", lanes_per_env=LANES)
        env.reset(seed=7)
        g = torch.Generator(device="cuda"); g.manual_seed(3)
        for k in range(K):
            a = torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1
            env.step(a)
        out[f"{task}_{control}"] = env.sim.f[:, :B].cpu().numpy()
np.savez(os.environ["OUT"], **out)
'''


def run(lib, path, B, K):
    env = dict(os.environ, PANDASIM_LIB=os.path.abspath(lib), ROOT=ROOT, OUT=path, B=str(B), K=str(K))
    subprocess.run([sys.executable, "-c", CHILD], env=env, check=True, timeout=900)
    return dict(np.load(path))


def main():
    a, b = sys.argv[1], sys.argv[2]
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    K = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    with tempfile.TemporaryDirectory() as d:
        ra, rb = run(a, os.path.join(d, "a.npz"), B, K), run(b, os.path.join(d, "b.npz"), B, K)
    same = True
    for k in ra:
        x, y = ra[k], rb[k]
        neq = ~((x == y) | (np.isnan(x) & np.isnan(y)))
        same &= not neq.any()
        print(f"{k:22s} differing floats {int(neq.sum()):8d} of {x.size}  envs {int(neq.any(0).sum()):5d}  "
              f"max |diff| {float(np.nanmax(np.abs(x - y))) if neq.any() else 0.0:.3e}", flush=True)
    print("bit-identical" if same else "DIFFERENT", os.path.basename(a), os.path.basename(b), f"B={B} K={K}")


if __name__ == "__main__":
    main()
