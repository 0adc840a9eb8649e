#!/usr/bin/env python
"""Runs an env for a few steps of the phase profiler's action stream and saves
the whole state (and the robot-contact cache ids) to an npz, so two builds of
the library can be compared bit for bit (PANDASIM_LIB selects the build):

  PANDASIM_LIB=.../libpandasim_prof.so python scripts/state_after_steps.py PandaPush-v3 65536 25 out.npz
  python scripts/state_after_steps.py --compare a.npz b.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "panda-lang-manip_amd"))


def run(env_id, B, steps, out):
    import torch

    import pandasim

    env = pandasim.make(env_id, num_envs=B)
    env.reset(seed=12345)
    g = torch.Generator(device="cuda")
    g.manual_seed(0xC0FFEE)
    for _ in range(steps):
        env.step(torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1, copy=False)
    torch.cuda.synchronize()
    np.savez_compressed(out, f=env.sim.f[:, :B].cpu().numpy())


def compare(a, b):
    fa, fb = np.load(a)["f"], np.load(b)["f"]
    diff = fa != fb
    rows = np.nonzero(diff.any(1))[0]
    print(f"{a} vs {b}: {int(diff.any(0).sum())} of {fa.shape[1]} envs differ; rows {rows.tolist()[:40]}; "
          f"max |d| {np.nanmax(np.abs(fa - fb)) if diff.any() else 0.0:.3e}")


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
