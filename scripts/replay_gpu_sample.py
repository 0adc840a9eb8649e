#!/usr/bin/env python
"""Replays dumped teacher-forced samples (gpurun_out/tf200/*.npz) on the GPU
with the one-lane and the 8/16-lane step kernels and prints each kernel's
distance from the fp64 oracle's step and from the dumped GPU observation --
whether a sample's difference belongs to one kernel or to the fp32 path.

  python scripts/replay_gpu_sample.py gpurun_out/tf200/push_ee_171_60.npz [...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "panda-lang-manip_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

import oracle as O  # noqa: E402
from helpers import oracle_env_from  # noqa: E402


def replay(path):
    from pandasim.envs import PandaVecEnv

    name = os.path.basename(path)[:-4]
    task, control = name.rsplit("_", 3)[0], name.rsplit("_", 3)[1]
    d = np.load(path)
    cfg = O.config(task, control)
    snap = {"f": d["f"][:, None], "goal": d["goal"][:, None], "rng": d["rng"][:, None],
            "elapsed": np.array([int(d["elapsed"])])}
    o, *_ = O.step(cfg, oracle_env_from(cfg, snap, 0), d["action"])
    out = [f"{name}: dumped GPU vs oracle {np.abs(d['gpu_obs'] - o)[:6].max():.2e}"]
    B = 64
    for lanes in (1, 8, 16):
        env = PandaVecEnv(task, "sparse", control, B, "cuda", lanes_per_env=lanes)
        env.autoreset = False
        env.reset(seed=1)
        env.sim.f[:, :B] = torch.from_numpy(np.repeat(d["f"][:, None], B, axis=1)).to(env.sim.f.dtype).cuda()
        env.sim.goal[:, :B] = torch.from_numpy(np.repeat(d["goal"][:, None], B, axis=1)).to(env.sim.goal.dtype).cuda()
        env.sim.elapsed[:B] = int(d["elapsed"]) % env.max_episode_steps
        env.sim._call("ps_mark_motor_rows_dirty", env.sim._ctx)
        a = torch.from_numpy(np.repeat(d["action"][None, :], B, axis=0)).cuda()
        obs, *_ = env.step(a)
        g = obs["observation"][0].cpu().numpy()
        out.append(f"lanes {lanes:2d}: vs oracle {np.abs(g - o)[:6].max():.2e}, vs dumped {np.abs(g - d['gpu_obs'])[:6].max():.2e}")
    print("; ".join(out), flush=True)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        replay(p)
