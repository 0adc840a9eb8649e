#!/usr/bin/env python
"""Scripted grasp-and-lift on PandaPickAndPlace-v3: the
end effector moves above the cube with the gripper open, descends to the
cube's centre, closes, and lifts to 0.15 m; a grasp succeeds when the cube is
above 0.08 m at the end (its rest height is 0.02 m).

  python scripts/grasp_success.py oracle [N] [ORACLE_DIR]   fp64 oracle, N envs
  python scripts/grasp_success.py gpu [N]                   fused GPU step, N envs

ORACLE_DIR selects another oracle build (e.g. one of an older commit's
geometry, for a before/after comparison).  Prints one JSON line.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PHASES = ((0, 15, "above"), (15, 25, "descend"), (25, 35, "close"), (35, 60, "lift"))


DZ = float(os.environ.get("GRASP_DZ", "0.0"))  # grasp height above the cube's centre


def tilt_deg(quat: np.ndarray) -> np.ndarray:
    """Angle between the cube's z axis and the world z axis, degrees."""
    x, y = quat[:, 0], quat[:, 1]
    return np.degrees(np.arccos(np.clip(1.0 - 2.0 * (x * x + y * y), -1.0, 1.0)))


def policy(s: int, ee: np.ndarray, cube: np.ndarray) -> np.ndarray:
    """Actions [B, 4] of step s from the ee and cube positions [B, 3]."""
    tgt = cube.copy()
    tgt[:, 2] += DZ
    grip = np.ones(len(ee))
    if s < 15:
        tgt[:, 2] += 0.06
    elif s < 25:
        pass
    elif s < 35:
        grip[:] = -1.0
    else:
        tgt[:, 2] = 0.15
        grip[:] = -1.0
    a = np.zeros((len(ee), 4), np.float32)
    a[:, :3] = np.clip(10.0 * (tgt - ee), -1, 1)
    a[:, 3] = grip
    return a


def run_oracle(n: int, oracle_dir: str) -> dict:
    sys.path.insert(0, oracle_dir)
    import oracle as O

    cfg = O.config("pick_and_place", "ee")
    envs = [O.new_env(cfg) for _ in range(n)]
    for i, e in enumerate(envs):
        O.reset(cfg, e, seed=1000 + i)
    t0 = time.perf_counter()
    for s in range(60):
        ee = np.array([O.link_state(cfg, e, 11)[0] for e in envs])
        cube = np.array([list(e.obj[0].pos) for e in envs])
        a = policy(s, ee, cube)
        for i, e in enumerate(envs):
            O.step(cfg, e, a[i])
    z = np.array([e.obj[0].pos[2] for e in envs])
    tilt = tilt_deg(np.array([list(e.obj[0].quat) for e in envs]))
    return {"path": "oracle", "oracle": oracle_dir, "envs": n, "grasp_dz": DZ, "success": float((z > 0.08).mean()),
            "cube_z_median": float(np.median(z)), "tilt_deg_median": float(np.median(tilt)),
            "tilt_deg_max": float(tilt.max()), "seconds": round(time.perf_counter() - t0, 1)}


def run_gpu(n: int) -> dict:
    import torch

    sys.path.insert(0, os.path.join(ROOT, "panda-lang-manip_amd"))
    from pandasim.envs import PandaVecEnv

    env = PandaVecEnv("pick_and_place", "sparse", "ee", n, "cuda", autoreset=False)
    env.reset(seed=(1000 + np.arange(n)).astype(np.uint64))
    for s in range(60):
        ee = env.sim.get_link_position("panda", 11).double().cpu().numpy()
        cube = env.sim.get_base_position("object").double().cpu().numpy()
        env.step(torch.from_numpy(policy(s, ee, cube)).cuda())
    z = env.sim.get_base_position("object")[:, 2].double().cpu().numpy()
    tilt = tilt_deg(env.sim.get_base_orientation("object").double().cpu().numpy())
    return {"path": "gpu", "envs": n, "lanes_per_env": env.lanes_per_env, "grasp_dz": DZ,
            "success": float((z > 0.08).mean()), "cube_z_median": float(np.median(z)),
            "tilt_deg_median": float(np.median(tilt)), "tilt_deg_max": float(tilt.max())}


if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else "oracle"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    if mode == "gpu":
        print(json.dumps(run_gpu(n)))
    else:
        print(json.dumps(run_oracle(n, sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "oracle"))))
