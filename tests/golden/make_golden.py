"""Generate the task-layer golden vectors from the reference's own task classes.

Run in the survey/build container (it needs /root/reference; the GPU box does
not have it):  python tests/golden/make_golden.py

What is imported from the reference: panda_gym.envs.tasks.{reach,push,
pick_and_place} (Task subclasses) and panda_gym.utils.  Their third-party
imports that are absent here (gymnasium, pybullet, pybullet_data,
pybullet_utils, cv2) are replaced by empty placeholder modules so that the
modules import; nothing from them is used by the code paths exercised below
(goal/object sampling, is_success, compute_reward).  The simulator handed to
the tasks is a recorder that only stores set_base_pose() calls.

The RNG is built exactly as gymnasium.utils.seeding.np_random does (gymnasium
0.26-0.28): Generator(PCG64(SeedSequence(seed))), and assigned to
task.np_random as RobotTaskEnv.reset does (panda_gym/envs/core.py:244).

Output: tests/golden/task_layer.npz (data only).
"""
from __future__ import annotations

import contextlib
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "task_layer.npz")


def _placeholder_modules():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class _Space:
        def __init__(self, *a, **k):
            pass

    class _Env:
        pass

    spaces = mod("gymnasium.spaces", Box=_Space, Dict=_Space, Space=_Space)
    seeding = mod("gymnasium.utils.seeding")
    utils = mod("gymnasium.utils", seeding=seeding)
    registration = mod("gymnasium.envs.registration", register=lambda **k: None)
    envs = mod("gymnasium.envs", registration=registration)
    mod("gymnasium", spaces=spaces, utils=utils, envs=envs, Env=_Env)
    mod("pybullet")
    mod("pybullet_data", getDataPath=lambda: "")
    bc = mod("pybullet_utils.bullet_client")
    mod("pybullet_utils", bullet_client=bc)
    mod("cv2")
    if not hasattr(np, "bool8"):
        np.bool8 = np.bool_  # removed in numpy 2; the reference tasks still name it


class RecorderSim:
    """Stands in for panda_gym.pybullet.PyBullet: records set_base_pose()."""

    def __init__(self):
        self.poses = {}

    @contextlib.contextmanager
    def no_rendering(self):
        yield

    def __getattr__(self, name):
        return lambda *a, **k: None

    def set_base_pose(self, body, position, orientation):
        self.poses[body] = (np.array(position, dtype=np.float64), np.array(orientation, dtype=np.float64))


def seeded_rng(seed):
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))


def main():
    sys.dont_write_bytecode = True
    _placeholder_modules()
    sys.path.insert(0, REF)
    from panda_gym.envs.tasks.pick_and_place import PickAndPlace
    from panda_gym.envs.tasks.push import Push
    from panda_gym.envs.tasks.reach import Reach

    seeds = [0, 1, 2, 7, 42, 6789, 12345, 13795, 657894, 794512, 2**31 - 1, 2**32 - 1, 2**32, 2**40 + 3,
             2**63 + 11, 2**64 - 1] + list(range(100, 300))
    seeds = np.array(seeds, dtype=np.uint64)
    out = {"seeds": seeds}
    n_resets = 4  # first reset seeded, the next ones continue the same generator
    for name, cls in [("reach", Reach), ("push", Push), ("pick_and_place", PickAndPlace)]:
        goals = np.zeros((len(seeds), n_resets, 3))
        objs = np.zeros((len(seeds), n_resets, 3))
        for i, s in enumerate(seeds):
            sim = RecorderSim()
            if cls is Reach:
                task = cls(sim, get_ee_position=lambda: np.zeros(3))
            else:
                task = cls(sim)
            task.np_random = seeded_rng(int(s))
            for r in range(n_resets):
                task.reset()
                goals[i, r] = task.goal
                if "object" in sim.poses:
                    objs[i, r] = sim.poses["object"][0]
        out[f"{name}_goal"] = goals
        out[f"{name}_object"] = objs

    # reward / success (utils.distance: fp32 achieved goal vs fp64 goal)
    rng = np.random.default_rng(2024)
    n = 4096
    dg = rng.uniform(-0.2, 0.2, size=(n, 3))
    ag = (dg + rng.normal(scale=0.04, size=(n, 3))).astype(np.float32)
    # points at distance ~0.05 to exercise the threshold
    direction = rng.normal(size=(512, 3))
    direction /= np.linalg.norm(direction, axis=1, keepdims=True)
    ag[:512] = (dg[:512] + direction * (0.05 + rng.uniform(-1e-6, 1e-6, size=(512, 1)))).astype(np.float32)
    ag[512] = dg[512].astype(np.float32)
    out["reward_ag"] = ag
    out["reward_dg"] = dg
    sim = RecorderSim()
    for reward_type in ["sparse", "dense"]:
        task = Push(sim, reward_type=reward_type)
        out[f"reward_{reward_type}"] = np.asarray(task.compute_reward(ag, dg, {}), dtype=np.float32)
        out["success"] = np.asarray(task.is_success(ag, dg), dtype=np.bool_)
    # HER-style batched call with fp32 desired goals and extra leading dims
    ag3 = ag[:1024].reshape(32, 32, 3)
    dg3 = dg[:1024].astype(np.float32).reshape(32, 32, 3)
    out["her_ag"] = ag3
    out["her_dg"] = dg3
    out["her_reward_sparse"] = np.asarray(Push(sim, reward_type="sparse").compute_reward(ag3, dg3, {}), np.float32)
    out["her_reward_dense"] = np.asarray(Push(sim, reward_type="dense").compute_reward(ag3, dg3, {}), np.float32)
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
