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
    from panda_gym.envs.tasks.flip import Flip
    from panda_gym.envs.tasks.pick_and_place import PickAndPlace
    from panda_gym.envs.tasks.push import Push
    from panda_gym.envs.tasks.reach import Reach
    from panda_gym.envs.tasks.slide import Slide
    from panda_gym.envs.tasks.stack import Stack

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

    # --- Slide, Stack, Flip (draws from task.np_random).
    # Flip's goal comes from scipy's Rotation.random() on numpy's unseeded
    # global RandomState (flip.py:70-72): only its object draws are seeded.
    for name, cls in [("slide", Slide), ("stack", Stack), ("flip", Flip)]:
        goals = np.zeros((len(seeds), n_resets, 6 if cls is Stack else 3))
        objs = np.zeros((len(seeds), n_resets, 6 if cls is Stack else 3))
        for i, s in enumerate(seeds):
            sim = RecorderSim()
            task = cls(sim)
            task.np_random = seeded_rng(int(s))
            for r in range(n_resets):
                task.reset()
                if cls is Stack:
                    goals[i, r] = task.goal
                    objs[i, r, :3] = sim.poses["object1"][0]
                    objs[i, r, 3:] = sim.poses["object2"][0]
                elif cls is Slide:
                    goals[i, r] = task.goal
                    objs[i, r] = sim.poses["object"][0]
                else:
                    objs[i, r] = sim.poses["object"][0]
                    assert np.array_equal(sim.poses["object"][1], np.zeros(3))  # Euler zeros
        if cls is not Flip:
            out[f"{name}_goal"] = goals
        out[f"{name}_object"] = objs

    rng = np.random.default_rng(2025)
    # Stack: 6-D goals, threshold 0.1 (stack.py:118-131)
    dg6 = rng.uniform(-0.2, 0.2, size=(n, 6))
    ag6 = (dg6 + rng.normal(scale=0.04, size=(n, 6))).astype(np.float32)
    dir6 = rng.normal(size=(512, 6))
    dir6 /= np.linalg.norm(dir6, axis=1, keepdims=True)
    ag6[:512] = (dg6[:512] + dir6 * (0.1 + rng.uniform(-1e-6, 1e-6, size=(512, 1)))).astype(np.float32)
    out["stack_ag"], out["stack_dg"] = ag6, dg6
    for reward_type in ["sparse", "dense"]:
        task = Stack(RecorderSim(), reward_type=reward_type)
        out[f"stack_reward_{reward_type}"] = np.asarray(task.compute_reward(ag6, dg6, {}), dtype=np.float32)
        out["stack_success"] = np.asarray(task.is_success(ag6, dg6), dtype=np.bool_)
    # Flip: angle_distance on single (float32 achieved, float64 desired)
    # quaternion pairs, as RobotTaskEnv.step calls it (core.py:285-288);
    # batched inputs would hit np.inner's outer-product semantics (utils.py:29)
    qd = rng.normal(size=(n, 4))
    qd /= np.linalg.norm(qd, axis=1, keepdims=True)
    qa = qd + rng.normal(scale=0.3, size=(n, 4))
    qa = (qa / np.linalg.norm(qa, axis=1, keepdims=True)).astype(np.float32)
    out["flip_ag"], out["flip_dg"] = qa, qd
    for reward_type in ["sparse", "dense"]:
        task = Flip(RecorderSim(), reward_type=reward_type)
        out[f"flip_reward_{reward_type}"] = np.array([task.compute_reward(a, d, {}) for a, d in zip(qa, qd)],
                                                     dtype=np.float32)
        out["flip_success"] = np.array([task.is_success(a, d) for a, d in zip(qa, qd)], dtype=np.bool_)
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
