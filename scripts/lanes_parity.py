#!/usr/bin/env python
"""Teacher-forced parity of one step-kernel variant (test_gpu_parity.py's
test_env_step_parity_teacher_forced workload: 64 envs, seeds 12345 + i, 10
steps of default_rng(7) actions, each GPU step judged against one oracle step
from the same state by tests/parity_judge.judge), for a library and a lanes-per-
env value the test suite does not parametrise -- the round-6 G = 2 experiment
(PANDASIM_LIB=scripts/bin/variants/lib_g2.so).

  PANDASIM_LIB=... python scripts/lanes_parity.py LANES TASK CONTROL
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "panda-lang-manip_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

import oracle as O  # noqa: E402
from helpers import oracle_config_for, oracle_env_from, snapshot  # noqa: E402
from parity_judge import FREE_GRIPPER, groups_for, judge  # noqa: E402


def main(lanes, task, control):
    from pandasim.envs import PandaVecEnv

    B, steps = 64, 10
    env = PandaVecEnv(task, "sparse", control, B, "cuda", lanes_per_env=lanes)
    assert env.lanes_per_env == lanes, env.lanes_per_env
    env.autoreset = False
    env.reset(seed=12345)
    cfg = oracle_config_for(env.sim.cfg)
    rng = np.random.default_rng(7)
    groups = groups_for(task, 7 if task in FREE_GRIPPER else 6)
    counts = {"tight": 0, "conditioned": 0, "bif": 0, "beyond": 0}
    for s in range(steps):
        snap = snapshot(env.sim)
        a = rng.uniform(-1, 1, size=(B, env.action_dim)).astype(np.float32)
        obs, *_ = env.step(torch.from_numpy(a).cuda())
        og = obs["observation"].cpu().numpy()
        for i in range(B):
            o, *_ = O.step(cfg, oracle_env_from(cfg, snap, i), a[i])
            cls, _ = judge(cfg, snap, i, a[i], o, og[i], groups, task)
            counts[cls] += 1
    print(f"lanes {lanes} {task} {control}: {counts}", flush=True)
    return counts["beyond"] == 0


if __name__ == "__main__":
    ok = main(int(sys.argv[1]), sys.argv[2], sys.argv[3])
    sys.exit(0 if ok else 1)
