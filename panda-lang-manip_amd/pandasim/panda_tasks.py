"""Env wiring of panda_gym/envs/panda_tasks.py:31-79 over the plugin path:
batched PandaSim + Panda(base=(-0.6, 0, 0)) + task, composed by RobotTaskEnv.

These are the unfused counterparts of the registered IDs (same robot, task,
scene and constants); ``pandasim.make(id, fused=False)`` builds them wrapped
in TimeLimit(50) as gym.make does.
"""
from __future__ import annotations

import numpy as np

from .core import RobotTaskEnv
from .robots import Panda
from .sim import PandaSim
from .tasks import PickAndPlace, Push, Reach

BASE = np.array([-0.6, 0.0, 0.0])


class PandaPickAndPlaceEnv(RobotTaskEnv):
    """panda_tasks.py:31-46."""

    def __init__(self, num_envs: int = 1, device="cuda", reward_type: str = "sparse", control_type: str = "ee"):
        sim = PandaSim(task=None, num_envs=num_envs, device=device)
        robot = Panda(sim, block_gripper=False, base_position=BASE, control_type=control_type)
        task = PickAndPlace(sim, reward_type=reward_type)
        super().__init__(robot, task)


class PandaPushEnv(RobotTaskEnv):
    """panda_tasks.py:49-62."""

    def __init__(self, num_envs: int = 1, device="cuda", reward_type: str = "sparse", control_type: str = "ee"):
        sim = PandaSim(task=None, num_envs=num_envs, device=device)
        robot = Panda(sim, block_gripper=True, base_position=BASE, control_type=control_type)
        task = Push(sim, reward_type=reward_type)
        super().__init__(robot, task)


class PandaReachEnv(RobotTaskEnv):
    """panda_tasks.py:65-79."""

    def __init__(self, num_envs: int = 1, device="cuda", reward_type: str = "sparse", control_type: str = "ee"):
        sim = PandaSim(task=None, num_envs=num_envs, device=device)
        robot = Panda(sim, block_gripper=True, base_position=BASE, control_type=control_type)
        task = Reach(sim, reward_type=reward_type, get_ee_position=robot.get_ee_position)
        super().__init__(robot, task)


ENV_CLASSES = {"reach": PandaReachEnv, "push": PandaPushEnv, "pick_and_place": PandaPickAndPlaceEnv}
