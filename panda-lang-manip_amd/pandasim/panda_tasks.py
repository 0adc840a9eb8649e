"""Env wiring of panda_gym/envs/panda_tasks.py:14-116 over the plugin path:
batched PandaSim + Panda(base=(-0.6, 0, 0)) + task, composed by RobotTaskEnv.

These are the unfused counterparts of the registered IDs (same robot, task,
scene and constants); ``pandasim.make(id, fused=False)`` builds them wrapped
in TimeLimit(50; Stack 100) as gym.make does.
"""
from __future__ import annotations

import numpy as np

from .core import RobotTaskEnv
from .robots import Panda
from .sim import PandaSim
from .tasks import Flip, PickAndPlace, Push, Reach, Slide, Stack

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


def _compose(env, num_envs, device, task_cls, block_gripper, control_type, reward_type):
    sim = PandaSim(task=None, num_envs=num_envs, device=device)
    robot = Panda(sim, block_gripper=block_gripper, base_position=BASE, control_type=control_type)
    RobotTaskEnv.__init__(env, robot, task_cls(sim, reward_type=reward_type))


class PandaFlipEnv(RobotTaskEnv):
    """panda_tasks.py:14-28."""

    def __init__(self, num_envs: int = 1, device="cuda", reward_type: str = "sparse", control_type: str = "ee"):
        _compose(self, num_envs, device, Flip, False, control_type, reward_type)


class PandaSlideEnv(RobotTaskEnv):
    """panda_tasks.py:82-96."""

    def __init__(self, num_envs: int = 1, device="cuda", reward_type: str = "sparse", control_type: str = "ee"):
        _compose(self, num_envs, device, Slide, True, control_type, reward_type)


class PandaStackEnv(RobotTaskEnv):
    """panda_tasks.py:99-113."""

    def __init__(self, num_envs: int = 1, device="cuda", reward_type: str = "sparse", control_type: str = "ee"):
        _compose(self, num_envs, device, Stack, False, control_type, reward_type)


ENV_CLASSES = {"reach": PandaReachEnv, "push": PandaPushEnv, "pick_and_place": PandaPickAndPlaceEnv,
               "slide": PandaSlideEnv, "stack": PandaStackEnv, "flip": PandaFlipEnv}
