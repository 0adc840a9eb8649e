"""Batched task plugins (panda_gym/envs/tasks/{reach,push,pick_and_place}.py).

Goals are [B, 3] float64 device tensors drawn from each env's own PCG64
stream in the reference's draw order (goal before object; PickAndPlace's
extra ``random() < 0.3``), so they are bit-identical to the reference's
numpy goals for the same seed.
"""
from __future__ import annotations

from typing import Any, Dict

import numpy as np
import torch

from .core import Task
from .utils import goal_reward_and_success


class _GoalTask(Task):
    """is_success / compute_reward shared by Reach, Push, PickAndPlace
    (reach.py:56-65, push.py:89-98, pick_and_place.py:87-96)."""

    reward_type: str
    distance_threshold: float

    def is_success(self, achieved_goal, desired_goal, info: Dict[str, Any] = {}) -> torch.Tensor:
        return goal_reward_and_success(achieved_goal, desired_goal, self.reward_type, self.distance_threshold)[1]

    def compute_reward(self, achieved_goal, desired_goal, info: Dict[str, Any] = {}) -> torch.Tensor:
        return goal_reward_and_success(achieved_goal, desired_goal, self.reward_type, self.distance_threshold)[0]


class Reach(_GoalTask):
    """reach.py:9-65."""

    def __init__(self, sim, get_ee_position, reward_type="sparse", distance_threshold=0.05, goal_range=0.3) -> None:
        super().__init__(sim)
        self.reward_type = reward_type
        self.distance_threshold = distance_threshold
        self.get_ee_position = get_ee_position
        self.goal_range_low = np.array([-goal_range / 2, -goal_range / 2, 0])
        self.goal_range_high = np.array([goal_range / 2, goal_range / 2, goal_range])
        with self.sim.no_rendering():
            self._create_scene()
            self.sim.place_visualizer(target_position=np.zeros(3), distance=0.9, yaw=45, pitch=-30)

    def _create_scene(self) -> None:
        self.sim.create_plane(z_offset=-0.4)
        self.sim.create_table(length=1.1, width=0.7, height=0.4, x_offset=-0.3)
        self.sim.create_sphere(body_name="target", radius=0.02, mass=0.0, ghost=True, position=np.zeros(3),
                               rgba_color=np.array([0.1, 0.9, 0.1, 0.3]))

    def get_obs(self) -> torch.Tensor:
        return torch.zeros(self.sim.num_envs, 0, device=self.sim.device)  # no task-specific observation

    def get_achieved_goal(self) -> torch.Tensor:
        return self.get_ee_position()

    def reset(self) -> None:
        self.goal = self._sample_goal()
        self.sim.set_base_pose("target", self.goal, np.array([0.0, 0.0, 0.0, 1.0]))

    def _sample_goal(self) -> torch.Tensor:
        return self.np_random.uniform(self.goal_range_low, self.goal_range_high)


class Push(_GoalTask):
    """push.py:9-98."""

    def __init__(self, sim, reward_type="sparse", distance_threshold=0.05, goal_xy_range=0.3,
                 obj_xy_range=0.3) -> None:
        super().__init__(sim)
        self.reward_type = reward_type
        self.distance_threshold = distance_threshold
        self.object_size = 0.04
        self.goal_range_low = np.array([-goal_xy_range / 2, -goal_xy_range / 2, 0])
        self.goal_range_high = np.array([goal_xy_range / 2, goal_xy_range / 2, 0])
        self.obj_range_low = np.array([-obj_xy_range / 2, -obj_xy_range / 2, 0])
        self.obj_range_high = np.array([obj_xy_range / 2, obj_xy_range / 2, 0])
        with self.sim.no_rendering():
            self._create_scene()
            self.sim.place_visualizer(target_position=np.zeros(3), distance=0.9, yaw=45, pitch=-30)

    def _create_scene(self) -> None:
        self.sim.create_plane(z_offset=-0.4)
        self.sim.create_table(length=1.1, width=0.7, height=0.4, x_offset=-0.3)
        self.sim.create_box(body_name="object", half_extents=np.ones(3) * self.object_size / 2, mass=1.0,
                            position=np.array([0.0, 0.0, self.object_size / 2]),
                            rgba_color=np.array([0.1, 0.9, 0.1, 1.0]))
        self.sim.create_box(body_name="target", half_extents=np.ones(3) * self.object_size / 2, mass=0.0,
                            ghost=True, position=np.array([0.0, 0.0, self.object_size / 2]),
                            rgba_color=np.array([0.1, 0.9, 0.1, 0.3]))

    def get_obs(self) -> torch.Tensor:
        return torch.cat([self.sim.get_base_position("object"), self.sim.get_base_rotation("object"),
                          self.sim.get_base_velocity("object"), self.sim.get_base_angular_velocity("object")],
                         dim=-1)

    def get_achieved_goal(self) -> torch.Tensor:
        return self.sim.get_base_position("object")

    def reset(self) -> None:
        self.goal = self._sample_goal()
        object_position = self._sample_object()
        self.sim.set_base_pose("target", self.goal, np.array([0.0, 0.0, 0.0, 1.0]))
        self.sim.set_base_pose("object", object_position, np.array([0.0, 0.0, 0.0, 1.0]))

    def _sample_goal(self) -> torch.Tensor:
        goal = torch.tensor([0.0, 0.0, self.object_size / 2], dtype=torch.float64, device=self.sim.device)
        return goal + self.np_random.uniform(self.goal_range_low, self.goal_range_high)

    def _sample_object(self) -> torch.Tensor:
        pos = torch.tensor([0.0, 0.0, self.object_size / 2], dtype=torch.float64, device=self.sim.device)
        return pos + self.np_random.uniform(self.obj_range_low, self.obj_range_high)


class PickAndPlace(Push):
    """pick_and_place.py:10-96 (Push's scene and observation; goal z ~
    U(0, 0.2), set to 0 with probability 0.3)."""

    def __init__(self, sim, reward_type="sparse", distance_threshold=0.05, goal_xy_range=0.3, goal_z_range=0.2,
                 obj_xy_range=0.3) -> None:
        super().__init__(sim, reward_type, distance_threshold, goal_xy_range, obj_xy_range)
        self.goal_range_high = np.array([goal_xy_range / 2, goal_xy_range / 2, goal_z_range])

    def _sample_goal(self) -> torch.Tensor:
        goal = torch.tensor([0.0, 0.0, self.object_size / 2], dtype=torch.float64, device=self.sim.device)
        noise = self.np_random.uniform(self.goal_range_low, self.goal_range_high)
        on_table = self.np_random.random() < 0.3
        noise[:, 2] = torch.where(on_table, torch.zeros_like(noise[:, 2]), noise[:, 2])
        return goal + noise
