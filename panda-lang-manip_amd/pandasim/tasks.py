"""Batched task plugins (panda_gym/envs/tasks/{reach,push,pick_and_place,
slide,stack,flip}.py).

Goals are [B, G] float64 device tensors drawn from each env's own PCG64
stream in the reference's draw order (goal before object; PickAndPlace's
extra ``random() < 0.3``; Stack's one goal noise and two object noises), so
they are bit-identical to the reference's numpy goals for the same seed.
Flip's goal is the reference's unseeded ``Rotation.random()``; here it comes
from each env's auxiliary stream (``PandaSim.random_rotation``), a uniform
unit quaternion like scipy's, reproducible from the seed.
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

    task_name = "push"

    def is_success(self, achieved_goal, desired_goal, info: Dict[str, Any] = {}) -> torch.Tensor:
        return goal_reward_and_success(achieved_goal, desired_goal, self.reward_type, self.distance_threshold,
                                       task=self.task_name)[1]

    def compute_reward(self, achieved_goal, desired_goal, info: Dict[str, Any] = {}) -> torch.Tensor:
        return goal_reward_and_success(achieved_goal, desired_goal, self.reward_type, self.distance_threshold,
                                       task=self.task_name)[0]


class Reach(_GoalTask):
    """reach.py:9-65."""

    task_name = "reach"

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

    task_name = "push"

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

    task_name = "pick_and_place"

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


def _object_obs(sim, body: str, rotation: str = "euler") -> torch.Tensor:
    return torch.cat([sim.get_base_position(body), sim.get_base_rotation(body, rotation),
                      sim.get_base_velocity(body), sim.get_base_angular_velocity(body)], dim=-1)


class Slide(_GoalTask):
    """slide.py:9-106: a low-friction cylinder (radius 0.03, height 0.03) on a
    1.4 m table; the goal lies 0.4 m further along x."""

    task_name = "slide"

    def __init__(self, sim, reward_type="sparse", distance_threshold=0.05, goal_xy_range=0.3, goal_x_offset=0.4,
                 obj_xy_range=0.3) -> None:
        super().__init__(sim)
        self.reward_type = reward_type
        self.distance_threshold = distance_threshold
        self.object_size = 0.06
        self.goal_range_low = np.array([-goal_xy_range / 2 + goal_x_offset, -goal_xy_range / 2, 0])
        self.goal_range_high = np.array([goal_xy_range / 2 + goal_x_offset, goal_xy_range / 2, 0])
        self.obj_range_low = np.array([-obj_xy_range / 2, -obj_xy_range / 2, 0])
        self.obj_range_high = np.array([obj_xy_range / 2, obj_xy_range / 2, 0])
        with self.sim.no_rendering():
            self._create_scene()
            self.sim.place_visualizer(target_position=np.zeros(3), distance=0.9, yaw=45, pitch=-30)

    def _create_scene(self) -> None:
        self.sim.create_plane(z_offset=-0.4)
        self.sim.create_table(length=1.4, width=0.7, height=0.4, x_offset=-0.1)
        self.sim.create_cylinder(body_name="object", mass=1.0, radius=self.object_size / 2,
                                 height=self.object_size / 2, position=np.array([0.0, 0.0, self.object_size / 2]),
                                 rgba_color=np.array([0.1, 0.9, 0.1, 1.0]), lateral_friction=0.04)
        self.sim.create_cylinder(body_name="target", mass=0.0, ghost=True, radius=self.object_size / 2,
                                 height=self.object_size / 2, position=np.array([0.0, 0.0, self.object_size / 2]),
                                 rgba_color=np.array([0.1, 0.9, 0.1, 0.3]))

    def get_obs(self) -> torch.Tensor:
        return _object_obs(self.sim, "object")

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


class Stack(_GoalTask):
    """stack.py:9-131: two cubes (2 kg, 1 kg); the 6-D goal stacks object2 on
    object1 at one shared xy noise."""

    task_name = "stack"

    def __init__(self, sim, reward_type="sparse", distance_threshold=0.1, goal_xy_range=0.3,
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
        half = np.ones(3) * self.object_size / 2
        self.sim.create_plane(z_offset=-0.4)
        self.sim.create_table(length=1.1, width=0.7, height=0.4, x_offset=-0.3)
        self.sim.create_box(body_name="object1", half_extents=half, mass=2.0,
                            position=np.array([0.0, 0.0, self.object_size / 2]),
                            rgba_color=np.array([0.1, 0.1, 0.9, 1.0]))
        self.sim.create_box(body_name="target1", half_extents=half, mass=0.0, ghost=True,
                            position=np.array([0.0, 0.0, 0.05]), rgba_color=np.array([0.1, 0.1, 0.9, 0.3]))
        self.sim.create_box(body_name="object2", half_extents=half, mass=1.0,
                            position=np.array([0.5, 0.0, self.object_size / 2]),
                            rgba_color=np.array([0.1, 0.9, 0.1, 1.0]))
        self.sim.create_box(body_name="target2", half_extents=half, mass=0.0, ghost=True,
                            position=np.array([0.5, 0.0, 0.05]), rgba_color=np.array([0.1, 0.9, 0.1, 0.3]))

    def get_obs(self) -> torch.Tensor:
        return torch.cat([_object_obs(self.sim, "object1"), _object_obs(self.sim, "object2")], dim=-1)

    def get_achieved_goal(self) -> torch.Tensor:
        return torch.cat([self.sim.get_base_position("object1"), self.sim.get_base_position("object2")], dim=-1)

    def reset(self) -> None:
        self.goal = self._sample_goal()
        object1_position, object2_position = self._sample_objects()
        quat = np.array([0.0, 0.0, 0.0, 1.0])
        self.sim.set_base_pose("target1", self.goal[:, :3], quat)
        self.sim.set_base_pose("target2", self.goal[:, 3:], quat)
        self.sim.set_base_pose("object1", object1_position, quat)
        self.sim.set_base_pose("object2", object2_position, quat)

    def _sample_goal(self) -> torch.Tensor:
        dev = self.sim.device
        goal1 = torch.tensor([0.0, 0.0, self.object_size / 2], dtype=torch.float64, device=dev)
        goal2 = torch.tensor([0.0, 0.0, 3 * self.object_size / 2], dtype=torch.float64, device=dev)
        noise = self.np_random.uniform(self.goal_range_low, self.goal_range_high)
        return torch.cat([goal1 + noise, goal2 + noise], dim=-1)

    def _sample_objects(self):
        dev = self.sim.device
        p1 = torch.tensor([0.0, 0.0, self.object_size / 2], dtype=torch.float64, device=dev)
        p2 = torch.tensor([0.0, 0.0, 3 * self.object_size / 2], dtype=torch.float64, device=dev)
        noise1 = self.np_random.uniform(self.obj_range_low, self.obj_range_high)
        noise2 = self.np_random.uniform(self.obj_range_low, self.obj_range_high)
        return p1 + noise1, p2 + noise2


class Flip(_GoalTask):
    """flip.py:11-91: reach a random orientation of the cube; the goal and the
    achieved goal are (x, y, z, w) quaternions, the metric 1 - <q, g>^2."""

    task_name = "flip"

    def __init__(self, sim, reward_type="sparse", distance_threshold=0.2, obj_xy_range=0.3) -> None:
        super().__init__(sim)
        self.reward_type = reward_type
        self.distance_threshold = distance_threshold
        self.object_size = 0.04
        self.obj_range_low = np.array([-obj_xy_range / 2, -obj_xy_range / 2, 0])
        self.obj_range_high = np.array([obj_xy_range / 2, obj_xy_range / 2, 0])
        with self.sim.no_rendering():
            self._create_scene()
            self.sim.place_visualizer(target_position=np.zeros(3), distance=0.9, yaw=45, pitch=-30)

    def _create_scene(self) -> None:
        half = np.ones(3) * self.object_size / 2
        self.sim.create_plane(z_offset=-0.4)
        self.sim.create_table(length=1.1, width=0.7, height=0.4, x_offset=-0.3)
        self.sim.create_box(body_name="object", half_extents=half, mass=1.0,
                            position=np.array([0.0, 0.0, self.object_size / 2]), texture="colored_cube.png")
        self.sim.create_box(body_name="target", half_extents=half, mass=0.0, ghost=True,
                            position=np.array([0.0, 0.0, 3 * self.object_size / 2]),
                            rgba_color=np.array([1.0, 1.0, 1.0, 0.5]), texture="colored_cube.png")

    def get_obs(self) -> torch.Tensor:
        return _object_obs(self.sim, "object", "quaternion")

    def get_achieved_goal(self) -> torch.Tensor:
        return self.sim.get_base_rotation("object", "quaternion").to(torch.float64)

    def reset(self) -> None:
        self.goal = self._sample_goal()
        object_position, object_orientation = self._sample_object()
        self.sim.set_base_pose("target", np.array([0.0, 0.0, 3 * self.object_size / 2]), self.goal)
        self.sim.set_base_pose("object", object_position, object_orientation)

    def _sample_goal(self) -> torch.Tensor:
        return self.sim.random_rotation()

    def _sample_object(self):
        pos = torch.tensor([0.0, 0.0, self.object_size / 2], dtype=torch.float64, device=self.sim.device)
        return pos + self.np_random.uniform(self.obj_range_low, self.obj_range_high), np.zeros(3)
