"""Batched Robot/Task plugin split (panda_gym/envs/core.py:11-335).

The same three classes as the reference -- ``PyBulletRobot`` (robot plugin),
``Task`` (task plugin) and ``RobotTaskEnv`` (their junction) -- with the same
method names, call order and error behaviour, acting on B envs at once: every
value that is a numpy array / Python float per env in the reference is a
device tensor with a leading batch dimension here, and ``sim`` is a
``pandasim.PandaSim`` (the batched counterpart of ``panda_gym.pybullet.PyBullet``).

This is the unfused path: each plugin call is one or a few kernel launches
through libpandasim.so (ps_link_state, ps_inverse_kinematics, ps_sim_step,
ps_base_state, ps_rng_*), so custom robots and tasks written against the
reference's plugin API run on the GPU unchanged in structure.  The registered
env IDs (``pandasim.make``) run the same algorithm fused into one kernel
(``PandaVecEnv``, ps_step); tests/test_gpu_plugins.py holds the two paths
against each other.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch


class BoxSpace:
    """Minimal ``gymnasium.spaces.Box`` stand-in (gymnasium is optional):
    per-env bounds ``low``/``high`` of ``shape``; ``sample(n)`` draws [n, *shape]."""

    def __init__(self, low: float, high: float, shape: Tuple[int, ...], dtype=np.float32):
        self.low = np.full(shape, low, dtype=dtype)
        self.high = np.full(shape, high, dtype=dtype)
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)

    def sample(self, n: int = 1, device="cpu", generator: Optional[torch.Generator] = None) -> torch.Tensor:
        lo = torch.as_tensor(self.low, device=device)
        hi = torch.as_tensor(self.high, device=device)
        return lo + (hi - lo) * torch.rand((n,) + self.shape, device=device, generator=generator)


def box(low: float, high: float, shape, dtype=np.float32):
    try:
        from gymnasium import spaces  # optional
        return spaces.Box(low, high, shape=tuple(shape), dtype=dtype)
    except Exception:
        return BoxSpace(low, high, tuple(shape), dtype)


class BatchedGenerator:
    """``task.np_random`` of B envs: each env draws from its own
    Generator(PCG64(SeedSequence(seed_i))) held in the sim state, with numpy's
    uniform()/random() arithmetic (core.py:244, reach.py:52, push.py:78)."""

    def __init__(self, sim):
        self.sim = sim

    def uniform(self, low, high) -> torch.Tensor:
        """[B, n] float64 (numpy returns shape (n,) per env)."""
        return self.sim.uniform(np.atleast_1d(low), np.atleast_1d(high))

    def random(self) -> torch.Tensor:
        """[B] float64 in [0, 1)."""
        return self.sim.uniform([0.0], [1.0])[:, 0]


def np_random(sim, seed=None) -> Tuple[BatchedGenerator, Optional[np.ndarray]]:
    """gymnasium.utils.seeding.np_random for B envs: env i is seeded with
    seed + i (an int) or seed[i] (a sequence).  seed None keeps each env's
    current stream (the reference draws OS entropy)."""
    seeds = None
    if seed is not None:
        if isinstance(seed, (int, np.integer)):
            seeds = np.uint64(int(seed) & 0xFFFFFFFFFFFFFFFF) + np.arange(sim.num_envs, dtype=np.uint64)
        else:
            seeds = np.asarray(seed, dtype=np.uint64).reshape(sim.num_envs)
        sim.seed(torch.from_numpy(seeds.view(np.int64)))
    return BatchedGenerator(sim), seeds


class PyBulletRobot(ABC):
    """Base class for robots (core.py:11-158).

    Args:
        sim (PandaSim): batched simulation.
        body_name (str): the robot's name in the simulation.
        file_name (str): URDF path.
        base_position: base position (x, y, z).
        action_space: per-env action space.
        joint_indices: controlled joint indices.
        joint_forces: motor forces of those joints.
    """

    def __init__(self, sim, body_name: str, file_name: str, base_position, action_space, joint_indices,
                 joint_forces) -> None:
        self.sim = sim
        self.body_name = body_name
        with self.sim.no_rendering():
            self._load_robot(file_name, base_position)
            self.setup()
        self.action_space = action_space
        self.joint_indices = np.asarray(joint_indices)
        self.joint_forces = np.asarray(joint_forces)

    def _load_robot(self, file_name: str, base_position) -> None:
        """core.py:40-52."""
        self.sim.loadURDF(body_name=self.body_name, fileName=file_name, basePosition=base_position,
                          useFixedBase=True)

    def setup(self) -> None:
        """Called after robot loading."""

    @abstractmethod
    def set_action(self, action: torch.Tensor) -> None:
        """Set the [B, A] action. Must be called just before sim.step()."""

    @abstractmethod
    def get_obs(self) -> torch.Tensor:
        """[B, r] robot observation."""

    @abstractmethod
    def reset(self) -> None:
        """Reset the robot."""

    def get_link_position(self, link: int) -> torch.Tensor:
        return self.sim.get_link_position(self.body_name, link)

    def get_link_orientation(self, link: int) -> torch.Tensor:
        return self.sim.get_link_orientation(self.body_name, link)

    def get_link_velocity(self, link: int) -> torch.Tensor:
        return self.sim.get_link_velocity(self.body_name, link)

    def get_joint_angle(self, joint: int) -> torch.Tensor:
        return self.sim.get_joint_angle(self.body_name, joint)

    def get_joint_velocity(self, joint: int) -> torch.Tensor:
        return self.sim.get_joint_velocity(self.body_name, joint)

    def control_joints(self, target_angles: torch.Tensor) -> None:
        """core.py:125-136: POSITION_CONTROL motors on joint_indices."""
        self.sim.control_joints(body=self.body_name, joints=self.joint_indices, target_angles=target_angles,
                                forces=self.joint_forces)

    def set_joint_angles(self, angles) -> None:
        """core.py:138-144."""
        self.sim.set_joint_angles(self.body_name, joints=self.joint_indices, angles=angles)

    def inverse_kinematics(self, link: int, position, orientation) -> torch.Tensor:
        """core.py:146-158 -> [B, 9]."""
        return self.sim.inverse_kinematics(self.body_name, link=link, position=position, orientation=orientation)


class Task(ABC):
    """Base class for tasks (core.py:161-196).  ``goal`` is a [B, g] tensor."""

    def __init__(self, sim) -> None:
        self.sim = sim
        self.goal: Optional[torch.Tensor] = None
        self.np_random = BatchedGenerator(sim)

    @abstractmethod
    def reset(self) -> None:
        """Sample a new goal (and object poses) for every env."""

    @abstractmethod
    def get_obs(self) -> torch.Tensor:
        """[B, t] task observation."""

    @abstractmethod
    def get_achieved_goal(self) -> torch.Tensor:
        """[B, g] achieved goal."""

    def get_goal(self) -> torch.Tensor:
        """core.py:183-188."""
        if self.goal is None:
            raise RuntimeError("No goal yet, call reset() first")
        return self.goal.clone()

    @abstractmethod
    def is_success(self, achieved_goal, desired_goal, info: Dict[str, Any] = {}) -> torch.Tensor:
        """[...] bool."""

    @abstractmethod
    def compute_reward(self, achieved_goal, desired_goal, info: Dict[str, Any] = {}) -> torch.Tensor:
        """[...] float32, vectorised over leading dims (HER)."""


class RobotTaskEnv:
    """Junction of a robot and a task (core.py:199-335), B envs per call.

    reset(seed) -> (obs dict of [B, .] float32, info); step(action [B, A]) ->
    (obs, reward [B] f32, terminated [B] bool, truncated [B] bool (all False:
    truncation is TimeLimit's job), info).
    """

    metadata = {"render_modes": ["rgb_array"]}

    def __init__(self, robot: PyBulletRobot, task: Task) -> None:
        assert robot.sim == task.sim, "The robot and the task must belong to the same simulation."
        self.sim = robot.sim
        self.robot = robot
        self.task = task
        self.num_envs = self.sim.num_envs
        self.device = self.sim.device
        observation, _ = self.reset()  # required for init; seed can be changed later
        obs_shape = tuple(observation["observation"].shape[1:])
        goal_shape = tuple(observation["achieved_goal"].shape[1:])
        self.observation_space = {"observation": box(-10.0, 10.0, obs_shape),
                                  "desired_goal": box(-10.0, 10.0, goal_shape),
                                  "achieved_goal": box(-10.0, 10.0, goal_shape)}
        self.action_space = self.robot.action_space
        self.compute_reward = self.task.compute_reward
        self._saved_goal: Dict[int, torch.Tensor] = {}

    def _get_obs(self) -> Dict[str, torch.Tensor]:
        """core.py:229-238."""
        robot_obs = self.robot.get_obs().to(torch.float32)
        task_obs = self.task.get_obs().to(torch.float32)
        observation = torch.cat([robot_obs, task_obs], dim=-1)
        achieved_goal = self.task.get_achieved_goal().to(torch.float32)
        return {"observation": observation, "achieved_goal": achieved_goal,
                "desired_goal": self.task.get_goal().to(torch.float32)}

    def reset(self, seed=None, options: Optional[dict] = None) -> Tuple[Dict[str, torch.Tensor], Dict[str, Any]]:
        """core.py:240-250."""
        self.task.np_random, _ = np_random(self.sim, seed)
        with self.sim.no_rendering():
            self.robot.reset()
            self.task.reset()
        observation = self._get_obs()
        info = {"is_success": self.task.is_success(observation["achieved_goal"], self.task.get_goal())}
        return observation, info

    def save_state(self) -> int:
        """core.py:252-260."""
        state_id = self.sim.save_state()
        self._saved_goal[state_id] = self.task.goal
        return state_id

    def restore_state(self, state_id: int) -> None:
        """core.py:262-269."""
        self.sim.restore_state(state_id)
        self.task.goal = self._saved_goal[state_id]

    def remove_state(self, state_id: int) -> None:
        """core.py:271-278."""
        self._saved_goal.pop(state_id)
        self.sim.remove_state(state_id)

    def step(self, action) -> Tuple[Dict[str, torch.Tensor], torch.Tensor, torch.Tensor, torch.Tensor,
                                    Dict[str, Any]]:
        """core.py:280-289."""
        action = torch.as_tensor(action, dtype=torch.float32, device=self.device).reshape(self.num_envs, -1)
        self.robot.set_action(action)
        self.sim.step()
        observation = self._get_obs()
        # An episode is terminated iff the agent has reached the target
        terminated = self.task.is_success(observation["achieved_goal"], self.task.get_goal()).to(torch.bool)
        truncated = torch.zeros_like(terminated)
        info = {"is_success": terminated}
        reward = self.task.compute_reward(observation["achieved_goal"], self.task.get_goal(), info)
        return observation, reward.to(torch.float32), terminated, truncated, info

    def close(self) -> None:
        self.sim.close()

    def render(self, mode: str = "human", width: int = 720, height: int = 480, target_position=None,
               distance: float = 1.4, yaw: float = 45, pitch: float = -30, roll: float = 0):
        """core.py:294-335.  The reference passes `mode` positionally into
        PyBullet.render's `width` (pybullet.py:149), so it cannot run; this
        returns what its docstring promises: "rgb_array" -> [B, height, width, 3]
        uint8 RGB of every env (getCameraImage), "human" -> None
        (there is no window)."""
        if mode != "rgb_array":
            return None
        target_position = np.zeros(3) if target_position is None else target_position
        view, proj, _ = self.sim.get_cam2world_transforms(width, height, target_position, distance, yaw, pitch, roll)
        return self.sim.get_camera_image(width, height, view, proj)[1]


class TimeLimit:
    """gymnasium.wrappers.TimeLimit as gym.make applies it (__init__.py:18-40):
    per-env elapsed counter, truncated = elapsed >= max_episode_steps."""

    def __init__(self, env: RobotTaskEnv, max_episode_steps: int):
        self.env = env
        self.max_episode_steps = int(max_episode_steps)
        self._elapsed = torch.zeros(env.num_envs, dtype=torch.int32, device=env.device)

    def __getattr__(self, name):
        return getattr(self.env, name)

    def reset(self, **kwargs):
        self._elapsed.zero_()
        return self.env.reset(**kwargs)

    def step(self, action):
        obs, reward, terminated, truncated, info = self.env.step(action)
        self._elapsed += 1
        truncated = truncated | (self._elapsed >= self.max_episode_steps)
        return obs, reward, terminated, truncated, info
