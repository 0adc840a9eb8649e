"""Vectorised drop-in for the panda_gym env surface (core.py:199-335).

``make("PandaPush-v3", num_envs=B)`` returns a ``PandaVecEnv`` whose
``reset``/``step`` run B envs per call through the fused HIP step kernel
(ps_step).  Semantics follow the reference:

* ``reset(seed=s)`` re-seeds env i with Generator(PCG64(SeedSequence(s + i)))
  (core.py:244; per-env offsets as gymnasium vector envs do) and samples goal
  then object exactly as the reference tasks; ``reset()`` without a seed
  continues each env's generator (the reference would draw OS entropy).
* ``step`` returns ``(obs, reward, terminated, truncated, info)`` with
  terminated = is_success, reward from compute_reward, truncated from the
  TimeLimit of the registration (50 steps, Stack 100; __init__.py:18-46).  With ``autoreset``
  (default) finished envs are reset inside the kernel; ``info`` then carries
  ``final_observation``/``final_achieved_goal`` for them.
* ``compute_reward(ag, dg, info)`` is vectorised over leading dims (HER).
"""
from __future__ import annotations

import ctypes as C
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch

from . import _lib as L
from .sim import PandaSim, _ptr

def _spaces(obs_dim: int, action_dim: int, goal_dim: int = 3):
    try:
        from gymnasium import spaces  # optional: not installed in the build image
    except Exception:  # pragma: no cover - depends on the environment
        return None, None
    obs = spaces.Dict(dict(
        observation=spaces.Box(-10.0, 10.0, shape=(obs_dim,), dtype=np.float32),
        desired_goal=spaces.Box(-10.0, 10.0, shape=(goal_dim,), dtype=np.float32),
        achieved_goal=spaces.Box(-10.0, 10.0, shape=(goal_dim,), dtype=np.float32),
    ))
    return obs, spaces.Box(-1.0, 1.0, shape=(action_dim,), dtype=np.float32)


class PandaVecEnv:
    metadata = {"render_modes": ["rgb_array"]}

    def __init__(self, task: str, reward_type: str = "sparse", control_type: str = "ee", num_envs: int = 1,
                 device="cuda", autoreset: bool = True, lanes_per_env: int = 0):
        self.task_name, self.reward_type, self.control_type = task, reward_type, control_type
        self.sim = PandaSim(task, control_type, reward_type, num_envs, device)
        # 0: the library picks 16 or 8 lanes per env for small batches, 1 above (ps_set_lanes_per_env)
        self.sim._call("ps_set_lanes_per_env", self.sim._ctx, int(lanes_per_env))
        self.lanes_per_env = self.sim._lib.ps_step_lanes(self.sim._ctx)
        self.num_envs = self.sim.num_envs
        self.device = self.sim.device
        self.autoreset = autoreset
        self.obs_dim, self.action_dim = self.sim.obs_dim, self.sim.action_dim
        self.goal_dim = self.sim.goal_dim
        self.observation_space, self.action_space = _spaces(self.obs_dim, self.action_dim, self.goal_dim)
        self.max_episode_steps = self.sim.max_episode_steps
        B, dev, G = self.num_envs, self.device, self.goal_dim
        self._obs = torch.zeros(B, self.obs_dim, device=dev)
        self._ag = torch.zeros(B, G, device=dev)
        self._dg = torch.zeros(B, G, device=dev)
        self._final_obs = torch.zeros(B, self.obs_dim, device=dev)
        self._final_ag = torch.zeros(B, G, device=dev)
        self._reward = torch.zeros(B, device=dev)
        self._term = torch.zeros(B, dtype=torch.uint8, device=dev)
        self._trunc = torch.zeros(B, dtype=torch.uint8, device=dev)
        self._saved_goals: Dict[int, torch.Tensor] = {}
        self._has_reset = False
        self._nonfinite: Optional[torch.Tensor] = None
        self._epstats: Optional[torch.Tensor] = None

    def set_nonfinite_guard(self, enabled: bool = True, reset: bool = False) -> None:
        """NaN/Inf guard of the fused step (ps_set_nonfinite_guard): step()'s
        info["nonfinite"] flags envs whose joint or object state is not finite;
        with reset=True they are also reset in-kernel and reported truncated."""
        if enabled:
            self._nonfinite = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.device)
        else:
            self._nonfinite = None
        self.sim._call("ps_set_nonfinite_guard", self.sim._ctx, _ptr(self._nonfinite), int(bool(enabled and reset)))

    def record_episode_statistics(self, enabled: bool = True) -> Optional[torch.Tensor]:
        """gymnasium's RecordEpisodeStatistics, fused into the step kernel
        (ps_set_episode_stats): returns the [4, B] float32 device buffer every
        following step() updates -- running return, last finished episode's
        return, its success (terminated 1, truncated 0), finished episodes --
        or None when disabled."""
        self._epstats = torch.zeros(4, self.num_envs, device=self.device) if enabled else None
        self.sim._call("ps_set_episode_stats", self.sim._ctx, _ptr(self._epstats))
        return self._epstats

    # ---------------------------------------------------------------- core
    def _obs_dict(self, obs=None, ag=None, dg=None):
        return {"observation": (self._obs if obs is None else obs).clone(),
                "achieved_goal": (self._ag if ag is None else ag).clone(),
                "desired_goal": (self._dg if dg is None else dg).clone()}

    def reset(self, seed=None, options: Optional[dict] = None, mask=None) -> Tuple[Dict[str, torch.Tensor], Dict]:
        """RobotTaskEnv.reset (core.py:240-250) for all envs (or `mask`)."""
        seeds = None
        if seed is not None:
            if isinstance(seed, (int, np.integer)):
                base = np.uint64(int(seed) & 0xFFFFFFFFFFFFFFFF)
                seeds_np = (base + np.arange(self.num_envs, dtype=np.uint64))
            else:
                seeds_np = np.asarray(seed, dtype=np.uint64).reshape(self.num_envs)
            seeds = torch.from_numpy(seeds_np.view(np.int64)).to(self.device)
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        self.sim._call("ps_reset", self.sim._ctx, _ptr(self.sim.state), _ptr(m), _ptr(seeds), _ptr(self._obs),
                       _ptr(self._ag), _ptr(self._dg), self.sim._stream())
        self._has_reset = True
        info = {"is_success": self.compute_success(self._ag, self.sim.goals())}
        return self._obs_dict(), info

    def step(self, actions, copy: bool = True) -> Tuple[Dict[str, torch.Tensor], torch.Tensor, torch.Tensor,
                                                         torch.Tensor, Dict]:
        """RobotTaskEnv.step (core.py:280-289) + TimeLimit, fused in one kernel.

        copy=False returns views of the env's output buffers (valid until the
        next step) and skips the clones."""
        if not self._has_reset:
            raise L.PandasimError("Cannot call env.step() before calling env.reset()")  # OrderEnforcing
        a = torch.as_tensor(actions, dtype=torch.float32, device=self.device).reshape(self.num_envs, self.action_dim)
        a = a.contiguous()
        self.sim._call("ps_step", self.sim._ctx, _ptr(self.sim.state), _ptr(a), _ptr(self._obs), _ptr(self._ag),
                       _ptr(self._dg), _ptr(self._reward), _ptr(self._term), _ptr(self._trunc), int(self.autoreset),
                       _ptr(self._final_obs), _ptr(self._final_ag), self.sim._stream())
        if not copy:
            obs = {"observation": self._obs, "achieved_goal": self._ag, "desired_goal": self._dg}
            info = {"final_observation": self._final_obs, "final_achieved_goal": self._final_ag}
            if self._nonfinite is not None:
                info["nonfinite"] = self._nonfinite
            return obs, self._reward, self._term, self._trunc, info
        term, trunc = self._term.bool(), self._trunc.bool()
        info = {"is_success": term.clone()}
        if self.autoreset:
            info["final_observation"] = self._final_obs.clone()
            info["final_achieved_goal"] = self._final_ag.clone()
        if self._nonfinite is not None:
            info["nonfinite"] = self._nonfinite.bool()
        return self._obs_dict(), self._reward.clone(), term, trunc, info

    # ----------------------------------------------------------- task API
    def compute_reward(self, achieved_goal, desired_goal, info: Any = None):
        """Task.compute_reward (push.py:93-98), any leading dims, on the GPU."""
        return self._reward_and_success(achieved_goal, desired_goal)[0]

    def compute_success(self, achieved_goal, desired_goal):
        """Task.is_success (push.py:89-91)."""
        return self._reward_and_success(achieved_goal, desired_goal)[1]

    def _reward_and_success(self, achieved_goal, desired_goal):
        from .utils import goal_reward_and_success

        return goal_reward_and_success(achieved_goal, desired_goal, self.reward_type, task=self.task_name)

    # ------------------------------------------------------- state snapshots
    def save_state(self) -> int:
        sid = self.sim.save_state()
        self._saved_goals[sid] = self._dg.clone()
        return sid

    def restore_state(self, state_id: int) -> None:
        self.sim.restore_state(state_id)
        self._dg.copy_(self._saved_goals[state_id])

    def remove_state(self, state_id: int) -> None:
        self._saved_goals.pop(state_id, None)
        self.sim.remove_state(state_id)

    def render(self, mode: str = "rgb_array", width: int = 720, height: int = 480, target_position=None,
               distance: float = 1.4, yaw: float = 45, pitch: float = -30, roll: float = 0):
        """RobotTaskEnv.render (core.py:294-335) for every env: "rgb_array" ->
        [B, height, width, 3] uint8; "human" -> None."""
        if mode != "rgb_array":
            return None
        target_position = np.zeros(3) if target_position is None else target_position
        view, proj, _ = self.sim.get_cam2world_transforms(width, height, target_position, distance, yaw, pitch, roll)
        return self.sim.get_camera_image(width, height, view, proj)[1]

    def close(self) -> None:
        self.sim.close()


# ------------------------------------------------------------- registration
# panda_gym/__init__.py:8-54: 6 tasks x {sparse, dense} x {ee, joints}
_TASK_IDS = {"Reach": "reach", "Push": "push", "Slide": "slide", "PickAndPlace": "pick_and_place",
             "Stack": "stack", "Flip": "flip"}
REGISTRY: Dict[str, Dict[str, Any]] = {}
for _reward in ("sparse", "dense"):
    for _control in ("ee", "joints"):
        for _name, _task in _TASK_IDS.items():
            _id = "Panda{}{}{}-v3".format(_name, "Joints" if _control == "joints" else "",
                                         "Dense" if _reward == "dense" else "")
            REGISTRY[_id] = dict(task=_task, reward_type=_reward, control_type=_control,
                                 max_episode_steps=100 if _name == "Stack" else 50)


def make(env_id: str, num_envs: int = 1, device="cuda", fused: bool = True, **kwargs):
    """gym.make(env_id) counterpart returning B envs.

    fused=True (default): PandaVecEnv, the whole step in one kernel (ps_step),
    TimeLimit and auto-reset inside.  fused=False: the Robot/Task plugin
    composition of panda_tasks.py (pandasim.panda_tasks) wrapped in
    TimeLimit(max_episode_steps), as gym.make builds the reference env."""
    if env_id not in REGISTRY:
        raise KeyError(f"unknown env id {env_id}")
    spec = REGISTRY[env_id]
    if not fused:
        from .core import TimeLimit
        from .panda_tasks import ENV_CLASSES

        env = ENV_CLASSES[spec["task"]](num_envs, device, spec["reward_type"], spec["control_type"], **kwargs)
        return TimeLimit(env, spec["max_episode_steps"])
    return PandaVecEnv(spec["task"], spec["reward_type"], spec["control_type"], num_envs, device, **kwargs)
