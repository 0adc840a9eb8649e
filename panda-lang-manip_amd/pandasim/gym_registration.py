"""gymnasium registration of the 24 env IDs (panda_gym/__init__.py:8-54).

The reference registers every ID with ``gymnasium.envs.registration.register``
at import time, so ``gym.make("PandaPush-v3")`` builds a single env wrapped in
``TimeLimit(max_episode_steps)``.  ``register_envs()`` does the same for
pandasim: same IDs, same ``kwargs`` (reward_type, control_type) and
``max_episode_steps`` (50, Stack 100), with entry points to the one-env
classes below.  It is explicit rather than an import side effect because
gymnasium is optional here (the build image lacks it); without gymnasium it
raises ImportError and the classes still work on their own.

The one-env classes present gymnasium's single-env API on top of
:class:`pandasim.envs.PandaVecEnv` with ``num_envs=1`` and no auto-reset:
``reset(seed, options) -> (obs, info)`` and ``step(action) -> (obs, reward,
terminated, truncated, info)`` with numpy observations (``Dict`` of float32
``observation``/``achieved_goal``/``desired_goal``, core.py:218-224), a float
reward and bool flags, ``info["is_success"]`` as core.py:280-289.  The
TimeLimit the fused kernel applies and the one gym.make adds truncate at the
same step.  Batched training should use :func:`pandasim.make` with many envs:
one env per call leaves the GPU idle.
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Tuple

import numpy as np

from .envs import REGISTRY, PandaVecEnv

try:  # optional dependency
    import gymnasium as _gym
except Exception:  # pragma: no cover - depends on the environment
    _gym = None

_Base = _gym.Env if _gym is not None else object

_CLASS_OF_TASK = {"reach": "PandaReachGymEnv", "push": "PandaPushGymEnv", "slide": "PandaSlideGymEnv",
                  "pick_and_place": "PandaPickAndPlaceGymEnv", "stack": "PandaStackGymEnv",
                  "flip": "PandaFlipGymEnv"}


class PandaGymEnv(_Base):
    """One env of ``task`` with gymnasium's API (RobotTaskEnv, core.py:202-335)."""

    metadata = {"render_modes": ["human", "rgb_array"]}
    task = "reach"

    def __init__(self, reward_type: str = "sparse", control_type: str = "ee", render_mode: Optional[str] = None,
                 device="cuda", **_: Any):
        self.render_mode = render_mode
        self._env = PandaVecEnv(self.task, reward_type, control_type, num_envs=1, device=device, autoreset=False)
        self.observation_space, self.action_space = self._env.observation_space, self._env.action_space
        self.np_random = None

    @staticmethod
    def _np(obs: Dict[str, Any]) -> Dict[str, np.ndarray]:
        return {k: v[0].detach().cpu().numpy().astype(np.float32) for k, v in obs.items()}

    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None) -> Tuple[Dict[str, np.ndarray], Dict]:
        obs, info = self._env.reset(seed=seed, options=options)
        return self._np(obs), {"is_success": bool(info["is_success"][0])}

    def step(self, action) -> Tuple[Dict[str, np.ndarray], float, bool, bool, Dict[str, Any]]:
        a = np.asarray(action, dtype=np.float32).reshape(1, -1)
        obs, reward, terminated, truncated, info = self._env.step(a)
        return (self._np(obs), float(reward[0]), bool(terminated[0]), bool(truncated[0]),
                {"is_success": bool(info["is_success"][0])})

    def compute_reward(self, achieved_goal, desired_goal, info: Any = None):
        """Task.compute_reward (core.py:226, HER): numpy in, numpy out."""
        r = self._env.compute_reward(np.asarray(achieved_goal), np.asarray(desired_goal), info)
        return r.detach().cpu().numpy()

    def save_state(self) -> int:
        return self._env.save_state()

    def restore_state(self, state_id: int) -> None:
        self._env.restore_state(state_id)

    def remove_state(self, state_id: int) -> None:
        self._env.remove_state(state_id)

    def render(self, width: int = 720, height: int = 480, **kwargs):
        if self.render_mode != "rgb_array":
            return None
        return self._env.render("rgb_array", width=width, height=height, **kwargs)[0].cpu().numpy()

    def close(self) -> None:
        self._env.close()


def _task_class(task: str) -> type:
    return type(_CLASS_OF_TASK[task], (PandaGymEnv,), {"task": task, "__doc__": f"One {task} env (gymnasium API)."})


PandaReachGymEnv = _task_class("reach")
PandaPushGymEnv = _task_class("push")
PandaSlideGymEnv = _task_class("slide")
PandaPickAndPlaceGymEnv = _task_class("pick_and_place")
PandaStackGymEnv = _task_class("stack")
PandaFlipGymEnv = _task_class("flip")


def registrations():
    """(id, entry_point, kwargs, max_episode_steps) of every ID, in the
    reference's registration order (panda_gym/__init__.py:8-54)."""
    out = []
    for reward_type in ("sparse", "dense"):
        for control_type in ("ee", "joints"):
            for name in ("Reach", "Push", "Slide", "PickAndPlace", "Stack", "Flip"):
                env_id = "Panda{}{}{}-v3".format(name, "Joints" if control_type == "joints" else "",
                                                 "Dense" if reward_type == "dense" else "")
                spec = REGISTRY[env_id]
                out.append((env_id, f"pandasim.gym_registration:{_CLASS_OF_TASK[spec['task']]}",
                            {"reward_type": reward_type, "control_type": control_type}, spec["max_episode_steps"]))
    return out


def register_envs(override: bool = False) -> list:
    """Register the 24 IDs with gymnasium; returns the IDs.  An ID already
    registered with pandasim's entry point is kept.  One registered by
    another package (panda_gym imported first: gym.make would build the
    reference's PyBullet env) raises RuntimeError, unless ``override=True``,
    which re-registers it to pandasim.  Raises ImportError when gymnasium is
    not installed."""
    if _gym is None:
        raise ImportError("gymnasium is not installed: pandasim.make(env_id, num_envs) needs no registry")
    from gymnasium.envs.registration import register, registry

    ids = []
    for env_id, entry_point, kwargs, steps in registrations():
        if env_id in registry:
            theirs = registry[env_id].entry_point
            if theirs == entry_point:
                ids.append(env_id)
                continue
            if not override:
                raise RuntimeError(f"{env_id} is already registered to {theirs!r} (panda_gym imported first?); "
                                   "call register_envs(override=True) to point it at pandasim")
            del registry[env_id]
        register(id=env_id, entry_point=entry_point, kwargs=kwargs, max_episode_steps=steps)
        ids.append(env_id)
    return ids
