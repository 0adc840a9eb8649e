"""Batched counterparts of panda_gym/utils.py:4-30 on device tensors.

``distance`` reproduces numpy's ``np.linalg.norm(a - b, axis=-1)`` for the
3-vectors of the goal-conditioned tasks bit for bit: the difference is taken
in the promoted dtype (float32 - float64 -> float64, as numpy), the three
squares are summed left to right, each elementwise torch op rounds once (no
contraction) and the root is correctly rounded.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch


def distance(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """utils.py:4-15."""
    a, b = torch.as_tensor(a), torch.as_tensor(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    d = a - b
    if d.shape[-1] != 3:
        return torch.sqrt((d * d).sum(-1))
    s = d[..., 0] * d[..., 0]
    s = s + d[..., 1] * d[..., 1]
    s = s + d[..., 2] * d[..., 2]
    return _sqrt_rn(s)


def _sqrt_rn(s: torch.Tensor) -> torch.Tensor:
    """Correctly rounded square root, as numpy's.  torch's CPU float64 sqrt is
    not (it is off by an ulp on ~1% of inputs), so CPU tensors go through
    numpy; on the GPU a float32 root is taken in float64 and rounded once
    (exact for sqrt), float64 uses the device's IEEE sqrt (checked against
    numpy in tests/test_gpu_plugins.py)."""
    if s.device.type == "cpu":
        return torch.from_numpy(np.sqrt(s.numpy()))
    if s.dtype == torch.float32:
        return torch.sqrt(s.double()).float()
    return torch.sqrt(s)


def goal_reward_and_success(achieved_goal, desired_goal, reward_type: str, distance_threshold: float):
    """compute_reward and is_success of reach.py:56-65 / push.py:89-98 in one
    pass.  On the GPU with the registered threshold this is the
    ps_compute_reward kernel (bit-exact with the reference goldens); anything
    else goes through ``distance``."""
    ag, dg = torch.as_tensor(achieved_goal), torch.as_tensor(desired_goal)
    if ag.is_cuda and ag.shape == dg.shape and ag.shape[-1] == 3 and distance_threshold == 0.05:
        from . import _lib as L
        from .sim import _ptr

        lead = ag.shape[:-1]
        adbl, ddbl = ag.dtype == torch.float64, dg.dtype == torch.float64
        ag = (ag if adbl else ag.to(torch.float32)).reshape(-1, 3).contiguous()
        dg = (dg if ddbl else dg.to(torch.float32)).reshape(-1, 3).contiguous()
        n = ag.shape[0]
        r = torch.empty(n, device=ag.device)
        ok = torch.empty(n, dtype=torch.uint8, device=ag.device)
        with torch.cuda.device(ag.device):
            stream = C.c_void_p(torch.cuda.current_stream(ag.device).cuda_stream)
            rc = L.lib().ps_compute_reward(0 if reward_type == "sparse" else 1, _ptr(ag), int(adbl), _ptr(dg),
                                           int(ddbl), _ptr(r), _ptr(ok), n, stream)
        L.check(rc, what="ps_compute_reward")
        return r.reshape(lead), ok.bool().reshape(lead)
    d = distance(ag, dg)
    r = -(d > distance_threshold).to(torch.float32) if reward_type == "sparse" else -d.to(torch.float32)
    return r, d < distance_threshold


def angle_distance(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """utils.py:18-30: 1 - <a, b>^2 over the last axis (Flip's quaternion goals)."""
    a, b = torch.as_tensor(a), torch.as_tensor(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    return 1 - (a * b).sum(-1) ** 2
