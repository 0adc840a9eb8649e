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
    s = d[..., 0] * d[..., 0]
    for k in range(1, d.shape[-1]):
        s = s + d[..., k] * d[..., k]
    return _sqrt_rn(s)


def angle_distance(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """utils.py:18-30: 1 - <a, b>^2 over the last axis (Flip's quaternion
    goals), the products summed left to right in the promoted dtype."""
    a, b = torch.as_tensor(a), torch.as_tensor(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    dt = torch.promote_types(a.dtype, b.dtype)
    a, b = a.to(dt), b.to(dt)
    dot = a[..., 0] * b[..., 0]
    for k in range(1, a.shape[-1]):
        dot = dot + a[..., k] * b[..., k]
    return 1 - dot * dot


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


TASK_IDS = {"reach": 0, "push": 1, "pick_and_place": 2, "slide": 3, "stack": 4, "flip": 5}
# registered goal sizes and thresholds (reach.py:14, push.py:13, stack.py:14, flip.py:15)
GOAL_DIM = {"reach": 3, "push": 3, "pick_and_place": 3, "slide": 3, "stack": 6, "flip": 4}
THRESHOLD = {"reach": 0.05, "push": 0.05, "pick_and_place": 0.05, "slide": 0.05, "stack": 0.1, "flip": 0.2}


def goal_reward_and_success(achieved_goal, desired_goal, reward_type: str, distance_threshold: float = None,
                            task: str = "push"):
    """compute_reward and is_success of reach.py:56-65 / push.py:89-98 /
    stack.py:118-131 / flip.py:80-91 in one pass.  On the GPU with the
    registered threshold this is the ps_compute_reward kernel (bit-exact with
    the reference goldens); anything else goes through ``distance`` /
    ``angle_distance``.  Flip's metric is applied per goal pair (the
    reference's np.inner would form the outer product of batched inputs)."""
    thr = THRESHOLD[task] if distance_threshold is None else distance_threshold
    ag, dg = torch.as_tensor(achieved_goal), torch.as_tensor(desired_goal)
    gd = GOAL_DIM[task]
    if ag.is_cuda and ag.shape == dg.shape and ag.shape[-1] == gd and thr == THRESHOLD[task]:
        from . import _lib as L
        from .sim import _ptr

        lead = ag.shape[:-1]
        adbl, ddbl = ag.dtype == torch.float64, dg.dtype == torch.float64
        ag = (ag if adbl else ag.to(torch.float32)).reshape(-1, gd).contiguous()
        dg = (dg if ddbl else dg.to(torch.float32)).reshape(-1, gd).contiguous()
        n = ag.shape[0]
        r = torch.empty(n, device=ag.device)
        ok = torch.empty(n, dtype=torch.uint8, device=ag.device)
        with torch.cuda.device(ag.device):
            stream = C.c_void_p(torch.cuda.current_stream(ag.device).cuda_stream)
            rc = L.lib().ps_compute_reward(TASK_IDS[task], 0 if reward_type == "sparse" else 1, _ptr(ag), int(adbl),
                                           _ptr(dg), int(ddbl), _ptr(r), _ptr(ok), n, stream)
        L.check(rc, what="ps_compute_reward")
        return r.reshape(lead), ok.bool().reshape(lead)
    d = angle_distance(ag, dg) if task == "flip" else distance(ag, dg)
    r = -(d > thr).to(torch.float32) if reward_type == "sparse" else -d.to(torch.float32)
    return r, d < thr
