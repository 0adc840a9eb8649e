"""Batched counterpart of panda_gym.pybullet.PyBullet (pybullet.py:16-799).

``PandaSim`` owns one structure-of-arrays state buffer (a torch uint8 tensor on
the GPU) for B identical scenes and exposes the subset of the PyBullet wrapper
that the Robot/Task plugins of the hot path call, each method acting on all B
scenes at once.  Compute goes through libpandasim.so (HIP, gfx950); simple
field reads/writes are tensor views of the state buffer.
"""
from __future__ import annotations

import ctypes as C
import itertools
from typing import Dict, Optional, Sequence

import torch

from . import _lib as L

TASKS = {"reach": 0, "push": 1, "pick_and_place": 2}
CONTROLS = {"ee": 0, "joints": 1}
REWARDS = {"sparse": 0, "dense": 1}
JOINT_TO_DOF = {0: 0, 1: 1, 2: 2, 3: 3, 4: 4, 5: 5, 6: 6, 9: 7, 10: 8}
DT_SUBSTEP = 1.0 / 500


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


class PandaSim:
    """B Panda scenes on one GPU (one process per GPU)."""

    def __init__(self, task: str = "reach", control_type: str = "ee", reward_type: str = "sparse", num_envs: int = 1,
                 device="cuda", n_substeps: int = 20, config: Optional[L.Config] = None):
        if not torch.cuda.is_available():
            raise L.PandasimError("PandaSim needs a ROCm GPU (there is no CPU fallback)")
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.num_envs = int(num_envs)
        self.n_substeps = int(n_substeps)
        self.cfg = config if config is not None else L.default_config(TASKS[task], CONTROLS[control_type],
                                                                      REWARDS[reward_type])
        self._lib = L.lib()
        ctx = C.c_void_p()
        L.check(self._lib.ps_create(C.byref(self.cfg), self.num_envs, self.device.index, C.byref(ctx)),
                what="ps_create")
        self._ctx = ctx
        self.layout = L.layout(self.num_envs)
        self.state = torch.zeros(self.layout.total_bytes, dtype=torch.uint8, device=self.device)
        self._bind_views()
        self._saved: Dict[int, torch.Tensor] = {}
        self._ids = itertools.count()
        self._call("ps_init_state", self._ctx, _ptr(self.state), self._stream())

    # ---------------------------------------------------------------- plumbing
    def _bind_views(self):
        lay, s = self.layout, self.state
        n = lay.stride
        self.f = s[lay.float_offset:lay.float_offset + L.NUM_FLOAT_ROWS * n * 4].view(torch.float32).view(
            L.NUM_FLOAT_ROWS, n)
        self.goal = s[lay.goal_offset:lay.goal_offset + 3 * n * 8].view(torch.float64).view(3, n)
        self.rng = s[lay.rng_offset:lay.rng_offset + 4 * n * 8].view(torch.int64).view(4, n)
        self.elapsed = s[lay.elapsed_offset:lay.elapsed_offset + n * 4].view(torch.int32)

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _call(self, name: str, *args):
        with torch.cuda.device(self.device):
            rc = getattr(self._lib, name)(*args)
        L.check(rc, self._ctx, name)

    def rows(self, row: int, count: int) -> torch.Tensor:
        """[B, count] view-copy of float rows (env-major)."""
        return self.f[row:row + count, :self.num_envs].t()

    def set_rows(self, row: int, values: torch.Tensor) -> None:
        values = torch.as_tensor(values, dtype=torch.float32, device=self.device)
        if values.dim() == 1:
            values = values.unsqueeze(0).expand(self.num_envs, -1)
        self.f[row:row + values.shape[1], :self.num_envs] = values.t()

    @property
    def obs_dim(self) -> int:
        return self._lib.ps_obs_dim(self._ctx)

    @property
    def action_dim(self) -> int:
        return self._lib.ps_action_dim(self._ctx)

    @property
    def dt(self) -> float:
        """pybullet.py:47-50: timestep * n_substeps (0.04 s)."""
        return DT_SUBSTEP * self.n_substeps

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._lib.ps_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ stepping
    def step(self) -> None:
        """pybullet.py:52-55: n_substeps stepSimulation() calls."""
        self._call("ps_sim_step", self._ctx, _ptr(self.state), self.n_substeps, self._stream())

    def save_state(self) -> int:
        """pybullet.py:61-68: in-memory snapshot; returns a state id."""
        sid = next(self._ids)
        self._saved[sid] = self.state.clone()
        return sid

    def restore_state(self, state_id: int) -> None:
        """pybullet.py:266-272.  Unknown/removed ids raise (pybullet.error in the reference)."""
        if state_id not in self._saved:
            raise L.PandasimError(f"restoreState: unknown state id {state_id}")
        self.state.copy_(self._saved[state_id])

    def remove_state(self, state_id: int) -> None:
        """pybullet.py:274-280."""
        if self._saved.pop(state_id, None) is None:
            raise L.PandasimError(f"removeState: unknown state id {state_id}")

    # -------------------------------------------------------------- getters
    def link_state(self, link: int):
        B = self.num_envs
        pos = torch.empty(B, 3, device=self.device)
        quat = torch.empty(B, 4, device=self.device)
        lv = torch.empty(B, 3, device=self.device)
        av = torch.empty(B, 3, device=self.device)
        self._call("ps_link_state", self._ctx, _ptr(self.state), int(link), _ptr(pos), _ptr(quat), _ptr(lv), _ptr(av),
                   self._stream())
        return pos, quat, lv, av

    def get_link_position(self, body: str, link: int) -> torch.Tensor:
        return self.link_state(link)[0]

    def get_link_orientation(self, body: str, link: int) -> torch.Tensor:
        return self.link_state(link)[1]

    def get_link_velocity(self, body: str, link: int) -> torch.Tensor:
        return self.link_state(link)[2]

    def get_link_angular_velocity(self, body: str, link: int) -> torch.Tensor:
        return self.link_state(link)[3]

    def get_joint_angle(self, body: str, joint: int) -> torch.Tensor:
        return self.f[L.F_Q + JOINT_TO_DOF[joint], :self.num_envs].clone()

    def get_joint_velocity(self, body: str, joint: int) -> torch.Tensor:
        return self.f[L.F_QD + JOINT_TO_DOF[joint], :self.num_envs].clone()

    def get_base_position(self, body: str) -> torch.Tensor:
        return self.rows(L.F_CPOS, 3).clone()

    def get_base_orientation(self, body: str) -> torch.Tensor:
        return self.rows(L.F_CQUAT, 4).clone()

    def get_base_velocity(self, body: str) -> torch.Tensor:
        return self.rows(L.F_CVEL, 3).clone()

    def get_base_angular_velocity(self, body: str) -> torch.Tensor:
        return self.rows(L.F_COMG, 3).clone()

    # -------------------------------------------------------------- setters
    def set_joint_angles(self, body: str, joints: Sequence[int], angles) -> None:
        """resetJointState (pybullet.py:441-460): position set, velocity zeroed."""
        angles = torch.as_tensor(angles, dtype=torch.float32, device=self.device)
        for k, j in enumerate(joints):
            d = JOINT_TO_DOF[int(j)]
            self.f[L.F_Q + d, :self.num_envs] = angles[..., k]
            self.f[L.F_QD + d, :self.num_envs] = 0.0

    def set_joint_angle(self, body: str, joint: int, angle) -> None:
        self.set_joint_angles(body, [joint], torch.as_tensor(angle, dtype=torch.float32).reshape(-1, 1)
                              if torch.as_tensor(angle).dim() else [angle])

    def set_base_pose(self, body: str, position, orientation) -> None:
        """resetBasePositionAndOrientation (pybullet.py:427-439); velocity kept."""
        self.set_rows(L.F_CPOS, position)
        self.set_rows(L.F_CQUAT, orientation)

    def control_joints(self, body: str, joints: Sequence[int], target_angles, forces) -> None:
        """setJointMotorControlArray(POSITION_CONTROL) (pybullet.py:462-477)."""
        t = torch.as_tensor(target_angles, dtype=torch.float32, device=self.device)
        for k, j in enumerate(joints):
            d = JOINT_TO_DOF[int(j)]
            self.f[L.F_MTARGET + d, :self.num_envs] = t[..., k]
            self.f[L.F_MKP + d, :self.num_envs] = 0.1
            self.f[L.F_MKD + d, :self.num_envs] = 1.0
            self.f[L.F_MVEL + d, :self.num_envs] = 0.0
            self.f[L.F_MIMP + d, :self.num_envs] = float(forces[k]) * DT_SUBSTEP

    def inverse_kinematics(self, body: str, link: int, position, orientation) -> torch.Tensor:
        """calculateInverseKinematics from the current joints (pybullet.py:479-497) -> [B, 9]."""
        B = self.num_envs
        pos = torch.as_tensor(position, dtype=torch.float32, device=self.device).expand(B, 3).contiguous()
        orn = torch.as_tensor(orientation, dtype=torch.float32, device=self.device).expand(B, 4).contiguous()
        out = torch.empty(B, 9, device=self.device)
        self._call("ps_inverse_kinematics", self._ctx, _ptr(self.state), int(link), _ptr(pos), _ptr(orn), _ptr(out),
                   self._stream())
        return out
