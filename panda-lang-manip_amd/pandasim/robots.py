"""Batched Panda robot plugin (panda_gym/envs/robots/panda.py:10-140)."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .core import PyBulletRobot, box


class Panda(PyBulletRobot):
    """Panda robot, B envs.

    Args:
        sim (PandaSim): batched simulation.
        block_gripper (bool): whether the gripper is blocked.
        base_position: base position (x, y, z); defaults to the origin.
        control_type (str): "ee" (end-effector displacement) or "joints".
    """

    def __init__(self, sim, block_gripper: bool = False, base_position: Optional[np.ndarray] = None,
                 control_type: str = "ee") -> None:
        base_position = base_position if base_position is not None else np.zeros(3)
        self.block_gripper = block_gripper
        self.control_type = control_type
        n_action = 3 if self.control_type == "ee" else 7  # (x, y, z) if "ee", else the 7 joints
        n_action += 0 if self.block_gripper else 1
        action_space = box(-1.0, 1.0, (n_action,))
        super().__init__(sim, body_name="panda", file_name="franka_panda/panda.urdf", base_position=base_position,
                         action_space=action_space, joint_indices=np.array([0, 1, 2, 3, 4, 5, 6, 9, 10]),
                         joint_forces=np.array([87.0, 87.0, 87.0, 87.0, 12.0, 120.0, 120.0, 170.0, 170.0]))
        self.fingers_indices = np.array([9, 10])
        self.neutral_joint_values = np.array([0.00, 0.41, 0.00, -1.85, 0.00, 2.26, 0.79, 0.00, 0.00])
        self.ee_link = 11
        self.sim.set_lateral_friction(self.body_name, self.fingers_indices[0], lateral_friction=1.0)
        self.sim.set_lateral_friction(self.body_name, self.fingers_indices[1], lateral_friction=1.0)
        self.sim.set_spinning_friction(self.body_name, self.fingers_indices[0], spinning_friction=0.001)
        self.sim.set_spinning_friction(self.body_name, self.fingers_indices[1], spinning_friction=0.001)

    def set_action(self, action: torch.Tensor) -> None:
        """panda.py:52-70."""
        action = torch.as_tensor(action, dtype=torch.float32, device=self.sim.device).clone()
        action = action.clamp(-1.0, 1.0)
        if self.control_type == "ee":
            target_arm_angles = self.ee_displacement_to_target_arm_angles(action[:, :3])
        else:
            target_arm_angles = self.arm_joint_ctrl_to_target_arm_angles(action[:, :7])
        if self.block_gripper:
            target_fingers_width = torch.zeros(action.shape[0], device=action.device)
        else:
            fingers_ctrl = action[:, -1] * 0.2  # limit maximum change in position
            target_fingers_width = self.get_fingers_width() + fingers_ctrl
        half = (target_fingers_width / 2).unsqueeze(-1)
        target_angles = torch.cat([target_arm_angles, half, half], dim=-1)
        self.control_joints(target_angles=target_angles)

    def ee_displacement_to_target_arm_angles(self, ee_displacement: torch.Tensor) -> torch.Tensor:
        """panda.py:72-92."""
        ee_displacement = ee_displacement[:, :3] * 0.05  # limit maximum change in position
        ee_position = self.get_ee_position()
        target_ee_position = ee_position + ee_displacement
        # Clip the height target (panda.py:86)
        target_ee_position[:, 2] = target_ee_position[:, 2].clamp(min=0.0)
        target_arm_angles = self.inverse_kinematics(link=self.ee_link, position=target_ee_position,
                                                    orientation=np.array([1.0, 0.0, 0.0, 0.0]))
        return target_arm_angles[:, :7]  # remove fingers angles

    def arm_joint_ctrl_to_target_arm_angles(self, arm_joint_ctrl: torch.Tensor) -> torch.Tensor:
        """panda.py:94-107."""
        arm_joint_ctrl = arm_joint_ctrl * 0.05  # limit maximum change in position
        current = torch.stack([self.get_joint_angle(joint=i) for i in range(7)], dim=-1)
        return current + arm_joint_ctrl

    def get_obs(self) -> torch.Tensor:
        """panda.py:109-119."""
        ee_position = self.get_ee_position()
        ee_velocity = self.get_ee_velocity()
        if not self.block_gripper:
            fingers_width = self.get_fingers_width()
            return torch.cat([ee_position, ee_velocity, fingers_width.unsqueeze(-1)], dim=-1)
        return torch.cat([ee_position, ee_velocity], dim=-1)

    def reset(self) -> None:
        self.set_joint_neutral()

    def set_joint_neutral(self) -> None:
        """panda.py:121-126."""
        self.set_joint_angles(self.neutral_joint_values)

    def get_fingers_width(self) -> torch.Tensor:
        """panda.py:128-132."""
        finger1 = self.sim.get_joint_angle(self.body_name, self.fingers_indices[0])
        finger2 = self.sim.get_joint_angle(self.body_name, self.fingers_indices[1])
        return finger1 + finger2

    def get_ee_position(self) -> torch.Tensor:
        return self.get_link_position(self.ee_link)

    def get_ee_velocity(self) -> torch.Tensor:
        return self.get_link_velocity(self.ee_link)
