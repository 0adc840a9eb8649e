"""Shared helpers for the parity tests: move state between the HIP path's SoA
state buffer and the oracle's per-env structs."""
import numpy as np
import oracle as O

TASK_NAMES = ["reach", "push", "pick_and_place"]


def oracle_config_for(sim_cfg):
    """oracle.Config mirroring a pandasim _lib.Config."""
    cfg = O.config(TASK_NAMES[sim_cfg.task], control="ee" if sim_cfg.control == 0 else "joints",
                   reward="sparse" if sim_cfg.reward == 0 else "dense")
    cfg.block_gripper = sim_cfg.block_gripper
    cfg.has_table, cfg.has_plane, cfg.has_cube = sim_cfg.has_table, sim_cfg.has_plane, sim_cfg.has_cube
    for k in range(3):
        cfg.base[k] = float(np.float32(sim_cfg.base[k]))
    cfg.cube_half = float(np.float32(sim_cfg.cube_half))
    cfg.cube_mass = float(np.float32(sim_cfg.cube_mass))
    return cfg


def snapshot(sim):
    """Host copy of the whole batched state (numpy)."""
    B = sim.num_envs
    return {
        "f": sim.f[:, :B].double().cpu().numpy(),
        "goal": sim.goal[:, :B].cpu().numpy(),
        "rng": sim.rng[:, :B].cpu().numpy().view(np.uint64),
        "elapsed": sim.elapsed[:B].cpu().numpy(),
    }


def oracle_env_from(cfg, snap, i):
    env = O.new_env(cfg)
    f = snap["f"][:, i]
    for d in range(9):
        env.q[d], env.qd[d] = f[d], f[9 + d]
        env.m_target[d], env.m_kp[d], env.m_kd[d] = f[18 + d], f[27 + d], f[36 + d]
        env.m_vel[d], env.m_maximp[d] = f[45 + d], f[54 + d]
    for k in range(3):
        env.cpos[k], env.cvel[k], env.comg[k] = f[63 + k], f[70 + k], f[73 + k]
        env.goal[k] = snap["goal"][k, i]
    for k in range(4):
        env.cquat[k] = f[66 + k]
        env.rng[k] = int(snap["rng"][k, i])
    env.elapsed = int(snap["elapsed"][i])
    return env
