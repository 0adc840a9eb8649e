"""Shared helpers for the parity tests: move state between the HIP path's SoA
state buffer and the oracle's per-env structs."""
import numpy as np
import oracle as O

TASK_NAMES = ["reach", "push", "pick_and_place", "slide", "stack", "flip"]
OBJECT_ROWS = (63, 76)
# contact-cache rows (include/pandasim.h PS_F_WG0..PS_F_WPN)
WG_ROWS, WR_ROW, WP_ROW, WPPT_ROW, WPN_ROW = (89, 94), 99, 104, 108, 120


def unpack_ids(x):
    """Four 5-bit slot ids of a packed id row (sum id_k 32^k)."""
    v = int(x)
    return [(v >> (5 * k)) & 31 for k in range(4)]


def oracle_config_for(sim_cfg):
    """oracle.Config mirroring a pandasim _lib.Config."""
    cfg = O.config(TASK_NAMES[sim_cfg.task], control="ee" if sim_cfg.control == 0 else "joints",
                   reward="sparse" if sim_cfg.reward == 0 else "dense")
    cfg.block_gripper = sim_cfg.block_gripper
    cfg.has_table, cfg.has_plane = sim_cfg.has_table, sim_cfg.has_plane
    cfg.n_objects, cfg.object_shape = sim_cfg.n_objects, sim_cfg.object_shape
    for k in range(3):
        cfg.base[k] = float(np.float32(sim_cfg.base[k]))
        cfg.object_half[k] = float(np.float32(sim_cfg.object_half[k]))
    for name in ("object_mass", "object2_mass", "object_friction", "table_cx", "table_hx", "table_hy"):
        setattr(cfg, name, float(np.float32(getattr(sim_cfg, name))))
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
    for b, r in enumerate(OBJECT_ROWS):
        o = env.obj[b]
        for k in range(3):
            o.pos[k], o.vel[k], o.omg[k] = f[r + k], f[r + 7 + k], f[r + 10 + k]
        for k in range(4):
            o.quat[k] = f[r + 3 + k]
    for k in range(snap["goal"].shape[0]):
        env.goal[k] = snap["goal"][k, i]
    for k in range(snap["rng"].shape[0]):
        env.rng[k] = int(snap["rng"][k, i])
    env.elapsed = int(snap["elapsed"][i])
    k = env.cache
    for b, r in enumerate(WG_ROWS):
        for s, idv in enumerate(unpack_ids(f[r + 4])):
            k.ground_lam[b][s], k.ground_id[b][s] = f[r + s], idv
    for s, idv in enumerate(unpack_ids(f[WR_ROW + 4])):
        k.robot_lam[s], k.robot_id[s] = f[WR_ROW + s], idv
    for s in range(4):
        k.pair_lam[s] = f[WP_ROW + s]
        for j in range(3):
            k.pair_pt[s][j] = f[WPPT_ROW + 3 * s + j]
    k.pair_n = int(f[WPN_ROW])
    return env
