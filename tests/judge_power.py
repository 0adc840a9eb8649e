"""Power of the parity classifier (test infrastructure, CPU only).

tests/parity_judge.judge decides whether a GPU env step agrees with the fp64
oracle.  Its allowances (the oracle's own sensitivity at fp32 resolution, the
ill-conditioned probes) could in principle absorb a real model error.  This
module replays the teacher-forced workloads of the GPU tests with a stand-in
for the GPU: the oracle itself, in fp32-like arithmetic (PGS impulses, M^-1
and the state rounded to fp32: oracle.set_fp32_solver / set_fp32_dynamics /
set_state_noise(-1)), optionally with a deliberate model error
(oracle.set_model_mutation, or the object's mass and friction in the config).
Every step is classified exactly as the GPU tests classify theirs.

Workloads (as in the GPU tests):
  * "random": test_gpu_parity.test_env_step_parity_teacher_forced -- 64 envs
    reset with seeds 12345 + i, 10 steps of U(-1, 1) actions from
    default_rng(7);
  * "push": test_gpu_parity.test_gripper_object_contact_parity's scripted
    push -- 64 envs, seeds 44 + i, 14 steps, the end effector driven over
    the object and then through it, the fingers closing from step 8;
  * "stack_push" (Stack): test_gpu_parity.test_judged_contact_workloads --
    seeds 44 + i, cube 2 set on cube 1 at rest, then the scripted push
    aimed at cube 2: the gripper comes down on the top cube and drags it
    over the bottom one (box-box normal and friction rows every step).
The stand-in's own trajectory is followed (as the GPU's is), and each step
starts from its state rounded to fp32 (the GPU's state storage).
"""
import ctypes

import numpy as np

import oracle as O
from helpers import OBJECT_ROWS, WG_ROWS, WP_ROW, WPN_ROW, WPPT_ROW, WR_ROW, oracle_env_from
from parity_judge import FREE_GRIPPER, TOL, _before, _obs_err, _within, groups_for, judge

N_ROWS = 121


def _pack_ids(ids):
    return float(sum(int(v) << (5 * k) for k, v in enumerate(ids)))


def snapshot_of(envs):
    """The SoA snapshot (tests/helpers.snapshot's layout) of oracle envs, the
    state rounded to fp32 as the GPU stores it."""
    B = len(envs)
    f = np.zeros((N_ROWS, B))
    goal = np.zeros((6, B))
    rng = np.zeros((5, B), np.uint64)
    elapsed = np.zeros(B, np.int64)
    for i, e in enumerate(envs):
        col = f[:, i]
        col[0:9], col[9:18] = e.q[:], e.qd[:]
        for k, name in enumerate(("m_target", "m_kp", "m_kd", "m_vel", "m_maximp")):
            col[18 + 9 * k:27 + 9 * k] = getattr(e, name)[:]
        for b, r in enumerate(OBJECT_ROWS):
            o = e.obj[b]
            col[r:r + 3], col[r + 3:r + 7], col[r + 7:r + 10], col[r + 10:r + 13] = o.pos[:], o.quat[:], o.vel[:], o.omg[:]
        k = e.cache
        for b, r in enumerate(WG_ROWS):
            col[r:r + 4] = k.ground_lam[b][:]
            col[r + 4] = _pack_ids(k.ground_id[b][:])
        col[WR_ROW:WR_ROW + 4] = k.robot_lam[:]
        col[WR_ROW + 4] = _pack_ids(k.robot_id[:])
        col[WP_ROW:WP_ROW + 4] = k.pair_lam[:]
        for s in range(4):
            col[WPPT_ROW + 3 * s:WPPT_ROW + 3 * s + 3] = k.pair_pt[s][:]
        col[WPN_ROW] = k.pair_n
        goal[:, i] = e.goal[:]
        rng[:, i] = [int(v) for v in e.rng]
        elapsed[i] = e.elapsed
    return {"f": f.astype(np.float32).astype(np.float64), "goal": goal, "rng": rng, "elapsed": elapsed}


def _copy_cfg(cfg, **overrides):
    c = O.Config()
    ctypes.memmove(ctypes.byref(c), ctypes.byref(cfg), ctypes.sizeof(cfg))
    for k, v in overrides.items():
        setattr(c, k, v)
    return c


MUTATIONS = {
    # name: (oracle hook kind, value) or ("config", field, factor)
    "none": None,
    "cube_mass_x1.02": ("config", "object_mass", 1.02),
    "cube_friction_0.51": ("config", "object_friction", 0.51 / 0.5),
    "motor_kp_x1.01": ("motor_kp_scale", 1.01),
    "link_damping_0.045": ("link_damping", 0.045),
    "finger_box_+0.5mm": ("finger_box_grow", 0.0005),
    # round 6: Stack's second cube and its cube-cube rows
    "cube2_mass_x1.02": ("config", "object2_mass", 1.02),
    "pair_friction_x1.02": ("pair_friction_scale", 1.02),
}


def _stand_in_step(cfg, env, action, mutation, fp32=True):
    """One env step of the GPU stand-in: the oracle in fp32-like arithmetic
    (fp32=False: in fp64), with `mutation` applied."""
    c = cfg
    if mutation is not None and mutation[0] == "config":
        c = _copy_cfg(cfg, **{mutation[1]: getattr(cfg, mutation[1]) * mutation[2]})
    elif mutation is not None:
        O.set_model_mutation(mutation[0], mutation[1])
    O.set_fp32_solver(fp32)
    O.set_fp32_dynamics(fp32)
    O.set_state_noise(-1.0 if fp32 else 0.0)
    try:
        return O.step(c, env, action)
    finally:
        O.set_state_noise(0.0)
        O.set_fp32_dynamics(False)
        O.set_fp32_solver(False)
        O.set_model_mutation("none")


def _push_actions(envs, body, s, action_dim, cfg):
    """test_gpu_contacts._push_policy on oracle envs."""
    a = np.zeros((len(envs), action_dim), np.float32)
    for i, e in enumerate(envs):
        pos, *_ = O.link_state(cfg, e, 11)
        obj = np.array(e.obj[body].pos)
        tgt = obj + np.array([0.0, 0.0, 0.06 if s < 6 else 0.0])
        if s >= 6:
            tgt[0] += 0.05
        a[i, :3] = np.clip(10.0 * (tgt - pos), -1, 1)
        if action_dim == 4:
            a[i, 3] = -1.0 if s >= 8 else 1.0
    return a


def stack_cubes(e):
    """Cube 2 at rest on top of cube 1 (face to face, cube size 0.04 m)."""
    for k in range(3):
        e.obj[1].pos[k] = e.obj[0].pos[k] + (0.04 if k == 2 else 0.0)
        e.obj[1].vel[k] = e.obj[1].omg[k] = 0.0
    for k in range(4):
        e.obj[1].quat[k] = e.obj[0].quat[k]


def classify_workload(task, control, workload, mutation_name, B=64, steps=None, stride=1):
    """Class counts of every (env, step) sample of a workload whose GPU
    stand-in carries `mutation_name` (MUTATIONS).  Returns (counts, worst
    per-group error of the non-tight samples, the mutation's own effect: the
    largest per-group move of the fp64 oracle's observation under it, and the
    number of samples where that effect alone leaves the tight bounds)."""
    mutation = MUTATIONS[mutation_name]
    cfg = O.config(task, control)
    seed0 = 12345 if workload == "random" else 44
    steps = steps or (10 if workload == "random" else 14)
    envs = []
    for i in range(B):
        e = O.new_env(cfg)
        O.reset(cfg, e, seed=seed0 + i)
        if workload == "stack_push":
            stack_cubes(e)
        envs.append(e)
    body = 1 if workload == "stack_push" else 0
    adim = O.action_dim(cfg)
    groups = groups_for(task, 7 if task in FREE_GRIPPER else 6)
    rng = np.random.default_rng(7)
    counts = {"tight": 0, "conditioned": 0, "bif": 0, "beyond": 0}
    worst = {k: 0.0 for k in groups}
    effect = {k: 0.0 for k in groups}
    visible = 0
    for s in range(steps):
        snap = snapshot_of(envs)
        if workload == "random":
            a = rng.uniform(-1, 1, size=(B, adim)).astype(np.float32)
        else:
            a = _push_actions([oracle_env_from(cfg, snap, i) for i in range(B)], body, s, adim, cfg)
        for i in range(0, B, stride):
            gpu = oracle_env_from(cfg, snap, i)
            og, *_ = _stand_in_step(cfg, gpu, a[i], mutation)
            o, *_ = O.step(cfg, oracle_env_from(cfg, snap, i), a[i])
            cls, errs = judge(cfg, snap, i, a[i], o, og, groups, task)
            counts[cls] += 1
            if mutation is not None:
                om, *_ = _stand_in_step(cfg, oracle_env_from(cfg, snap, i), a[i], mutation, fp32=False)
                eff = {k: _obs_err(om, o, k, idx, task) for k, idx in groups.items()}
                bf = _before(snap, i, task)
                visible += any(not _within(eff[k], o, groups, k, TOL[task], bf) for k in groups)
                for k in groups:
                    effect[k] = max(effect[k], eff[k])
            if cls != "tight":
                for k, v in errs.items():
                    worst[k] = max(worst[k], v)
            envs[i] = gpu
        for i in range(B):  # envs not sampled this step follow the stand-in too
            if i % stride:
                e = oracle_env_from(cfg, snap, i)
                _stand_in_step(cfg, e, a[i], mutation)
                envs[i] = e
    return counts, worst, effect, visible


__all__ = ["MUTATIONS", "classify_workload", "snapshot_of", "stack_cubes"]
