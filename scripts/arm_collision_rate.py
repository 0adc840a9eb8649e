#!/usr/bin/env python
"""How often do the arm links (PyBullet links 0-6, panda_link1-7) reach the
table or the objects?  (VERDICT r04 missing 3 / item 6.)

PyBullet collides every link of the Panda with the table and the objects
(envs/core.py:47-52 loads panda.urdf with its collision meshes; robots/
panda.py:37).  The build collides only the gripper (three boxes from the
reference's hand and finger hulls) and a wrist sphere on link 7
(include/panda_model.h PM_BOX_TABLE, PM_WRIST_SPHERE).  This script runs the
fp64 oracle (CPU, test infrastructure) on random-action rollouts with
autoreset and, after every env step, tests the arm's capsule proxies of the
render path (oracle/render_oracle.py ARM_CAPSULES; the fixed base's capsule
is left out: the base does not move; the hand is collided already) against
the table box and the objects, reporting the fraction of env-steps in which
any of them intersects, by capsule, with the depth.

  python scripts/arm_collision_rate.py [envs] [steps] > profiles/r05_arm_collision_rate.jsonl
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle")]

import oracle as O  # noqa: E402
import render_oracle as RO  # noqa: E402

N_SAMPLES = 33  # points per capsule axis (spacing <= 1.6 cm on the longest link)
# the render path's arm capsules of links that move (render_oracle.ARM_CAPSULES
# without the fixed base's); the hand (link 8) is collided as its hull boxes,
# and the render path's flange-to-palm capsule reaches 2 cm between the fingers,
# so it is no arm-link proxy
CAPS = [(a, b, r) for a, b, r in RO.ARM_CAPSULES if a >= 0]
CAP_NAMES = [f"frames {a}-{b} (r {r})" for a, b, r in CAPS]


def box_distance(p, c, Rb, h):
    """Distance of points p [..., n, 3] from boxes (centres c [..., 1, 3],
    rotations Rb [..., 3, 3], half extents h [3])."""
    loc = np.einsum("...ni,...ij->...nj", p - c, Rb)  # box frame
    d = np.maximum(np.abs(loc) - h, 0.0)
    return np.linalg.norm(d, axis=-1)


def quat_mats(q):
    x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return np.stack([np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
                     np.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
                     np.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)], -2)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    O.lib().po_set_threads(int(os.environ.get("OMP_NUM_THREADS", "8")))
    Lf = O.lib().po_link_frames
    Lf.argtypes = [C.POINTER(O.Config), C.POINTER(O.Env), C.c_void_p, C.c_void_p]
    Rbuf, obuf = (C.c_double * 108)(), (C.c_double * 36)()
    for env_id, task, control in [("PandaPush-v3", "push", "ee"), ("PandaPushJoints-v3", "push", "joints"),
                                  ("PandaReachJoints-v3", "reach", "joints"), ("PandaReach-v3", "reach", "ee"),
                                  ("PandaPickAndPlace-v3", "pick_and_place", "ee")]:
        t0 = time.time()
        cfg = O.config(task, control)
        envs = (O.Env * B)()
        for i in range(B):
            O.lib().po_init_env(C.byref(cfg), C.byref(envs[i]))
            O.reset(cfg, envs[i], seed=12345 + i)
        na, od, gd = O.action_dim(cfg), O.obs_dim(cfg), O.goal_dim(cfg)
        obs, ag, dg = np.zeros((B, od), np.float32), np.zeros((B, gd), np.float32), np.zeros((B, gd), np.float32)
        rew = np.zeros(B, np.float32)
        te, tr = np.zeros(B, np.uint8), np.zeros(B, np.uint8)
        rng = np.random.default_rng(0xC0FFEE)
        table_c = np.array([cfg.table_cx, 0.0, -0.2])
        table_h = np.array([cfg.table_hx, cfg.table_hy, 0.2])
        obj_h = np.array([cfg.object_half[k] for k in range(3)])
        hit_any = hit_table = hit_obj = near = 0
        per_cap = np.zeros(len(CAP_NAMES), np.int64)
        depth_hist = {"<1mm": 0, "1-5mm": 0, ">=5mm": 0}
        max_depth = 0.0
        fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
        for s in range(T):
            a = rng.uniform(-1, 1, size=(B, na)).astype(np.float32)
            O.lib().po_step_batch(C.byref(cfg), envs, B, fp(a), fp(obs), fp(ag), fp(dg), fp(rew),
                                  te.ctypes.data_as(C.POINTER(C.c_uint8)), tr.ctypes.data_as(C.POINTER(C.c_uint8)),
                                  1, None)
            o = np.zeros((B, 12, 3))
            for i in range(B):
                Lf(C.byref(cfg), C.byref(envs[i]), Rbuf, obuf)
                o[i] = np.frombuffer(obuf, np.float64).reshape(12, 3)
            t_ = np.linspace(0.0, 1.0, N_SAMPLES)[None, :, None]
            dt = np.zeros((B, len(CAPS)))
            do = np.full((B, len(CAPS)), -1.0)
            objs = [(np.array([envs[i].obj[b].pos[:] for i in range(B)]),
                     quat_mats(np.array([envs[i].obj[b].quat[:] for i in range(B)]))) for b in range(cfg.n_objects)]
            for ci, (ca, cb, r) in enumerate(CAPS):
                pts = o[:, ca][:, None] + t_ * (o[:, cb] - o[:, ca])[:, None]  # [B, n, 3]
                dt[:, ci] = r - box_distance(pts, table_c[None, None], np.eye(3)[None], table_h).min(1)
                for pos, Rq in objs:
                    d = r - box_distance(pts, pos[:, None], Rq, obj_h).min(1)
                    do[:, ci] = np.maximum(do[:, ci], d)
            deep = np.maximum(dt, do)  # [B, caps]
            hit = deep.max(1) > 0
            near += int((deep.max(1) > -0.01).sum())
            per_cap += (deep > 0).sum(0)
            hit_any += int(hit.sum())
            hit_table += int((dt.max(1) > 0).sum())
            hit_obj += int((do.max(1) > 0).sum())
            dm = deep.max(1)[hit]
            depth_hist["<1mm"] += int((dm < 1e-3).sum())
            depth_hist["1-5mm"] += int(((dm >= 1e-3) & (dm < 5e-3)).sum())
            depth_hist[">=5mm"] += int((dm >= 5e-3).sum())
            if hit.any():
                max_depth = max(max_depth, float(dm.max()))
        n = B * T
        rec = {"env_id": env_id, "envs": B, "steps": T, "autoreset": True, "actions": "U(-1,1), default_rng(0xC0FFEE)",
               "env_steps_with_arm_intersection": hit_any, "fraction": hit_any / n,
               "fraction_table": hit_table / n, "fraction_objects": hit_obj / n,
               "fraction_within_1cm": near / n,
               "per_capsule": {CAP_NAMES[k]: int(per_cap[k]) for k in range(len(CAP_NAMES))},
               "deepest_per_env_step": depth_hist, "max_depth_m": round(max_depth, 5),
               "seconds": round(time.time() - t0, 1)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
