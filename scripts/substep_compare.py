#!/usr/bin/env python
"""Substep-by-substep comparison of one dumped teacher-forced sample
(gpurun_out/tf200/*.npz): the GPU's plugin-path substep (ps_sim_step with one
substep, the step's motor targets from the dumped state after it) against
the oracle's po_substep from the same state, printing after each of the 20
substeps the largest joint and object differences and both gripper-contact
caches -- where in the step a GPU/oracle difference starts.

  python scripts/substep_compare.py scratch_samples/push_ee_171_60.npz
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "panda-lang-manip_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

import oracle as O  # noqa: E402
from helpers import WG_ROWS, WR_ROW, oracle_env_from, unpack_ids  # noqa: E402


def main(path):
    from pandasim.envs import PandaVecEnv

    name = os.path.basename(path)[:-4]
    task, control = name.rsplit("_", 3)[0], name.rsplit("_", 3)[1]
    d = np.load(path)
    f0 = d["f"].astype(np.float64).copy()
    f0[18:27] = d["gpu_f_after"][18:27]  # this step's motor targets (set_action)
    cfg = O.config(task, control)
    snap = {"f": f0[:, None], "goal": d["goal"][:, None], "rng": d["rng"][:, None],
            "elapsed": np.array([int(d["elapsed"])])}
    e = oracle_env_from(cfg, snap, 0)
    B = 64
    env = PandaVecEnv(task, "sparse", control, B, "cuda", lanes_per_env=1)
    env.autoreset = False
    env.reset(seed=1)
    env.sim.f[:, :B] = torch.from_numpy(np.repeat(f0[:, None], B, axis=1)).to(env.sim.f.dtype).cuda()
    env.sim._call("ps_mark_motor_rows_dirty", env.sim._ctx)
    env.sim.n_substeps = 1
    for s in range(20):
        env.sim.step()
        O.lib().po_substep(C.byref(cfg), C.byref(e), None)
        g = env.sim.f[:, 0].double().cpu().numpy()
        dq = np.abs(g[0:9] - np.array(e.q[:9])).max()
        dqd = np.abs(g[9:18] - np.array(e.qd[:9])).max()
        dobj = np.abs(g[63:66] - np.array(e.obj[0].pos)).max()
        dov = np.abs(g[70:73] - np.array(e.obj[0].vel)).max()
        dow = np.abs(g[73:76] - np.array(e.obj[0].omg)).max()
        gg = [round(float(x), 5) for x in g[WG_ROWS[0]:WG_ROWS[0] + 4]]
        og = [round(e.cache.ground_lam[0][k], 5) for k in range(4)]
        gid = unpack_ids(g[WR_ROW + 4])
        glam = [round(float(x), 5) for x in g[WR_ROW:WR_ROW + 4]]
        oid = [e.cache.robot_id[k] for k in range(4)]
        olam = [round(e.cache.robot_lam[k], 5) for k in range(4)]
        print(f"substep {s:2d}: |dq| {dq:.2e} |dqd| {dqd:.2e} |dobj| {dobj:.2e} |dv_obj| {dov:.2e} |dw_obj| {dow:.2e}  "
              f"gpu robot {list(zip(gid, glam))}  oracle {list(zip(oid, olam))}  ground0 gpu {gg} oracle {og}",
              flush=True)
    print("final vs the fused step's state:", float(np.abs(env.sim.f[0:18, 0].double().cpu().numpy() -
                                                       d["gpu_f_after"][0:18]).max()))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
