#!/usr/bin/env python
"""The group solver's row dump (-DPS_DEBUG_ROW_DUMP builds: scripts/build_variants.py
dump, groups_o3_dump) of one fused step from a reset, for each library given,
and the first record where the libraries differ per lane (the -O3 group-kernel
investigation).  Records per lane and substep (0, 1): the
solver inputs (motor rhs, 1/den, limit rhs per DoF; ground rows' rhs and 1/den;
gripper rows' rhs, 1/den, warm start; the gates), then each row's impulse
change in the first iteration pair, then that pair's residual.

usage: python scripts/row_dump.py TASK CONTROL LANES lib_a.so lib_b.so [...]
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROWS, LANES_DUMPED = 256, 4096
CHILD = r'''
import ctypes as C, os, sys, numpy as np, torch
sys.path.insert(0, os.path.join(os.environ["ROOT"], "panda-lang-manip_amd"))
from pandasim.envs import PandaVecEnv
task, control, lanes, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
B = 64
env = PandaVecEnv(task, "sparse", control, B, "cuda", lanes_per_env=lanes, autoreset=False)
env.reset(seed=12345)
lib = env.sim._lib
buf = np.zeros(4096 * 2 * 256, np.float32)
lib.ps_debug_row_dump.argtypes = [C.c_void_p, C.c_int]
assert lib.ps_debug_row_dump(buf.ctypes.data, 1) == 0
a = np.random.default_rng(7).uniform(-1, 1, size=(B, env.action_dim)).astype(np.float32)
env.step(torch.from_numpy(a).cuda())
assert lib.ps_debug_row_dump(buf.ctypes.data, 0) == 0
np.savez(out, dump=buf.reshape(4096, 2, 256), q=env.sim.f[0:18, :B].double().cpu().numpy())
'''


def main(task, control, lanes, libs):
    res = []
    for i, lib in enumerate(libs):
        out = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"row_dump_{task}_{control}_{lanes}_{i}.npz")  # 8 MB each: not under gpurun_out
        env = dict(os.environ, PANDASIM_LIB=os.path.abspath(lib), ROOT=ROOT)
        p = subprocess.run([sys.executable, "-c", CHILD, task, control, str(lanes), out], env=env,
                           capture_output=True, text=True, timeout=300)
        if p.returncode:
            print(lib, "failed", p.stderr[-2000:])
            return 1
        res.append(np.load(out))
    a, b = res[0], res[-1]
    n_lanes = 64 * lanes
    da, db = a["dump"][:n_lanes], b["dump"][:n_lanes]
    both = ~(np.isnan(da) & np.isnan(db))
    diff = both & ~np.isclose(da, db, rtol=1e-5, atol=1e-7, equal_nan=True)
    q_err = np.abs(a["q"] - b["q"]).max(axis=0)
    summary = {"task": task, "control": control, "lanes": lanes, "libs": [os.path.basename(l) for l in libs],
               "q_qd_max_diff": float(q_err.max()), "envs_off_1e-3": int((q_err > 1e-3).sum()),
               "lanes_with_a_differing_record": int(diff.any(axis=(1, 2)).sum())}
    first = []
    for lane in range(n_lanes):
        for st in range(2):
            idx = np.nonzero(diff[lane, st])[0]
            if len(idx):
                k = int(idx[0])
                first.append((lane, st, k, float(da[lane, st, k]), float(db[lane, st, k])))
                break
    first.sort(key=lambda t: (t[1], t[2]))
    summary["earliest"] = first[:12]
    print(json.dumps(summary))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4:]))
