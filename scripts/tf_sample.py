#!/usr/bin/env python
"""Replays a dumped teacher-forced sample (tests/test_gpu_contacts.py
test_teacher_forced_200_steps -> gpurun_out/tf200/<task>_<control>_<step>_<env>.npz)
with the oracle on the CPU and prints where the GPU step and the oracle step
part: observation groups, joint state, and the contact caches (slot ids and
impulses).

  python scripts/tf_sample.py gpurun_out/tf200/push_ee_49_50.npz [...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import oracle as O  # noqa: E402
from helpers import oracle_env_from  # noqa: E402
from test_gpu_contacts import gpu_cache, oracle_cache  # noqa: E402


def replay(path):
    name = os.path.basename(path)[:-4]
    task, rest = name.rsplit("_", 3)[0], name.rsplit("_", 3)[1:]
    control = rest[0]
    d = np.load(path)
    cfg = O.config(task, control)
    snap = {"f": d["f"][:, None], "goal": d["goal"][:, None],
            "rng": d["rng"][:, None] if "rng" in d else np.zeros((4, 1), np.uint64),
            "elapsed": np.array([int(d["elapsed"]) if "elapsed" in d else 0])}
    e = oracle_env_from(cfg, snap, 0)
    o, *_ = O.step(cfg, e, d["action"])
    g = d["gpu_obs"]
    print(f"== {name}: obs max |gpu - oracle| {np.abs(g - o).max():.2e} at {int(np.abs(g - o).argmax())}")
    fa = d["gpu_f_after"]
    dq = np.abs(fa[0:9] - np.array(e.q[:9]))
    dqd = np.abs(fa[9:18] - np.array(e.qd[:9]))
    fmt = {"float_kind": lambda x: f"{x:.1e}"}
    print(f"   q  err {np.array2string(dq, formatter=fmt)}\n   qd err {np.array2string(dqd, formatter=fmt)}")
    gc, oc = gpu_cache(fa[:, None], 0), oracle_cache(e)
    for k in gc:
        print(f"   {k:8s} gpu {[(int(i), round(float(l), 5)) for i, l in gc[k]] if k != 'pair' else len(gc[k])}")
        print(f"   {'':8s} ora {[(int(i), round(float(l), 5)) for i, l in oc[k]] if k != 'pair' else len(oc[k])}")
    # the oracle's own conditioning: the same step with the state moved at fp32
    # resolution (test_gpu_parity.FP32_PROBES) and with per-substep state noise
    from parity_judge import FP32_PROBES

    moves = []
    for p in FP32_PROBES:
        e2 = oracle_env_from(cfg, snap, 0)
        p(e2)
        o2, *_ = O.step(cfg, e2, d["action"])
        moves.append(np.abs(o2 - o).max())
    for seed in range(4):
        e2 = oracle_env_from(cfg, snap, 0)
        O.set_state_noise(1.0, seed=seed + 1)
        o2, *_ = O.step(cfg, e2, d["action"])
        O.set_state_noise(0.0)
        moves.append(np.abs(o2 - o).max())
    noise = ", ".join(f"{m:.1e}" for m in moves[-4:])
    print(f"   oracle moved by fp32 probes: max {max(moves[:-4]):.2e}; by 1-ulp state noise: {noise}")
    before = gpu_cache(d["f"][:, None], 0)
    print(f"   robot cache before the step {[(int(i), round(float(l), 5)) for i, l in before['robot']]}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        replay(p)
