#!/usr/bin/env python
"""CPU-only calibration of the free-run yardstick (tests/test_gpu_contacts.py
test_free_running_200_steps): the fp64 oracle from the free runs' initial
states (reset seeds 2024 + i, state rounded to fp32 as the GPU stores it) and
action stream, against itself perturbed at fp32 resolution in several ways --
one and two fp32 ulps of per-substep state noise, the state rounded to fp32
after every substep (the GPU's storage), and that rounding plus one ulp of
noise.  Prints, per case and perturbation, the fraction of env-steps whose ee
and object positions stay within 1e-3 m of the unperturbed run (the fraction
the GPU run is held to).

  python scripts/free_run_yardstick.py [push:ee reach:joints ...]
"""
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import oracle as O  # noqa: E402

B, T, SEED = 64, 200, 2024
PERTURBATIONS = {"ulp1": (1.0, 3), "ulp2": (2.0, 3), "fp32_state": (-1.0, 1)}


def _obs_index(task):
    nobj = {"reach": 0, "stack": 2}.get(task, 1)
    robot_dim = 6 if task in ("reach", "push", "slide") else 7
    per = 13 if task == "flip" else 12
    return [0, 1, 2] + [robot_dim + per * b + k for b in range(nobj) for k in range(3)]


def _round_state(e, nobj):
    for d in range(9):
        e.q[d], e.qd[d] = float(np.float32(e.q[d])), float(np.float32(e.qd[d]))
    for b in range(nobj):
        o = e.obj[b]
        for k in range(3):
            o.pos[k], o.vel[k], o.omg[k] = (float(np.float32(x)) for x in (o.pos[k], o.vel[k], o.omg[k]))
        for k in range(4):
            o.quat[k] = float(np.float32(o.quat[k]))


def run_case(case):
    task, control = case.split(":")
    cfg = O.config(task, control)
    nobj = {"reach": 0, "stack": 2}.get(task, 1)
    idx = _obs_index(task)

    def fresh():
        envs = []
        for i in range(B):
            e = O.new_env(cfg)
            O.reset(cfg, e, seed=SEED + i)
            _round_state(e, nobj)
            envs.append(e)
        return envs

    rng = np.random.default_rng(SEED)
    actions = rng.uniform(-1, 1, size=(T, B, O.action_dim(cfg))).astype(np.float32)
    ref = fresh()
    runs = {f"{name}#{r}": (ulps, fresh()) for name, (ulps, n) in PERTURBATIONS.items() for r in range(n)}
    within = {k: 0 for k in runs}
    for s in range(T):
        for i in range(B):
            o, *_ = O.step(cfg, ref[i], actions[s, i])
            for r, (key, (ulps, envs)) in enumerate(runs.items()):
                O.set_state_noise(ulps, seed=((s * B + i) * 2 + 1) + r * 1000003)
                op, *_ = O.step(cfg, envs[i], actions[s, i])
                O.set_state_noise(0.0)
                within[key] += bool(np.abs(op[idx] - o[idx]).max() <= 1e-3)
    return case, {k: round(v / (B * T), 4) for k, v in within.items()}


if __name__ == "__main__":
    cases = sys.argv[1:] or ["push:ee", "pick_and_place:ee", "reach:joints", "push:joints"]
    with ProcessPoolExecutor(min(len(cases), 4)) as ex:
        for case, fr in ex.map(run_case, cases):
            print(json.dumps({"case": case, "fraction_within_1e-3": fr}), flush=True)
