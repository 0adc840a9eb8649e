#!/usr/bin/env python
"""Power of the parity classifier on the CPU: the class
counts of the GPU tests' teacher-forced workloads when the "GPU" is the oracle
in fp32-like arithmetic with a deliberate model error (tests/judge_power.py),
and the smallest error of each kind that still yields 'beyond' samples.

  python scripts/judge_power_scan.py > profiles/r05_judge_power.jsonl
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import judge_power as J  # noqa: E402

CASES = [
    # (task, control, workload, mutations)
    ("reach", "ee", "random", ["none", "motor_kp_x1.01", "link_damping_0.045"]),
    ("push", "ee", "push", ["link_damping_0.045"]),
    ("reach", "joints", "random", ["none", "motor_kp_x1.01", "link_damping_0.045"]),
    ("push", "ee", "random", ["none", "motor_kp_x1.01", "link_damping_0.045", "cube_mass_x1.02",
                              "cube_friction_0.51", "finger_box_+0.5mm"]),
    ("pick_and_place", "ee", "random", ["none", "motor_kp_x1.01", "link_damping_0.045", "finger_box_+0.5mm"]),
    ("push", "ee", "push", ["none", "cube_mass_x1.02", "cube_friction_0.51", "finger_box_+0.5mm"]),
    ("pick_and_place", "ee", "push", ["none", "cube_mass_x1.02", "cube_friction_0.51", "finger_box_+0.5mm"]),
    ("slide", "ee", "push", ["none", "cube_mass_x1.02", "cube_friction_0.51", "finger_box_+0.5mm"]),
]

# effect-size ladders: the smallest value of each kind with beyond samples
LADDERS = [
    ("push", "ee", "random", "motor_kp_scale", [1.0003, 1.001, 1.003]),
    ("reach", "ee", "random", "link_damping", [0.08, 0.2, 0.5]),
    ("push", "ee", "push", "link_damping", [0.045, 0.06, 0.1, 0.2]),
    ("push", "ee", "push", "object_mass", [1.001, 1.003, 1.01]),
    ("push", "ee", "push", "object_friction", [1.001, 1.003, 1.01]),
    ("push", "ee", "push", "finger_box_grow", [0.00002, 0.00005, 0.0001, 0.0002]),
]


def run(task, control, workload, name, B):
    t = time.time()
    counts, worst, effect, visible = J.classify_workload(task, control, workload, name, B=B)
    rec = {"task": task, "control": control, "workload": workload, "mutation": name, "envs": B, "counts": counts,
           "worst_not_tight": {k: float(f"{v:.3g}") for k, v in worst.items()},
           "mutation_effect_fp64": {k: float(f"{v:.3g}") for k, v in effect.items()},
           "samples_effect_beyond_tight": visible, "seconds": round(time.time() - t, 1)}
    print(json.dumps(rec), flush=True)
    return counts


def main():
    B = int(os.environ.get("JUDGE_POWER_ENVS", "64"))
    for task, control, workload, muts in CASES:
        for m in muts:
            run(task, control, workload, m, B)
    for task, control, workload, kind, values in LADDERS:
        for v in values:
            if kind in ("object_mass", "object_friction"):
                J.MUTATIONS[f"{kind}_x{v}"] = ("config", kind, v)
            else:
                J.MUTATIONS[f"{kind}_{v}"] = (kind, v)
            name = f"{kind}_x{v}" if kind in ("object_mass", "object_friction") else f"{kind}_{v}"
            run(task, control, workload, name, B)


if __name__ == "__main__":
    main()
