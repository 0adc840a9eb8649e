"""Algorithmic FLOP count of the env step (bench.py's ``roofline.fp32``,
DESIGN.md §7).

The cost of each primitive is counted from the formulas the step kernel
evaluates (``csrc/ps_physics.h``, ``csrc/pandasim.hip``): an FMA is 2 FLOPs,
add/sub/mul 1, div/sqrt/rsqrt/rcp/sin/cos/atan2 1 each; comparisons, min/max,
selects and moves are not counted, and zero entries of the constant URDF
origin rotations are counted as if they were not known (the algorithm's
3x3 product, not what the compiler folds).  How often each primitive runs is
workload-dependent (PGS iterations, rows and contacts per substep, IK
iterations per step): those counts come from the fp64 oracle stepping a
sample of the same workload (``oracle.Stats``, ``po_stats``), i.e. each env's
own iteration count, not the wave-max the SIMD executes.
"""
from __future__ import annotations

# ---- per substep, independent of contacts (ps_physics.h substep())
FK = 7 * 83 + 3 * 63 + 2 * 84          # child_frame x 12 (revolute / fixed / prismatic)
BIAS_FORCES = 7 * 357 + 2 * 63 + 250 + 2 * 370 + 7 * 23  # RNEA with fused FK: arm links, hand, fingers, tau
GEOMETRY = FK + 30 + 8 * 21            # second FK, finger axes, 8 sphere centres
MASS_MATRIX = 10 * 66 + 9 * 72 + 14 * 17 + 6 + 7 * 30 + 20 * 28  # CRBA: link comps, combines, entries
SPD_INVERSE = 285 + 285 + 330          # Cholesky, L^-1, L^-T L^-1 (9x9)
UNCONSTRAINED = 9 * 20                 # v1 = qd - h M^-1 bias
JOINT_ROWS = 9 * 15                    # limit / motor row rhs (control_joints state)
INTEGRATE_ROBOT = 9 * 4
PER_OBJECT = 70 + 8 * 18 + 70          # body_dyn + damping, support points, integration (exp-map quaternion)
SPHERE_TESTS_PER_OBJECT = 8 * 40       # closest point of the solid to each sphere
SPHERE_TESTS_GROUND = 8 * 3

# ---- per active contact, per substep (row setup)
GROUND_CONTACT_SETUP = 110             # r, 3 rows: r x dir, I^-1, denominators, rhs
ROBOT_CONTACT_SETUP = 40 + 10 + 3 * 365  # contact frame, plane space, 3 x (J, M^-1 J^T, den, rel, rhs)
PAIR_CONTACT_SETUP = 60 + 10 + 3 * 60  # box-box clip share, plane space, 3 two-body rows

# ---- per row visit of the PGS loop (one iteration over one row; friction pairs included)
MOTOR_ROW = 23
LIMIT_ROW = 24
GROUND_ROW = 19 + 42                   # normal + friction-cone pair, object-only rows
ROBOT_ROW = 67 + 142                   # normal + friction-cone pair, 9 robot + 6 object DoFs
PAIR_ROW = 50 + 110                    # normal + friction-cone pair, two objects

# ---- per env step
IK_ITERATION = 1800                    # FK, orientation error, 6x7 Jacobian, J^T J + damping, 7x7 Cholesky solve
STEP_FIXED = 2500                      # set_action FK, observation (FK + link velocity + Euler), reward


def flops_per_env_step(stats: dict, n_objects: int) -> dict:
    """Algorithmic FLOPs per env step from oracle work counters (po_stats as
    a dict) summed over a sample; returns the total and its split."""
    steps = max(1, stats["steps"])
    sub = stats["substeps"] / steps
    per_sub_fixed = (BIAS_FORCES + GEOMETRY + MASS_MATRIX + SPD_INVERSE + UNCONSTRAINED + JOINT_ROWS
                     + INTEGRATE_ROBOT + n_objects * (PER_OBJECT + SPHERE_TESTS_PER_OBJECT) + SPHERE_TESTS_GROUND)
    setup = (stats["ground_contacts"] * GROUND_CONTACT_SETUP + stats["robot_contacts"] * ROBOT_CONTACT_SETUP
             + stats["pair_contacts"] * PAIR_CONTACT_SETUP) / steps
    pgs = (stats["motor_visits"] * MOTOR_ROW + stats["limit_visits"] * LIMIT_ROW + stats["ground_visits"] * GROUND_ROW
           + stats["robot_visits"] * ROBOT_ROW + stats["pair_visits"] * PAIR_ROW) / steps
    ik = stats["ik_iterations"] / steps * IK_ITERATION
    split = {"dynamics_and_rows": sub * per_sub_fixed + setup, "pgs": pgs, "ik": ik, "step": float(STEP_FIXED)}
    split = {k: round(v) for k, v in split.items()}
    return {"flops_per_env_step": int(sum(split.values())), "split": split,
            "pgs_iterations_per_substep": round(stats["pgs_iterations"] / max(1, stats["substeps"]), 2),
            "ik_iterations_per_step": round(stats["ik_iterations"] / steps, 2)}
