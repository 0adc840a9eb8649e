"""The per-sample parity classifier of the teacher-forced tests (test
infrastructure, no GPU needed): one fused env step of the HIP path against one
fp64 oracle step from the same state.

Moved out of tests/test_gpu_parity.py (round 5) so that the CPU suite can show
it has power: tests/test_judge_power.py feeds it "GPU" observations from an
oracle with a deliberate 1-2 % model error and requires 'beyond' samples, and
from the unmutated oracle in fp32 arithmetic and requires none.  Any change to
the bounds or the classes below must keep that test green.

Per-component tolerances of the fused env step (fp32 GPU vs fp64 oracle from
the same state).  Reach/Push/Slide measure ~1e-6 m / ~1e-4 m/s.  The tasks
with a free gripper (PickAndPlace, Stack, Flip) meet those bounds except on
samples at a finger-limit bifurcation: fingers resting exactly at their lower
limit (q = 0 after every reset) under a closing command sit at |q| ~ 1e-22,
and a joint-limit row exists only while the penetration is <= 0
(btMultiBodyJointLimitConstraint::createConstraintRows skips rows with
positive penetration), so on a substep where rounding leaves q > 0 the 170 N
finger motor drives the finger ~7 mm past the limit in one substep and the
reaction moves the hand.  Which substeps that happens on is decided by
rounding: in the fp64 oracle alone a 1e-9 relative change of one joint moves
the end effector by 8e-4 m; the same holds at the upper limit
(0.04 m) for an opening command.  Such samples are found with the oracle
alone (_ill_conditioned) and held to the loose bounds; every other sample to
the tight ones, or to the tight ones plus the oracle's own sensitivity to the
fp32 resolution of the state (_sensitivity).
"""
import numpy as np

import oracle as O
from helpers import OBJECT_ROWS, oracle_env_from

FREE_GRIPPER = ("pick_and_place", "stack", "flip")  # panda_tasks.py:26,43,111

_TIGHT = dict(ee_pos=2e-5, ee_vel=2e-3, width=2e-4, obj_pos=2e-5, obj_rot=1e-4, obj_vel=1e-4, obj_avel=2e-3)
_LOOSE = dict(ee_pos=3e-3, ee_vel=2e-1, width=1e-2, obj_pos=1e-3, obj_rot=5e-3, obj_vel=5e-2, obj_avel=2e-1)
_TIGHT2 = dict(_TIGHT, **{f"obj2_{k[4:]}": v for k, v in _TIGHT.items() if k.startswith("obj_")})
TOL = {"reach": _TIGHT, "push": _TIGHT, "slide": _TIGHT, "pick_and_place": _TIGHT, "stack": _TIGHT2, "flip": _TIGHT}
LOOSE = dict(_LOOSE, **{f"obj2_{k[4:]}": v for k, v in _LOOSE.items() if k.startswith("obj_")})

# Conditioning-scaled bound: a sample beyond the tight bounds is still within
# them once the oracle's own sensitivity to the fp32 resolution of the state is
# allowed for -- the largest move of its observation over four runs with
# NOISE_K fp32 ulps of noise on every state component per substep and one run
# whose state is rounded to fp32 after every substep (the GPU's state storage;
# oracle.set_state_noise).  NOISE_K = 2: the fp32 path rounds its arithmetic as
# well as its state, and the free runs' yardstick uses the same two ulps
# (tests/test_gpu_contacts.py ULP_NOISE, scripts/free_run_yardstick.py).
NOISE_K = 2.0

STEP_DT = 20 / 500  # one env step: 20 substeps of 1/500 s (core.py n_substeps, timestep)

# Done flags (core.py:285 terminated = is_success; push.py:89-91 d < 0.05 on
# the fp32 achieved goal against the fp64 goal; stack.py:118-131 6-D, 0.1;
# flip.py:80-91 1 - <q, g>^2, 0.2).  LIPSCHITZ bounds |d(a) - d(b)| / |a - b|.
THRESHOLD = {"reach": 0.05, "push": 0.05, "pick_and_place": 0.05, "slide": 0.05, "stack": 0.1, "flip": 0.2}
LIPSCHITZ = {"flip": 2.0}


def goal_distance(task, ag, dg):
    """The reference's distance of the fp32 achieved goal (cast to fp64) from
    the fp64 goal (utils.py:4-33)."""
    a = np.asarray(ag, np.float32).astype(np.float64)
    d = np.asarray(dg, np.float64)
    if task == "flip":
        return 1.0 - np.inner(a, d) ** 2
    return float(np.linalg.norm(a - d, axis=-1))


def terminated_rule(task, ag, dg):
    return bool(goal_distance(task, ag, dg) < THRESHOLD[task])


def done_flags_ok(task, te_gpu, ag_gpu, te_oracle, ag_oracle, dg):
    """(ok, mismatch): the GPU's terminated flag must be the reference's rule
    applied to the GPU's own achieved goal, bit for bit; it may differ from the
    oracle's flag only when the oracle's distance lies within the two achieved
    goals' difference of the threshold (|d_o - thr| <= L |ag_gpu - ag_o|): the
    two runs' goals straddle it."""
    if bool(te_gpu) != terminated_rule(task, ag_gpu, dg):
        return False, False
    if bool(te_gpu) == bool(te_oracle):
        return True, False
    d_o = goal_distance(task, ag_oracle, dg)
    gap = np.linalg.norm(np.asarray(ag_gpu, np.float64) - np.asarray(ag_oracle, np.float64))
    return bool(abs(d_o - THRESHOLD[task]) <= LIPSCHITZ.get(task, 1.0) * gap), True


def groups_for(task, robot_dim):
    """Observation slices: robot (panda.py:109-119), then the task's object
    blocks (position, rotation -- a quaternion for Flip --, velocity, angular
    velocity; Stack has two)."""
    g = {"ee_pos": [0, 1, 2], "ee_vel": [3, 4, 5]}
    if robot_dim == 7:
        g["width"] = [6]
    k = robot_dim
    nrot = 4 if task == "flip" else 3
    for b in range({"reach": 0, "stack": 2}.get(task, 1)):
        p = "obj_" if b == 0 else "obj2_"
        g[p + "pos"] = list(range(k, k + 3))
        g[p + "rot"] = list(range(k + 3, k + 3 + nrot))
        k += 3 + nrot
        g[p + "vel"] = list(range(k, k + 3))
        g[p + "avel"] = list(range(k + 3, k + 6))
        k += 6
    return g


def _fp32_probes():
    """State changes at fp32 resolution: each finger's position by one fp32
    ulp of its range (4e-9 m) and its velocity by 1e-7 relative, either sign;
    joint 2 by 1e-7 relative; each arm joint by one fp32 ulp of its angle,
    either sign (an arm joint pressed against its limit by a motor target
    beyond it flips its limit row like a finger does)."""
    probes = []
    for d in (7, 8):
        for sg in (1.0, -1.0):
            probes.append(lambda e, d=d, sg=sg: e.q.__setitem__(d, e.q[d] + sg * 4e-9))
            probes.append(lambda e, d=d, sg=sg: e.qd.__setitem__(d, e.qd[d] * (1 + sg * 1e-7) + sg * 1e-9))
    probes.append(lambda e: e.q.__setitem__(1, e.q[1] * (1 + 1e-7)))
    for d in range(7):
        for sg in (1.0, -1.0):
            probes.append(lambda e, d=d, sg=sg: e.q.__setitem__(
                d, float(np.nextafter(np.float32(e.q[d]), np.float32(sg * np.inf)))))
    return probes


FP32_PROBES = _fp32_probes()


def _within(err, o, groups, k, tol, before=None):
    """err <= tol[k], relative for the object velocities: an impact that spins
    a cube up to ~30 rad/s within one step -- or stops such a spin: `before`
    holds the groups' magnitudes at the start of the step -- is resolved by
    the 50-iteration PGS to ~1e-4 relative, so their bound is atol + 1e-3 x
    the larger magnitude; an object's rotation accrues that angular-velocity
    allowance over the step (+ STEP_DT x 1e-3 |omega|)."""
    before = before or {}
    bound = tol[k]
    if k.startswith("obj") and k.endswith(("_vel", "_avel")):
        bound += 1e-3 * max(np.abs(o[groups[k]]).max(), before.get(k, 0.0))
    if k.startswith("obj") and k.endswith("_rot"):
        ka = k[:-4] + "_avel"
        bound += STEP_DT * 1e-3 * max(np.linalg.norm(o[groups[ka]]), before.get(ka, 0.0))
    return err <= bound


def _before(snap, i, task):
    """The objects' velocity magnitudes (largest component) at the start of
    the step, keyed like groups_for (for _within)."""
    out = {}
    f = snap["f"][:, i]
    for b, r in enumerate(OBJECT_ROWS[:{"reach": 0, "stack": 2}.get(task, 1)]):
        p = "obj_" if b == 0 else "obj2_"
        out[p + "vel"] = float(np.abs(f[r + 7:r + 10]).max())
        out[p + "avel"] = float(np.abs(f[r + 10:r + 13]).max())
    return out


def _euler_matrix(e):
    """R = Rz(yaw) Ry(pitch) Rx(roll) of pybullet's getEulerFromQuaternion."""
    (cr, cp, cy), (sr, sp, sy) = np.cos(e), np.sin(e)
    return np.array([[cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr],
                     [sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr],
                     [-sp, cp * sr, cp * cr]])


def _obs_err(a, b, k, idx, task):
    """max |a - b| over a group.  Euler angles (every task but Flip, whose
    rotation is a quaternion) are compared as the angle between the two
    orientations: +-pi is one orientation, and at pitch +-pi/2 (a cube
    resting on a side face) roll and yaw are not separately determined."""
    a, b = np.asarray(a, np.float64)[idx], np.asarray(b, np.float64)[idx]
    if k.endswith("_rot") and task != "flip":
        fro = np.linalg.norm(_euler_matrix(a) - _euler_matrix(b))
        return float(2.0 * np.arcsin(min(fro / (2.0 * np.sqrt(2.0)), 1.0)))
    return float(np.abs(a - b).max())


def _ill_conditioned(cfg, snap, i, action, o_ref, groups, tol, task=""):
    """True when the oracle's own step from env i of `snap` is not determined
    to the tight bounds at fp32 resolution: one of FP32_PROBES (the state
    changed at fp32 resolution) or a per-substep finger-position noise of
    4e-9 m -- one fp32 ulp of the finger range, the resolution at which the
    fp32 path places a finger pressed against its limit (oracle.set_finger_noise),
    or a constant 4e-9 m per-substep offset of the fingers either way
    (oracle.set_finger_bias: a finger limit row that flips on one substep, e.g.
    the substep a blocked finger strikes the table), or (Stack) the box-box
    clip lines moved by 4e-9 m either way (oracle.set_clip_bias) -- moves its
    observation beyond them."""
    runs = ([(p, None, 0.0, 0.0) for p in FP32_PROBES] + [(None, seed, 0.0, 0.0) for seed in range(4)] +
            [(None, None, b, 0.0) for b in (4e-9, -4e-9)])
    if task == "stack":
        # Stack's box-box clip lines moved by 4e-9 m either way (round 6): a
        # vertex of the incident face on a clip line to within the fp32 path's
        # rounding (cubes side by side, a corner on the other's face edge) is
        # kept by one precision and cut by the other; the polygon then starts
        # at another vertex and the pair rows run in another order.  Replayed
        # on the 200-step sample stack_joints_64_44, the oracle
        # with the lines moved out by 4e-9 m reproduces the GPU's pair order,
        # its ground-impulse split and its 1.30e-3 rad yaw difference.
        runs += [(None, None, 0.0, cb) for cb in (4e-9, -4e-9)]
    try:
        for probe, seed, bias, clip in runs:
            e = oracle_env_from(cfg, snap, i)
            if probe is not None:
                probe(e)
            O.set_finger_noise(4e-9 if seed is not None else 0.0, 0 if seed is None else seed)
            O.set_finger_bias(bias)
            O.set_clip_bias(clip)
            o, *_ = O.step(cfg, e, action)
            if any(not _within(_obs_err(o, o_ref, k, idx, task), o_ref, groups, k, tol, _before(snap, i, task))
                   for k, idx in groups.items()):
                return True
    finally:
        O.set_finger_noise(0.0)
        O.set_finger_bias(0.0)
        O.set_clip_bias(0.0)
    return False


def _sensitivity(cfg, snap, i, action, o_ref, groups, task):
    sens = {k: 0.0 for k in groups}
    try:
        for ulps, seed in [(NOISE_K, 1), (NOISE_K, 2), (NOISE_K, 3), (NOISE_K, 4), (-1.0, 0)]:
            O.set_state_noise(ulps, seed)
            o, *_ = O.step(cfg, oracle_env_from(cfg, snap, i), action)
            for k, idx in groups.items():
                sens[k] = max(sens[k], _obs_err(o, o_ref, k, idx, task))
    finally:
        O.set_state_noise(0.0)
    return sens


def judge(cfg, snap, i, action, o, og, groups, task):
    """Classifies one teacher-forced sample (GPU observation og vs oracle o):
    'tight' within the tight bounds; 'conditioned' within them once the
    oracle's sensitivity (_sensitivity) is added; 'bif' at a branch the oracle itself
    cannot resolve at fp32 resolution (its answer leaves the tight bounds
    under the state noise of _sensitivity, or under _ill_conditioned's probes:
    held to the loose bounds); 'beyond' otherwise.  Returns (class, per-group
    errors)."""
    tol = TOL[task]
    bf = _before(snap, i, task)
    errs = {k: _obs_err(og, o, k, idx, task) for k, idx in groups.items()}
    bad = [k for k in groups if not _within(errs[k], o, groups, k, tol, bf)]
    if not bad:
        return "tight", errs
    sens = _sensitivity(cfg, snap, i, action, o, groups, task)
    if all(_within(errs[k] - sens[k], o, groups, k, tol, bf) for k in bad):
        return "conditioned", errs
    # the oracle's own answer leaves the tight bounds under fp32-resolution
    # state noise (a limit row or contact that flickers on some substeps and
    # not on others), or under one of the probes
    if any(not _within(sens[k], o, groups, k, tol, bf) for k in groups) or \
            _ill_conditioned(cfg, snap, i, action, o, groups, tol, task):
        return "bif", errs
    return "beyond", errs


# Rates the teacher-forced tests may not exceed (ADVICE
# r04): a blocked gripper (Reach/Push/Slide) measured at most 14 conditioned +
# 3 ill-conditioned of 12 800 in 200-step teacher forcing (profiles/r04p,
# r04y) and none of 640 in the 10-step tests; the free-gripper tasks reach
# finger-limit branches on ~4 % of their samples.
NOT_TIGHT_CAP = {"blocked": 0.005, "free": 0.08}


def not_tight_cap(task):
    return NOT_TIGHT_CAP["free" if task in FREE_GRIPPER else "blocked"]
