"""GPU parity of the warm-started contact solver and of the long-horizon
behaviour of the fused step (warm start / persistent contacts,
reset semantics, 200-step ee-control free runs, full-size and 1000-step
rollouts).

* The contact cache (Bullet's persistent manifolds + warm starting, DESIGN.md
  §5) lives in the SoA state rows PS_F_WG0..PS_F_WPN.  After each
  teacher-forced GPU step the cache the kernel wrote is compared with the
  cache the fp64 oracle wrote from the same state: slot ids exactly, normal
  impulses to a tolerance.
* set_base_pose / reset place objects at rest (resetBasePositionAndOrientation
  zeroes the base velocity) and empty the cache.
* Free runs: the fp32 GPU path and the fp64 oracle from the same initial
  states and actions.  Before the first contact or joint-limit event of an
  env the dynamics are smooth and the two must agree to 1e-5 m (event-onset
  tests); after it they are chaotic, so the long-horizon bound is an absolute
  floor plus the oracle's own conditioning at fp32 resolution (ULP_NOISE).
"""
import copy
import os

import numpy as np
import pytest
import torch

from helpers import WG_ROWS, WPN_ROW, WPPT_ROW, WP_ROW, WR_ROW, oracle_config_for, oracle_env_from, snapshot, \
    unpack_ids

import oracle as O

pytestmark = pytest.mark.gpu

OBJECT_TASKS = ["push", "pick_and_place", "slide", "stack", "flip"]


def make_env(task, control, n, reward="sparse", autoreset=False):
    from pandasim.envs import PandaVecEnv

    env = PandaVecEnv(task, reward, control, n, "cuda")
    env.autoreset = autoreset
    return env


def gpu_cache(f, i):
    """The cache rows of env i (snapshot 'f' columns) as slot lists."""
    out = {}
    for b, r in enumerate(WG_ROWS):
        out[f"ground{b}"] = list(zip(unpack_ids(f[r + 4, i]), f[r:r + 4, i]))
    out["robot"] = list(zip(unpack_ids(f[WR_ROW + 4, i]), f[WR_ROW:WR_ROW + 4, i]))
    n = int(f[WPN_ROW, i])
    out["pair"] = [(tuple(f[WPPT_ROW + 3 * s:WPPT_ROW + 3 * s + 3, i]), f[WP_ROW + s, i]) for s in range(n)]
    return out


def oracle_cache(env):
    k = env.cache
    out = {}
    for b in range(2):
        out[f"ground{b}"] = [(k.ground_id[b][s], k.ground_lam[b][s]) for s in range(4)]
    out["robot"] = [(k.robot_id[s], k.robot_lam[s]) for s in range(4)]
    out["pair"] = [(tuple(k.pair_pt[s][j] for j in range(3)), k.pair_lam[s]) for s in range(k.pair_n)]
    return out


def _push_policy(env, body):
    B = env.num_envs

    def policy(s):
        ee = env.sim.get_link_position("panda", 11).cpu().numpy()
        obj = env.sim.get_base_position(body).cpu().numpy()
        tgt = obj + np.array([0.0, 0.0, 0.06 if s < 6 else 0.0])
        if s >= 6:
            tgt[:, 0] += 0.05
        a = np.zeros((B, env.action_dim), np.float32)
        a[:, :3] = np.clip(10.0 * (tgt - ee), -1, 1)
        if env.action_dim == 4:
            a[:, 3] = -1.0 if s >= 8 else 1.0
        return a

    return policy


def _pair_point_sensitivity(cfg, snap, i, action, po, c):
    """Largest move of the oracle's c-th cached box-box point when the step is
    re-run with one fp32 ulp of state noise per substep (four seeds) and with
    the state rounded to fp32 every substep."""
    spread = 0.0
    try:
        for ulps, seed in [(1.0, 1), (1.0, 2), (1.0, 3), (1.0, 4), (-1.0, 0)]:
            O.set_state_noise(ulps, seed)
            e = oracle_env_from(cfg, snap, i)
            O.step(cfg, e, action)
            k = e.cache
            if c < k.pair_n:
                spread = max(spread, float(np.abs(np.subtract([k.pair_pt[c][j] for j in range(3)], po)).max()))
            else:
                spread = max(spread, 1.0)  # the point itself comes and goes
    finally:
        O.set_state_noise(0.0)
    return spread


@pytest.mark.parametrize("task", OBJECT_TASKS)
def test_contact_cache_parity(task):
    """Teacher-forced steps of a scripted push into the object: the cache
    (slot ids and normal impulses) the GPU writes equals the oracle's.  A
    box-box point (Stack) more than 1e-4 m off must be within NOISE_K x the
    oracle's own spread of it at the state's fp32 resolution (a pushed stack
    can sit at a near-tie between clipping candidates), on at most 1 % of the
    env-steps."""
    B, steps = 64, 14
    env = make_env(task, "ee", B)
    env.reset(seed=44)
    cfg = oracle_config_for(env.sim.cfg)
    policy = _push_policy(env, "object1" if task == "stack" else "object")
    from parity_judge import NOISE_K

    ids_equal = total = hits = n_cond = 0
    lam_err = []
    for s in range(steps):
        snap = snapshot(env.sim)
        a = policy(s)
        env.step(torch.from_numpy(a).cuda())
        after = snapshot(env.sim)
        for i in range(0, B, 2):
            e = oracle_env_from(cfg, snap, i)
            O.step(cfg, e, a[i])
            g, o = gpu_cache(after["f"], i), oracle_cache(e)
            total += 1
            same = all([sid for sid, _ in g[k]] == [sid for sid, _ in o[k]] for k in ("ground0", "ground1", "robot"))
            same = same and len(g["pair"]) == len(o["pair"])
            if not same:
                continue
            ids_equal += 1
            for k in ("ground0", "ground1", "robot"):
                for (sid, lg), (_, lo) in zip(g[k], o[k]):
                    if sid:
                        hits += 1
                        lam_err.append(abs(lg - lo) / max(abs(lo), 1e-3))
            for c, ((pg, lg), (po, lo)) in enumerate(zip(g["pair"], o["pair"])):
                d = float(np.abs(np.subtract(pg, po)).max())
                if d > 1e-4:
                    # the oracle's own spread of this point at the state's
                    # fp32 resolution (parity_judge.judge's perturbations)
                    sens = _pair_point_sensitivity(cfg, snap, i, a[i], po, c)
                    print(f"  {task} step {s} env {i} pair point {c}: |GPU - oracle| {d:.1e} m, "
                          f"oracle spread {sens:.1e} m")
                    assert d <= 1e-4 + NOISE_K * sens, (s, i, c, d, sens)
                    n_cond += 1
                lam_err.append(abs(lg - lo) / max(abs(lo), 1e-3))
    lam_err = np.array(lam_err)
    print(task, f"cache ids equal in {ids_equal}/{total} env-steps; {hits} cached contacts; "
                f"normal impulse rel err median {np.median(lam_err):.1e} p99 {np.quantile(lam_err, 0.99):.1e}; "
                f"pair points beyond 1e-4 m within the oracle's spread: {n_cond}")
    assert n_cond <= 0.01 * total
    assert hits > total  # warm starting is exercised (on average > 1 cached contact per env-step)
    # the contact sets of the two precisions can differ at the margins on rare samples
    assert ids_equal >= 0.95 * total
    assert np.median(lam_err) < 1e-3 and np.quantile(lam_err, 0.95) < 5e-2


@pytest.mark.parametrize("task", ["push", "stack"])
def test_reset_places_objects_at_rest(task):
    """resetBasePositionAndOrientation zeroes the base velocity: after a push
    sets the object moving, both reset paths (ps_reset and the in-kernel
    autoreset) start the episode with zero object velocity in the state and in
    the observation, and with an empty contact cache."""
    B = 64
    env = make_env(task, "ee", B, autoreset=True)
    env.reset(seed=9)
    policy = _push_policy(env, "object1" if task == "stack" else "object")
    for s in range(10):
        env.step(torch.from_numpy(policy(s)).cuda())
    vel = env.sim.get_base_velocity("object1" if task == "stack" else "object")
    assert (vel.norm(dim=1) > 1e-3).float().mean() > 0.3  # objects are moving
    # explicit reset of every other env
    mask = torch.zeros(B, dtype=torch.uint8, device="cuda")
    mask[::2] = 1
    obs, _ = env.reset(mask=mask)
    f = env.sim.f[:, :B]
    nobj = 2 if task == "stack" else 1
    for b, row in enumerate([63, 76][:nobj]):
        assert torch.all(f[row + 7:row + 13, ::2] == 0)
    assert torch.all(f[89:121, ::2] == 0)
    o = obs["observation"][::2]
    robot_dim = 6 if task == "push" else 7
    for b in range(nobj):
        base = robot_dim + b * 12
        assert torch.all(o[:, base + 6:base + 12] == 0)
    # autoreset: run to the TimeLimit; the envs reset in-kernel start at rest
    for s in range(env.max_episode_steps):
        obs, r, te, tr, info = env.step(torch.from_numpy(policy(10)).cuda())
        done = (te | tr)
        if done.any():
            o = obs["observation"][done]
            for b in range(nobj):
                base = robot_dim + b * 12
                assert torch.all(o[:, base + 6:base + 12] == 0)
            assert torch.all(env.sim.f[89:121, :B][:, done] == 0)


# Yardstick of the free runs: the fp64 oracle perturbed at the fp32
# resolution of the state, ULP_NOISE fp32 ulps per state component per
# substep (oracle.set_state_noise).  A second oracle run with this noise shows
# how far two runs that differ only by fp32 rounding drift apart.  Two ulps:
# the fp32 path rounds its arithmetic as well as its state, which the
# per-step bounds allow for with the same factor (parity_judge.NOISE_K);
# scripts/free_run_yardstick.py measures the ensembles on the CPU
# (profiles/r04_free_run_yardstick.jsonl: with one ulp Push ee 87-92 %, with
# two 83-84 %, with the state rounded to fp32 every substep 91 %).
ULP_NOISE = 2.0
# After the first event the runs are chaotic, and which env leaves the 1e-3 band
# first is a coin flip between two runs that differ by rounding (one env of 64
# is 1.6 points of the fraction): the yardstick is an ensemble of ULP_RUNS
# perturbed oracle runs (independent noise), and the GPU's fraction is held to
# the ensemble's lowest less 2 points.
ULP_RUNS = 3
# Free-run floors (absolute, next to the relative yardstick): fraction of
# env-steps whose ee/object positions are within 1e-3 m of the oracle, 64 envs
# x 200 steps, seed 2024.  Each floor is the lowest of the CPU yardstick's
# three oracle runs perturbed by ULP_NOISE fp32 ulps per substep from the same
# initial states (scripts/free_run_yardstick.py,
# profiles/r04_free_run_yardstick.jsonl: Push ee 83.3 %, PickAndPlace ee
# 61.9 %, Reach joints 94.8 %, Push joints 93.2 %) less one point,
# so it is set by how far two runs that differ only by fp32 rounding part, not
# by a GPU measurement (round 5: 85.2, 75.9, 97.1, 92.7 %,
# profiles/r05a_pytest_gpu.log).  Every env that leaves the 1e-3 band does so
# after a contact event; the hull-derived gripper boxes of round 4 touch the
# table and the object more often than round 3's sphere pads did, which is the
# accepted cause of the lower fractions.
FREE_RUN_FLOOR = {("push", "ee"): 0.82, ("pick_and_place", "ee"): 0.61,
                  ("reach", "joints"): 0.94, ("push", "joints"): 0.92}
# Regression guard next to the yardstick floor: the GPU's own
# fraction on the round-5 final library (profiles/r05at_pytest_gpu.log) less
# 3 points.  The yardstick floor
# says how far rounding alone may take the runs apart; this one fails a build
# whose agreement drops well below what the path measured, e.g. PickAndPlace
# falling 14 points to its floor.
FREE_RUN_MEASURED = {("push", "ee"): 0.8788, ("pick_and_place", "ee"): 0.7516,
                     ("reach", "joints"): 0.9642, ("push", "joints"): 0.9523}
FREE_RUN_REGRESSION = 0.03
_RUNS = {}


def _obs_index(task):
    nobj = {"reach": 0, "stack": 2}.get(task, 1)
    robot_dim = 6 if task in ("reach", "push", "slide") else 7  # + finger width (panda.py:109-119)
    per = 13 if task == "flip" else 12
    return nobj, [0, 1, 2] + [robot_dim + per * b + k for b in range(nobj) for k in range(3)]


def _free_run(task, control, B=64, T=200, seed=2024, open_gripper=False):
    """GPU vs oracle free run from the same initial states and actions.
    Returns per env-step arrays [T, B]: the GPU's error against the oracle
    (max over ee and object positions), the error of an oracle run perturbed
    by ULP_NOISE, whether the reference oracle's discrete state (contact
    features, joint-limit rows: po_env.event_sig) has changed at any substep
    up to and including that step, and whether the GPU's contact-cache ids
    equal the oracle's after that step."""
    key = (task, control, B, T, seed, open_gripper)
    if key in _RUNS:
        return _RUNS[key]
    env = make_env(task, control, B)
    env.reset(seed=seed)
    if open_gripper:
        # fingers half open (0.02 m each, off both limits) and gripper action 0
        # (width target = current width): no finger-limit branch is reachable
        env.sim.f[7:9, :B] = 0.02
    cfg = oracle_config_for(env.sim.cfg)
    snap = snapshot(env.sim)
    ref = [oracle_env_from(cfg, snap, i) for i in range(B)]
    pert = [[oracle_env_from(cfg, snap, i) for i in range(B)] for _ in range(ULP_RUNS)]
    rng = np.random.default_rng(seed)
    nobj, idx = _obs_index(task)
    err_gpu = np.zeros((T, B))
    err_ulp = np.zeros((ULP_RUNS, T, B))
    event = np.zeros((T, B), bool)
    fevent = np.zeros((T, B), bool)
    kinds = np.zeros((T, B), np.int8)
    ids_equal = np.zeros((T, B), bool)
    for s in range(T):
        a = rng.uniform(-1, 1, size=(B, env.action_dim)).astype(np.float32)
        if open_gripper:
            a[:, -1] = 0.0
        obs, *_ = env.step(torch.from_numpy(a).cuda())
        og = obs["observation"].cpu().numpy()
        f = env.sim.f[:, :B].double().cpu().numpy()
        for i in range(B):
            o, *_ = O.step(cfg, ref[i], a[i])
            err_gpu[s, i] = np.abs(og[i, idx] - o[idx]).max()
            event[s, i] = ref[i].event_changes > 0
            fevent[s, i] = ref[i].finger_changes > 0
            kinds[s, i] = ref[i].event_kinds
            gc, oc = gpu_cache(f, i), oracle_cache(ref[i])
            ids_equal[s, i] = all([k for k, _ in gc[g]] == [k for k, _ in oc[g]] for g in ("ground0", "ground1", "robot")) \
                and len(gc["pair"]) == len(oc["pair"])
            for k in range(ULP_RUNS):
                O.set_state_noise(ULP_NOISE, seed=((s * B + i) * 2 + 1) + k * 1000003)
                op, *_ = O.step(cfg, pert[k][i], a[i])
                O.set_state_noise(0.0)
                err_ulp[k, s, i] = np.abs(op[idx] - o[idx]).max()
    _RUNS[key] = (err_gpu, err_ulp, event, fevent, ids_equal)
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed(f"gpurun_out/free_run_{task}_{control}{'_open' if open_gripper else ''}.npz", err_gpu=err_gpu,
                        err_ulp=err_ulp, event=event, fevent=fevent, kinds=kinds, ids_equal=ids_equal)
    return _RUNS[key]


def _report(task, control, err_gpu, err_ulp, event):
    """err_ulp: [ULP_RUNS, T, B]; returns the GPU's fraction within 1e-3 and
    the lowest fraction of the perturbed oracle runs."""
    pre = ~event
    frac = float((err_gpu <= 1e-3).mean())
    fracs = [float((e <= 1e-3).mean()) for e in err_ulp]
    first = np.where(event.any(0), event.argmax(0), event.shape[0])
    print(f"{task} {control}: GPU within 1e-3 of the oracle in {frac * 100:.2f} % of env-steps (worst "
          f"{err_gpu.max():.1e} m); oracle + {ULP_NOISE:g} fp32 ulp/substep noise, {len(fracs)} runs: "
          f"{', '.join(f'{f * 100:.2f}' for f in fracs)} % (worst {err_ulp.max():.1e}); pre-event env-steps "
          f"{int(pre.sum())} / {pre.size} (first event: median step {int(np.median(first))}), pre-event max error "
          f"GPU {err_gpu[pre].max() if pre.any() else 0:.2e} m, oracle+ulp {err_ulp[0][pre].max() if pre.any() else 0:.2e} m")
    return frac, min(fracs)


# Pre-event bound: until the first event the only difference between the
# fp32 GPU run and the fp64 oracle is rounding, which the integrating ee
# (targets are relative to the current position) accumulates as a random
# walk over the event-free span.  The GPU must stay within an absolute bound
# and within PRE_EVENT_ULP_RATIO x the deviation of an oracle run perturbed by
# ULP_NOISE fp32 ulps per state component per substep.  Measured
# (profiles/r03*_pytest_gpu.log, one ulp of noise then): 200-step runs Push
# 7.2e-6 m (oracle+ulp 7.1e-6), PickAndPlace with the gripper held 5.5e-6
# (8.0e-6) -- the 1e-5 m of the north star; the bench config, whose
# event-free spans run up to a 50-step episode, 2.0e-5 m (oracle+ulp 3.3e-5).
PRE_EVENT_ULP_RATIO = 1.0


def _check_pre_event(name, err_gpu, err_ulp, pre, abs_tol, ids_equal=None):
    assert pre.sum() >= 0.05 * pre.size, f"{name}: too few pre-event env-steps for the check to mean anything"
    g, u = float(err_gpu[pre].max()), float(err_ulp[pre].max())
    print(f"{name}: pre-event env-steps {int(pre.sum())}/{pre.size}, max error GPU {g:.2e} m, oracle+ulp {u:.2e} m")
    assert g <= abs_tol
    assert g <= PRE_EVENT_ULP_RATIO * u
    if ids_equal is not None:
        assert ids_equal[pre].all()


def test_event_onset_parity_push_ee():
    """Until the oracle's discrete state first changes (a contact appears or
    breaks, an arm joint-limit row switches: po_env.event_sig), the dynamics
    are smooth and the fp32 GPU path tracks the fp64 oracle to rounding:
    ee and object positions on every pre-event env-step of a 200-step free
    run (ee control, 64 envs), with the GPU's contact-cache ids equal to the
    oracle's (core.py:280-289, panda.py:72-92).  Push blocks the gripper: its
    fingers rest on their stop with the motor target at the stop, so their
    limit row's on/off flicker (decided at the 1e-22 level) is not an event
    here (the PickAndPlace test below excludes it by construction)."""
    err_gpu, err_ulp, event, fevent, ids_equal = _free_run("push", "ee")
    _report("push", "ee", err_gpu, err_ulp, event)
    _check_pre_event("push ee", err_gpu, err_ulp[0], ~event, 1e-5, ids_equal)


def test_event_onset_parity_pick_and_place_ee():
    """PickAndPlace (free gripper) with the fingers held half open (gripper
    action 0, both fingers 0.02 m from their limits), so the finger-limit
    branches that make PickAndPlace chaotic at fp32 resolution
    cannot occur; events are then contacts and any joint-limit row.  With a
    random gripper action the first finger-limit change falls on step 0 for
    nearly every env (reported, not asserted)."""
    err_gpu, err_ulp, event, fevent, ids_equal = _free_run("pick_and_place", "ee", open_gripper=True)
    _report("pick_and_place", "ee (gripper open, held)", err_gpu, err_ulp, event | fevent)
    _check_pre_event("pick_and_place ee (gripper held open)", err_gpu, err_ulp[0], ~(event | fevent), 1e-5, ids_equal)
    e2 = _free_run("pick_and_place", "ee")
    _report("pick_and_place", "ee (random gripper; finger-limit changes are events)", e2[0], e2[1], e2[2] | e2[3])


@pytest.mark.parametrize("task,control", [("push", "ee"), ("pick_and_place", "ee"), ("reach", "joints"),
                                          ("push", "joints")])
def test_free_running_200_steps(task, control):
    """The north star's horizon: 200 free-running steps, 64 envs.  After the
    first contact or joint-limit event the trajectories are chaotic (a finger
    at its limit flips branch at the 1e-22 level), so the
    fraction of env-steps within 1e-3 m of the oracle is held (a) to an
    absolute floor per task and (b) against the oracle's own conditioning at
    fp32 resolution: ULP_RUNS oracle runs perturbed by ULP_NOISE every
    substep, whose lowest fraction the GPU must reach less 2 points."""
    err_gpu, err_ulp, event, _, _ = _free_run(task, control)
    frac, frac_ulp = _report(task, control, err_gpu, err_ulp, event)
    assert frac >= FREE_RUN_FLOOR[(task, control)]
    assert frac >= FREE_RUN_MEASURED[(task, control)] - FREE_RUN_REGRESSION
    assert frac >= frac_ulp - 0.02


# Teacher forcing over the north star's horizon: every step of a 200-step run
# (the GPU's own trajectory, random actions) is replayed by the oracle from the
# GPU's state before it, so a systematic difference on any contact
# configuration the run reaches shows as a step error, where a free run only
# shows chaos.  Bounds are test_gpu_parity's per-step ones.
# The 200-step samples beyond the tight bounds on the product library, each
# replayed from its dump (scripts/tf_sample.py, scripts/substep_compare.py,
# profiles/r06c_substep_compare.log).  Round 5's 0.1 % allowance
# is gone: any other beyond sample fails.  (Round 6's other one, Stack joints
# step 64 env 44, is a box-box clip-line tie the classifier now recognises:
# parity_judge._ill_conditioned's clip-bias probe.)
TF200_EXEMPT = {
    ("pick_and_place", "ee-random-gripper", 87, 15):
        "the cube has left the table and slides (0.29 m/s) and spins on its side on the plane; its four "
        "coplanar ground contacts are statically indeterminate, the GPU's and the oracle's normal impulses "
        "among them part by 0.3-3 % from the first substep, and the spin error grows steadily to 2.5e-3 rad/s "
        "(1.3 % of 0.19 rad/s; bound 2.26e-3) with positions within 6e-7 m; no oracle probe at fp32 "
        "resolution (state noise, fp32 solver, PGS exit +-1..8 iterations) moves it beyond 1.4e-4 rad/s",
}
LONG_TF_CASES = [("reach", "joints"), ("push", "ee"), ("push", "joints"), ("pick_and_place", "ee"), ("slide", "ee"),
                 ("stack", "ee"), ("flip", "ee"),
                 # round 5: joint control of the other scenes, and a free gripper
                 # under random gripper actions (finger-limit branches included)
                 ("slide", "joints"), ("stack", "joints"), ("pick_and_place", "ee-random-gripper")]
FREE_GRIPPER_TASKS = ("pick_and_place", "stack", "flip")


@pytest.mark.parametrize("task,control", LONG_TF_CASES)
def test_teacher_forced_200_steps(task, control):
    """64 envs x 200 steps, seed 2024 (the free runs' start): each GPU step vs
    one oracle step from the same state.  Samples beyond the tight bounds are
    dumped (state before and after, action, GPU observation) to
    gpurun_out/tf200/ and listed; none may exceed them (parity_judge.judge:
    beyond the tight bounds even after the oracle's own sensitivity to the
    state's fp32 resolution is allowed for, and not at a branch the oracle
    cannot resolve at that resolution) but the replayed ones of TF200_EXEMPT,
    and no non-ill-conditioned one the loose ones.
    The free-gripper runs (PickAndPlace, Stack, Flip) hold the gripper half
    open (action 0), as in the event-onset test, so the finger-limit
    bifurcations stay out; the "ee-random-gripper" case keeps
    the random gripper action, so those branches are in, held to the 10-step
    test's free-gripper caps (8 % ill-conditioned, 2 % conditioned)."""
    from parity_judge import LOOSE, groups_for as _groups, judge as _judge

    B, T = 64, 200
    random_gripper = control == "ee-random-gripper"
    control = "ee" if random_gripper else control
    env = make_env(task, control, B)
    env.reset(seed=2024)
    free = task in FREE_GRIPPER_TASKS and not random_gripper
    if free:
        env.sim.f[7:9, :B] = 0.02
    cfg = oracle_config_for(env.sim.cfg)
    groups = _groups(task, 7 if task in FREE_GRIPPER_TASKS else 6)
    rng = np.random.default_rng(2024)
    out = os.path.join("gpurun_out", "tf200")
    os.makedirs(out, exist_ok=True)
    worst = {k: 0.0 for k in groups}
    counts = {"tight": 0, "conditioned": 0, "bif": 0, "beyond": 0}
    beyond = []
    for s in range(T):
        snap = snapshot(env.sim)
        a = rng.uniform(-1, 1, size=(B, env.action_dim)).astype(np.float32)
        if free:
            a[:, -1] = 0.0
        obs, *_ = env.step(torch.from_numpy(a).cuda())
        og = obs["observation"].cpu().numpy()
        after = None
        for i in range(B):
            e = oracle_env_from(cfg, snap, i)
            o, *_ = O.step(cfg, e, a[i])
            cls, errs = _judge(cfg, snap, i, a[i], o, og[i], groups, task)
            counts[cls] += 1
            for k, err in errs.items():
                assert err <= LOOSE[k] or cls == "bif", (k, err, s, i, cls)
                if cls != "bif":
                    worst[k] = max(worst[k], err)
            if cls == "beyond":
                beyond.append((s, i, {k: f"{v:.1e}" for k, v in errs.items()}))
                if after is None:
                    after = env.sim.f[:, :B].double().cpu().numpy()
                if len(beyond) <= 40:
                    np.savez(os.path.join(out, f"{task}_{control}_{s}_{i}.npz"), f=snap["f"][:, i],
                             goal=snap["goal"][:, i], rng=snap["rng"][:, i], elapsed=snap["elapsed"][i], action=a[i],
                             gpu_obs=og[i], gpu_f_after=after[:, i], oracle_obs=o)
    print(task, control + (" (random gripper)" if random_gripper else ""), counts, "worst (not ill-conditioned)",
          {k: f"{v:.2e}" for k, v in worst.items()}, "beyond:", beyond[:20])
    # no allowance: every beyond sample must be a listed,
    # replayed one (TF200_EXEMPT)
    name = control + ("-random-gripper" if random_gripper else "")
    unexplained = [b for b in beyond if (task, name, b[0], b[1]) not in TF200_EXEMPT]
    assert not unexplained, unexplained
    if random_gripper:
        assert counts["bif"] <= 0.08 * B * T and counts["conditioned"] <= 0.02 * B * T
    else:
        # measured at most 14 conditioned + 3 ill-conditioned of 12 800 (Push ee,
        # profiles/r04p_pytest_gpu.log); ADVICE r04: cap them near that rate
        assert counts["conditioned"] + counts["bif"] <= 0.0025 * B * T


def test_event_onset_parity_at_bench_config():
    """The bench workload (PandaPush-v3, 65 536 envs, ee, autoreset, seeds
    12345 + i, the bench's action stream) for 100 steps, 64 sampled envs
    stepped alongside by the oracle (autoreset too): on every env-step before
    the env's first event of an episode (reset starts a new event-free span)
    ee and object positions agree to rounding (_check_pre_event: 5e-5 m, the
    spans are up to an episode long, and an oracle perturbed by ULP_NOISE
    fp32 ulps per substep)."""
    B, T = 65536, 100
    env = make_env("push", "ee", B, autoreset=True)
    env.reset(seed=(12345 + np.arange(B)).astype(np.uint64))
    cfg = oracle_config_for(env.sim.cfg)
    sample = np.linspace(0, B - 1, 64).astype(int)
    snap = snapshot(env.sim)
    ref = [oracle_env_from(cfg, snap, int(i)) for i in sample]
    pert = [oracle_env_from(cfg, snap, int(i)) for i in sample]
    g = torch.Generator(device="cuda")
    g.manual_seed(0xC0FFEE)
    actions = torch.rand(T, B, 3, device="cuda", generator=g) * 2 - 1
    _, idx = _obs_index("push")
    err_gpu = np.zeros((T, len(ref)))
    err_ulp = np.zeros((T, len(ref)))
    pre = np.zeros((T, len(ref)), bool)
    resets = 0
    for s in range(T):
        obs, r, te, tr, info = env.step(actions[s])
        og = obs["observation"][torch.from_numpy(sample).cuda()].cpu().numpy()
        a = actions[s][torch.from_numpy(sample).cuda()].cpu().numpy()
        for j, e in enumerate(ref):
            o, ag, dg, rr, t_e, t_r = O.step(cfg, e, a[j], autoreset=True)
            O.set_state_noise(ULP_NOISE, seed=(s * len(ref) + j) * 2 + 1)
            op, *_ = O.step(cfg, pert[j], a[j], autoreset=True)
            O.set_state_noise(0.0)
            pre[s, j] = e.event_changes == 0
            err_gpu[s, j] = np.abs(og[j, idx] - o[idx]).max()
            err_ulp[s, j] = np.abs(op[idx] - o[idx]).max()
            if t_e or t_r:
                # the reset starts a new event-free span (both runs reset to
                # the same state: the reset draws are bit-exact)
                e.event_changes, e.event_sig = 0, 0
                pert[j] = copy.deepcopy(e)
                resets += 1
    print(f"bench config: {resets} resets")
    assert resets >= len(ref)
    _check_pre_event("bench config (PandaPush-v3 x65536, 64 sampled envs, 100 steps)", err_gpu, err_ulp, pre, 5e-5)


def test_reach_at_config_size():
    """BASELINE config C2 (PandaReach, 4096 envs): finite bounded observations,
    exact TimeLimit/autoreset bookkeeping over 60 steps, then 32 sampled envs
    teacher-forced against the oracle."""
    from parity_judge import LOOSE, groups_for as _groups, judge as _judge

    B = 4096
    for control in ("ee", "joints"):
        env = make_env("reach", control, B, autoreset=True)
        env.reset(seed=77)
        g = torch.Generator(device="cuda")
        g.manual_seed(3)
        for s in range(60):
            obs, r, te, tr, info = env.step(torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1)
            assert torch.isfinite(obs["observation"]).all()
            assert (obs["observation"].abs() < 10).all()
        el = env.sim.elapsed[:B]
        assert int(el.max()) < env.max_episode_steps and int(el.min()) >= 0
        cfg = oracle_config_for(env.sim.cfg)
        snap = snapshot(env.sim)
        a = (torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1)
        obs, *_ = env.step(a)
        og, a = obs["observation"].cpu().numpy(), a.cpu().numpy()
        counts = {"tight": 0, "conditioned": 0, "bif": 0, "beyond": 0}
        for i in np.linspace(0, B - 1, 32).astype(int):
            o, ag, dg, rr, t_e, t_r = O.step(cfg, oracle_env_from(cfg, snap, i), a[i], autoreset=True)
            if t_e or t_r:  # reset in this step: the new episode's first observation
                assert np.abs(og[i, :3] - o[:3]).max() < 2e-5, (control, i)
                assert np.abs(og[i, 3:6] - o[3:6]).max() < 2e-3, (control, i)
                continue
            # the tight bounds, or the oracle's own conditioning (a fingertip on
            # the table, a joint at its limit: parity_judge.judge)
            cls, errs = _judge(cfg, snap, i, a[i], o, og[i], _groups("reach", 6), "reach")
            counts[cls] += 1
            assert cls != "beyond", (control, i, errs)
            assert cls != "bif" or all(v <= LOOSE[k] for k, v in errs.items()), (control, i, errs)
        print("reach", control, counts)


@pytest.mark.parametrize("task", ["push", "pick_and_place"])
def test_push_and_pick_and_place_at_config_size(task):
    """BASELINE configs C3 (PandaPush-v3) and C4 (PandaPickAndPlace-v3) at
    their own size, 8 192 envs, on the kernel the library picks for it
    (lanes_per_env = 0 resolves to the 8-lane group kernel): 60 autoreset
    steps with finite, bounded observations and exact TimeLimit bookkeeping,
    then 3 steps of 64 evenly spaced envs teacher-forced against the oracle
    at the tight bounds of test_env_step_parity_teacher_forced (test_gpu_parity
    ._judge): samples the oracle itself cannot resolve at fp32 resolution
    (finger- and joint-limit branches) are held to the loose bounds instead,
    at most 8 % of them."""
    from parity_judge import FREE_GRIPPER, LOOSE, done_flags_ok, groups_for as _groups, judge as _judge

    from pandasim.envs import PandaVecEnv

    B = 8192
    env = PandaVecEnv(task, "sparse", "ee", B, "cuda", lanes_per_env=0)
    assert env.lanes_per_env == 8
    env.autoreset = True
    env.reset(seed=2024)
    g = torch.Generator(device="cuda")
    g.manual_seed(17)
    steps_in_episode = torch.zeros(B, dtype=torch.int64, device="cuda")
    for s in range(60):
        obs, r, te, tr, info = env.step(torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1)
        steps_in_episode += 1
        assert torch.equal(tr, steps_in_episode == env.max_episode_steps)
        steps_in_episode[te | tr] = 0
        assert torch.isfinite(obs["observation"]).all()
        # a gripper strike can spin a cube to ~100 rad/s (the fp64 oracle does
        # too: 116 rad/s in 8 192 PickAndPlace envs); a blow-up is far beyond
        assert (obs["observation"].abs() < 1000).all()
    assert torch.equal(env.sim.elapsed[:B].long(), steps_in_episode)
    env.autoreset = False
    cfg = oracle_config_for(env.sim.cfg)
    groups = _groups(task, 7 if task in FREE_GRIPPER else 6)
    sample = np.linspace(0, B - 1, 64).astype(int)
    worst = {k: 0.0 for k in groups}
    counts = {"tight": 0, "conditioned": 0, "bif": 0, "beyond": 0}
    flag_mismatch = terminated = 0
    for s in range(3):
        snap = snapshot(env.sim)
        a = torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1
        obs, r, te, tr, _ = env.step(a)
        og, a = obs["observation"].cpu().numpy(), a.cpu().numpy()
        te, tr = te.cpu().numpy(), tr.cpu().numpy()
        agg = obs["achieved_goal"].cpu().numpy()
        # every env's terminated flag is the reference's rule on its own
        # achieved goal (core.py:285, push.py:89-91), bit for bit
        from parity_judge import terminated_rule
        goal = env.sim.goal[:3, :B].t().cpu().numpy()
        rule = np.array([terminated_rule(task, agg[i], goal[i]) for i in range(B)])
        assert np.array_equal(te.astype(bool), rule), (s, np.nonzero(te.astype(bool) != rule))
        terminated += int(te.sum())
        for i in sample:
            o, ag, dg, rr, t_e, t_r = O.step(cfg, oracle_env_from(cfg, snap, i), a[i])
            assert t_r == bool(tr[i]), (s, i)
            ok, mismatch = done_flags_ok(task, te[i], agg[i], t_e, ag, snap["goal"][:3, i])
            assert ok, (s, i, bool(te[i]), t_e)
            flag_mismatch += mismatch
            cls, errs = _judge(cfg, snap, i, a[i], o, og[i], groups, task)
            counts[cls] += 1
            assert cls != "beyond", (task, s, i, errs)
            for k, err in errs.items():
                assert cls != "bif" or err <= LOOSE[k], (task, s, i, k, err)
                if cls != "bif":
                    worst[k] = max(worst[k], err)
    print(task, f"{B} envs, 8 lanes:", {k: f"{v:.1e}" for k, v in worst.items()}, counts,
          f"terminated {terminated} of {3 * B}; sampled mismatches with the oracle (straddling) {flag_mismatch}")
    assert counts["bif"] <= 0.08 * 3 * len(sample)


def test_bench_config_after_60_steps():
    """The bench's exact workload (PandaPush-v3, 65 536 envs, ee, autoreset)
    after 60 steps -- past the first TimeLimit, mid-episode contacts in the
    batch -- then 64 sampled envs teacher-forced against the oracle."""
    B = 65536
    env = make_env("push", "ee", B, autoreset=True)
    env.reset(seed=12345)
    g = torch.Generator(device="cuda")
    g.manual_seed(0xC0FFEE)
    for s in range(60):
        obs, *_ = env.step(torch.rand(B, 3, device="cuda", generator=g) * 2 - 1, copy=False)
    assert torch.isfinite(obs["observation"]).all()
    cfg = oracle_config_for(env.sim.cfg)
    snap = snapshot(env.sim)
    a = torch.rand(B, 3, device="cuda", generator=g) * 2 - 1
    obs, r, te, tr, _ = env.step(a)
    og, a = obs["observation"].cpu().numpy(), a.cpu().numpy()
    te, tr = te.cpu().numpy(), tr.cpu().numpy()
    cached = 0
    for i in np.linspace(0, B - 1, 64).astype(int):
        e = oracle_env_from(cfg, snap, i)
        cached += sum(1 for k in range(4) if e.cache.ground_id[0][k] or e.cache.robot_id[k])
        o, ag, dg, rr, t_e, t_r = O.step(cfg, e, a[i], autoreset=True)
        assert t_r == bool(tr[i]) and t_e == bool(te[i]), i
        assert np.abs(og[i, :3] - o[:3]).max() < 2e-5, i
        assert np.abs(og[i, 6:9] - o[6:9]).max() < 2e-5, i
    assert cached > 64  # the sampled envs carry warm-start contacts into the step


@pytest.mark.parametrize("env_id", ["PandaReach-v3", "PandaPushDense-v3", "PandaSlideJoints-v3",
                                    "PandaPickAndPlace-v3", "PandaStack-v3", "PandaFlipJointsDense-v3"])
def test_1000_random_steps_with_resets(env_id):
    """envs_test.py:6-14 at the reference's length: 1000 random steps with
    reset on done (in-kernel autoreset), 64 envs; every episode boundary
    follows the TimeLimit and everything stays finite.  (All 24 IDs run the
    12-step smoke of test_gpu_envs.py; these six cover every task and both
    control and reward variants at full length.)"""
    import pandasim

    B = 64
    env = pandasim.make(env_id, num_envs=B)
    env.reset(seed=0)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    steps_in_episode = torch.zeros(B, dtype=torch.int64, device="cuda")
    episodes = 0
    for _ in range(1000):
        obs, r, te, tr, info = env.step(torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1,
                                        copy=False)
        steps_in_episode += 1
        done = (te.bool() | tr.bool())
        assert torch.equal(tr.bool(), steps_in_episode == env.max_episode_steps)
        episodes += int(done.sum())
        steps_in_episode[done] = 0
        assert torch.isfinite(obs["observation"]).all()
    assert episodes >= B * (1000 // env.max_episode_steps)


def test_nonfinite_guard_flags_and_resets():
    """NaN/Inf guard: a corrupted env is flagged; with
    reset=True it restarts from a reset state and is reported truncated,
    while every other env steps exactly as without the guard."""
    B = 64
    a = torch.rand(3, B, 3, device="cuda") * 2 - 1
    ref = make_env("push", "ee", B)
    ref.reset(seed=3)
    env = make_env("push", "ee", B)
    env.reset(seed=3)
    env.set_nonfinite_guard(True, reset=False)
    env.sim.f[0, 5] = float("nan")  # joint 0 of env 5
    ref.sim.f[0, 5] = 0.0
    obs, r, te, tr, info = env.step(a[0])
    o_ref, *_ = ref.step(a[0])
    flags = info["nonfinite"]
    assert bool(flags[5]) and int(flags.sum()) == 1
    keep = torch.ones(B, dtype=torch.bool, device="cuda")
    keep[5] = False
    assert torch.equal(obs["observation"][keep], o_ref["observation"][keep])
    # flag + reset: env 5 restarts (finite, elapsed 0, truncated), the rest are untouched
    env.set_nonfinite_guard(True, reset=True)
    obs, r, te, tr, info = env.step(a[1])
    o_ref, _, _, tr_ref, _ = ref.step(a[1])
    assert bool(info["nonfinite"][5]) and bool(tr[5])
    assert torch.isfinite(obs["observation"][5]).all()
    assert int(env.sim.elapsed[5]) == 0
    assert torch.equal(obs["observation"][keep], o_ref["observation"][keep])
    assert torch.equal(tr[keep], tr_ref[keep])
    obs, r, te, tr, info = env.step(a[2])
    assert not info["nonfinite"].any() and torch.isfinite(obs["observation"]).all()
    env.set_nonfinite_guard(False)
    obs, r, te, tr, info = env.step(a[2])
    assert "nonfinite" not in info


@pytest.mark.parametrize("task,lanes", [("push", 1), ("slide", 1), ("stack", 1), ("pick_and_place", 1),
                                        ("push", 8), ("pick_and_place", 16)])
def test_gripper_work_lists_are_lane_independent(task, lanes):
    """The gripper candidates are evaluated on whichever lane of the wave the
    work list assigns (ps_physics.h robot_candidates): an env's step must not
    depend on which other envs share its wave, nor on a partial last wave
    (one-lane kernels: lanes past the batch end have returned).  A scripted
    push into the object (contact-rich) from the same seeds, in batches of
    128, 100 (a partial second wave) and 36 (the partial wave alone): every
    env's state is equal bit for bit across the three."""
    from pandasim.envs import PandaVecEnv

    seeds = (777 + np.arange(128)).astype(np.uint64)
    body = "object1" if task == "stack" else "object"
    runs = {}
    for lo, hi in ((0, 128), (0, 100), (64, 100)):
        B = hi - lo
        env = PandaVecEnv(task, "sparse", "ee", B, "cuda", lanes_per_env=lanes)
        assert env.lanes_per_env == lanes
        env.autoreset = False
        env.reset(seed=seeds[lo:hi])
        policy = _push_policy(env, body)
        contacts = 0
        for s in range(14):
            env.step(torch.from_numpy(policy(s)).cuda())
            ids = env.sim.f[WR_ROW + 4, :B].cpu().numpy()
            contacts += int((ids != 0).sum())
        assert contacts > 0  # the gripper rows are exercised
        runs[(lo, hi)] = env.sim.f[:, :B].cpu().numpy()
    full = runs[(0, 128)]
    assert np.array_equal(runs[(0, 100)], full[:, :100])
    assert np.array_equal(runs[(64, 100)], full[:, 64:100])
