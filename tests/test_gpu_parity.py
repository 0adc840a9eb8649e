"""GPU parity tests: the HIP path (through libpandasim.so's C ABI) against the
fp64 CPU oracle and the reference's golden vectors / known-answer tests.

Tolerances (fp32 kernel vs fp64 oracle; BASELINE north star: 1e-3):
  * task layer (goal/object sampling, rewards, success, TimeLimit): bit-exact;
  * KATs: atol 1e-3 as in /root/reference/test/pybullet_test.py;
  * engine step (20 substeps) from identical state + motors: joint positions
    2e-4, joint velocities 5e-3, object position 5e-4;
  * IK: median 1e-5 rad, max 2e-3 rad (the 1e-4 stopping rule);
  * fused env step from identical state: positions 5e-4, velocities 2e-2
    (velocity = 50/s x IK target error).
"""
import os

import numpy as np
import pytest
import torch

from helpers import OBJECT_ROWS, oracle_config_for, oracle_env_from, snapshot
from pandasim._lib import NUM_FLOAT_ROWS as L_ROWS

import oracle as O

pytestmark = pytest.mark.gpu

ALL_TASKS = ["reach", "push", "pick_and_place", "slide", "stack", "flip"]
OBJECT_TASKS = ALL_TASKS[1:]
TASKS = [(t, c) for t in ALL_TASKS for c in ("ee", "joints")]
from parity_judge import FREE_GRIPPER, LOOSE, NOISE_K, TOL, done_flags_ok, not_tight_cap
from parity_judge import groups_for as _groups
from parity_judge import judge as _judge


@pytest.fixture(scope="module")
def ps():
    import pandasim

    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return pandasim


def make_env(ps, task, control, n, reward="sparse", lanes=0):
    from pandasim.envs import PandaVecEnv

    return PandaVecEnv(task, reward, control, n, "cuda", lanes_per_env=lanes)


# ps_step kernels: one env per lane, and groups of 16 or 8 lanes per env (not Stack)
LANES = [1, 16, 8]
TASKS_LANES = [(t, c, l) for t, c in TASKS for l in LANES if not (t == "stack" and l > 1)]


# ------------------------------------------------------------ known answers
def kat_sim(ps, **overrides):
    from pandasim import _lib as L
    from pandasim.sim import PandaSim

    cfg = L.default_config(0, 0, 0)
    cfg.has_table = cfg.has_plane = 0
    cfg.base[0] = 0.0
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return PandaSim(config=cfg, num_envs=4)


def test_kat_link_position(ps):  # pybullet_test.py:124-136
    sim = kat_sim(ps)
    pos = sim.get_link_position("panda", 1).cpu().numpy()
    assert np.allclose(pos, [0.0, 0.060, 0.373], atol=1e-3)


def test_kat_joint5_motor(ps):  # pybullet_test.py:139-204
    sim = kat_sim(ps)
    sim.control_joints("panda", [5], [0.3], [5.0])
    sim.step()
    pos, orn, v, w = [t.cpu().numpy() for t in sim.link_state(5)]
    assert np.allclose(orn, [0.707, -0.02, 0.02, 0.707], atol=1e-3)
    assert np.allclose(v, [-0.0068, 0.0000, 0.1186], atol=1e-3)
    assert np.allclose(w, [0.000, -2.969, 0.000], atol=1e-3)
    assert np.allclose(sim.get_joint_angle("panda", 5).cpu().numpy(), 0.063, atol=1e-3)


def test_kat_inverse_kinematics(ps):  # pybullet_test.py:254-266
    sim = kat_sim(ps)
    q = sim.inverse_kinematics("panda", 6, [0.4, 0.5, 0.6], [0.707, -0.02, 0.02, 0.707]).cpu().numpy()
    assert np.allclose(q, [1.000, 1.223, -1.113, -0.021, -0.917, 0.666, -0.499, 0.0, 0.0], atol=1e-3)


def test_kat_box_free_fall(ps):  # pybullet_test.py:56-64 (robot parked far away: no contact)
    from pandasim.sim import PandaSim

    sim = PandaSim(task=None, num_envs=4)
    sim.loadURDF(body_name="panda", fileName="franka_panda/panda.urdf", basePosition=[10.0, 0.0, 0.0],
                 useFixedBase=True)
    sim.create_box(body_name="my_box", half_extents=[0.5, 0.5, 0.5], mass=1.0, position=[0.0, 0.0, 0.0])
    sim.step()
    assert np.allclose(sim.get_base_velocity("my_box").cpu().numpy(), [0.0, 0.0, -0.392], atol=1e-3)
    assert np.allclose(sim.get_base_orientation("my_box").cpu().numpy(), [0, 0, 0, 1], atol=1e-3)


# ------------------------------------------------------------ task layer
@pytest.mark.parametrize("task", ALL_TASKS)
def test_reset_goldens_bit_exact(ps, golden, task):
    """Goal and object draws of 216 seeds x 4 successive resets against the
    reference's own numpy draws (tests/golden/make_golden.py).  Flip's goal is
    the reference's unseeded Rotation.random(); it is checked against the
    oracle's auxiliary stream instead (parity of the restatement)."""
    seeds = golden["seeds"]
    B = len(seeds)
    env = make_env(ps, task, "ee", B)
    G = env.goal_dim
    cfg = oracle_config_for(env.sim.cfg)
    oenvs = [O.new_env(cfg) for _ in range(B)]
    for r in range(golden[f"{task}_object"].shape[1]):
        obs, _ = env.reset(seed=seeds if r == 0 else None)
        goal = env.sim.goal[:G, :B].t().cpu().numpy()
        if task == "flip":
            for i in range(B):
                O.reset(cfg, oenvs[i], seed=int(seeds[i]) if r == 0 else None)
            assert np.array_equal(goal, np.array([list(e.goal)[:4] for e in oenvs]))
            assert np.allclose(np.linalg.norm(goal, axis=1), 1.0, atol=1e-12)
        else:
            assert np.array_equal(goal, golden[f"{task}_goal"][:, r])
            assert np.array_equal(obs["desired_goal"].cpu().numpy(), golden[f"{task}_goal"][:, r].astype(np.float32))
        if task == "stack":
            pos = torch.cat([env.sim.get_base_position("object1"), env.sim.get_base_position("object2")], -1)
        elif task != "reach":
            pos = env.sim.get_base_position("object")
        if task != "reach":
            assert np.array_equal(pos.cpu().numpy(), golden[f"{task}_object"][:, r].astype(np.float32))


def test_compute_reward_goldens_bit_exact(ps, golden):
    for reward_type in ["sparse", "dense"]:
        env = make_env(ps, "push", "ee", 8, reward=reward_type)
        ag = torch.from_numpy(golden["reward_ag"]).cuda()
        dg = torch.from_numpy(golden["reward_dg"]).cuda()
        r = env.compute_reward(ag, dg, {}).cpu().numpy()
        assert np.array_equal(r.view(np.uint32), golden[f"reward_{reward_type}"].view(np.uint32))
        s = env.compute_success(ag, dg).cpu().numpy()
        assert np.array_equal(s, golden["success"])
        her = env.compute_reward(torch.from_numpy(golden["her_ag"]).cuda(), torch.from_numpy(golden["her_dg"]).cuda())
        assert her.shape == (32, 32)
        assert np.array_equal(her.cpu().numpy().view(np.uint32), golden[f"her_reward_{reward_type}"].view(np.uint32))


@pytest.mark.parametrize("task", ["stack", "flip"])
def test_compute_reward_goldens_stack_flip(ps, golden, task):
    """stack.py:118-131 (6-D distance, threshold 0.1) and flip.py:80-91
    (1 - <q, g>^2, threshold 0.2) against the reference's functions."""
    for reward_type in ["sparse", "dense"]:
        env = make_env(ps, task, "ee", 8, reward=reward_type)
        ag = torch.from_numpy(golden[f"{task}_ag"]).cuda()
        dg = torch.from_numpy(golden[f"{task}_dg"]).cuda()
        r = env.compute_reward(ag, dg, {}).cpu().numpy()
        want = golden[f"{task}_reward_{reward_type}"]
        assert np.array_equal(r.view(np.uint32), want.view(np.uint32))
        assert np.array_equal(env.compute_success(ag, dg).cpu().numpy(), golden[f"{task}_success"])


# ------------------------------------------------------------ physics parity
def _oracle_ik_batch(cfg, snap, link, pos, orn):
    out = []
    for i in range(snap["f"].shape[1]):
        out.append(O.inverse_kinematics(cfg, snap["f"][:9, i], link, pos[i], orn[i]))
    return np.array(out)


@pytest.mark.parametrize("task", ["reach", "push"])
def test_ik_parity(ps, task):
    """calculateInverseKinematics: GPU fp32 vs oracle fp64 from the same joints.

    The DLS loop stops once |p - p*| <= 1e-4, so the two precisions may stop
    one iteration apart; targets then still agree to ~1e-3 rad."""
    B = 256
    env = make_env(ps, task, "ee", B)
    env.autoreset = False
    env.reset(seed=5)
    rng = np.random.default_rng(3)
    for _ in range(3):
        env.step(torch.from_numpy(rng.uniform(-1, 1, size=(B, 3)).astype(np.float32)).cuda())
    cfg = oracle_config_for(env.sim.cfg)
    snap = snapshot(env.sim)
    ee = env.sim.get_link_position("panda", 11).cpu().numpy()
    target = ee + rng.uniform(-0.05, 0.05, size=(B, 3))
    orn = np.tile([1.0, 0.0, 0.0, 0.0], (B, 1))
    q_gpu = env.sim.inverse_kinematics("panda", 11, target, orn).cpu().numpy()
    q_ref = _oracle_ik_batch(cfg, snap, 11, target, orn)
    err = np.abs(q_gpu - q_ref).max(axis=1)
    assert np.median(err) < 1e-5
    assert np.all(err < 2e-3)


# Engine-step tolerances (fp32 GPU vs fp64 oracle from the same state and
# motors).  Reach and Push are well conditioned: every sample must meet the
# tight bounds.  PickAndPlace's free fingers (0.1 kg prismatic joints under
# 170 N motors, touching the 1 kg cube) make its contact events
# ill-conditioned: in the oracle alone a 2e-7-relative state perturbation
# moves finger q by 1.2e-4 and qd by 1.4e-2 in one step, and a
# contact that the two precisions resolve on different substeps moves the
# whole arm.  There, 95 % of the (env, step) samples must meet the tight
# bounds and all of them the loose ones.
SIM_TIGHT = dict(q=2e-4, qd=5e-3)
SIM_LOOSE = dict(q=1e-2, qd=1.0)


def _object_rows(task):
    return {"reach": [], "stack": [63, 76]}.get(task, [63])


OBJ_ATOL = {"push": 5e-4, "slide": 5e-4}


def _sim_step_sensitivity(cfg, snap, i, ref):
    """Largest move of the oracle's joint positions and velocities after one
    engine step (20 substeps) from env i of `snap` under one fp32 ulp of
    state noise per substep (four seeds) and with the state rounded to fp32
    every substep (test_gpu_parity._sensitivity for the engine step)."""
    sq = sqd = 0.0
    try:
        for ulps, seed in [(1.0, 1), (1.0, 2), (1.0, 3), (1.0, 4), (-1.0, 0)]:
            O.set_state_noise(ulps, seed)
            e = oracle_env_from(cfg, snap, i)
            O.sim_step(cfg, e)
            sq = max(sq, float(np.abs(np.array(e.q) - np.array(ref.q)).max()))
            sqd = max(sqd, float(np.abs(np.array(e.qd) - np.array(ref.qd)).max()))
    finally:
        O.set_state_noise(0.0)
    return sq, sqd


@pytest.mark.parametrize("task", ALL_TASKS)
def test_sim_step_parity_same_motors(ps, task):
    """Engine step (20 substeps) from identical joints, motors and object."""
    B = 128
    env = make_env(ps, task, "ee", B)
    env.autoreset = False
    env.reset(seed=21)
    cfg = oracle_config_for(env.sim.cfg)
    rng = np.random.default_rng(5)
    err_q, err_qd, conditioned = [], [], []
    for s in range(8):
        env.step(torch.from_numpy(rng.uniform(-1, 1, size=(B, env.action_dim)).astype(np.float32)).cuda())
        snap = snapshot(env.sim)  # motors hold the targets of this step's set_action
        env.sim.step()
        after = snapshot(env.sim)
        for i in range(0, B, 4):
            e = oracle_env_from(cfg, snap, i)
            O.sim_step(cfg, e)
            eq = np.abs(after["f"][0:9, i] - np.array(e.q)).max()
            eqd = np.abs(after["f"][9:18, i] - np.array(e.qd)).max()
            err_q.append(eq)
            err_qd.append(eqd)
            cond = False
            if eq >= SIM_TIGHT["q"] or eqd >= SIM_TIGHT["qd"]:
                # within the tight bounds once NOISE_K x the oracle's own
                # spread at the state's fp32 resolution is allowed for (_judge)
                sq, sqd = _sim_step_sensitivity(cfg, snap, i, e)
                cond = eq < SIM_TIGHT["q"] + NOISE_K * sq and eqd < SIM_TIGHT["qd"] + NOISE_K * sqd
            conditioned.append(cond)
            for b, row in enumerate(_object_rows(task)):
                assert np.allclose(after["f"][row:row + 3, i], np.array(e.obj[b].pos),
                                   atol=OBJ_ATOL.get(task, 5e-3)), (s, i, b)
    err_q, err_qd, conditioned = np.array(err_q), np.array(err_qd), np.array(conditioned)
    tight = (err_q < SIM_TIGHT["q"]) & (err_qd < SIM_TIGHT["qd"])
    print(task, f"max q {err_q.max():.1e} qd {err_qd.max():.1e}; tight {tight.mean() * 100:.1f} % of {tight.size}, "
                f"within the oracle's conditioning {conditioned.sum()}")
    if task in FREE_GRIPPER:
        assert tight.mean() >= 0.95
        assert err_q.max() < SIM_LOOSE["q"] and err_qd.max() < SIM_LOOSE["qd"]
    else:
        assert (tight | conditioned).all(), (err_q.max(), err_qd.max())
        assert conditioned.mean() <= 0.02


# The per-sample classifier (tight / conditioned / ill-conditioned / beyond)
# and its bounds live in tests/parity_judge.py, where the CPU suite checks that
# it reports deliberate 1-2 % model errors as failures
# (tests/test_judge_power.py).


@pytest.mark.parametrize("task,control,lanes", TASKS_LANES)
def test_env_step_parity_teacher_forced(ps, task, control, lanes):
    """Each fused GPU env step vs one oracle env step from the same state,
    classified by parity_judge.judge.  No sample may be beyond the tight
    bounds; a blocked gripper (Reach/Push/Slide) may leave at most 0.5 % of
    them conditioned or ill-conditioned, a free one 8 % ill-conditioned
    (finger-limit branches) and 2 % conditioned.  Done flags: `terminated` is
    the reference's rule on the GPU's own achieved goal bit for bit, and
    differs from the oracle's only where the two achieved goals straddle the
    threshold (parity_judge.done_flags_ok); `truncated` equal."""
    B, steps = 64, 10
    env = make_env(ps, task, control, B, lanes=lanes)
    assert env.lanes_per_env == lanes
    env.autoreset = False
    env.reset(seed=12345)
    cfg = oracle_config_for(env.sim.cfg)
    rng = np.random.default_rng(7)
    groups = _groups(task, 7 if task in FREE_GRIPPER else 6)
    assert max(max(v) for v in groups.values()) == env.obs_dim - 1
    worst = {k: 0.0 for k in groups}
    worst_bif = {k: 0.0 for k in groups}
    counts = {"tight": 0, "conditioned": 0, "bif": 0, "beyond": 0}
    beyond, flag_bad = [], []
    flag_mismatch = 0
    G = env.goal_dim
    for s in range(steps):
        snap = snapshot(env.sim)
        a = rng.uniform(-1, 1, size=(B, env.action_dim)).astype(np.float32)
        obs, r, te, tr, _ = env.step(torch.from_numpy(a).cuda())
        og, te, tr = obs["observation"].cpu().numpy(), te.cpu().numpy(), tr.cpu().numpy()
        agg = obs["achieved_goal"].cpu().numpy()
        for i in range(B):
            e = oracle_env_from(cfg, snap, i)
            o, ag, dg, rr, t_e, t_r = O.step(cfg, e, a[i])
            cls, errs = _judge(cfg, snap, i, a[i], o, og[i], groups, task)
            counts[cls] += 1
            for k, err in errs.items():
                if cls == "bif":
                    worst_bif[k] = max(worst_bif[k], err)
                else:
                    worst[k] = max(worst[k], err)
            if cls == "beyond":
                beyond.append((s, i, {k: f"{v:.2e}" for k, v in errs.items()}))
                if os.environ.get("PANDASIM_DUMP_SAMPLES"):
                    np.savez(os.path.join(os.environ["PANDASIM_DUMP_SAMPLES"], f"{task}_{control}_{s}_{i}.npz"),
                             f=snap["f"][:, i], goal=snap["goal"][:, i], action=a[i], gpu_obs=og[i])
            assert t_r == bool(tr[i])
            ok, mismatch = done_flags_ok(task, te[i], agg[i], t_e, ag, snap["goal"][:G, i])
            flag_mismatch += mismatch
            if not ok:
                flag_bad.append((s, i, bool(te[i]), t_e))
    print(task, control, f"lanes {lanes}", counts, "worst", {k: f"{v:.2e}" for k, v in worst.items()},
          "ill-conditioned worst", {k: f"{v:.2e}" for k, v in worst_bif.items()}, "beyond", beyond[:8],
          f"terminated mismatches (straddling the threshold) {flag_mismatch}")
    assert not beyond
    assert not flag_bad, flag_bad
    for k, v in worst_bif.items():
        assert v <= LOOSE[k], (k, v)
    if task in FREE_GRIPPER:
        assert counts["bif"] <= not_tight_cap(task) * B * steps
        assert counts["conditioned"] <= 0.02 * B * steps
    else:
        assert counts["bif"] + counts["conditioned"] <= not_tight_cap(task) * B * steps


def test_reach_free_running_parity(ps):
    """Contact-free Reach, joint control (no IK stopping rule): 30 steps free-running."""
    B = 16
    env = make_env(ps, "reach", "joints", B)
    env.autoreset = False
    env.reset(seed=3)
    cfg = oracle_config_for(env.sim.cfg)
    snap = snapshot(env.sim)
    oenvs = [oracle_env_from(cfg, snap, i) for i in range(B)]
    rng = np.random.default_rng(11)
    for s in range(30):
        a = rng.uniform(-1, 1, size=(B, 7)).astype(np.float32)
        obs, *_ = env.step(torch.from_numpy(a).cuda())
        og = obs["observation"].cpu().numpy()
        for i in range(B):
            o, *_ = O.step(cfg, oenvs[i], a[i])
            assert np.allclose(og[i, :3], o[:3], atol=1e-3), (s, i)
            assert np.allclose(og[i, 3:], o[3:], atol=2e-2), (s, i)


@pytest.mark.parametrize("task", ALL_TASKS)
def test_autoreset_continues_generator(ps, task):
    """Every in-kernel reset (success or TimeLimit) draws the next goal/object
    from the env's own PCG64 stream: after n resets the goal equals the
    oracle's n-th unseeded reset after reset(seed) -- bit-exact."""
    B = 32
    env = make_env(ps, task, "ee", B)
    env.reset(seed=100)
    cfg = oracle_config_for(env.sim.cfg)
    zeros = torch.zeros(B, env.action_dim, device="cuda")
    n_resets = np.zeros(B, int)
    for s in range(env.max_episode_steps + 10):
        obs, r, te, tr, info = env.step(zeros)
        n_resets += (te | tr).cpu().numpy().astype(int)
    assert (n_resets >= 1).all()
    G = env.goal_dim
    goal = env.sim.goal[:G, :B].t().cpu().numpy()
    for i in range(B):
        e = O.new_env(cfg)
        O.reset(cfg, e, seed=100 + i)
        for _ in range(n_resets[i]):
            O.reset(cfg, e, seed=None)
        assert np.array_equal(goal[i], np.array(e.goal)[:G])


def test_determinism_and_save_restore(ps):
    B = 128
    a = torch.rand(6, B, 3, device="cuda") * 2 - 1
    outs = []
    for _ in range(2):
        env = make_env(ps, "push", "ee", B)
        env.reset(seed=6789)
        for k in range(6):
            obs, *_ = env.step(a[k])
        outs.append(obs["observation"].cpu())
    assert torch.equal(outs[0], outs[1])
    env = make_env(ps, "reach", "ee", B)
    env.reset(seed=1)
    sid = env.save_state()
    o1, *_ = env.step(a[0])
    env.reset(seed=2)
    env.restore_state(sid)
    o2, *_ = env.step(a[0])
    for k in o1:
        assert torch.equal(o1[k], o2[k])
    env.remove_state(sid)
    with pytest.raises(Exception):
        env.restore_state(sid)


@pytest.mark.parametrize("task", OBJECT_TASKS)
def test_large_batch_properties(ps, task):
    """At the bench size: finite, bounded observations and exact TimeLimit."""
    B = 65536
    env = make_env(ps, task, "ee", B)
    env.reset(seed=12345)
    for s in range(5):
        obs, r, te, tr, _ = env.step(torch.rand(B, env.action_dim, device="cuda") * 2 - 1)
    o = obs["observation"]
    assert torch.isfinite(o).all()
    # a gripper strike can spin the 4 cm cube to ~100 rad/s and throw it off
    # the table (the oracle reproduces these states: DESIGN.md §6); a blow-up
    # would be far beyond
    assert (o.abs() < 1000).all()
    for body in (("object1", "object2") if task == "stack" else ("object",)):
        assert (env.sim.get_base_position(body)[:, 2] > -0.45).all()
    assert not tr.any()
    assert int(env.sim.elapsed[:B].max()) <= 5 and int(env.sim.elapsed[:B].min()) >= 0


# ------------------------------------------------------------ contact-rich parity
def _teacher_forced_objects(env, cfg, actions_fn, steps, stride=2):
    """Per step: snapshot, one fused GPU step, one oracle step of every
    `stride`-th env from the snapshot; returns per-(env, step) max errors of
    the object positions and of the joint positions."""
    B = env.num_envs
    rows = _object_rows(env.task_name)
    e_obj, e_q = [], []
    for s in range(steps):
        snap = snapshot(env.sim)
        a = actions_fn(s)
        env.step(torch.from_numpy(a).cuda())
        after = snapshot(env.sim)
        for i in range(0, B, stride):
            e = oracle_env_from(cfg, snap, i)
            O.step(cfg, e, a[i])
            e_q.append(np.abs(after["f"][0:9, i] - np.array(e.q)).max())
            e_obj.append(max(np.abs(after["f"][r:r + 3, i] - np.array(e.obj[b].pos)).max()
                             for b, r in enumerate(rows)))
    return np.array(e_obj), np.array(e_q)


def test_box_on_box_parity(ps):
    """Stack's cube-on-cube contact (box-box face clipping): object2 dropped
    onto object1 with xy offsets up to 3/4 of the cube and yaw up to 45 deg,
    teacher-forced against the oracle for 12 env steps (resting, sliding off
    and tipping cases)."""
    B = 64
    env = make_env(ps, "stack", "ee", B)
    env.autoreset = False
    env.reset(seed=31)
    rng = np.random.default_rng(8)
    p1 = env.sim.get_base_position("object1").double()
    off = torch.from_numpy(rng.uniform(-0.03, 0.03, size=(B, 2))).cuda()
    p2 = p1.clone()
    p2[:, :2] += off
    p2[:, 2] = 0.02 + 0.04 + torch.from_numpy(rng.uniform(0.0, 0.004, size=B)).cuda()
    yaw = torch.from_numpy(rng.uniform(-np.pi / 4, np.pi / 4, size=B)).cuda()
    q2 = torch.stack([torch.zeros_like(yaw), torch.zeros_like(yaw), torch.sin(yaw / 2), torch.cos(yaw / 2)], -1)
    env.sim.set_base_pose("object2", p2, q2)
    # park the arm high above the table so only the cubes interact
    cfg = oracle_config_for(env.sim.cfg)
    up = np.zeros((B, env.action_dim), np.float32)
    up[:, 2] = 1.0
    e_obj, e_q = _teacher_forced_objects(env, cfg, lambda s: up, 12, stride=1)
    z2 = env.sim.get_base_position("object2")[:, 2].cpu().numpy()
    print("box-on-box", f"max obj {e_obj.max():.1e}; resting {(z2 > 0.05).mean() * 100:.0f} %")
    assert (z2 > 0.05).any() and (z2 < 0.05).any()  # both outcomes are exercised
    assert (e_obj < 1e-3).mean() >= 0.95 and e_obj.max() < 1e-2


def test_airborne_cube_has_no_ground_rows(ps):
    """Stack's ground-row gates are per wave: lanes whose cube has no ground
    contact still run the rows some other lane of the wave has.  Those rows
    must be exact no-ops.  Half the wave rests both cubes on the table (the
    gates open); the other half holds the pair 0.3 m up with cube 2 sunk 3 mm
    into cube 1, so the pair rows push cube 1 down in the solve.  A ground row
    left live there would push back (its 1/den is the cube's mass at a zero
    offset); against the oracle, the airborne cubes must match."""
    B = 64
    env = make_env(ps, "stack", "ee", B)
    env.autoreset = False
    env.reset(seed=5)
    p1 = env.sim.get_base_position("object1").double()
    air = torch.arange(B, device=p1.device) >= B // 2
    p1[air, 2] = 0.3
    p2 = p1.clone()
    p2[:, 2] = p1[:, 2] + 0.04 - torch.where(air, 0.003, 0.0)
    q = torch.zeros(B, 4, dtype=torch.float64, device=p1.device)
    q[:, 3] = 1.0
    env.sim.set_base_pose("object1", p1, q)
    env.sim.set_base_pose("object2", p2, q)
    cfg = oracle_config_for(env.sim.cfg)
    up = np.zeros((B, env.action_dim), np.float32)
    up[:, 2] = 1.0
    e_obj, _ = _teacher_forced_objects(env, cfg, lambda s: up, 2, stride=1)
    e_air = e_obj.reshape(-1, B)[:, B // 2:]  # (step, env) order
    print("airborne pair", f"max obj err {np.max(e_air):.1e} (all lanes {np.max(e_obj):.1e})")
    assert np.max(e_air) < 1e-3


@pytest.mark.parametrize("task", OBJECT_TASKS)
def test_gripper_object_contact_parity(ps, task):
    """Scripted pushes into the object (P-control of the end effector towards
    the object, then through it): robot-object contacts on every env,
    teacher-forced against the oracle.  Contact onsets are ill-conditioned
    (DESIGN.md §6), so 95 % of the samples meet the tight bounds and all the
    loose ones."""
    B = 64
    env = make_env(ps, task, "ee", B)
    env.autoreset = False
    env.reset(seed=44)
    cfg = oracle_config_for(env.sim.cfg)
    body = "object1" if task == "stack" else "object"

    def policy(s):
        ee = env.sim.get_link_position("panda", 11).cpu().numpy()
        obj = env.sim.get_base_position(body).cpu().numpy()
        tgt = obj + np.array([0.0, 0.0, 0.06 if s < 6 else 0.0])
        if s >= 6:
            tgt[:, 0] += 0.05  # push through the object
        a = np.zeros((B, env.action_dim), np.float32)
        a[:, :3] = np.clip(10.0 * (tgt - ee), -1, 1)
        if env.action_dim == 4:
            a[:, 3] = -1.0 if s >= 8 else 1.0  # close the fingers late
        return a

    p0 = env.sim.get_base_position(body).cpu().numpy()
    e_obj, e_q = _teacher_forced_objects(env, cfg, policy, 14)
    moved = np.linalg.norm(env.sim.get_base_position(body).cpu().numpy() - p0, axis=1)
    print(task, f"contact: max obj {e_obj.max():.1e} q {e_q.max():.1e}; moved {np.mean(moved > 1e-3) * 100:.0f} %")
    assert np.mean(moved > 1e-3) > 0.5  # the gripper did reach the objects
    assert (e_obj < 1e-3).mean() >= 0.95 and (e_q < SIM_TIGHT["q"] * 10).mean() >= 0.95
    assert e_obj.max() < 2e-2 and e_q.max() < SIM_LOOSE["q"] * 5


# Contact-rich workloads classified like the random-action tests (round 6,
# VERDICT r05 item 3): the ones tests/judge_power.py shows the classifier can
# fail on -- Stack with cube 2 resting on cube 1 and the gripper dragging the
# top cube over the bottom one ("stack_push": cube 2's mass and the cube-cube
# friction x 1.02 are reported beyond), and the scripted push of Flip's cube
# (its mass and friction x 1.02 move the quaternion observation beyond the
# bounds).  The fp32 stand-in of tests/judge_power.py leaves 3.2 % (Stack)
# and 2.9 % (Flip) of these samples conditioned and none beyond
# (profiles/r06_judge_power.log); caps: 6 % conditioned, 8 % ill-conditioned,
# 1 % ill-conditioned beyond the loose bounds.
JUDGED_CONTACT_CAPS = {"conditioned": 0.06, "bif": 0.08}


@pytest.mark.parametrize("task,workload", [("stack", "stack_push"), ("flip", "push"), ("stack", "push")])
def test_judged_contact_workloads(ps, task, workload):
    B, steps = 64, 14
    env = make_env(ps, task, "ee", B)
    env.autoreset = False
    env.reset(seed=44)
    if workload == "stack_push":
        p1 = env.sim.get_base_position("object1").double()
        p2 = p1.clone()
        p2[:, 2] += 0.04  # cube 2 face to face on cube 1, at rest (judge_power.stack_cubes)
        env.sim.set_base_pose("object2", p2, env.sim.get_base_orientation("object1").double())
    body = {"stack_push": "object2", "push": "object1" if task == "stack" else "object"}[workload]
    from test_gpu_contacts import _push_policy

    policy = _push_policy(env, body)
    cfg = oracle_config_for(env.sim.cfg)
    groups = _groups(task, 7)
    counts = {"tight": 0, "conditioned": 0, "bif": 0, "beyond": 0}
    beyond, past_loose = [], []
    p0 = env.sim.get_base_position(body).cpu().numpy()
    for s in range(steps):
        snap = snapshot(env.sim)
        a = policy(s)
        obs, *_ = env.step(torch.from_numpy(a).cuda())
        og = obs["observation"].cpu().numpy()
        after = None
        for i in range(B):
            o, *_ = O.step(cfg, oracle_env_from(cfg, snap, i), a[i])
            cls, errs = _judge(cfg, snap, i, a[i], o, og[i], groups, task)
            counts[cls] += 1
            if cls == "beyond":
                beyond.append((s, i, {k: f"{v:.1e}" for k, v in errs.items()}))
                # dumped for scripts/tf_sample.py / substep_compare.py
                after = env.sim.f[:, :B].double().cpu().numpy() if after is None else after
                out = os.path.join("gpurun_out", "judged")
                os.makedirs(out, exist_ok=True)
                np.savez(os.path.join(out, f"{task}_ee_{s}_{i}.npz"), f=snap["f"][:, i], goal=snap["goal"][:, i],
                         rng=snap["rng"][:, i], elapsed=snap["elapsed"][i], action=a[i], gpu_obs=og[i],
                         gpu_f_after=after[:, i], oracle_obs=o)
            if cls == "bif" and any(v > LOOSE[k] for k, v in errs.items()):
                past_loose.append((s, i, {k: f"{v:.1e}" for k, v in errs.items() if v > LOOSE[k]}))
    moved = np.linalg.norm(env.sim.get_base_position(body).cpu().numpy() - p0, axis=1)
    print(task, workload, counts, f"moved {np.mean(moved > 1e-3) * 100:.0f} %", "beyond", beyond[:8],
          "ill-conditioned past the loose bounds", past_loose)
    assert np.mean(moved > 1e-3) > 0.5  # the gripper did reach the cube
    n = B * steps
    # Resting stacked cubes: a body's velocity after the solve is fixed only
    # to the PGS stopping rule's resolution (Bullet exits once every row's
    # (dl / dinv)^2 <= 1e-7: a last row velocity change of up to 3.2e-4 m/s,
    # 1.6e-2 rad/s over the cube's 0.02 m contact offsets), and each of the
    # two runs stops somewhere within it: twice that between them.  Replayed
    # (round 6, stack_push steps 2 and 5, envs 9 and 22: the oracle's own
    # probes move them by <= 1.4e-3 rad/s): positions and rotations agree to
    # 3e-7 m / 2e-5 rad, velocities part by at most 3.7e-4 m/s and 1.2e-2
    # rad/s.  Such samples (every other group tight, the objects' velocities
    # within 6.4e-4 m/s and 3.2e-2 rad/s) are counted apart, at most 0.5 %; no
    # other beyond.
    def at_resolution(errs):
        objv = [k for k in errs if k.startswith("obj") and k.endswith(("_vel", "_avel"))]
        return all(v <= TOL[task][k] for k, v in errs.items() if k not in objv) and \
            all(errs[k] <= (6.4e-4 if k.endswith("_vel") else 3.2e-2) for k in objv)
    resolution = [b for b in beyond if at_resolution({k: float(v) for k, v in b[2].items()})]
    assert len(beyond) == len(resolution), [b for b in beyond if b not in resolution]
    assert len(resolution) <= 0.005 * n
    assert counts["conditioned"] <= JUDGED_CONTACT_CAPS["conditioned"] * n
    assert counts["bif"] <= JUDGED_CONTACT_CAPS["bif"] * n
    # a cube balanced on an edge of the other (tipping) is a branch the oracle
    # cannot resolve at fp32 resolution; where it tips the two runs part by
    # more than the loose bounds (round 6: stack_push step 8 env 25)
    assert len(past_loose) <= 0.01 * n


@pytest.mark.parametrize("B,lanes", [(1, 1), (70, 1), (1, 16), (7, 16), (70, 16), (1, 8), (13, 8), (70, 8)])
def test_ragged_batch_parity(ps, B, lanes):
    """Batches that are not a multiple of the wave (one env; 70 = a full
    64-lane wave plus 6 lanes; with 16 lanes per env, 7 envs = a wave of 4
    plus 3 envs and a dummy group; with 8, 13 envs = a wave of 8 plus 5 and
    three dummy groups): every env, including the ragged wave's,
    steps like the oracle from the same state."""
    env = make_env(ps, "push", "ee", B, lanes=lanes)
    env.autoreset = False
    env.reset(seed=4242)
    cfg = oracle_config_for(env.sim.cfg)
    rng = np.random.default_rng(11)
    groups = _groups("push", 6)
    for _ in range(3):
        snap = snapshot(env.sim)
        a = rng.uniform(-1, 1, size=(B, env.action_dim)).astype(np.float32)
        obs, *_ = env.step(torch.from_numpy(a).cuda())
        og = obs["observation"].cpu().numpy()
        for i in sorted({0, B - 1, B // 2}):
            o, *_ = O.step(cfg, oracle_env_from(cfg, snap, i), a[i])
            for k, idx in groups.items():
                assert np.abs(og[i, idx] - o[idx]).max() <= TOL["push"][k], (B, i, k)


GROUP_TASKS = [(t, c) for t, c in TASKS if t != "stack"]


@pytest.mark.parametrize("B", [64, 1000])
@pytest.mark.parametrize("task,control", GROUP_TASKS)
def test_group_kernels_match_one_lane(ps, task, control, B):
    """The 16- and 8-lane group kernels against the one-lane kernel over the
    same step from the same reset (no gripper contact yet): the robot's rows
    (q, qd: rows 0-17) of every env equal bit for bit, every other row within
    1e-4 (the object's ground rows sum J.v over the group's lanes in another
    order).  They run the same rows in the same order and, built with the same
    flags (-O3), the same arithmetic (profiles/r04b_groups_o3.log: all ten
    pairs 0.0 apart in q, qd).  Round 3's -O3 Slide group kernels were off by
    6.8e-3 to 2.1e-1 rad/s in the joint velocities; any such
    recurrence, or codegen drift, fails here.  Contact states:
    test_group_kernels_match_one_lane_in_contact.  1 000 envs: 125 and 250
    group blocks, so the XCD-aware block order (ps_common.h step_block:
    tiles of 4 waves at 8 lanes up to block 96, then the blocks' own order;
    the whole range at 16) maps every env to one group, each once."""
    res = {}
    for lanes in (1, 8, 16):
        env = make_env(ps, task, control, B, lanes=lanes)
        assert env.lanes_per_env == lanes
        env.autoreset = False
        env.reset(seed=12345)
        a = np.random.default_rng(7).uniform(-1, 1, size=(B, env.action_dim)).astype(np.float32)
        env.step(torch.from_numpy(a).cuda())
        res[lanes] = env.sim.f[:, :B].double().cpu().numpy()
    for lanes in (8, 16):
        diff = np.abs(res[lanes] - res[1])
        print(f"{task} {control} {lanes} lanes vs 1: max {diff.max():.1e} over rows {np.nonzero(diff.max(1))[0].tolist()}")
        # the robot's rows bit for bit; the object's (and its ground contacts'
        # cached impulses) to rounding: a group sums a ground row's J.v in
        # another order than the one-lane solver (1.6e-5 at most measured,
        # profiles/r04c_pytest_gpu.log)
        assert np.array_equal(res[lanes][0:18], res[1][0:18]), (lanes, float(diff[0:18].max()))
        assert diff.max() <= 1e-4, (lanes, float(diff.max()))


def _contact_policy(env, task):
    """Drives the end effector into contact: over the object and through it
    (test_gpu_contacts._push_policy), or for Reach down onto the table, the
    fingers closing late (free gripper)."""
    B = env.num_envs

    def policy(s):
        ee = env.sim.get_link_position("panda", 11).cpu().numpy()
        if task == "reach":
            tgt = ee.copy()
            tgt[:, 2] = -0.05
        else:
            obj = env.sim.get_base_position("object").cpu().numpy()
            tgt = obj + np.array([0.0, 0.0, 0.06 if s < 6 else 0.0])
            if s >= 6:
                tgt[:, 0] += 0.05
        a = np.zeros((B, env.action_dim), np.float32)
        a[:, :3] = np.clip(10.0 * (tgt - ee), -1, 1)
        if env.action_dim == 4:
            a[:, 3] = -1.0 if s >= 8 else 1.0
        return a

    return policy


@pytest.mark.parametrize("task,control", GROUP_TASKS)
def test_group_kernels_match_one_lane_in_contact(ps, task, control):
    """As test_group_kernels_match_one_lane, from a mid-rollout state with
    gripper-object and gripper-table contacts: an
    ee-control one-lane run pushes into the object (Reach: presses onto the
    table) for 9 steps; that state is stepped once more by the one-lane, 8-lane
    and 16-lane kernels with the same action.  Every env without a gripper
    contact row in the state before or after keeps the robot rows (q, qd)
    bit for bit.  In the others a gripper contact row's J.v is a group sum in
    another order than the one-lane solver's, so they round differently and a
    contact amplifies it (measured: up to 3e-3 rad/s in qd and 4e-2 in the
    object's velocities after one step, profiles/r05a_pytest_gpu.log); each
    kernel's step is therefore held against the oracle from the same state, by
    parity_judge.judge: no sample beyond, and the one-lane kernel's own caps on
    the other classes."""
    from helpers import WR_ROW

    B = 64
    drv = make_env(ps, task, "ee", B, lanes=1)
    drv.autoreset = False
    drv.reset(seed=44)
    policy = _contact_policy(drv, task)
    for s in range(9):
        drv.step(torch.from_numpy(policy(s)).cuda())
    state0 = drv.sim.state.clone()
    env = make_env(ps, task, control, B, lanes=1)
    env.autoreset = False
    env.reset(seed=44)
    a = np.random.default_rng(9).uniform(-1, 1, size=(B, env.action_dim)).astype(np.float32)
    if control == "ee":
        a[:, :3] = policy(9)[:, :3]
    res, obs = {}, {}
    for lanes in (1, 8, 16):
        env.sim.state.copy_(state0)
        if lanes == 1:
            snap = snapshot(env.sim)
        env.sim._call("ps_set_lanes_per_env", env.sim._ctx, lanes)
        assert env.sim._lib.ps_step_lanes(env.sim._ctx) == lanes
        env.sim._call("ps_mark_motor_rows_dirty", env.sim._ctx)
        o, *_ = env.step(torch.from_numpy(a).cuda())
        res[lanes] = env.sim.f[:, :B].double().cpu().numpy()
        obs[lanes] = o["observation"].cpu().numpy()
    contact = (snap["f"][WR_ROW + 4] != 0) | (res[1][WR_ROW + 4] != 0)
    assert contact.sum() >= 4, int(contact.sum())  # the gripper rows are exercised
    for lanes in (8, 16):
        diff = np.abs(res[lanes] - res[1])
        rob = diff[0:18].max(0)
        print(f"{task} {control} {lanes} lanes vs 1 in contact ({int(contact.sum())} of {B} envs with gripper "
              f"contacts): robot rows max {rob.max():.1e} (contact envs), "
              f"{rob[~contact].max() if (~contact).any() else 0.0:.1e} (others); other rows max "
              f"{diff[18:].max():.1e}; envs bit-equal in q, qd: {int((rob == 0).sum())}")
        assert np.array_equal(res[lanes][0:18, ~contact], res[1][0:18, ~contact]), lanes
    cfg = oracle_config_for(env.sim.cfg)
    groups = _groups(task, 7 if task in FREE_GRIPPER else 6)
    counts = {lanes: {"tight": 0, "conditioned": 0, "bif": 0, "beyond": 0} for lanes in (1, 8, 16)}
    for i in range(B):
        o, *_ = O.step(cfg, oracle_env_from(cfg, snap, i), a[i])
        for lanes in (1, 8, 16):
            cls, errs = _judge(cfg, snap, i, a[i], o, obs[lanes][i], groups, task)
            counts[lanes][cls] += 1
            assert cls != "beyond", (lanes, i, errs)
            assert cls != "bif" or all(v <= LOOSE[k] for k, v in errs.items()), (lanes, i, errs)
    print(task, control, "in contact, against the oracle:", counts)
    for lanes in (1, 8, 16):
        c = counts[lanes]
        if task in FREE_GRIPPER:
            assert c["bif"] <= not_tight_cap(task) * B and c["conditioned"] <= 0.05 * B
        else:
            assert c["bif"] + c["conditioned"] <= 0.05 * B
