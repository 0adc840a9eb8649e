"""CPU tests: pin the oracle (fp64 CPU restatement) before trusting it.

* Physics known-answer tests transcribed from the reference's own suite,
  /root/reference/test/pybullet_test.py (atol 1e-3 as there).
* Task-layer golden vectors generated from the reference's task classes
  (tests/golden/make_golden.py): bit-exact.
* numpy SeedSequence/PCG64 restatement vs numpy itself: bit-exact.
* seed_test.py / save_and_restore_test.py behaviours.
"""
import copy
import os

import numpy as np
import oracle as O
import pytest


def kat_config():
    # PyBullet() + loadURDF("franka_panda/panda.urdf", basePosition=0, useFixedBase=True), no other bodies
    return O.config("reach", base=(0.0, 0.0, 0.0), has_table=0, has_plane=0, n_objects=0)


def test_dt():  # pybullet_test.py:30-35
    assert O.lib() is not None
    assert abs(20 * (1.0 / 500) - 0.04) < 1e-12


def test_get_link_position():  # pybullet_test.py:124-136
    cfg = kat_config()
    env = O.new_env(cfg)
    pos, *_ = O.link_state(cfg, env, 1)
    assert np.allclose(pos, [0.000, 0.060, 0.373], atol=1e-3)


@pytest.fixture(scope="module")
def joint5_after_step():  # pybullet_test.py:139-204: control_joints([5],[0.3],[5.0]) + step()
    cfg = kat_config()
    env = O.new_env(cfg)
    O.control_joints(env, [5], [0.3], [5.0])
    O.sim_step(cfg, env)
    return cfg, env


def test_get_link_orientation(joint5_after_step):  # :139-153
    cfg, env = joint5_after_step
    _, orn, _, _ = O.link_state(cfg, env, 5)
    assert np.allclose(orn, [0.707, -0.02, 0.02, 0.707], atol=1e-3)


def test_get_link_velocity(joint5_after_step):  # :156-170
    cfg, env = joint5_after_step
    _, _, v, _ = O.link_state(cfg, env, 5)
    assert np.allclose(v, [-0.0068, 0.0000, 0.1186], atol=1e-3)


def test_get_link_angular_velocity(joint5_after_step):  # :173-187
    cfg, env = joint5_after_step
    _, _, _, w = O.link_state(cfg, env, 5)
    assert np.allclose(w, [0.000, -2.969, 0.000], atol=1e-3)


def test_get_joint_angle(joint5_after_step):  # :190-204
    _, env = joint5_after_step
    assert np.allclose(env.q[5], 0.063, atol=1e-3)


def test_inverse_kinematics():  # pybullet_test.py:254-266
    cfg = kat_config()
    q = O.inverse_kinematics(cfg, np.zeros(9), 6, [0.4, 0.5, 0.6], [0.707, -0.02, 0.02, 0.707])
    assert np.allclose(q, [1.000, 1.223, -1.113, -0.021, -0.917, 0.666, -0.499, 0.0, 0.0], atol=1e-3)


def test_box_free_fall_velocity():  # pybullet_test.py:56-64 (1 kg box, half extents 0.5, one step())
    cfg = O.config("push", base=(0, 0, 0), has_table=0, has_plane=0, has_robot=0, object_half=(0.5, 0.5, 0.5),
                   object_mass=1.0)
    env = O.new_env(cfg)
    O.sim_step(cfg, env)
    assert np.allclose(np.array(env.obj[0].vel), [0.0, 0.0, -0.392], atol=1e-3)
    assert np.allclose(np.array(env.obj[0].omg), 0.0, atol=1e-3)  # :89-97
    e = np.zeros(3)
    O.lib().po_euler_from_quaternion(np.array(env.obj[0].quat).ctypes.data_as(O.C.POINTER(O.C.c_double)),
                                     e.ctypes.data_as(O.C.POINTER(O.C.c_double)))
    assert np.allclose(e, 0.0, atol=1e-3)  # :78-86
    assert np.allclose(np.array(env.obj[0].quat), [0, 0, 0, 1], atol=1e-3)  # :67-75


def test_set_joint_angles_roundtrip():  # pybullet_test.py:221-251
    cfg = kat_config()
    env = O.new_env(cfg)
    env.q[3], env.q[4] = 0.4, 0.5
    assert env.q[3] == 0.4 and env.q[4] == 0.5


def test_euler_from_quaternion_branches():
    for q in ([0, 0, 0, 1], [0.707, -0.02, 0.02, 0.707], [0, 0.7071068, 0, 0.7071068], [0, -0.7071068, 0, 0.7071068]):
        q = np.array(q, float) / np.linalg.norm(q)
        e = np.zeros(3)
        O.lib().po_euler_from_quaternion(q.ctypes.data_as(O.C.POINTER(O.C.c_double)),
                                         e.ctypes.data_as(O.C.POINTER(O.C.c_double)))
        # reconstruct (XYZ fixed axes: R = Rz(yaw) Ry(pitch) Rx(roll))
        h = e / 2  # btQuaternion::setEulerZYX (getQuaternionFromEuler)
        cr, sr, cp, sp, cy, sy = np.cos(h[0]), np.sin(h[0]), np.cos(h[1]), np.sin(h[1]), np.cos(h[2]), np.sin(h[2])
        w = cr * cp * cy + sr * sp * sy
        x = sr * cp * cy - cr * sp * sy
        y = cr * sp * cy + sr * cp * sy
        z = cr * cp * sy - sr * sp * cy
        r = np.array([x, y, z, w])
        assert min(np.abs(r - q).max(), np.abs(r + q).max()) < 1e-4


def test_neutral_pose_observation():
    # Panda.reset -> neutral joints (panda.py:121-126); ee = grasptarget COM
    cfg = O.config("reach")
    env = O.new_env(cfg)
    obs, ag, dg = O.reset(cfg, env, seed=0)
    assert np.allclose(obs[:3], [0.0384397, 0.0, 0.1974001], atol=1e-6)
    assert np.all(obs[3:6] == 0.0)
    assert np.array_equal(ag, obs[:3])


@pytest.mark.parametrize("seed", [0, 1, 2**32 - 1, 2**32, 2**63 + 7, 2**64 - 1])
def test_pcg64_matches_numpy(seed):
    st = O.pcg64_seed(seed)
    bg = np.random.PCG64(np.random.SeedSequence(seed))
    assert [O.pcg64_next(st) for _ in range(16)] == [int(bg.random_raw()) for _ in range(16)]


@pytest.mark.parametrize("task", ["reach", "push", "pick_and_place", "slide", "stack", "flip"])
def test_goal_sampling_golden(task, golden):
    cfg = O.config(task)
    for i, s in enumerate(golden["seeds"]):
        env = O.new_env(cfg)
        for r in range(golden[f"{task}_object"].shape[1]):
            O.reset(cfg, env, seed=int(s) if r == 0 else None)
            if task != "flip":  # Flip's goal is not seeded in the reference (flip.py:70-72)
                assert np.array_equal(np.array(env.goal)[:O.goal_dim(cfg)], golden[f"{task}_goal"][i, r])
            if task == "stack":
                assert np.array_equal(np.array(env.obj[0].pos), golden["stack_object"][i, r, :3])
                assert np.array_equal(np.array(env.obj[1].pos), golden["stack_object"][i, r, 3:])
            elif task != "reach":
                assert np.array_equal(np.array(env.obj[0].pos), golden[f"{task}_object"][i, r])


def test_flip_goal_is_a_unit_quaternion_stream():
    cfg = O.config("flip")
    env = O.new_env(cfg)
    goals = []
    for r in range(400):
        O.reset(cfg, env, seed=77 if r == 0 else None)
        goals.append(np.array(env.goal[:4]))
    g = np.array(goals)
    assert np.allclose(np.linalg.norm(g, axis=1), 1.0)
    # uniform over rotations: E[q_i^2] = 1/4, components symmetric
    assert np.allclose((g ** 2).mean(0), 0.25, atol=0.05) and np.allclose(g.mean(0), 0.0, atol=0.1)
    env2 = O.new_env(cfg)
    O.reset(cfg, env2, seed=77)
    assert np.array_equal(np.array(env2.goal[:4]), g[0])  # seeded: reproducible


@pytest.mark.parametrize("task", ["stack", "flip"])
def test_stack_flip_reward_goldens(task, golden):
    ag, dg = golden[f"{task}_ag"], golden[f"{task}_dg"]
    for rt in ("sparse", "dense"):
        r = np.array([O.compute_reward(rt, a, d, task=task) for a, d in zip(ag, dg)], np.float32)
        assert np.array_equal(r.view(np.uint32), golden[f"{task}_reward_{rt}"].view(np.uint32)), rt
    su = np.array([O.is_success(a, d, task=task) for a, d in zip(ag, dg)])
    assert np.array_equal(su, golden[f"{task}_success"])


def test_reward_and_success_golden(golden):
    ag, dg = golden["reward_ag"], golden["reward_dg"]
    sp = np.array([O.compute_reward("sparse", a, d) for a, d in zip(ag, dg)], np.float32)
    de = np.array([O.compute_reward("dense", a, d) for a, d in zip(ag, dg)], np.float32)
    su = np.array([O.is_success(a, d) for a, d in zip(ag, dg)])
    assert np.array_equal(sp.view(np.uint32), golden["reward_sparse"].view(np.uint32))
    assert np.array_equal(de.view(np.uint32), golden["reward_dense"].view(np.uint32))
    assert np.array_equal(su, golden["success"])


def _rollout(task, seed, actions, control="ee"):
    cfg = O.config(task, control=control)
    env = O.new_env(cfg)
    O.reset(cfg, env, seed=seed)
    out = None
    for a in actions:
        out = O.step(cfg, env, np.asarray(a, np.float32), autoreset=True)
    return out


@pytest.mark.parametrize("task,seed,na", [("reach", 12345, 3), ("push", 6789, 3), ("pick_and_place", 794512, 4)])
def test_seed_determinism(task, seed, na):  # seed_test.py:7-122
    actions = np.random.default_rng(seed).uniform(-1, 1, size=(6, na))
    a = _rollout(task, seed, actions)
    b = _rollout(task, seed, actions)
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y)


def test_save_and_restore_bit_equal():  # save_and_restore_test.py:9-27
    cfg = O.config("reach")
    env = O.new_env(cfg)
    O.reset(cfg, env, seed=3)
    saved = copy.deepcopy(env)
    action = np.array([0.3, -0.2, 0.5], np.float32)
    o1 = O.step(cfg, env, action)
    O.reset(cfg, env, seed=99)
    env = copy.deepcopy(saved)
    o2 = O.step(cfg, env, action)
    for x, y in zip(o1[:3], o2[:3]):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("task", ["reach", "push", "pick_and_place"])
def test_random_rollout_is_finite_and_bounded(task):  # envs_test.py:6-14 (shortened)
    cfg = O.config(task)
    env = O.new_env(cfg)
    O.reset(cfg, env, seed=1)
    rng = np.random.default_rng(0)
    na = O.action_dim(cfg)
    resets = 0
    for _ in range(120):
        obs, ag, dg, r, te, tr = O.step(cfg, env, rng.uniform(-1, 1, na).astype(np.float32), autoreset=True)
        assert np.all(np.isfinite(obs)) and np.all(np.abs(obs) < 10.0)
        resets += te or tr
    assert resets >= 2  # TimeLimit(50) fired


def _perturbed_step_spread(task, control, steps=2, n=32, rel=6e-8):
    cfg = O.config(task, control=control)
    rng = np.random.default_rng(7)
    worst = np.zeros(O.obs_dim(cfg))
    for s in range(steps):
        a = rng.uniform(-1, 1, size=(n, O.action_dim(cfg))).astype(np.float32)
        for i in range(n):
            e = O.new_env(cfg)
            O.reset(cfg, e, seed=12345 + i)
            for k in range(s):
                O.step(cfg, e, a[(i + k) % n])
            e2 = copy.deepcopy(e)
            pr = np.random.default_rng(i)
            for d in range(9):
                e2.q[d] *= 1 + rel * pr.standard_normal()
                e2.qd[d] *= 1 + rel * pr.standard_normal()
            o1, *_ = O.step(cfg, e, a[i])
            o2, *_ = O.step(cfg, e2, a[i])
            worst = np.maximum(worst, np.abs(o1 - o2))
    return worst


def test_pick_and_place_conditioning():
    """Documents the model's conditioning that sets the GPU parity bounds:
    fp32-ulp-sized state perturbations move Push's ee by <1e-5 but
    PickAndPlace's ee/finger width by ~1e-4..1e-3 in the fp64 oracle itself."""
    push = _perturbed_step_spread("push", "ee")
    pnp = _perturbed_step_spread("pick_and_place", "ee")
    assert push[:3].max() < 1e-5
    assert pnp[:3].max() > 10 * push[:3].max()


@pytest.mark.parametrize("task", ["push", "stack"])
def test_threaded_batch_step_matches_serial(task):
    """po_step_batch over OpenMP threads (bench.py's cpu_baseline leg) gives the
    serial loop's results bit for bit: envs share no mutable state."""
    cfg = O.config(task)
    n, na, od = 24, O.action_dim(cfg), O.obs_dim(cfg)
    fp = lambda a: a.ctypes.data_as(O.C.POINTER(O.C.c_float))
    u8 = lambda a: a.ctypes.data_as(O.C.POINTER(O.C.c_uint8))
    acts = np.random.default_rng(5).uniform(-1, 1, size=(4, n, na)).astype(np.float32)
    outs = []
    for threads in (1, 4):
        assert O.lib().po_set_threads(threads) >= 1
        envs = (O.Env * n)()
        for i in range(n):
            O.lib().po_init_env(O.C.byref(cfg), O.C.byref(envs[i]))
            O.lib().po_reset(O.C.byref(cfg), O.C.byref(envs[i]), 1, 100 + i, None, None, None)
        obs = np.zeros((n, od), np.float32)
        ag, dg = np.zeros((n, 6), np.float32), np.zeros((n, 6), np.float32)
        rew, te, tr = np.zeros(n, np.float32), np.zeros(n, np.uint8), np.zeros(n, np.uint8)
        for a in acts:
            O.lib().po_step_batch(O.C.byref(cfg), envs, n, fp(a), fp(obs), fp(ag), fp(dg), fp(rew), u8(te), u8(tr),
                                  1, None)
        outs.append((obs.copy(), rew.copy()))
    O.lib().po_set_threads(1)
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])


def test_oracle_clean_under_asan_ubsan():
    """the CPU restatement built with AddressSanitizer and
    UndefinedBehaviorSanitizer (oracle/Makefile `asan`, any report fatal),
    driven through every entry point, all tasks and both control modes."""
    import subprocess

    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    subprocess.run(["make", "-s", "-C", here, "asan"], check=True)
    out = subprocess.run([os.path.join(here, "build", "asan_check")], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "clean" in out.stdout


def test_finger_limit_branch_sensitivity():
    """The mechanism behind the free-gripper tolerances (DESIGN.md §6,
    tests/test_gpu_parity.py TOL): in the first step of the teacher-forced
    test's PickAndPlace batch (seeds 12345 + i), envs whose action closes the
    gripper onto its lower limit from q = 0.  For some of them a 1e-9 relative
    change of joint 2 moves the end effector by more than 1e-4 m after one
    step, because on some substep a finger lands on the free side of its limit
    (the row is skipped) in one run and not in the other, and the 170 N motor
    drives it millimetres past the limit within one substep.  Prints the
    per-substep trace of the first such env (profiles/r02a_finger_limit_trace.txt)."""
    import ctypes as C

    cfg = O.config("pick_and_place", "ee")
    B = 64
    envs = [O.new_env(cfg) for _ in range(B)]
    for i, e in enumerate(envs):
        O.reset(cfg, e, seed=12345 + i)
    acts = np.random.default_rng(7).uniform(-1, 1, size=(B, 4)).astype(np.float32)
    found = []
    for i in range(B):
        a = acts[i]
        if a[3] >= 0:
            continue  # opening: no closing onto the limit
        runs = []
        for eps in (0.0, 1e-9):
            e = O.Env()
            C.memmove(C.byref(e), C.byref(envs[i]), C.sizeof(O.Env))
            e.q[1] *= 1 + eps
            p, *_ = O.link_state(cfg, e, 11)
            tgt = np.array([p[k] + float(np.float32(a[k] * np.float32(0.05))) for k in range(3)])
            qik = O.inverse_kinematics(cfg, np.array(e.q), 11, tgt, [1, 0, 0, 0])
            w = (e.q[7] + e.q[8]) + float(np.float32(a[3] * np.float32(0.2)))
            O.control_joints(e, [0, 1, 2, 3, 4, 5, 6, 9, 10], list(qik[:7]) + [w / 2, w / 2],
                             [87, 87, 87, 87, 12, 120, 120, 170, 170])
            trace = []
            for _ in range(20):
                O.lib().po_substep(C.byref(cfg), C.byref(e), None)
                trace.append((np.array(e.q), np.array(e.qd)))
            runs.append((trace, O.link_state(cfg, e, 11)[0]))
        overshoot = ([min(q[7], q[8]) < -5e-3 for q, _ in runs[0][0]], [min(q[7], q[8]) < -5e-3 for q, _ in runs[1][0]])
        if np.abs(runs[0][1] - runs[1][1]).max() > 1e-4 and overshoot[0] != overshoot[1]:
            found.append(i)
            if len(found) == 1:
                print(f"env {i}")
                for s, ((q0, v0), (q1, v1)) in enumerate(zip(runs[0][0], runs[1][0])):
                    print(f"substep {s:2d}: |dq| {np.abs(q0 - q1).max():.1e} |dqd| {np.abs(v0 - v1).max():.1e}  "
                          f"fingers q {q0[7]:+.3e} {q0[8]:+.3e} / {q1[7]:+.3e} {q1[8]:+.3e}")
    print("envs whose finger-limit branch flips under a 1e-9 change of joint 2:", found)
    assert found


def test_event_signature_tracks_contact_and_limit_changes():
    """po_env.event_sig (test bookkeeping for the event-onset parity tests):
    unchanged while the discrete state is (a cube resting on the table, the
    arm in free motion), counted once a contact appears (a box dropped onto
    the table) and it is part of no physics (same trajectory with and
    without reading it)."""
    cfg = O.config("push")
    env = O.new_env(cfg)
    O.reset(cfg, env, seed=4)
    O.step(cfg, env, np.zeros(3, np.float32))
    assert env.event_sig >> 63 == 1 and env.event_changes == 0  # resting cube: 4 ground contacts
    # lift the cube 5 cm and let it fall: the ground contacts break, then re-form
    env.obj[0].pos[2] += 0.05
    for _ in range(10):
        O.step(cfg, env, np.zeros(3, np.float32))
    assert env.event_changes >= 2
    # a joint-limit row appearing is an event: drive joint 0 to its upper limit
    jc = O.config("reach", control="joints")
    e = O.new_env(jc)
    O.reset(jc, e, seed=0)
    O.step(jc, e, np.zeros(7, np.float32))
    base = e.event_changes
    e.q[0] = 2.9671 + 1e-3  # joint 0 upper limit (panda_model.h PM_DOF_TABLE)
    O.step(jc, e, np.zeros(7, np.float32))
    assert e.event_changes > base and e.event_kinds & 2
    assert env.event_kinds & 1  # the cube's ground contacts changed above


def test_state_noise_hook_moves_state_by_fp32_ulps():
    """po_set_state_noise: every state component moves by at most `ulps`
    fp32 ulps per substep and the hook is off at 0 (bit-equal to no hook)."""
    cfg = O.config("push")
    a = np.array([0.2, -0.1, 0.3], np.float32)
    e0, e1, e2 = O.new_env(cfg), O.new_env(cfg), O.new_env(cfg)
    for e in (e0, e1, e2):
        O.reset(cfg, e, seed=9)
    O.sim_step(cfg, e0)
    O.set_state_noise(0.0)
    O.sim_step(cfg, e1)
    assert np.array_equal(np.array(e0.q), np.array(e1.q)) and np.array_equal(np.array(e0.qd), np.array(e1.qd))
    O.set_state_noise(1.0, seed=3)
    try:
        O.lib().po_substep(O.C.byref(cfg), O.C.byref(e2), None)
    finally:
        O.set_state_noise(0.0)
    e3 = O.new_env(cfg)
    O.reset(cfg, e3, seed=9)
    O.lib().po_substep(O.C.byref(cfg), O.C.byref(e3), None)
    for x, y in ((e2.q, e3.q), (e2.qd, e3.qd), (e2.obj[0].pos, e3.obj[0].pos)):
        x, y = np.array(x), np.array(y)
        ulp = np.spacing(np.abs(y).astype(np.float32)).astype(np.float64)
        assert np.all(np.abs(x - y) <= ulp * 1.0000001)
        assert np.any(x != y)


# ------------------------------------------------------------------------------
# Lagrangian-mechanics identities.  The oracle's mass matrix is a sum over
# links of J^T m J + Jw^T I Jw (panda_oracle.c), its bias forces a world-frame
# recursive Newton-Euler pass, and its link COM positions plain FK: three
# separate code paths, so these identities pin its dynamics without any
# PyBullet output (the GPU kernels -- composite-rigid-body M, prefix-sum RNEA --
# are held to the oracle by tests/test_gpu_parity.py).
def _link_masses():
    import re
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                           "panda_model.h")) as f:
        h = f.read()
    body = h[h.index("#define PM_LINK_TABLE(X)"):h.index("/* DoF -> link index")]
    rows = re.findall(r"X\(([^)]*)\)", body.replace("\\\n", " "))
    masses = {}
    for r in rows:
        f = [x.strip() for x in r.split(",")]
        if f[0].isdigit():
            masses[int(f[0])] = float(f[13])
    return masses


def _random_q(rng):
    lo = np.array([-2.9, -1.7, -2.9, -3.0, -2.9, 0.0, -2.9, 0.0, 0.0])
    hi = np.array([2.9, 1.7, 2.9, -0.1, 2.9, 3.7, 2.9, 0.04, 0.04])
    return lo + (hi - lo) * rng.random(9)


def test_mass_matrix_is_symmetric_positive_definite():
    cfg, rng = kat_config(), np.random.default_rng(1)
    for _ in range(20):
        M = O.mass_matrix(cfg, _random_q(rng))
        assert np.allclose(M, M.T, atol=1e-14)
        assert np.linalg.eigvalsh(M).min() > 0


def test_gravity_torque_is_the_potential_gradient():
    """h(q, 0) = dV/dq with V = sum_i m_i g z_i over the links' COM heights."""
    cfg, rng = kat_config(), np.random.default_rng(2)
    masses = _link_masses()
    assert len(masses) == 12 and all(masses[i] > 0 for i in (0, 1, 2, 3, 4, 5, 6, 8, 9, 10))

    def potential(q):
        env = O.new_env(cfg)
        env.q[:] = q
        return sum(m * 9.81 * O.link_state(cfg, env, link)[0][2] for link, m in masses.items() if m > 0)

    for _ in range(10):
        q = _random_q(rng)
        g = O.bias_forces(cfg, q, np.zeros(9))
        eps = 1e-6
        grad = np.array([(potential(q + eps * e) - potential(q - eps * e)) / (2 * eps) for e in np.eye(9)])
        assert np.allclose(g, grad, rtol=1e-6, atol=1e-7), (g, grad)


def test_coriolis_terms_follow_from_the_mass_matrix():
    """The part of h(q, qd) even in qd, less gravity, is C(q, qd) qd with
    (C qd)_i = sum_jk (dM_ij/dq_k - 1/2 dM_jk/dq_i) qd_j qd_k (Christoffel
    symbols of M).  btMultiBody's link damping is odd in the velocity
    (m d (1 + |v|) v), so it cancels in h(q, qd) + h(q, -qd)."""
    cfg, rng = kat_config(), np.random.default_rng(3)
    for _ in range(10):
        q, qd = _random_q(rng), rng.normal(0.0, 1.0, 9)
        even = 0.5 * (O.bias_forces(cfg, q, qd) + O.bias_forces(cfg, q, -qd)) - O.bias_forces(cfg, q, np.zeros(9))
        eps = 1e-6
        dM = np.stack([(O.mass_matrix(cfg, q + eps * e) - O.mass_matrix(cfg, q - eps * e)) / (2 * eps)
                       for e in np.eye(9)])  # dM[k] = dM/dq_k
        cqd = np.einsum("kij,j,k->i", dM, qd, qd) - 0.5 * np.einsum("ijk,j,k->i", dM, qd, qd)
        assert np.allclose(even, cqd, rtol=1e-5, atol=1e-7), (even, cqd)


# ---- contact mechanics identities (independent of PyBullet: Coulomb friction
# and statics).  The contact constants the oracle shares with the kernels
# (include/panda_model.h) cannot show up in GPU-vs-oracle tests; these pin the
# oracle's contact solve to mechanics itself.

def _sliding_run(task, v0, steps=80, settle=25):
    """The task's object alone on its table (no robot), settled, then given a
    horizontal velocity v0 (m/s, 2-vector); returns (cfg, mu, p0, positions,
    velocities, angular velocities) per step."""
    cfg = O.config(task, has_robot=0, has_plane=0)
    env = O.new_env(cfg)
    O.reset(cfg, env, seed=1)
    for _ in range(settle):
        O.sim_step(cfg, env)
    p0 = np.array(env.obj[0].pos)
    env.obj[0].vel[0], env.obj[0].vel[1] = v0
    ps, vs, ws = [], [], []
    for _ in range(steps):
        O.sim_step(cfg, env)
        ps.append(np.array(env.obj[0].pos))
        vs.append(np.array(env.obj[0].vel))
        ws.append(np.array(env.obj[0].omg))
    # friction coefficients multiply (object x table 0.5; panda_oracle.c contact setup)
    mu = cfg.object_friction * 0.5
    return cfg, mu, p0, np.array(ps), np.array(vs), np.array(ws)


@pytest.mark.parametrize("task,v0,tol", [("push", (-0.5, 0.0), 0.02), ("push", (-0.6, 0.45), 0.02),
                                         ("pick_and_place", (-1.0, 0.0), 0.02), ("slide", (-0.3, 0.1), 0.06)])
def test_sliding_object_decelerates_at_mu_g(task, v0, tol):
    """A cube (cylinder for Slide) sliding on the table: Coulomb friction
    decelerates it at mu g along its velocity, it stops after v0^2 / (2 mu g),
    and it neither lifts, sinks nor turns (the four corner contacts share the
    load).  tol: relative (the cylinder's ground contacts tilt its friction
    cone's support by a few percent)."""
    cfg, mu, p0, ps, vs, ws = _sliding_run(task, v0)
    g = 9.81
    speed0 = float(np.hypot(*v0))
    speed = np.hypot(vs[:, 0], vs[:, 1])
    t = 0.04 * (np.arange(len(speed)) + 1)
    moving = speed > 0.1 * speed0
    decel = -np.polyfit(t[moving], speed[moving], 1)[0]
    assert abs(decel - mu * g) <= tol * mu * g, (decel, mu * g)
    dist = float(np.hypot(*(ps[-1, :2] - p0[:2])))
    assert abs(dist - speed0 ** 2 / (2 * mu * g)) <= 2.5 * tol * speed0 ** 2 / (2 * mu * g), dist
    assert speed[-1] < 1e-3  # at rest again
    # the path is straight along v0
    d = (ps[-1, :2] - p0[:2]) / dist
    assert abs(d @ np.array(v0) / speed0 - 1.0) < 1e-3
    assert np.all(np.abs(ps[:, 2] - p0[2]) < 2e-4) and np.all(np.abs(ws) < 0.05)


@pytest.mark.parametrize("task", ["push", "slide", "pick_and_place"])
def test_resting_object_normal_impulses_carry_its_weight(task):
    """Statics of the warm-started solve: a settled object's ground normal
    impulses (the contact cache the next substep starts from) sum to m g dt
    per substep, and it does not drift faster than the solver resolves: PGS
    stops at a squared row residual of 1e-7, so a tangential creep below
    sqrt(1e-7) = 3.2e-4 m/s is left alone by the friction rows (a cube settles
    with ~3e-5 m/s of creep, as Bullet's early-terminated solve allows)."""
    cfg = O.config(task, has_robot=0, has_plane=0)
    env = O.new_env(cfg)
    O.reset(cfg, env, seed=3)
    for _ in range(25):
        O.sim_step(cfg, env)
    p = np.array(env.obj[0].pos)
    for _ in range(25):
        O.sim_step(cfg, env)
    lam = sum(env.cache.ground_lam[0][k] for k in range(4))
    assert abs(lam - cfg.object_mass * 9.81 / 500) < 1e-9 * cfg.object_mass
    assert np.all(np.abs(np.array(env.obj[0].pos) - p) < 1e-4)
    assert abs(env.obj[0].pos[2] - p[2]) < 1e-8
    assert np.all(np.abs(np.array(env.obj[0].vel)) < 1e-4)
