"""CPU tests of the host layer's task logic (pandasim.tasks / utils / core):
draw order, goal arithmetic, distance, reward and success against the
reference task goldens, with a recording stand-in for PandaSim whose per-env
generators are numpy's own PCG64 (the device kernels are covered by the -m gpu
tests)."""
import os
import numpy as np
import pytest
import torch

from pandasim.core import TimeLimit, np_random
from pandasim.tasks import Flip, PickAndPlace, Push, Reach, Slide, Stack
from pandasim.utils import angle_distance, distance


class FakeSim:
    """Scene calls are recorded; uniform() draws from numpy Generators."""

    def __init__(self, n):
        self.num_envs, self.device = n, torch.device("cpu")
        self.gens = [np.random.Generator(np.random.PCG64(np.random.SeedSequence(i))) for i in range(n)]
        self.calls = []
        self.poses = {}

    def no_rendering(self):
        import contextlib
        return contextlib.nullcontext()

    def __getattr__(self, name):
        if name.startswith(("create_", "place_")):
            return lambda *a, **k: self.calls.append(name)
        raise AttributeError(name)

    def seed(self, seeds):
        self.gens = [np.random.Generator(np.random.PCG64(np.random.SeedSequence(int(s)))) for s in
                     seeds.numpy().view(np.uint64)]

    def uniform(self, low, high):
        return torch.from_numpy(np.stack([g.uniform(low, high) for g in self.gens]))

    def random_rotation(self):
        return torch.tensor([[0.0, 0.0, 0.0, 1.0]] * self.num_envs, dtype=torch.float64)

    def set_base_pose(self, body, position, orientation):
        self.poses[body] = torch.as_tensor(position).clone()
        self.orns = getattr(self, "orns", {})
        self.orns[body] = torch.as_tensor(np.asarray(orientation) if not torch.is_tensor(orientation)
                                          else orientation).clone()

    def get_base_position(self, body):
        return self.poses[body].to(torch.float32)


CLASSES = {"push": Push, "pick_and_place": PickAndPlace, "slide": Slide, "stack": Stack, "flip": Flip}


@pytest.mark.parametrize("task", ["reach", "push", "pick_and_place", "slide", "stack", "flip"])
def test_task_reset_draw_order_matches_goldens(golden, task):
    seeds = golden["seeds"]
    sim = FakeSim(len(seeds))
    if task == "reach":
        t = Reach(sim, get_ee_position=lambda: torch.zeros(len(seeds), 3))
    else:
        t = CLASSES[task](sim)
    assert "create_table" in sim.calls and "create_plane" in sim.calls
    for r in range(golden[f"{task}_object"].shape[1]):
        if r == 0:
            t.np_random, _ = np_random(sim, seeds)
        t.reset()
        if task == "flip":
            assert np.array_equal(sim.orns["target"].numpy(), t.get_goal().numpy())
            assert np.array_equal(sim.orns["object"], np.zeros(3))  # flip.py:77: Euler zeros
        elif task == "stack":
            assert np.array_equal(t.get_goal().numpy(), golden["stack_goal"][:, r])
            assert np.array_equal(sim.poses["target1"].numpy(), golden["stack_goal"][:, r, :3])
            assert np.array_equal(sim.poses["target2"].numpy(), golden["stack_goal"][:, r, 3:])
            got = np.concatenate([sim.poses["object1"].numpy(), sim.poses["object2"].numpy()], -1)
            assert np.array_equal(got, golden["stack_object"][:, r])
            continue
        else:
            assert np.array_equal(t.get_goal().numpy(), golden[f"{task}_goal"][:, r])
            assert np.array_equal(sim.poses["target"].numpy(), golden[f"{task}_goal"][:, r])
        if task != "reach":
            assert np.array_equal(sim.poses["object"].numpy(), golden[f"{task}_object"][:, r])


@pytest.mark.parametrize("task", ["stack", "flip"])
def test_stack_flip_reward_success_goldens_host(golden, task):
    """The host fallback of goal_reward_and_success (CPU tensors): Stack's
    6-D distance and Flip's 1 - <q, g>^2 against the reference's functions."""
    ag, dg = torch.from_numpy(golden[f"{task}_ag"]), torch.from_numpy(golden[f"{task}_dg"])
    for rt in ("sparse", "dense"):
        t = CLASSES[task](FakeSim(1), reward_type=rt)
        r = t.compute_reward(ag, dg, {}).numpy()
        assert np.array_equal(r.view(np.uint32), golden[f"{task}_reward_{rt}"].view(np.uint32)), rt
        assert np.array_equal(t.is_success(ag, dg).numpy(), golden[f"{task}_success"])


def test_distance_reward_success_goldens(golden):
    ag, dg = torch.from_numpy(golden["reward_ag"]), torch.from_numpy(golden["reward_dg"])
    assert np.array_equal(distance(ag, dg).numpy(), np.linalg.norm(golden["reward_ag"] - golden["reward_dg"], axis=-1))
    for rt in ("sparse", "dense"):
        t = Push(FakeSim(1), reward_type=rt)
        r = t.compute_reward(ag, dg, {}).numpy()
        assert r.dtype == np.float32
        assert np.array_equal(r.view(np.uint32), golden[f"reward_{rt}"].view(np.uint32))
        her = t.compute_reward(torch.from_numpy(golden["her_ag"]), torch.from_numpy(golden["her_dg"]), {}).numpy()
        assert np.array_equal(her.view(np.uint32), golden[f"her_reward_{rt}"].view(np.uint32))
    assert np.array_equal(Push(FakeSim(1)).is_success(ag, dg).numpy(), golden["success"])


def test_float32_distance_is_correctly_rounded():
    rng = np.random.default_rng(0)
    a = rng.uniform(-1, 1, size=(4096, 3)).astype(np.float32)
    b = rng.uniform(-1, 1, size=(4096, 3)).astype(np.float32)
    got = distance(torch.from_numpy(a), torch.from_numpy(b)).numpy()
    assert got.dtype == np.float32
    assert np.array_equal(got, np.linalg.norm(a - b, axis=-1))


def test_angle_distance():
    a = np.array([[0.0, 0.0, 0.0, 1.0], [0.0, 0.0, 1.0, 0.0]])
    b = np.array([[0.0, 0.0, 0.0, 1.0], [0.0, 0.0, 0.0, 1.0]])
    assert np.allclose(angle_distance(torch.from_numpy(a), torch.from_numpy(b)).numpy(), [0.0, 1.0])


def test_distance_shape_mismatch_asserts():  # utils.py:14
    with pytest.raises(AssertionError):
        distance(torch.zeros(2, 3), torch.zeros(3, 3))


def test_time_limit_wrapper():
    class Dummy:
        num_envs, device = 3, torch.device("cpu")

        def reset(self, **kw):
            return {}, {}

        def step(self, a):
            z = torch.zeros(3, dtype=torch.bool)
            return {}, torch.zeros(3), z, z, {}

    env = TimeLimit(Dummy(), 2)
    env.reset()
    assert not env.step(None)[3].any()
    assert env.step(None)[3].all()
    env.reset()
    assert not env.step(None)[3].any()


def _model_header():
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                           "panda_model.h")) as f:
        return f.read()


def _link_aabbs(h):
    """{link: (lx, ly, lz)} of PM_LINK_TABLE (the last three numbers of each row)."""
    import re
    out = {}
    body = h[h.index("#define PM_LINK_TABLE(X)"):h.index("/* DoF -> link index")]
    for m in re.finditer(r"X\((\d+),([^)]*)\)", body.replace("\\\n", " ")):
        vals = [v.strip() for v in m.group(2).split(",")]
        out[int(m.group(1))] = tuple(float(v) for v in vals[-3:])
    return out


def _boxes(h):
    import re
    body = h[h.index("#define PM_BOX_TABLE(X)"):h.index("#define PM_BOX_CONTACTS")]
    return [tuple(float(v) for v in m.groups()) for m in re.finditer(
        r"X\((\d+), ([-0-9.]+), ([-0-9.]+), ([-0-9.]+), ([-0-9.]+), ([-0-9.]+), ([-0-9.]+), ([-0-9.]+)\)", body)]


def test_gripper_proxies_follow_the_reference_hulls():
    """The hand and finger constants of include/panda_model.h against the
    hulls the reference ships (tests/golden/panda_gripper_hulls.npz, from
    contact_graspnet/gripper_models/panda_gripper/{hand,finger}.stl by
    tests/golden/make_gripper_golden.py, mapped to the URDF frames):
      * inertia AABBs (PyBullet derives link inertia from the collision
        AABB): hand = its hull above the flange plane (z >= 0) + Bullet's
        1 mm convex margin per side; fingers = the finger hull's extents.
        The 34 hand vertices below z = 0 are left out for a measured reason:
        with them the joint-5 KAT's angular velocity is -2.949 instead of the
        reference's -2.969 +- 1e-3;
      * collision boxes: each finger the finger hull's AABB (link 10 turned by
        pi about z), the palm the AABB of the hand hull at z >= 0.03;
      * the obj's fingers, placed fully open, are the same hull at the finger
        joint origin (z = 0.0584) +- the 0.04 m opening;
      * the pads cover contact-graspnet's finger control points
        (gripper_control_points/panda.npy: z = 0.0753 .. 0.1053 m in the hand
        frame, 0.0527 m either side of the centre line, gripper open)."""
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "panda_gripper_hulls.npz"))
    hand, finger = g["hand"], g["finger_left"]
    h = _model_header()
    aabb = _link_aabbs(h)
    up = hand[hand[:, 2] >= 0.0]
    assert len(up) == 68 and len(hand) == 102
    assert np.allclose(aabb[8], up.max(0) - up.min(0) + 0.002, atol=1e-4), aabb[8]
    ext = finger.max(0) - finger.min(0)
    assert np.allclose(aabb[9], ext, atol=1e-4) and np.allclose(aabb[10], ext, atol=1e-4)
    boxes = _boxes(h)
    assert [int(b[0]) for b in boxes] == [9, 10, 8]
    c, hh = (finger.max(0) + finger.min(0)) / 2, (finger.max(0) - finger.min(0)) / 2
    assert np.allclose(boxes[0][1:4], c, atol=1e-4) and np.allclose(boxes[0][4:7], hh, atol=1e-4)
    assert np.allclose(boxes[1][1:4], c * [-1, -1, 1], atol=1e-4) and np.allclose(boxes[1][4:7], hh, atol=1e-4)
    palm = hand[hand[:, 2] >= 0.03]
    assert np.allclose(boxes[2][1:4], (palm.max(0) + palm.min(0)) / 2, atol=1e-4)
    assert np.allclose(boxes[2][4:7], (palm.max(0) - palm.min(0)) / 2, atol=1e-4)
    assert boxes[0][7] == boxes[1][7] == 1.0 and boxes[2][7] == 0.5  # panda.py:47-48; Bullet's default
    # the obj's fingers at full opening: the left hull at +y, the right one turned by pi
    fa, fb = g["obj_finger_a"], g["obj_finger_b"]
    left, right = (fa, fb) if fa[:, 1].mean() > 0 else (fb, fa)
    place = lambda f, sy: f * [sy, sy, 1] + [0.0, sy * 0.04, 0.0584]
    assert np.allclose(np.sort(left, 0), np.sort(place(finger, 1), 0), atol=2e-4)
    assert np.allclose(np.sort(right, 0), np.sort(place(finger, -1), 0), atol=2e-4)
    # the pads cover the control points (gripper open, finger joint at z 0.0584)
    fy0, fy1 = 0.04 + boxes[0][2] - boxes[0][5], 0.04 + boxes[0][2] + boxes[0][5]
    fz0, fz1 = 0.0584 + boxes[0][3] - boxes[0][6], 0.0584 + boxes[0][3] + boxes[0][6]
    assert fy0 <= 0.0527 <= fy1 and fz0 <= 0.0753 and 0.1053 <= fz1


def test_gymnasium_registration_mirrors_the_reference(monkeypatch):
    """register_envs() registers the reference's 24 IDs
    (panda_gym/__init__.py:8-54: 6 tasks x {sparse, dense} x {ee, joints},
    kwargs reward_type/control_type, max_episode_steps 50, Stack 100) with
    gymnasium -- checked against a stand-in registry, as gymnasium is not
    installed in this image."""
    import importlib
    import importlib.util
    import sys
    import types

    calls = []
    gym = types.ModuleType("gymnasium")
    gym.Env = type("Env", (), {})
    envs_mod = types.ModuleType("gymnasium.envs")
    reg_mod = types.ModuleType("gymnasium.envs.registration")
    reg_mod.registry = {}

    def register(id, entry_point, kwargs, max_episode_steps):
        calls.append((id, entry_point, kwargs, max_episode_steps))
        reg_mod.registry[id] = types.SimpleNamespace(entry_point=entry_point)  # gymnasium's EnvSpec field

    reg_mod.register = register
    gym.envs = envs_mod
    envs_mod.registration = reg_mod
    for name, mod in (("gymnasium", gym), ("gymnasium.envs", envs_mod), ("gymnasium.envs.registration", reg_mod)):
        monkeypatch.setitem(sys.modules, name, mod)
    import pandasim.gym_registration as GR

    GR = importlib.reload(GR)
    try:
        ids = GR.register_envs()
        expected = []
        for reward_type in ("sparse", "dense"):
            for control_type in ("ee", "joints"):
                for name, steps in (("Reach", 50), ("Push", 50), ("Slide", 50), ("PickAndPlace", 50), ("Stack", 100),
                                    ("Flip", 50)):
                    expected.append(("Panda{}{}{}-v3".format(name, "Joints" if control_type == "joints" else "",
                                                             "Dense" if reward_type == "dense" else ""),
                                     {"reward_type": reward_type, "control_type": control_type}, steps, name))
        assert ids == [e[0] for e in expected] and len(set(ids)) == 24
        for (cid, entry, kwargs, steps), (eid, ekw, esteps, name) in zip(calls, expected):
            assert (cid, kwargs, steps) == (eid, ekw, esteps)
            mod, cls = entry.split(":")
            assert mod == "pandasim.gym_registration" and cls == f"Panda{name}GymEnv"
            assert issubclass(getattr(GR, cls), gym.Env)
        # idempotent: a second call registers nothing new
        n = len(calls)
        GR.register_envs()
        assert len(calls) == n
        # an ID another package registered (panda_gym imported first) is not
        # silently kept: it raises, and override=True points it at pandasim
        reg_mod.registry["PandaPush-v3"] = types.SimpleNamespace(entry_point="panda_gym.envs:PandaPushEnv")
        with pytest.raises(RuntimeError, match="panda_gym"):
            GR.register_envs()
        GR.register_envs(override=True)
        assert reg_mod.registry["PandaPush-v3"].entry_point == "pandasim.gym_registration:PandaPushGymEnv"
        assert len(calls) == n + 1
    finally:
        monkeypatch.undo()
        importlib.reload(GR)
    if importlib.util.find_spec("gymnasium") is None:
        with pytest.raises(ImportError):
            GR.register_envs()


def test_bench_pmc_fields_are_tied_to_the_binary(tmp_path):
    """bench.py takes roofline.traffic, valu_issue and fp32_executed from the
    committed PMC summary only while the library it loaded is the binary the
    counters were measured on (the sha256 summarize_profiles.py records);
    a mismatched or absent hash leaves the fields out ("stale")."""
    import importlib.util
    import json

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    lib = tmp_path / "libpandasim.so"
    lib.write_bytes(b"\x7fELF built once")
    good = bench.file_sha256(str(lib))
    entry = {"bytes_per_launch": 45_000_000, "valu_insts_per_launch": 10**9, "source": "profiles/x_summary.json"}
    pmc = tmp_path / "pmc_traffic.json"
    pmc.write_text(json.dumps({"W": dict(entry, lib_sha256=good), "V": dict(entry, lib_sha256="0" * 64),
                               "U": entry}))
    e, info = bench.pmc_entry("W", str(lib), str(pmc))
    assert info["status"] == "current" and e["bytes_per_launch"] == 45_000_000
    for w in ("V", "U"):  # measured on another binary, or on an unrecorded one
        e, info = bench.pmc_entry(w, str(lib), str(pmc))
        assert e is None and info["status"] == "stale"
    e, info = bench.pmc_entry("absent", str(lib), str(pmc))
    assert e is None and info["status"] == "missing"
    lib.write_bytes(b"\x7fELF rebuilt")  # the library changed after the profile
    e, info = bench.pmc_entry("W", str(lib), str(pmc))
    assert e is None and info["status"] == "stale" and info["measured_on"] == good


def test_bench_fp32_roofline_without_the_cpu_leg():
    """N > 1 (and --no-cpu-baseline) lines carry roofline.fp32 from the
    committed oracle work counts (profiles/oracle_work_counts.json, written by
    scripts/oracle_work_counts.py): present for every task, and the FLOPs per
    env-step they give match the ones the bench's own CPU leg measured."""
    import bench

    for task in ("reach", "push", "pick_and_place", "slide", "stack", "flip"):
        w = bench.committed_work_counts(task)
        assert w and w["substeps"] > 0 and w["pgs_iterations"] > 0, task
    r = bench.fp32_roofline(bench.committed_work_counts("push"), 1, 2.1e7)
    assert 5.0e5 < r["flops_per_env_step"] < 6.5e5
    assert bench.committed_work_counts("no such task") is None


def test_rim_point_culling_skips_only_invalid_candidates():
    """BoxCyl::visit (csrc/ps_physics.h) skips a cap's rim points for a wave
    when no lane's box reaches within the margin (+0.1 mm) of the cap's plane
    (DESIGN.md §12.11).  The argument: a point on the plane z = +-hh of the
    cylinder frame is at least |bc.z -+ hh| - ez from a box whose extent along
    z is bc.z +- ez, so every such rim point is an invalid candidate (distance
    >= the margin) and cannot change the picks.  Checked on random poses of
    the palm and finger boxes around the Slide cylinder, including poses
    right at the cut-off."""
    h = _model_header()
    margin = 0.005
    assert "#define PM_CONTACT_MARGIN_ROBOT 0.005" in h
    r, hh = 0.03, 0.015  # PM_SLIDE_OBJECT_SIZE / 2 radius and height: half extents (r, r, hh)
    rng = np.random.default_rng(5)
    ang = np.arange(8) * (np.pi / 4)
    skipped = 0
    for box in _boxes(h):
        xh = np.array(box[4:7])
        for _ in range(4000):
            q = rng.normal(size=4)
            q /= np.linalg.norm(q)
            w, x, y, z = q
            R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                          [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                          [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
            ez = np.abs(R[2]) @ xh
            reach = ez + margin + 1e-4
            bc = rng.uniform(-0.12, 0.12, size=3)
            if rng.random() < 0.5:  # put the box's face near a cap's plane
                cap = rng.choice([-1.0, 1.0])
                bc[2] = cap * hh + rng.choice([-1.0, 1.0]) * (reach + rng.uniform(-2e-3, 2e-3))
            for cap in (-1.0, 1.0):
                if abs(bc[2] - cap * hh) <= reach:
                    continue
                skipped += 1
                p = np.stack([r * np.cos(ang), r * np.sin(ang), np.full(8, cap * hh)], 1)
                lp = (p - bc) @ R  # the points in the box frame
                dist = np.linalg.norm(lp - np.clip(lp, -xh, xh), axis=1)
                assert dist.min() >= margin, (box, bc, cap, dist.min())
    assert skipped > 1000
