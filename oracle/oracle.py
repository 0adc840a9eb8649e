"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (panda_oracle.c).

The oracle is the fp64 CPU restatement the HIP path is checked against.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
import this module; the product package never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libpanda_oracle.so")

TASKS = {"reach": 0, "push": 1, "pick_and_place": 2, "slide": 3, "stack": 4, "flip": 5}


class Config(C.Structure):
    _fields_ = [
        ("task", C.c_int32), ("control", C.c_int32), ("reward", C.c_int32), ("block_gripper", C.c_int32),
        ("has_table", C.c_int32), ("has_plane", C.c_int32), ("n_objects", C.c_int32), ("object_shape", C.c_int32),
        ("has_robot", C.c_int32), ("reserved", C.c_int32),
        ("base", C.c_double * 3), ("object_half", C.c_double * 3),
        ("object_mass", C.c_double), ("object2_mass", C.c_double), ("object_friction", C.c_double),
        ("table_cx", C.c_double), ("table_hx", C.c_double), ("table_hy", C.c_double),
    ]


class Body(C.Structure):
    _fields_ = [("pos", C.c_double * 3), ("quat", C.c_double * 4), ("vel", C.c_double * 3), ("omg", C.c_double * 3)]


class Cache(C.Structure):
    """po_cache: the warm start's contact cache (slots per group, ids 1 + feature, 0 = empty)."""
    _fields_ = [
        ("ground_lam", (C.c_double * 4) * 2), ("robot_lam", C.c_double * 4), ("pair_lam", C.c_double * 4),
        ("pair_pt", (C.c_double * 3) * 4), ("ground_id", (C.c_int32 * 4) * 2), ("robot_id", C.c_int32 * 4),
        ("pair_n", C.c_int32), ("reserved", C.c_int32),
    ]


class Env(C.Structure):
    _fields_ = [
        ("q", C.c_double * 9), ("qd", C.c_double * 9),
        ("m_target", C.c_double * 9), ("m_kp", C.c_double * 9), ("m_kd", C.c_double * 9),
        ("m_vel", C.c_double * 9), ("m_maximp", C.c_double * 9),
        ("obj", Body * 2), ("goal", C.c_double * 6), ("elapsed", C.c_int64), ("rng", C.c_uint64 * 5),
        ("cache", Cache),
        # test bookkeeping (po_substep): discrete-state signature and its changes
        ("event_sig", C.c_uint64), ("event_changes", C.c_int64),
        ("finger_sig", C.c_uint64), ("finger_changes", C.c_int64),
        ("contact_sig", C.c_uint64), ("limit_sig", C.c_uint64), ("event_kinds", C.c_int64),
    ]


class Stats(C.Structure):
    """po_stats: work counters (panda_oracle.h)."""
    _fields_ = [(n, C.c_int64) for n in (
        "substeps", "pgs_iterations", "rows", "contacts",
        "motor_rows", "limit_rows", "ground_contacts", "robot_contacts", "pair_contacts",
        "motor_visits", "limit_visits", "ground_visits", "robot_visits", "pair_visits",
        "steps", "ik_iterations")]

    def as_dict(self) -> dict:
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


def build() -> str:
    """Compile the oracle with its Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P, D, I = C.POINTER, C.c_double, C.c_int
        L.po_default_config.argtypes = [P(Config), I, I, I]
        L.po_init_env.argtypes = [P(Config), P(Env)]
        L.po_link_state.argtypes = [P(Config), P(Env), I, P(D), P(D), P(D), P(D)]
        L.po_inverse_kinematics.argtypes = [P(Config), P(D), I, P(D), P(D), P(D)]
        L.po_control_joints.argtypes = [P(Env), I, P(C.c_int32), P(D), P(D)]
        L.po_substep.argtypes = [P(Config), P(Env), P(Stats)]
        L.po_sim_step.argtypes = [P(Config), P(Env), P(Stats)]
        L.po_euler_from_quaternion.argtypes = [P(D), P(D)]
        L.po_obs_dim.argtypes = [P(Config)]
        L.po_action_dim.argtypes = [P(Config)]
        L.po_goal_dim.argtypes = [P(Config)]
        L.po_max_episode_steps.argtypes = [P(Config)]
        L.po_flip_goal.argtypes = [P(C.c_uint64), P(D)]
        F, U8 = P(C.c_float), P(C.c_uint8)
        L.po_reset.argtypes = [P(Config), P(Env), I, C.c_uint64, F, F, F]
        L.po_get_obs.argtypes = [P(Config), P(Env), F, F, F]
        L.po_step.argtypes = [P(Config), P(Env), F, F, F, F, F, U8, U8, I, F, F, P(Stats)]
        L.po_step_batch.argtypes = [P(Config), P(Env), I, F, F, F, F, F, U8, U8, I, P(Stats)]
        L.po_set_threads.argtypes = [I]
        L.po_set_threads.restype = I
        L.po_compute_reward.argtypes = [I, I, F, P(D)]
        L.po_compute_reward.restype = C.c_float
        L.po_is_success.argtypes = [I, F, P(D)]
        L.po_is_success.restype = C.c_uint8
        L.po_pcg64_seed.argtypes = [C.c_uint64, P(C.c_uint64)]
        L.po_pcg64_next.argtypes = [P(C.c_uint64)]
        L.po_pcg64_next.restype = C.c_uint64
        L.po_pcg64_double.argtypes = [P(C.c_uint64)]
        L.po_pcg64_double.restype = C.c_double
        L.po_mass_matrix.argtypes = [P(Config), P(D), P(D)]
        L.po_bias_forces.argtypes = [P(Config), P(D), P(D), P(D)]
        L.po_link_inertia.argtypes = [I, P(D)]
        L.po_set_link_aabb.argtypes = [I, D, D, D]
        L.po_set_finger_noise.argtypes = [D, C.c_uint64]
        L.po_set_finger_bias.argtypes = [D]
        L.po_set_state_noise.argtypes = [D, C.c_uint64]
        L.po_set_pgs_log.argtypes = [C.c_void_p, C.c_int64]
        L.po_set_pgs_log.restype = C.c_int64
        L.po_set_model_mutation.argtypes = [I, D]
        L.po_set_fp32_solver.argtypes = [I]
        L.po_set_fp32_dynamics.argtypes = [I]
        L.po_set_pgs_shift.argtypes = [I]
        L.po_set_clip_bias.argtypes = [D]
        _lib = L
    return _lib


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _fp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def config(task="reach", control="ee", reward="sparse", **overrides) -> Config:
    cfg = Config()
    lib().po_default_config(C.byref(cfg), TASKS[task], 0 if control == "ee" else 1, 0 if reward == "sparse" else 1)
    for k, v in overrides.items():
        if k in ("base", "object_half"):
            for i in range(3):
                getattr(cfg, k)[i] = v[i]
        else:
            setattr(cfg, k, v)
    return cfg


def new_env(cfg: Config) -> Env:
    env = Env()
    lib().po_init_env(C.byref(cfg), C.byref(env))
    return env


def env_to_dict(env: Env) -> dict:
    return {name: np.array(getattr(env, name)) if not isinstance(getattr(env, name), int) else getattr(env, name)
            for name, _ in Env._fields_}


def link_state(cfg, env, link):
    pos, quat, v, w = np.zeros(3), np.zeros(4), np.zeros(3), np.zeros(3)
    lib().po_link_state(C.byref(cfg), C.byref(env), link, _dp(pos), _dp(quat), _dp(v), _dp(w))
    return pos, quat, v, w


def inverse_kinematics(cfg, q_start, link, pos, orn):
    q0 = np.ascontiguousarray(q_start, dtype=np.float64)
    p = np.ascontiguousarray(pos, dtype=np.float64)
    o = np.ascontiguousarray(orn, dtype=np.float64)
    out = np.zeros(9)
    lib().po_inverse_kinematics(C.byref(cfg), _dp(q0), link, _dp(p), _dp(o), _dp(out))
    return out


def control_joints(env, joints, targets, forces):
    j = np.ascontiguousarray(joints, dtype=np.int32)
    t = np.ascontiguousarray(targets, dtype=np.float64)
    f = np.ascontiguousarray(forces, dtype=np.float64)
    lib().po_control_joints(C.byref(env), len(j), j.ctypes.data_as(C.POINTER(C.c_int32)), _dp(t), _dp(f))


def sim_step(cfg, env, stats: Stats | None = None):
    lib().po_sim_step(C.byref(cfg), C.byref(env), C.byref(stats) if stats is not None else None)


def obs_dim(cfg) -> int:
    return lib().po_obs_dim(C.byref(cfg))


def action_dim(cfg) -> int:
    return lib().po_action_dim(C.byref(cfg))


def goal_dim(cfg) -> int:
    return lib().po_goal_dim(C.byref(cfg))


def max_episode_steps(cfg) -> int:
    return lib().po_max_episode_steps(C.byref(cfg))


def reset(cfg, env, seed=None):
    od, gd = obs_dim(cfg), goal_dim(cfg)
    obs, ag, dg = np.zeros(od, np.float32), np.zeros(gd, np.float32), np.zeros(gd, np.float32)
    lib().po_reset(C.byref(cfg), C.byref(env), 0 if seed is None else 1, 0 if seed is None else int(seed),
                   _fp(obs), _fp(ag), _fp(dg))
    return obs, ag, dg


def get_obs(cfg, env):
    od, gd = obs_dim(cfg), goal_dim(cfg)
    obs, ag, dg = np.zeros(od, np.float32), np.zeros(gd, np.float32), np.zeros(gd, np.float32)
    lib().po_get_obs(C.byref(cfg), C.byref(env), _fp(obs), _fp(ag), _fp(dg))
    return obs, ag, dg


def step(cfg, env, action, autoreset=False, stats: Stats | None = None):
    od, gd = obs_dim(cfg), goal_dim(cfg)
    a = np.ascontiguousarray(action, dtype=np.float32)
    obs, ag, dg = np.zeros(od, np.float32), np.zeros(gd, np.float32), np.zeros(gd, np.float32)
    fo, fa = np.zeros(od, np.float32), np.zeros(gd, np.float32)
    r = np.zeros(1, np.float32)
    te, tr = np.zeros(1, np.uint8), np.zeros(1, np.uint8)
    lib().po_step(C.byref(cfg), C.byref(env), _fp(a), _fp(obs), _fp(ag), _fp(dg), _fp(r),
                  te.ctypes.data_as(C.POINTER(C.c_uint8)), tr.ctypes.data_as(C.POINTER(C.c_uint8)),
                  int(autoreset), _fp(fo), _fp(fa), C.byref(stats) if stats is not None else None)
    return obs, ag, dg, float(r[0]), bool(te[0]), bool(tr[0])


def compute_reward(reward_type: str, ag, dg, task: str = "push"):
    a = np.ascontiguousarray(ag, dtype=np.float32)
    d = np.ascontiguousarray(dg, dtype=np.float64)
    return lib().po_compute_reward(TASKS[task], 0 if reward_type == "sparse" else 1, _fp(a), _dp(d))


def is_success(ag, dg, task: str = "push") -> bool:
    a = np.ascontiguousarray(ag, dtype=np.float32)
    d = np.ascontiguousarray(dg, dtype=np.float64)
    return bool(lib().po_is_success(TASKS[task], _fp(a), _dp(d)))


def flip_goal(aux_state: int):
    """(new aux state, quaternion) of the Flip goal stream."""
    st = (C.c_uint64 * 1)(aux_state)
    q = np.zeros(4)
    lib().po_flip_goal(st, _dp(q))
    return int(st[0]), q


def pcg64_seed(seed: int) -> np.ndarray:
    st = np.zeros(4, np.uint64)
    lib().po_pcg64_seed(C.c_uint64(seed), st.ctypes.data_as(C.POINTER(C.c_uint64)))
    return st


def pcg64_next(st: np.ndarray) -> int:
    return int(lib().po_pcg64_next(st.ctypes.data_as(C.POINTER(C.c_uint64))))


def mass_matrix(cfg, q):
    qq = np.ascontiguousarray(q, dtype=np.float64)
    M = np.zeros(81)
    lib().po_mass_matrix(C.byref(cfg), _dp(qq), _dp(M))
    return M.reshape(9, 9)


def bias_forces(cfg, q, qd):
    qq = np.ascontiguousarray(q, dtype=np.float64)
    vv = np.ascontiguousarray(qd, dtype=np.float64)
    h = np.zeros(9)
    lib().po_bias_forces(C.byref(cfg), _dp(qq), _dp(vv), _dp(h))
    return h


def set_finger_noise(amplitude: float, seed: int = 0):
    """Test hook: per-substep finger-position noise (panda_oracle.c)."""
    lib().po_set_finger_noise(float(amplitude), int(seed))


def set_finger_bias(b: float):
    """Test hook: a constant per-substep offset b of both finger positions
    (panda_oracle.c po_set_finger_bias)."""
    lib().po_set_finger_bias(float(b))


def set_fp32_solver(on: bool):
    """Test hook: round the PGS's accumulated impulses and velocity change to
    fp32 after every row update (panda_oracle.c po_set_fp32_solver)."""
    lib().po_set_fp32_solver(int(bool(on)))


def set_fp32_dynamics(on: bool):
    """Test hook: M^-1 in fp32 arithmetic (panda_oracle.c po_set_fp32_dynamics)."""
    lib().po_set_fp32_dynamics(int(bool(on)))


def set_link_aabb(link, lx, ly, lz):
    lib().po_set_link_aabb(link, lx, ly, lz)


MUTATIONS = {"none": 0, "motor_kp_scale": 1, "link_damping": 2, "finger_box_grow": 3, "pair_friction_scale": 4}


def set_model_mutation(kind: str, value: float = 0.0):
    """Test hook: a deliberate model error (panda_oracle.c po_set_model_mutation):
    'motor_kp_scale' (kp x value), 'link_damping' (every body's k1 = k2 := value),
    'finger_box_grow' (finger boxes' half extents + value m),
    'pair_friction_scale' (Stack's cube-cube friction x value); 'none' restores
    the model.  The objects' masses and friction are Config fields."""
    lib().po_set_model_mutation(MUTATIONS[kind], float(value))


def set_state_noise(ulps: float, seed: int = 0):
    """Test hook: fp32-resolution noise of u * ulp32(x), |u| <= ulps, on every
    state component after each substep (panda_oracle.c po_set_state_noise);
    ulps < 0 rounds the state to fp32 after each substep instead."""
    lib().po_set_state_noise(float(ulps), int(seed))


def set_pgs_shift(k: int):
    """Test hook (panda_oracle.c po_set_pgs_shift): every substep's PGS exits k
    iterations after its stopping rule is first met (k > 0), or with the
    impulses of the iteration before (k < 0); 0 restores Bullet's rule."""
    lib().po_set_pgs_shift(int(k))


def set_clip_bias(m: float):
    """Test hook (panda_oracle.c po_set_clip_bias): Stack's box-box clip lines
    moved outward by m metres (a vertex on a clip line to within rounding
    changes side, and the clipped polygon starts at another vertex)."""
    lib().po_set_clip_bias(float(m))
