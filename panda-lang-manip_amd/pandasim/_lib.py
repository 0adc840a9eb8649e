"""ctypes binding of libpandasim.so (include/pandasim.h).

The library is built in-tree (``python -m pandasim.build`` or
``__graft_entry__.build()``) and loaded from this package directory.  There is
no CPU fallback: if the library or a GPU is missing, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PANDASIM_LIB", os.path.join(HERE, "libpandasim.so"))

PS_OK = 0
PS_MAX_UNIFORM = 8
ERRORS = {-1: "PS_ERR_ARG", -2: "PS_ERR_HIP", -3: "PS_ERR_UNSUPPORTED"}

# float row indices of the SoA state (include/pandasim.h)
F_Q, F_QD, F_MTARGET, F_MKP, F_MKD, F_MVEL, F_MIMP = 0, 9, 18, 27, 36, 45, 54
F_CPOS, F_CQUAT, F_CVEL, F_COMG = 63, 66, 70, 73
F_C2POS, F_C2QUAT, F_C2VEL, F_C2OMG = 76, 79, 83, 86
OBJECT_ROWS = (F_CPOS, F_C2POS)  # pos, quat (+3), vel (+7), omg (+10) of object 0 / 1
# warm-start contact cache (ground of object 0 / 1, gripper, object-object)
F_WG0, F_WG0ID, F_WG1, F_WG1ID, F_WR, F_WRID, F_WP, F_WPPT, F_WPN = 89, 93, 94, 98, 99, 103, 104, 108, 120
NUM_FLOAT_ROWS = 121
NUM_RNG_ROWS = 5
MAX_GOAL_DIM = 6
SHAPE_BOX, SHAPE_CYLINDER = 0, 1


class Config(C.Structure):
    _fields_ = [
        ("task", C.c_int32), ("control", C.c_int32), ("reward", C.c_int32), ("block_gripper", C.c_int32),
        ("has_table", C.c_int32), ("has_plane", C.c_int32), ("n_objects", C.c_int32), ("object_shape", C.c_int32),
        ("base", C.c_float * 3), ("object_half", C.c_float * 3),
        ("object_mass", C.c_float), ("object2_mass", C.c_float), ("object_friction", C.c_float),
        ("table_cx", C.c_float), ("table_hx", C.c_float), ("table_hy", C.c_float),
    ]


class Visual(C.Structure):
    """ps_visual (include/pandasim.h): colours by role and ghost-target shapes."""
    _fields_ = [("rgba", (C.c_float * 4) * 8), ("target_shape", C.c_int32 * 2), ("target_half", (C.c_float * 3) * 2)]


VISUAL_SPHERE = 2
ROLES = ("plane", "table", "object1", "object2", "target1", "target2", "robot", "background")


class Layout(C.Structure):
    _fields_ = [
        ("num_envs", C.c_int64), ("stride", C.c_int64), ("float_offset", C.c_int64), ("goal_offset", C.c_int64),
        ("rng_offset", C.c_int64), ("elapsed_offset", C.c_int64), ("total_bytes", C.c_int64),
    ]


class PandasimError(RuntimeError):
    pass


_lib = None


def exported_symbols():
    return [
        "ps_abi_version", "ps_default_config", "ps_state_layout", "ps_create", "ps_destroy", "ps_last_error",
        "ps_obs_dim", "ps_action_dim", "ps_goal_dim", "ps_max_episode_steps", "ps_init_state", "ps_reset",
        "ps_step", "ps_sim_step", "ps_link_state", "ps_inverse_kinematics", "ps_compute_reward", "ps_rng_seed",
        "ps_rng_uniform", "ps_rng_rotation", "ps_base_state", "ps_camera", "ps_render", "ps_deproject_image",
        "ps_deproject_pixels", "ps_set_nonfinite_guard", "ps_set_lanes_per_env", "ps_step_lanes",
        "ps_mark_motor_rows_dirty", "ps_set_episode_stats",
    ]


def check_fresh(path: str) -> None:
    """Refuse a library built from other sources than the ones next to it
    (build.py's content stamp).  The product library and the named variants
    (libpandasim_<variant>.so) must carry a stamp equal to the sha256 of the
    current csrc/ and include/ files plus their flags; a library at any other
    path (an experiment under PANDASIM_LIB) is checked only if it has a stamp
    and its variant is known."""
    from . import build as B

    name = os.path.basename(path)
    variant = None
    if os.path.abspath(path) == os.path.abspath(B.OUT):
        variant = ""
    elif name.startswith("libpandasim_") and name.endswith(".so") and name[12:-3] in B.VARIANTS:
        variant = name[12:-3]
    if variant is None or not os.path.isdir(B.CSRC):
        return
    have = B.read_stamp(path)
    if have is None:
        if os.path.abspath(path) == os.path.abspath(B.OUT):
            raise PandasimError(f"{path} has no build stamp: rebuild it with `python -m pandasim.build`")
        return
    if have != B.fingerprint(variant):
        raise PandasimError(f"{path} is stale: its stamp does not match the sources in {B.CSRC} and "
                            f"{B.INCLUDE}; rebuild it with `python -m pandasim.build`")


def lib():
    """Load libpandasim.so (raises if it has not been built or is stale)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PandasimError(f"{LIB_PATH} not found: build it with `python -m pandasim.build` (hipcc, gfx950)")
    check_fresh(LIB_PATH)
    L = C.CDLL(LIB_PATH)
    V, I, I64, P = C.c_void_p, C.c_int, C.c_int64, C.POINTER
    L.ps_abi_version.restype = I
    L.ps_default_config.argtypes = [I, I, I, P(Config)]
    L.ps_state_layout.argtypes = [I64, P(Layout)]
    L.ps_create.argtypes = [P(Config), I64, I, P(V)]
    L.ps_destroy.argtypes = [V]
    L.ps_destroy.restype = None
    L.ps_last_error.argtypes = [V]
    L.ps_last_error.restype = C.c_char_p
    L.ps_obs_dim.argtypes = [V]
    L.ps_action_dim.argtypes = [V]
    L.ps_goal_dim.argtypes = [V]
    L.ps_max_episode_steps.argtypes = [V]
    L.ps_init_state.argtypes = [V, V, V]
    L.ps_reset.argtypes = [V, V, V, V, V, V, V, V]
    L.ps_step.argtypes = [V, V, V, V, V, V, V, V, V, I, V, V, V]
    L.ps_sim_step.argtypes = [V, V, I, V]
    L.ps_set_nonfinite_guard.argtypes = [V, V, I]
    L.ps_set_lanes_per_env.argtypes = [V, I]
    L.ps_step_lanes.argtypes = [V]
    L.ps_mark_motor_rows_dirty.argtypes = [V]
    L.ps_set_episode_stats.argtypes = [V, V]
    L.ps_link_state.argtypes = [V, V, I, V, V, V, V, V]
    L.ps_inverse_kinematics.argtypes = [V, V, I, V, V, V, V]
    L.ps_compute_reward.argtypes = [I, I, V, I, V, I, V, V, I64, V]
    L.ps_rng_seed.argtypes = [V, V, V, V, V]
    L.ps_rng_uniform.argtypes = [V, V, V, I, P(C.c_double), P(C.c_double), V, V]
    L.ps_rng_rotation.argtypes = [V, V, V, V, V]
    L.ps_base_state.argtypes = [V, V, I, V, V, V, V, V, V]
    F, D = P(C.c_float), P(C.c_double)
    L.ps_camera.argtypes = [F, C.c_float, C.c_float, C.c_float, C.c_float, I, I, F, F, D]
    L.ps_render.argtypes = [V, V, F, F, I, I, P(Visual), V, V, V, V]
    L.ps_deproject_image.argtypes = [V, V, D, I, I, V, V, V, V]
    L.ps_deproject_pixels.argtypes = [V, V, V, I, D, I, I, V, V]
    for name in exported_symbols():
        getattr(L, name).restype = getattr(L, name).restype if name in ("ps_destroy", "ps_last_error") else I
    _lib = L
    return L


def check(rc: int, ctx=None, what: str = "") -> None:
    if rc != PS_OK:
        msg = ""
        if ctx is not None:
            raw = lib().ps_last_error(ctx)
            msg = raw.decode() if raw else ""
        raise PandasimError(f"{what} failed: {ERRORS.get(rc, rc)} {msg}".strip())


def layout(num_envs: int) -> Layout:
    lay = Layout()
    check(lib().ps_state_layout(int(num_envs), C.byref(lay)), what="ps_state_layout")
    return lay


def default_config(task: int, control: int, reward: int) -> Config:
    cfg = Config()
    check(lib().ps_default_config(task, control, reward, C.byref(cfg)), what="ps_default_config")
    return cfg
