"""CPU tests of the drop-in boundary: libpandasim.so loads, exports every
symbol include/pandasim.h declares, and the host logic (layout, registry,
configuration) behaves; no kernel is launched."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def L():
    from pandasim import _lib

    return _lib


def header_symbols():
    src = open(os.path.join(ROOT, "include", "pandasim.h")).read()
    return sorted(set(re.findall(r"\b(ps_[a-z_]+)\s*\(", src)))


def test_library_exports_every_header_symbol(L):
    lib = L.lib()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(L.exported_symbols()) == syms


def test_abi_version(L):
    assert L.lib().ps_abi_version() == 1


def test_state_layout(L):
    lay = L.layout(1000)
    assert lay.stride == 1024
    assert lay.goal_offset == 76 * 1024 * 4
    assert lay.rng_offset == lay.goal_offset + 3 * 1024 * 8
    assert lay.total_bytes == lay.rng_offset + 4 * 1024 * 8 + 1024 * 4
    assert lay.goal_offset % 8 == 0 and lay.rng_offset % 8 == 0


def test_default_configs(L):
    for task in range(3):
        cfg = L.default_config(task, 0, 1)
        assert cfg.block_gripper == (task != 2)  # panda_tasks.py:46,62,78
        assert cfg.has_cube == (task != 0)
        assert abs(cfg.base[0] + 0.6) < 1e-7
    bad = L.Config()
    assert L.lib().ps_default_config(5, 0, 0, C.byref(bad)) < 0


def test_create_and_dims_without_gpu(L):
    lib = L.lib()
    cfg = L.default_config(2, 0, 0)
    ctx = C.c_void_p()
    assert lib.ps_create(C.byref(cfg), 8, 0, C.byref(ctx)) == 0
    assert lib.ps_obs_dim(ctx) == 19 and lib.ps_action_dim(ctx) == 4
    lib.ps_destroy(ctx)
    cfg = L.default_config(0, 1, 0)
    assert lib.ps_create(C.byref(cfg), 8, 0, C.byref(ctx)) == 0
    assert lib.ps_obs_dim(ctx) == 6 and lib.ps_action_dim(ctx) == 7
    lib.ps_destroy(ctx)
    assert lib.ps_create(C.byref(cfg), 0, 0, C.byref(ctx)) < 0


def test_registry_has_all_24_ids():
    from pandasim import REGISTRY, make

    assert len(REGISTRY) == 24
    assert REGISTRY["PandaPushJointsDense-v3"] == dict(task="push", reward_type="dense", control_type="joints",
                                                       max_episode_steps=50)
    assert REGISTRY["PandaStack-v3"]["max_episode_steps"] == 100
    with pytest.raises(NotImplementedError):
        make("PandaSlide-v3")


def test_no_silent_cpu_fallback():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from pandasim import PandasimError, make

    with pytest.raises(PandasimError):
        make("PandaReach-v3", num_envs=4)
