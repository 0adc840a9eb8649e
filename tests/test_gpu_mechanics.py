"""Contact mechanics on the GPU (the plugin path's ps_sim_step, robot
present at its initial pose, far above the object): the identities the oracle
is pinned to in tests/test_oracle.py (Coulomb sliding, statics of the
warm-started solve) hold for the fp32 kernels, and the sliding trajectories
agree with the fp64 oracle run of the same scene."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

G = 9.81


def _scene(env_id, B, seed):
    import pandasim

    env = pandasim.make(env_id, num_envs=B, lanes_per_env=1)
    env.reset(seed=seed)
    return env, env.sim


def _velocities(B, rng, lo=0.5, hi=1.0):
    """Speeds lo-hi m/s pointing into the table (the -x half-plane, so the
    object stops before an edge)."""
    speed = rng.uniform(lo, hi, B)
    ang = rng.uniform(np.pi * 0.75, np.pi * 1.25, B)
    return np.stack([speed * np.cos(ang), speed * np.sin(ang)], axis=1)


@pytest.mark.parametrize("env_id,mu,tol,speeds", [("PandaPush-v3", 0.25, 0.02, (0.5, 1.0)),
                                                  ("PandaPickAndPlace-v3", 0.25, 0.02, (0.5, 1.0)),
                                                  ("PandaSlide-v3", 0.02, 0.06, (0.15, 0.3))])
def test_gpu_sliding_object_decelerates_at_mu_g(env_id, mu, tol, speeds):
    from pandasim import _lib as L

    B, T = 64, 60
    env, sim = _scene(env_id, B, seed=100)
    for _ in range(25):
        sim.step()
    p0 = sim.rows(L.F_CPOS, 3).clone()
    v0 = _velocities(B, np.random.default_rng(5), *speeds)
    vel = sim.rows(L.F_CVEL, 3).clone()
    vel[:, :2] = torch.as_tensor(v0, dtype=torch.float32, device=vel.device)
    sim.set_rows(L.F_CVEL, vel)
    ps, vs = [], []
    for _ in range(T):
        sim.step()
        ps.append(sim.rows(L.F_CPOS, 3).clone())
        vs.append(sim.rows(L.F_CVEL, 3).clone())
    ps = torch.stack(ps).double().cpu().numpy()  # [T, B, 3]
    vs = torch.stack(vs).double().cpu().numpy()
    t = 0.04 * (np.arange(T) + 1)
    p0 = p0.double().cpu().numpy()
    for i in range(B):
        speed0 = float(np.hypot(*v0[i]))
        speed = np.hypot(vs[:, i, 0], vs[:, i, 1])
        moving = speed > 0.1 * speed0
        assert moving.sum() >= 4, i
        decel = -np.polyfit(t[moving], speed[moving], 1)[0]
        assert abs(decel - mu * G) <= tol * mu * G, (i, decel, mu * G)
        stop = speed0 ** 2 / (2 * mu * G)
        dist = float(np.hypot(*(ps[-1, i, :2] - p0[i, :2])))
        assert abs(dist - stop) <= 2.5 * tol * stop, (i, dist, stop)
        assert speed[-1] < 1e-3 and np.all(np.abs(ps[:, i, 2] - p0[i, 2]) < 3e-4)


@pytest.mark.parametrize("env_id", ["PandaPush-v3", "PandaSlide-v3"])
def test_gpu_resting_object_normal_impulses_carry_its_weight(env_id):
    """The warm start's cache rows hold the last substep's normal impulses:
    for a settled object they sum to m g dt (fp32)."""
    from pandasim import _lib as L

    B = 256
    env, sim = _scene(env_id, B, seed=7)
    for _ in range(50):
        sim.step()
    lam = sim.rows(L.F_WG0, 4).double().sum(dim=1)
    m = float(sim.cfg.object_mass)
    assert torch.allclose(lam, torch.full_like(lam, m * G / 500), rtol=2e-4, atol=0), (lam.min(), lam.max())
    assert sim.rows(L.F_CVEL, 3).abs().max() < 1e-4


def test_gpu_sliding_matches_the_oracle():
    """The same slide through the fp64 oracle (robot included): object
    positions within 2e-4 m over 60 steps of friction-limited sliding."""
    import oracle as O
    from pandasim import _lib as L

    B, T, seed = 16, 60, 300
    env, sim = _scene("PandaPush-v3", B, seed)
    cfg = O.config("push")
    oenvs = [O.new_env(cfg) for _ in range(B)]
    for i, e in enumerate(oenvs):
        O.reset(cfg, e, seed=seed + i)
    for _ in range(25):
        sim.step()
        for e in oenvs:
            O.sim_step(cfg, e)
    v0 = _velocities(B, np.random.default_rng(9))
    vel = sim.rows(L.F_CVEL, 3).clone()
    vel[:, :2] = torch.as_tensor(v0, dtype=torch.float32, device=vel.device)
    sim.set_rows(L.F_CVEL, vel)
    v32 = vel.double().cpu().numpy()
    for i, e in enumerate(oenvs):
        e.obj[0].vel[0], e.obj[0].vel[1] = float(v32[i, 0]), float(v32[i, 1])
    worst = 0.0
    for _ in range(T):
        sim.step()
        for e in oenvs:
            O.sim_step(cfg, e)
        gp = sim.rows(L.F_CPOS, 3).double().cpu().numpy()
        op = np.array([list(e.obj[0].pos) for e in oenvs])
        worst = max(worst, float(np.abs(gp - op).max()))
    assert worst < 2e-4, worst
    assert math.isfinite(worst)
