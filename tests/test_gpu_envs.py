"""Every registered env ID through the fused path (the reference's
test/envs_test.py:6-14: make, reset, random steps), and the §8(e) shard
claim: a batch split into per-rank shards (shard_seeds) steps env for env
like the unsplit batch."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ids():
    from pandasim.envs import REGISTRY

    return sorted(REGISTRY)


@pytest.mark.parametrize("env_id", _ids())
def test_every_registered_id_runs(env_id):
    import pandasim

    B = 64
    env = pandasim.make(env_id, num_envs=B)
    obs, info = env.reset(seed=0)
    assert set(obs) == {"observation", "achieved_goal", "desired_goal"}
    assert obs["observation"].shape == (B, env.obs_dim) and obs["observation"].dtype == torch.float32
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    for _ in range(12):
        a = torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1
        obs, r, te, tr, info = env.step(a)
        for k in obs:
            assert torch.isfinite(obs[k]).all(), (env_id, k)
        # Box(-10, 10) (core.py:218-224) is a declared bound the reference does not
        # enforce: a cube squeezed out of the closing fingers spins at > 10 rad/s
        assert obs["observation"].abs().max() < 100.0
        assert r.shape == (B,) and te.shape == (B,) and tr.shape == (B,)
        if "Dense" in env_id:
            assert (r <= 0).all()
        else:
            assert set(torch.unique(r).tolist()) <= {-1.0, 0.0}


@pytest.mark.parametrize("env_id", ["PandaPush-v3", "PandaStack-v3"])
def test_sharded_batch_matches_unsplit_batch(env_id):
    """The bench's 8-GPU partition (65 536 envs per GPU: the one-env-per-lane
    kernel) with 4 shards; lanes_per_env is fixed so that the shards and the
    full batch run the same kernel."""
    import pandasim
    from pandasim.dist import shard_seeds

    B, W = 256, 4
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    acts = torch.rand(6, B, 3 if "Push" in env_id else 4, device="cuda", generator=g) * 2 - 1
    full = pandasim.make(env_id, num_envs=B, lanes_per_env=1)
    full.reset(seed=shard_seeds(12345, B, 1, 0).numpy().astype("uint64"))
    shards = []
    for r in range(W):
        e = pandasim.make(env_id, num_envs=B // W, lanes_per_env=1)
        e.reset(seed=shard_seeds(12345, B, W, r).numpy().astype("uint64"))
        shards.append(e)
    for k in range(6):
        of, *_ = full.step(acts[k])
        parts = [e.step(acts[k][r * (B // W):(r + 1) * (B // W)])[0] for r, e in enumerate(shards)]
        for key in of:
            joined = torch.cat([p[key] for p in parts])
            assert torch.equal(of[key], joined), (env_id, k, key)


@pytest.mark.parametrize("lanes", [16, 8])
def test_group_kernel_shards_bit_identical(lanes):
    """The 16- and 8-lane kernels are batch-size independent too: 4 shards of
    24 envs step bit for bit like the 96-env batch (ragged last waves included)."""
    import pandasim
    from pandasim.dist import shard_seeds

    B, W = 96, 4
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    acts = torch.rand(5, B, 4, device="cuda", generator=g) * 2 - 1
    full = pandasim.make("PandaPickAndPlace-v3", num_envs=B, lanes_per_env=lanes)
    full.reset(seed=shard_seeds(77, B, 1, 0).numpy().astype("uint64"))
    shards = []
    for r in range(W):
        e = pandasim.make("PandaPickAndPlace-v3", num_envs=B // W, lanes_per_env=lanes)
        e.reset(seed=shard_seeds(77, B, W, r).numpy().astype("uint64"))
        shards.append(e)
    for k in range(5):
        of, *_ = full.step(acts[k])
        parts = [e.step(acts[k][r * (B // W):(r + 1) * (B // W)])[0] for r, e in enumerate(shards)]
        for key in of:
            assert torch.equal(of[key], torch.cat([p[key] for p in parts])), (k, key)


def test_motor_gain_rows_follow_the_fused_step():
    """env.step sets POSITION_CONTROL with PyBullet's gains on all nine joints
    (panda.py:52-107, pybullet.py:462-477).  The fused step writes the gain rows
    only when they may differ (ps_mark_motor_rows_dirty): a fresh state's
    default velocity motors, and after the plugin path's control_joints."""
    import pandasim
    from pandasim import _lib as L

    B = 8
    env = pandasim.make("PandaPush-v3", num_envs=B)
    env.reset(seed=3)
    f = env.sim.f
    assert torch.all(f[L.F_MKP:L.F_MKP + 9, :B] == 0.0)  # k_init_state: default velocity motors
    a = torch.zeros(B, env.action_dim, device="cuda")
    env.step(a)

    def gains():
        return f[L.F_MKP:L.F_MVEL + 9, :B].clone(), f[L.F_MIMP:L.F_MIMP + 9, :B].clone()

    kp_kd_vel, imp = gains()
    assert torch.allclose(kp_kd_vel[:9], torch.full_like(kp_kd_vel[:9], 0.1))
    assert torch.all(kp_kd_vel[9:18] == 1.0) and torch.all(kp_kd_vel[18:] == 0.0)
    # the plugin path changes joint 5's motor; the next fused step restores all nine
    env.sim.control_joints("panda", [5], [0.3], [5.0])
    f[L.F_MKD + 5, :B] = 0.5  # a gain no writer of the fused path uses
    env.step(a)
    kp_kd_vel2, imp2 = gains()
    assert torch.equal(kp_kd_vel2, kp_kd_vel) and torch.equal(imp2, imp)


@pytest.mark.parametrize("cls_name,env_id", [("PandaPushGymEnv", "PandaPush-v3"),
                                             ("PandaStackGymEnv", "PandaStackJointsDense-v3")])
def test_one_env_gymnasium_api(cls_name, env_id):
    """The gym.make entry points (pandasim.gym_registration): numpy obs dicts,
    float rewards, bool flags, the TimeLimit truncation, and the same bits as
    a one-env PandaVecEnv without auto-reset."""
    import pandasim
    from pandasim import gym_registration as GR
    from pandasim.envs import REGISTRY

    spec = REGISTRY[env_id]
    env = getattr(GR, cls_name)(reward_type=spec["reward_type"], control_type=spec["control_type"])
    ref = pandasim.make(env_id, num_envs=1, autoreset=False)
    obs, info = env.reset(seed=3)
    robs, _ = ref.reset(seed=3)
    assert set(obs) == {"observation", "achieved_goal", "desired_goal"} and isinstance(info["is_success"], bool)
    for k in obs:
        assert obs[k].dtype == np.float32 and np.array_equal(obs[k], robs[k][0].cpu().numpy())
    rng = np.random.default_rng(0)
    steps = spec["max_episode_steps"]
    for t in range(steps):
        a = rng.uniform(-1, 1, env._env.action_dim).astype(np.float32)
        obs, r, te, tr, info = env.step(a)
        robs, rr, rte, rtr, _ = ref.step(torch.as_tensor(a, device="cuda").reshape(1, -1))
        assert isinstance(r, float) and isinstance(te, bool) and isinstance(tr, bool)
        assert r == float(rr[0]) and te == bool(rte[0]) and tr == bool(rtr[0])
        for k in obs:
            assert np.array_equal(obs[k], robs[k][0].cpu().numpy()), (t, k)
        assert tr == (t == steps - 1)
    her = env.compute_reward(obs["achieved_goal"][None], obs["desired_goal"][None])
    # HER recomputes from the float32 goals of the observation; the step used
    # the float64 desired goal (as numpy does in the reference): rounding apart
    assert her.shape == (1,) and abs(float(her[0]) - r) <= 1e-6


@pytest.mark.parametrize("lanes", [1, 8])
def test_fused_episode_statistics_match_the_torch_ones(lanes):
    """ps_set_episode_stats (RecordEpisodeStatistics inside the step kernel)
    keeps the same bits as pandasim.dist.EpisodeStats updated from step()'s
    outputs: running return, last return, last success, episode count, across
    TimeLimit resets and successes."""
    import pandasim
    from pandasim.dist import EpisodeStats

    B = 700
    env = pandasim.make("PandaReachDense-v3", num_envs=B, lanes_per_env=lanes)
    env.reset(seed=21)
    fused = env.record_episode_statistics()
    ref = EpisodeStats(B, "cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(4)
    for _ in range(120):
        _, r, te, tr, _ = env.step(torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1, copy=False)
        ref.update(r, te, tr)
    assert torch.equal(fused[0], ref.running)
    assert torch.equal(fused[1:], ref.packed())
    assert int(fused[3].min()) >= 2  # at least the two TimeLimits
    env.record_episode_statistics(False)
    env.step(torch.zeros(B, env.action_dim, device="cuda"))
    assert torch.equal(fused[1:], ref.packed())  # off: the buffer is left alone


@pytest.mark.parametrize("lanes", [1, 8])
def test_fused_episode_statistics_restart_on_reset(lanes):
    """An explicit reset() mid-episode -- of every env and of a masked subset
    -- zeroes the running return (k_reset), as gymnasium's
    RecordEpisodeStatistics does: the abandoned episode's partial return does
    not carry into the next one.  Compared bit for bit with EpisodeStats whose
    running return is cleared on the same resets."""
    import pandasim
    from pandasim.dist import EpisodeStats

    B = 300
    env = pandasim.make("PandaPushDense-v3", num_envs=B, lanes_per_env=lanes)
    env.reset(seed=5)
    fused = env.record_episode_statistics()
    ref = EpisodeStats(B, "cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    mask = torch.zeros(B, dtype=torch.bool, device="cuda")
    mask[::3] = True

    def steps(n):
        for _ in range(n):
            _, r, te, tr, _ = env.step(torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1,
                                       copy=False)
            ref.update(r, te, tr)

    steps(7)
    assert float((fused[0][mask] != 0).float().mean()) > 0.9  # mid-episode (a few may have just succeeded)
    env.reset(mask=mask)
    ref.reset(mask)
    assert torch.equal(fused[0][mask], torch.zeros(int(mask.sum()), device="cuda"))
    assert torch.equal(fused[0], ref.running)
    steps(60)  # across a TimeLimit of the un-reset envs
    env.reset()
    ref.reset()
    assert not fused[0].any()
    steps(5)
    assert torch.equal(fused[0], ref.running)
    assert torch.equal(fused[1:], ref.packed())
