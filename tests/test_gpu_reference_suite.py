"""The reference's own test files, at their own parameters, on the HIP path.

* ``test/seed_test.py:7-122`` -- one env per task (Reach, Push, Slide,
  PickAndPlace, Stack) built as ``gym.make`` builds it (the one-env gymnasium
  classes of ``pandasim.gym_registration``), ``reset(seed=<the file's seed>)``,
  the file's six actions with ``reset()`` on done, twice.  The reference
  asserts the two final observations ``allclose``; here they must be equal bit
  for bit, every step of the first run is replayed by the fp64 oracle from the
  GPU's state before it and classified by ``parity_judge.judge`` (no sample
  beyond the tight bounds), and the final observation of a free-running oracle
  from the same reset and actions must agree to the north star's 1e-3.  The
  oracle perturbed by two fp32 ulps per substep parts from itself by at most
  2.2e-5 on these trajectories (no done flag, few contacts), so 1e-3 is a
  bound the GPU cannot meet by luck alone and cannot miss by chaos.
* ``test/envs_test.py:6-134`` -- every registered ID (24), 1000 random steps of
  one env with ``reset()`` on done.  The reference asserts that nothing raises;
  here every observation must be finite, ``truncated`` must fall exactly on
  the TimeLimit, and every unseeded ``reset()`` must draw the goal the
  oracle's generator draws after the same number of resets (bit for bit; Flip's
  goal from the auxiliary stream).

Actions are sampled like ``env.action_space.sample()`` (a float32 ``Box(-1, 1)``);
gymnasium is absent from the image, so numpy's uniform draw stands in.
"""
import zlib

import numpy as np
import pytest
import torch

import oracle as O
from helpers import oracle_config_for, oracle_env_from, snapshot
from parity_judge import FREE_GRIPPER, LOOSE, groups_for, judge

pytestmark = pytest.mark.gpu

# test/seed_test.py: (gym id, seed, the six actions) of each test function
SEED_CASES = {
    "reach": ("PandaReach-v3", 12345,  # seed_test.py:7-29
              [[-0.931, 0.979, -0.385], [-0.562, 0.391, -0.532], [0.042, 0.254, -0.624],
               [0.465, 0.745, 0.284], [-0.237, 0.995, -0.425], [0.67, 0.472, 0.972]]),
    "push": ("PandaPush-v3", 6789,  # seed_test.py:32-54
             [[0.925, 0.352, -0.014], [0.400, -0.018, -0.042], [0.308, 0.189, -0.943],
              [-0.556, 0.209, 0.907], [-0.862, -0.243, 0.835], [-0.552, -0.262, 0.317]]),
    "slide": ("PandaSlide-v3", 13795,  # seed_test.py:57-78
              [[0.245, 0.786, 0.329], [-0.414, 0.343, -0.839], [0.549, 0.047, -0.857],
               [0.744, -0.507, 0.092], [-0.202, -0.939, -0.945], [-0.97, -0.616, 0.472]]),
    "pick_and_place": ("PandaPickAndPlace-v3", 794512,  # seed_test.py:81-103
                       [[0.429, -0.287, 0.804, -0.592], [0.351, -0.136, 0.296, -0.223],
                        [-0.187, 0.706, -0.988, 0.972], [-0.389, -0.249, 0.374, -0.389],
                        [-0.191, -0.297, -0.739, 0.633], [0.093, 0.242, -0.11, -0.949]]),
    "stack": ("PandaStack-v3", 657894,  # seed_test.py:106-122
              [[-0.609, 0.73, -0.433, 0.76], [0.414, 0.327, 0.275, -0.196], [-0.3, 0.589, -0.712, 0.683],
               [0.772, 0.333, -0.537, -0.253], [0.784, -0.014, -0.997, -0.118], [-0.12, -0.958, -0.744, -0.98]]),
}


def _gym_make(env_id):
    """gym.make(env_id) of the reference: one env of the ID's task, reward and
    control type, TimeLimit applied by the fused step."""
    from pandasim import gym_registration as GR
    from pandasim.envs import REGISTRY

    spec = REGISTRY[env_id]
    cls = getattr(GR, GR._CLASS_OF_TASK[spec["task"]])
    return cls(reward_type=spec["reward_type"], control_type=spec["control_type"]), spec


def _flat(obs):
    return np.concatenate([obs["observation"], obs["achieved_goal"], obs["desired_goal"]])


@pytest.mark.parametrize("task", list(SEED_CASES))
def test_seed_test_at_its_own_parameters(task):
    env_id, seed, actions = SEED_CASES[task]
    env, _ = _gym_make(env_id)
    cfg = oracle_config_for(env._env.sim.cfg)
    groups = groups_for(task, 7 if task in FREE_GRIPPER else 6)
    finals, counts, beyond = [], {"tight": 0, "conditioned": 0, "bif": 0, "beyond": 0}, []
    for run in range(2):
        env.reset(seed=seed)
        for k, action in enumerate(actions):
            a = np.asarray(action, np.float32)
            snap = snapshot(env._env.sim) if run == 0 else None
            observation, _, terminated, truncated, _ = env.step(action)
            if run == 0:
                o, ag, dg, _, t_e, t_r = O.step(cfg, oracle_env_from(cfg, snap, 0), a)
                assert (t_e, t_r) == (terminated, truncated), (k, t_e, t_r)
                cls, errs = judge(cfg, snap, 0, a, o, observation["observation"], groups, task)
                counts[cls] += 1
                if cls == "beyond":
                    beyond.append((k, errs))
                assert cls != "bif" or all(v <= LOOSE[g] for g, v in errs.items()), (k, errs)
                assert np.array_equal(observation["desired_goal"], dg.astype(np.float32)), k
            if terminated or truncated:
                observation, _ = env.reset()
        finals.append(observation)
    print(task, counts, beyond)
    assert not beyond
    # seed_test.py's assertion, bit for bit
    for key in ("observation", "achieved_goal", "desired_goal"):
        assert np.array_equal(finals[0][key], finals[1][key]), key
        assert np.allclose(finals[0][key], finals[1][key])
    # the whole six-step trajectory against a free-running oracle from the same reset
    e = O.new_env(cfg)
    O.reset(cfg, e, seed=seed)
    for action in actions:
        o, ag, dg, _, t_e, t_r = O.step(cfg, e, np.asarray(action, np.float32), autoreset=True)
    err = np.abs(_flat(finals[0]) - np.concatenate([o, ag, dg]).astype(np.float32)).max()
    print(task, f"free-running oracle vs GPU after 6 steps: {err:.2e}")
    assert err < 1e-3


def _ids():
    from pandasim.envs import REGISTRY

    return sorted(REGISTRY)


@pytest.mark.parametrize("env_id", _ids())
def test_envs_test_at_its_own_parameters(env_id):
    """envs_test.py:6-14 run_env: reset(), 1000 x (sample, step, reset on done)."""
    env, spec = _gym_make(env_id)
    cfg = oracle_config_for(env._env.sim.cfg)
    rng = np.random.default_rng(zlib.crc32(env_id.encode()))
    steps = spec["max_episode_steps"]
    G = env._env.goal_dim
    env.reset(seed=1000)
    oe = O.new_env(cfg)
    O.reset(cfg, oe, seed=1000)
    assert np.array_equal(env._env.sim.goal[:G, 0].cpu().numpy(), np.array(oe.goal)[:G])
    in_episode = resets = 0
    for _ in range(1000):
        action = rng.uniform(-1.0, 1.0, env._env.action_dim).astype(np.float32)  # action_space.sample()
        observation, reward, terminated, truncated, info = env.step(action)
        in_episode += 1
        for v in observation.values():
            assert np.isfinite(v).all()
        assert truncated == (in_episode == steps)
        assert isinstance(reward, float) and info["is_success"] == terminated
        if terminated or truncated:
            env.reset()
            resets += 1
            in_episode = 0
            O.reset(cfg, oe, seed=None)  # the oracle's generator, after as many resets
            assert np.array_equal(env._env.sim.goal[:G, 0].cpu().numpy(), np.array(oe.goal)[:G]), resets
    env.close()
    print(env_id, f"{resets} resets in 1000 steps")
    assert resets >= 1000 // steps
