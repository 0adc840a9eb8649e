"""The in-contact scenario of tests/test_gpu_parity.py::
test_group_kernels_match_one_lane_in_contact for one library (PANDASIM_LIB):
the one-lane step from the mid-push state, each env judged against the oracle;
prints every env that is not 'tight' with its errors and the oracle's object
speeds.  Usage: python scripts/incontact_probe.py [task] [control]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "panda-lang-manip_amd")]
import oracle as O  # noqa: E402
from helpers import oracle_config_for, oracle_env_from, snapshot  # noqa: E402
from parity_judge import FREE_GRIPPER, groups_for, judge  # noqa: E402
from pandasim.envs import PandaVecEnv  # noqa: E402
from test_gpu_parity import _contact_policy  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "push"
control = sys.argv[2] if len(sys.argv) > 2 else "ee"
B = 64
drv = PandaVecEnv(task, "sparse", "ee", B, "cuda", lanes_per_env=1)
drv.autoreset = False
drv.reset(seed=44)
policy = _contact_policy(drv, task)
for s in range(9):
    drv.step(torch.from_numpy(policy(s)).cuda())
state0 = drv.sim.state.clone()
env = PandaVecEnv(task, "sparse", control, B, "cuda", lanes_per_env=1)
env.autoreset = False
env.reset(seed=44)
a = np.random.default_rng(9).uniform(-1, 1, size=(B, env.action_dim)).astype(np.float32)
if control == "ee":
    a[:, :3] = policy(9)[:, :3]
env.sim.state.copy_(state0)
snap = snapshot(env.sim)
env.sim._call("ps_mark_motor_rows_dirty", env.sim._ctx)
o, *_ = env.step(torch.from_numpy(a).cuda())
obs = o["observation"].cpu().numpy()
cfg = oracle_config_for(env.sim.cfg)
groups = groups_for(task, 7 if task in FREE_GRIPPER else 6)
counts = {"tight": 0, "conditioned": 0, "bif": 0, "beyond": 0}
for i in range(B):
    oo, *_ = O.step(cfg, oracle_env_from(cfg, snap, i), a[i])
    cls, errs = judge(cfg, snap, i, a[i], oo, obs[i], groups, task)
    counts[cls] += 1
    if cls != "tight":
        big = {k: f"{v:.2e}" for k, v in errs.items() if v > 1e-6}
        print(i, cls, big, "oracle avel", np.round(oo[groups["obj_avel"]], 4) if "obj_avel" in groups else "")
print(os.path.basename(os.environ.get("PANDASIM_LIB", "libpandasim.so")), task, control, counts, flush=True)
