# Group kernels (16 and 8 lanes per env) against the one-lane kernel: q/qd after
# one step from the same reset, per task and control (diagnostic; the GPU test
# is tests/test_gpu_parity.py::test_group_kernels_match_one_lane).
import sys, numpy as np, torch
sys.path.insert(0, 'panda-lang-manip_amd')
from pandasim.envs import PandaVecEnv
B = 64
for task in ("slide", "push", "pick_and_place", "reach"):
    for control in ("joints", "ee"):
        res = {}
        for lanes in (1, 8, 16):
            env = PandaVecEnv(task, "sparse", control, B, "cuda", lanes_per_env=lanes)
            env.autoreset = False
            env.reset(seed=12345)
            rng = np.random.default_rng(7)
            a = rng.uniform(-1, 1, size=(B, env.action_dim)).astype(np.float32)
            env.step(torch.from_numpy(a).cuda())
            res[lanes] = env.sim.f[0:18, :B].double().cpu().numpy()
        print(task, control, "q/qd max diff vs 1 lane: 8 lanes %.1e, 16 lanes %.1e" % (
            np.abs(res[8] - res[1]).max(), np.abs(res[16] - res[1]).max()), flush=True)
