import sys, os, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "panda-lang-manip_amd"))
from pandasim.envs import PandaVecEnv
g = dict(np.load(os.path.join(ROOT, "tests/golden/task_layer.npz")))
seeds = g["seeds"]
for task in ["reach", "push", "pick_and_place"]:
    env = PandaVecEnv(task, "sparse", "ee", len(seeds), "cuda")
    for r in range(4):
        env.reset(seed=seeds if r == 0 else None)
        goal = env.sim.goal[:, :len(seeds)].t().cpu().numpy()
        bad = np.where(~np.all(goal == g[f"{task}_goal"][:, r], axis=1))[0]
        print(task, r, "bad", len(bad), bad[:10])
        for i in bad[:3]:
            print("  seed", seeds[i], goal[i].view(np.uint64), g[f"{task}_goal"][i, r].view(np.uint64), goal[i] - g[f"{task}_goal"][i, r])
