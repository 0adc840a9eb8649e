"""Capture pre-step states of envs whose observation leaves |x| < 10 (for oracle replay)."""
import sys, os, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "panda-lang-manip_amd"))
from pandasim.envs import PandaVecEnv
out = {}
for task in ["push", "pick_and_place"]:
    B = 65536
    env = PandaVecEnv(task, "sparse", "ee", B, "cuda")
    env.reset(seed=12345)
    g = torch.Generator(device="cuda"); g.manual_seed(1)
    for s in range(8):
        pre = env.sim.state.clone()
        a = torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1
        obs, r, te, tr, info = env.step(a)
        o = info["final_observation"]
        bad = torch.nonzero((o.abs() >= 10).any(dim=1) | ~torch.isfinite(o).all(dim=1)).flatten()
        print(task, s, "bad", bad.numel(), bad[:8].tolist(), flush=True)
        if bad.numel() and f"{task}_idx" not in out:
            idx = bad[:16]
            f = pre[:env.sim.layout.goal_offset].view(torch.float32).view(76, -1)[:, idx].cpu().numpy()
            gl = pre[env.sim.layout.goal_offset:env.sim.layout.rng_offset].view(torch.float64).view(3, -1)[:, idx].cpu().numpy()
            out[f"{task}_idx"] = idx.cpu().numpy(); out[f"{task}_f"] = f; out[f"{task}_goal"] = gl
            out[f"{task}_act"] = a[idx].cpu().numpy(); out[f"{task}_obs"] = o[idx].cpu().numpy(); out[f"{task}_step"] = np.array(s)
np.savez(os.path.join(ROOT, "gpurun_out", "blowup.npz"), **out)
