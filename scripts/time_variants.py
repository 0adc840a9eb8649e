"""Time the fused step kernel of several libpandasim builds (phase breakdown)."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time, torch
sys.path.insert(0, os.path.join(os.environ["ROOT"], "panda-lang-manip_amd"))
import pandasim
out = {}
for task in os.environ.get("TASKS", "push").split(","):
    env_id = {"reach": "PandaReach-v3", "push": "PandaPush-v3", "pick_and_place": "PandaPickAndPlace-v3",
              "stack": "PandaStack-v3", "flip": "PandaFlip-v3", "slide": "PandaSlide-v3"}[task]
    B = int(os.environ.get("B", "65536"))
    env = pandasim.make(env_id, num_envs=B, lanes_per_env=int(os.environ.get("LANES", "0")))
    env.reset(seed=12345)
    g = torch.Generator(device="cuda"); g.manual_seed(0)
    acts = torch.rand(30, B, env.action_dim, device="cuda", generator=g) * 2 - 1
    for k in range(5): env.step(acts[k], copy=False)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for k in range(5, 30): env.step(acts[k], copy=False)
    e.record(); torch.cuda.synchronize()
    out[task] = s.elapsed_time(e) / 25
print("RESULT", __import__("json").dumps(out))
'''
res = {}
for lib in sys.argv[1:]:
    env = dict(os.environ, PANDASIM_LIB=os.path.abspath(lib), ROOT=ROOT)
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
    line = [l for l in p.stdout.splitlines() if l.startswith("RESULT")]
    res[os.path.basename(lib)] = json.loads(line[0][7:]) if line else p.stderr[-500:]
    print(os.path.basename(lib), res[os.path.basename(lib)], flush=True)
