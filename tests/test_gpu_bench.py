"""bench.py end to end on the GPU: the multi-rank path (torch.distributed.run,
per-rank seeds, barriers, the rank-0 gather of episode statistics,
max-over-ranks timing, rank 0's JSON line) rehearsed with 2 ranks on the one
GPU under gloo (RCCL refuses two ranks per GPU), and the single-rank line's
roofline blocks.  8-GPU runs are the driver's; these keep the N>1 code path
exercised."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_line(stdout: str) -> dict:
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_gloo_rehearsal():
    # plain `python bench.py --gpus 2`, as the driver's N-GPU run may invoke it:
    # bench.py itself starts the two ranks (torch.distributed.run child)
    env = dict(os.environ, PANDASIM_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "256", "--no-cpu-baseline"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = _json_line(out.stdout)
    assert line["n_gpus"] == 2 and line["steps"] == 3 and line["warmup"] == 1
    assert line["config"]["global_batch"] == 512 and line["config"]["batch_per_gpu"] == 256
    assert line["episodes"]["gathered_envs"] == 512  # rank 0 holds both shards
    assert line["value"] > 0 and line["scaling"] == "weak"


def test_bench_under_explicit_torchrun():
    env = dict(os.environ, PANDASIM_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "128", "--no-cpu-baseline"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = _json_line(out.stdout)
    assert line["n_gpus"] == 2 and line["episodes"]["gathered_envs"] == 256


def test_bench_single_rank_roofline_blocks():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--batch", "4096",
           "--cpu-seconds", "1.5"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = _json_line(out.stdout)
    rf = line["roofline"]
    assert rf["bound"] == "hbm" and rf["bytes_per_env_step"] == 630 and 0 < rf["frac"] < 1
    fp = rf["fp32"]
    assert fp["flops_per_env_step"] > 1e5 and 0 < fp["frac"] < 1 and fp["peak_tflops"] == 157.3
    assert set(fp["split"]) == {"dynamics_and_rows", "pgs", "ik", "step"}
    cb = line["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1


_RCCL_ONE_RANK = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.path.join(os.environ["ROOT"], "panda-lang-manip_amd"))
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
assert dist.get_backend() == "nccl"
import pandasim
from pandasim.dist import EpisodeStats, gather_to_rank0, max_over_ranks
B = 300
env = pandasim.make("PandaPush-v3", num_envs=B, device=dev)
env.reset(seed=5)
stats = EpisodeStats(B, dev)
g = torch.Generator(device=dev)
g.manual_seed(3)
for _ in range(55):
    _, r, te, tr, _ = env.step(torch.rand(B, 3, device=dev, generator=g) * 2 - 1, copy=False)
    stats.update(r, te, tr)
local = stats.packed()
full = gather_to_rank0(local)
assert full is not None and torch.equal(full, local), "RCCL gather changed the statistics"
assert int(local[2].sum()) >= B  # every env finished an episode (TimeLimit 50)
assert max_over_ranks(1.25, dev) == 1.25
dist.barrier()
dist.destroy_process_group()
print("RCCL_OK")
"""


def test_rccl_one_rank_gather_and_max():
    """The bench's collectives (pandasim.dist: the all_gather of shard sizes,
    the gather of episode statistics to rank 0, the max-over-ranks timer)
    through a real RCCL ("nccl") process group.  One box has one GPU and RCCL
    takes one rank per GPU, so this is world size 1; the 2-rank path is
    rehearsed under gloo above and the 8-GPU run is the driver's."""
    env = dict(os.environ, ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = subprocess.run([sys.executable, "-c", _RCCL_ONE_RANK], capture_output=True, text=True, timeout=240,
                         env=env, cwd=ROOT)
    assert out.returncode == 0 and "RCCL_OK" in out.stdout, (out.stdout[-1500:], out.stderr[-3000:])
