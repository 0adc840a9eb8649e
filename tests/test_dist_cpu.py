"""N>1 path on the CPU (gloo, world size 2 and 3): the batch partition owns
every env exactly once with the single-GPU seeds, and the only collective
(episode statistics to rank 0) reassembles the global batch in env order.
No kernel is launched: per-rank step outputs are synthetic tensors."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pandasim.dist import EpisodeStats, gather_to_rank0, max_over_ranks, shard_range, shard_seeds


def test_shard_range_partitions_the_batch():
    for B in (7, 8, 65536, 524288, 1000003):
        for W in (1, 2, 3, 4, 8):
            if B < W:
                continue
            owned = []
            for r in range(W):
                s, n = shard_range(B, W, r)
                owned.append((s, n))
            assert owned[0][0] == 0
            for (s0, n0), (s1, _) in zip(owned, owned[1:]):
                assert s1 == s0 + n0
            assert owned[-1][0] + owned[-1][1] == B
            assert max(n for _, n in owned) - min(n for _, n in owned) <= 1
    with pytest.raises(ValueError):
        shard_range(2, 4, 0)
    with pytest.raises(ValueError):
        shard_range(8, 2, 2)


def test_shard_seeds_match_single_gpu_run():
    full = shard_seeds(12345, 524288, 1, 0)
    parts = torch.cat([shard_seeds(12345, 524288, 8, r) for r in range(8)])
    assert torch.equal(full, parts)
    assert int(parts[65536]) == 12345 + 65536  # rank 1's first env (bench.py)


def test_episode_stats_update():
    st = EpisodeStats(3, "cpu")
    z = torch.zeros(3, dtype=torch.uint8)
    st.update(torch.tensor([-1.0, -1.0, 0.0]), z, z)
    st.update(torch.tensor([-1.0, 0.0, 0.0]), torch.tensor([0, 1, 0], dtype=torch.uint8),
              torch.tensor([1, 0, 0], dtype=torch.uint8))
    p = st.packed()
    assert p[0].tolist() == [-2.0, -1.0, 0.0]
    assert p[1].tolist() == [0.0, 1.0, 0.0]
    assert p[2].tolist() == [1.0, 1.0, 0.0]
    assert st.running.tolist() == [0.0, 0.0, 0.0]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, global_batch, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        start, n = shard_range(global_batch, world, rank)
        seeds = shard_seeds(12345, global_batch, world, rank)
        st = EpisodeStats(n, "cpu")
        # synthetic per-env outputs that depend only on the global env id
        gid = torch.arange(start, start + n)
        for k in range(5):
            r = -((gid + k) % 3 == 0).float()
            te = ((gid + k) % 4 == 0).to(torch.uint8)
            tr = torch.full((n,), int(k == 4), dtype=torch.uint8)
            st.update(r, te, tr)
        full = gather_to_rank0(st.packed())
        full_seeds = gather_to_rank0(seeds.to(torch.float64))
        t = max_over_ranks(float(rank + 1), "cpu")
        if rank == 0:
            q.put((full.tolist(), full_seeds.tolist(), t))
        else:
            assert full is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,B", [(2, 24), (3, 36), (3, 37), (2, 5)])
def test_gloo_gather_reassembles_global_batch(world, B):
    """Equal and uneven shards (37 over 3 ranks: 13, 12, 12)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, seeds, t = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the same statistics computed on one process over the whole batch
    st = EpisodeStats(B, "cpu")
    gid = torch.arange(B)
    for k in range(5):
        st.update(-((gid + k) % 3 == 0).float(), ((gid + k) % 4 == 0).to(torch.uint8),
                  torch.full((B,), int(k == 4), dtype=torch.uint8))
    assert torch.equal(torch.tensor(full), st.packed())
    assert seeds == [12345.0 + g for g in range(B)]
    assert t == float(world)


# ---- bench.py's multi-rank launch (no GPU: these exit before importing torch)
def _bench(args, env_extra=None):
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], capture_output=True, text=True,
                          timeout=60, env=env, cwd=root)


def test_bench_gpus_n_launches_n_ranks_as_a_child():
    import json

    out = _bench(["--gpus", "8", "--steps", "7", "--warmup", "2", "--print-launch"])
    assert out.returncode == 0, out.stderr
    cmd = json.loads(out.stdout.strip().splitlines()[-1])["launch"]
    i = cmd.index("torch.distributed.run")
    assert cmd[i - 1] == "-m"
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--nnodes=1")]
    script = cmd.index(next(a for a in cmd if a.endswith("bench.py")))
    assert cmd[script + 1:] == ["--gpus", "8", "--steps", "7", "--warmup", "2"]


def test_bench_refuses_world_size_other_than_gpus():
    out = _bench(["--gpus", "1", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode != 0 and "WORLD_SIZE=2" in (out.stderr + out.stdout)
    out = _bench(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode != 0 and "--gpus 4" in (out.stderr + out.stdout)
