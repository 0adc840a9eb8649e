#!/usr/bin/env python
"""Benchmark: batched env-steps/s of PandaPush-v3 on MI355X (BASELINE.json metric).

Workload: PandaPush-v3 (sparse, ee control), 65 536
envs per GPU (weak scaling; 524 288 at 8 GPUs), env i of rank r seeded with
12345 + r*B + i, i.i.d. U(-1, 1) fp32 actions from a Philox stream seeded
0xC0FFEE + rank, auto-reset on terminated|truncated.  One "step" = one fused
RobotTaskEnv.step() of every env (20 physics substeps + IK + obs + reward).

Launch: python bench.py [--gpus N --steps K --warmup W].  For N > 1 the
script starts `torch.distributed.run --nproc-per-node N` as a child process
(one rank per GPU, RCCL) unless it already runs under torch.distributed.run
(WORLD_SIZE set, which must equal N).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "panda-lang-manip_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_PEAK_TFLOPS = 157.3


def contact_cache_floats(n_objects: int) -> int:
    """Contact-cache rows a task's step reads and writes (include/pandasim.h
    PS_F_WG0..): 4 impulses + 1 id row per object's ground contacts and for
    the gripper contacts; Stack adds 4 impulses, 12 points and a count."""
    return 5 * n_objects + 5 + (17 if n_objects == 2 else 0)


def algorithmic_bytes_per_env_step(obs_dim: int, action_dim: int, goal_dim: int = 3, n_objects: int = 1) -> int:
    """Bytes one env-step must move through HBM:
    read q,qd (18 f32), 13 f32 per object, the contact cache, goal (f64),
    TimeLimit counter, action; write q,qd, the 9 motor targets and 9 max
    impulses (the gain rows are invariant, pandasim.hip store_motor_targets),
    objects, the contact cache, counter, obs, ag, dg (f32), reward, 2 flags,
    final_obs + final_ag.  PandaPush-v3: 630 B."""
    cache = contact_cache_floats(n_objects) * 4
    read = 18 * 4 + 13 * 4 * n_objects + cache + goal_dim * 8 + 4 + action_dim * 4
    write = (18 * 4 + 18 * 4 + 13 * 4 * n_objects + cache + 4 + obs_dim * 4 + 2 * goal_dim * 4 + 4 + 2
             + obs_dim * 4 + goal_dim * 4)
    return read + write


def host_threads() -> int:
    """Host threads this process may use: the affinity mask, capped by
    OMP_NUM_THREADS (16 on the GPU box, whose nproc shows the whole machine)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(task: str, seconds: float):
    """The oracle (fp64 C restatement) on a bounded sample of the same workload:
    a third of the time on 1 host thread, the rest on every host thread this
    process may use (OpenMP over envs, oracle/panda_oracle.c po_step_batch).
    `value`/`cores` are the all-threads figure; `value_1core` the scalar one."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    cfg = O.config(task)
    threads = host_threads()
    na, od = O.action_dim(cfg), O.obs_dim(cfg)
    fp = lambda a: a.ctypes.data_as(O.C.POINTER(O.C.c_float))
    u8 = lambda a: a.ctypes.data_as(O.C.POINTER(O.C.c_uint8))

    def run(n_threads, n_env, budget):
        used = O.lib().po_set_threads(n_threads)
        envs = (O.Env * n_env)()
        for i in range(n_env):
            O.lib().po_init_env(O.C.byref(cfg), O.C.byref(envs[i]))
            O.lib().po_reset(O.C.byref(cfg), O.C.byref(envs[i]), 1, 12345 + i, None, None, None)
        rng = np.random.default_rng(0xC0FFEE)
        obs = np.zeros((n_env, od), np.float32)
        ag = np.zeros((n_env, 3), np.float32)
        dg = np.zeros((n_env, 3), np.float32)
        rew = np.zeros(n_env, np.float32)
        te = np.zeros(n_env, np.uint8)
        tr = np.zeros(n_env, np.uint8)
        steps = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget:
            a = rng.uniform(-1, 1, size=(n_env, na)).astype(np.float32)
            O.lib().po_step_batch(O.C.byref(cfg), envs, n_env, fp(a), fp(obs), fp(ag), fp(dg), fp(rew), u8(te),
                                  u8(tr), 1, None)
            steps += 1
        dt = time.perf_counter() - t0
        return n_env * steps / dt, used, steps, dt

    v1, _, s1, d1 = run(1, 64, seconds / 3)
    work = oracle_work_counts(O, cfg)
    n_env = 16 * threads
    vn, used, sn, dn = run(threads, n_env, seconds * 2 / 3)
    O.lib().po_set_threads(1)
    return work, {"value": round(vn, 2), "unit": "env-steps/s", "cores": used, "kind": "port",
            "value_1core": round(v1, 2), "phase_split_1core": cpu_phase_split(O, task),
            "c1_reach_dense_1env": cpu_reach_dense_1env(O),
            "cpu_model": cpu_model(),
            "sample": f"{n_env} envs x {sn} steps of {task} (ee, sparse) in {dn:.1f} s on {used} host threads "
                      f"(OpenMP over envs) + 64 envs x {s1} steps in {d1:.1f} s on 1 thread; fp64 oracle, "
                      f"PyBullet not installed on the box"}


def oracle_work_counts(O, cfg, n_env: int = 64, steps: int = 60) -> dict:
    """Work counters (po_stats: PGS iterations and rows per substep, contacts,
    IK iterations) of the oracle stepping a sample of the bench workload --
    seeds 12345 + i, U(-1, 1) actions, auto-reset -- for the FLOP roofline."""
    import numpy as np

    envs = [O.new_env(cfg) for _ in range(n_env)]
    for i, e in enumerate(envs):
        O.reset(cfg, e, seed=12345 + i)
    rng = np.random.default_rng(0xC0FFEE)
    st = O.Stats()
    for _ in range(steps):
        for e in envs:
            O.step(cfg, e, rng.uniform(-1, 1, O.action_dim(cfg)).astype(np.float32), autoreset=True, stats=st)
    return st.as_dict()


WORK_COUNTS = "profiles/oracle_work_counts.json"


def committed_work_counts(task: str):
    """oracle_work_counts() of `task` as committed by scripts/oracle_work_counts.py
    (a data file: nothing under oracle/ runs), or None."""
    try:
        with open(os.path.join(ROOT, WORK_COUNTS)) as f:
            return json.load(f).get(task)
    except (OSError, ValueError):
        return None


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_phase_split(O, task: str, n_env: int = 16, steps: int = 3):
    """Share of one CPU env-step (fp64 oracle, 1 thread) in Panda.set_action's
    IK, the 20 substeps and the rest (obs, reward, TimeLimit) -- SURVEY.md §8(d)."""
    import numpy as np

    cfg = O.config(task)
    envs = [O.new_env(cfg) for _ in range(n_env)]
    for i, e in enumerate(envs):
        O.reset(cfg, e, seed=12345 + i)
    rng = np.random.default_rng(1)
    t_step = t_ik = t_sim = 0.0
    for _ in range(steps):
        for e in envs:
            a = rng.uniform(-1, 1, O.action_dim(cfg)).astype(np.float32)
            t0 = time.perf_counter()
            pos, _, _, _ = O.link_state(cfg, e, 11)
            O.inverse_kinematics(cfg, np.array(e.q[:]), 11, pos + 0.05 * a[:3], np.array([1.0, 0.0, 0.0, 0.0]))
            t1 = time.perf_counter()
            O.sim_step(cfg, e)
            t2 = time.perf_counter()
            O.step(cfg, e, a, autoreset=True)
            t3 = time.perf_counter()
            t_ik += t1 - t0
            t_sim += t2 - t1
            t_step += t3 - t2
    k = 1e6 / (n_env * steps)
    return {"unit": "us per env-step", "step": round(t_step * k, 1), "ik": round(t_ik * k, 1),
            "substeps": round(t_sim * k, 1), "note": "ik and substeps timed separately on the same states "
            "(substeps with the previous step's motors); their sum can exceed step by the PGS-iteration spread"}


def cpu_reach_dense_1env(O, seconds: float = 1.0):
    """BASELINE configs[0]: PandaReachDense-v3, 1 env, on the CPU (fp64 oracle)."""
    import numpy as np

    cfg = O.config("reach", reward="dense")
    env = O.new_env(cfg)
    O.reset(cfg, env, seed=12345)
    rng = np.random.default_rng(0)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        O.step(cfg, env, rng.uniform(-1, 1, 3).astype(np.float32), autoreset=True)
        n += 1
    return {"value": round(n / (time.perf_counter() - t0), 1), "unit": "env-steps/s", "cores": 1}


def fp32_roofline(work: dict, n_objects: int, env_steps_per_s_per_gpu: float) -> dict:
    """Algorithmic FP32 FLOP rate of one GPU against the vector peak
    (pandasim/roofline.py: per-primitive costs x the oracle's work counts on
    a sample of the same workload)."""
    from pandasim.roofline import flops_per_env_step

    f = flops_per_env_step(work, n_objects)
    achieved = f["flops_per_env_step"] * env_steps_per_s_per_gpu / 1e12
    return dict(f, achieved_tflops=round(achieved, 3), peak_tflops=VALU_PEAK_TFLOPS,
                frac=round(achieved / VALU_PEAK_TFLOPS, 4), unit="TFLOP/s",
                note="algorithmic FLOPs (each env's own PGS iterations) over the packed-FMA vector peak; "
                     "the kernel mixes scalar v_fma_f32 with v_pk_fma_f32 (DESIGN.md 12.12) and runs the PGS "
                     "to the wave's slowest env: roofline.fp32_executed has the counted work")


def file_sha256(path: str):
    import hashlib

    try:
        h = hashlib.sha256()
        with open(path, "rb") as f:
            for chunk in iter(lambda: f.read(1 << 20), b""):
                h.update(chunk)
        return h.hexdigest()
    except OSError:
        return None


def pmc_entry(workload: str, lib_path: str, path: str | None = None):
    """The committed rocprofv3 PMC figures of k_step for `workload`
    (profiles/pmc_traffic.json, scripts/summarize_profiles.py) and their
    status.  They describe one binary: the entry records the sha256 of the
    libpandasim.so it was measured on, and it is used only when that equals
    the hash of the library this process loaded ("current"); otherwise
    ("stale", or "missing") the PMC-derived fields are left out of the line."""
    path = path or os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        entry = json.load(open(path)).get(workload)
    except Exception:
        entry = None
    lib_hash = file_sha256(lib_path)
    if entry is None:
        return None, {"status": "missing", "lib_sha256": lib_hash}
    status = "current" if entry.get("lib_sha256") and entry.get("lib_sha256") == lib_hash else "stale"
    info = {"status": status, "lib_sha256": lib_hash, "measured_on": entry.get("lib_sha256"),
            "source": entry.get("source")}
    return (entry if status == "current" else None), info


def launch_command(n: int, argv) -> list:
    """The child command of `bench.py --gpus N` (N > 1): torch.distributed.run
    with one process per GPU on this node, rendezvous on 127.0.0.1, each rank
    running this script with the same arguments."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    argv = [a for a in argv if a != "--print-launch"]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--env-id", default="PandaPush-v3")
    ap.add_argument("--batch", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--lanes", type=int, default=0, help="lanes per env of the step kernel: 1, 8, 16, 0 = auto")
    ap.add_argument("--print-launch", action="store_true",
                    help="print the child command that --gpus N > 1 would start, and exit")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus > 1 or args.print_launch):
        # N ranks requested from a plain `python bench.py --gpus N`: start them as
        # a child torch.distributed.run (one process per GPU) before anything
        # here touches the GPU, wait for it and exit with its status
        cmd = launch_command(args.gpus, sys.argv[1:])
        if args.print_launch:
            print(json.dumps({"launch": cmd}))
            return
        import subprocess

        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        raise SystemExit(subprocess.run(cmd, env=env).returncode)
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU "
                         f"(plain `python bench.py --gpus {args.gpus}` starts them)")

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; the modulo only matters when rehearsing N ranks on
    # fewer GPUs (PANDASIM_DIST_BACKEND=gloo: RCCL refuses two ranks per GPU)
    dev = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        backend = os.environ.get("PANDASIM_DIST_BACKEND", "nccl")  # "nccl" is RCCL on ROCm
        if backend == "nccl" and world > torch.cuda.device_count():
            raise SystemExit(f"bench.py: {world} ranks but {torch.cuda.device_count()} GPUs visible; RCCL needs one "
                             "GPU per rank (PANDASIM_DIST_BACKEND=gloo rehearses more ranks than GPUs)")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")

    import pandasim
    from pandasim.dist import gather_to_rank0, max_over_ranks, shard_seeds
    from pandasim.envs import REGISTRY

    B = args.batch
    env = pandasim.make(args.env_id, num_envs=B, device=dev, lanes_per_env=args.lanes)
    spec = REGISTRY[args.env_id]
    # rank r owns global envs [r*B, (r+1)*B), env g seeded 12345 + g
    env.reset(seed=shard_seeds(12345, world * B, world, rank).numpy().astype("uint64"))
    gen = torch.Generator(device=dev)
    gen.manual_seed(0xC0FFEE + rank)
    n_act = args.warmup + args.steps
    actions = torch.rand(n_act, B, env.action_dim, device=dev, generator=gen) * 2 - 1
    # episode returns and successes, accumulated inside the step kernel
    # (RecordEpisodeStatistics fused: ps_set_episode_stats); rows 1-3 are
    # EpisodeStats.packed()'s layout
    eps = env.record_episode_statistics()

    for k in range(args.warmup):
        obs, r, te, tr, info = env.step(actions[k], copy=False)
    gather_to_rank0(eps[1:].contiguous())  # also loads the collective path
    eps.zero_()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    stops = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        a = actions[args.warmup + k]
        starts[k].record()
        obs, r, te, tr, info = env.step(a, copy=False)
        stops[k].record()
    # the one collective of the path: episode statistics to rank 0 (RCCL over xGMI)
    episode_stats = gather_to_rank0(eps[1:].contiguous())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(s.elapsed_time(e) for s, e in zip(starts, stops)) / args.steps
    elapsed = max_over_ranks(elapsed, dev)

    total_env_steps = world * B * args.steps
    value = total_env_steps / elapsed
    bytes_env = algorithmic_bytes_per_env_step(env.obs_dim, env.action_dim, env.goal_dim, env.sim.cfg.n_objects)
    achieved = bytes_env * B / (kernel_ms * 1e-3) / 1e9
    workload = f"{args.env_id} x{B}/gpu"
    from pandasim import _lib as _L

    pmc, pmc_info = pmc_entry(workload, _L.LIB_PATH)
    pmc = pmc or {}
    out = {
        "metric": "env steps/sec (batched) PandaPush-v3 at 1/2/4/8 MI355X vs PyBullet CPU",
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": dist.get_world_size() if world > 1 else 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded resets, U(-1,1) actions)",
        "config": {"workload": workload, "env_id": args.env_id, "task": spec["task"],
                   "control": spec["control_type"], "reward": spec["reward_type"], "batch_per_gpu": B,
                   "global_batch": world * B, "substeps": 20, "parallelism": f"batch shard x{world}",
                   "lanes_per_env": env.lanes_per_env},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": pmc.get("bytes_per_launch"),
                     "kernel": f"k_step<{spec['task'].upper()},{spec['control_type'].upper()},{env.lanes_per_env}>",
                     "kernel_ms": round(kernel_ms, 4),
                     "bytes_per_env_step": bytes_env, "pmc": pmc_info},
    }
    # The binding limit is VALU issue, not HBM: one wave per
    # SIMD at 65 536 envs (1 024 waves on 1 024 SIMDs) issues at most one VALU
    # instruction per 4 cycles (MI355X_MICROARCH.md, 'vector-instruction ISSUE
    # cost'), two or more waves per SIMD one per 2 cycles.
    valu = pmc.get("valu_insts_per_launch")
    if valu:
        rate = valu / (kernel_ms * 1e-3)
        simds, clk = 256 * 4, 2.4e9
        out["roofline"]["valu_issue"] = {
            "achieved": round(rate / 1e9, 2), "unit": "G wave-instr/s",
            "peak_one_wave_per_simd": round(simds * clk / 4 / 1e9, 2), "peak_dual_issue": round(simds * clk / 2 / 1e9, 2),
            "frac_one_wave_per_simd": round(rate / (simds * clk / 4), 4),
            "valu_insts_per_launch": valu, "source": "profiles/pmc_traffic.json (SQ_INSTS_VALU)"}
    executed = pmc.get("fp32_flops_executed_per_launch")
    if executed:
        rate = executed / (kernel_ms * 1e-3) / 1e12
        out["roofline"]["fp32_executed"] = {
            "achieved_tflops": round(rate, 3), "peak_tflops": VALU_PEAK_TFLOPS, "frac": round(rate / VALU_PEAK_TFLOPS, 4),
            "flops_per_launch": executed,
            "source": "profiles/pmc_traffic.json: " + pmc.get("fp32_flops_counter", "SQ_INSTS_VALU_*_F32") +
                      ", x 64 lanes",
            "packed_included": "packed included" in pmc.get("fp32_flops_counter", "")}
    if rank == 0:
        ep = episode_stats.double().cpu()
        done = ep[2] > 0
        out["episodes"] = {"envs_with_finished_episode": int(done.sum()),
                           "mean_last_return": round(float(ep[0][done].mean()), 4) if done.any() else None,
                           "last_success_rate": round(float(ep[1][done].mean()), 4) if done.any() else None,
                           "gathered_envs": int(ep.shape[1])}
        work = None
        if world == 1 and not args.no_cpu_baseline:
            work, out["cpu_baseline"] = cpu_baseline(spec["task"], args.cpu_seconds)
        else:
            # N > 1 (the CPU baseline is rank 0's at N = 1 only) or no CPU leg:
            # the FLOP roofline from the committed work counts of the same
            # oracle sample (scripts/oracle_work_counts.py)
            work = committed_work_counts(spec["task"])
        if work is not None:
            out["roofline"]["fp32"] = fp32_roofline(work, env.sim.cfg.n_objects, value / world)
            if world > 1 or args.no_cpu_baseline:
                out["roofline"]["fp32"]["work_source"] = WORK_COUNTS
            ex = out["roofline"].get("fp32_executed")
            if ex and ex["packed_included"]:
                # executed (PMC) over algorithmic FLOPs per launch: the share of
                # issue spent on lanes whose env has already converged, gated
                # rows a lane lacks, and the like -- only from a
                # counter that weighs the packed instructions right (round 6:
                # SQ_INSTS_VALU_FLOPS_FP32; the old instruction counters took a
                # v_pk_fma_f32 for one FMA)
                algo = out["roofline"]["fp32"]["flops_per_env_step"] * B
                ex["executed_over_algorithmic"] = round(ex["flops_per_launch"] / algo, 3)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
