#!/usr/bin/env python
"""Per-env PGS iteration counts of the one-lane step kernel (diagnostic build
libpandasim_prof.so, PhaseTimer::itp): runs the bench workload (seeded
resets, U(-1, 1) actions) and asks how much of the wave's PGS issue a
different env-to-wave assignment would save.

A wave's PGS runs until its slowest lane has converged, so its cost per
substep is the max over its 64 lanes; the lane mean is the floor.  The
assignment tested: before each step, the envs of a window of W consecutive
envs are sorted by their iteration total of the previous step and dealt to
the window's W / 64 waves in that order.  Prints, per step, the wave cost of
the identity assignment and of the sorted one at each W, in iterations per
wave-substep, and saves the counts (uint8 [step, substep, env]) to
gpurun_out/iter_dump_<env>.npz."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "panda-lang-manip_amd"))
os.environ["PANDASIM_LIB"] = os.path.join(ROOT, "panda-lang-manip_amd", "pandasim", "libpandasim_prof.so")

import torch  # noqa: E402

import pandasim  # noqa: E402
from pandasim import _lib as L  # noqa: E402

DUMP_ENVS = 131072
WINDOWS = (128, 256, 512, 1024, 4096, 65536)


def wave_cost(it, order=None):
    """it: [substeps, B] iterations; order: env of each lane (None: identity)."""
    x = it if order is None else it[:, order]
    s, b = x.shape
    return x.reshape(s, b // 64, 64).max(axis=2).mean()


def sorted_order(key, W):
    B = key.shape[0]
    order = np.empty(B, dtype=np.int64)
    for w0 in range(0, B, W):
        idx = np.arange(w0, min(w0 + W, B))
        order[w0:w0 + len(idx)] = idx[np.argsort(-key[idx], kind="stable")]
    return order


def main():
    env_id = sys.argv[1] if len(sys.argv) > 1 else "PandaPush-v3"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 24
    assert B <= DUMP_ENVS and B % 64 == 0
    env = pandasim.make(env_id, num_envs=B, lanes_per_env=1)
    env.reset(seed=12345)
    lib = L.lib()
    lib.ps_debug_env_iters.argtypes = [C.c_void_p]
    buf = np.zeros(5 * DUMP_ENVS, dtype=np.uint32)
    g = torch.Generator(device="cuda")
    g.manual_seed(0xC0FFEE)
    counts = np.zeros((steps, 20, B), dtype=np.uint8)
    for k in range(steps + 5):
        env.step(torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1, copy=False)
        torch.cuda.synchronize()
        if k < 5:
            continue
        assert lib.ps_debug_env_iters(buf.ctypes.data) == 0
        w = buf.reshape(5, DUMP_ENVS)[:, :B]
        # byte j of the 20 (newest first) -> substep 19 - j
        for j in range(20):
            counts[k - 5, 19 - j] = (w[j // 4] >> (8 * (j % 4))) & 0xFF
    print(f"{env_id} B={B}: PGS iterations per lane-substep mean {counts.mean():.2f}, "
          f"share at the cap 50: {(counts >= 50).mean() * 100:.1f} %")
    tot = counts.astype(np.int32).sum(axis=1)  # [step, env]
    for s in range(steps):
        it = counts[s].astype(np.int32)
        line = [f"step {s:2d}: lane mean {it.mean():5.2f}  identity {wave_cost(it):5.2f}"]
        if s > 0:
            for W in WINDOWS:
                line.append(f"W{W} {wave_cost(it, sorted_order(tot[s - 1], W)):5.2f}")
            line.append(f"oracle-W256 {wave_cost(it, sorted_order(tot[s], 256)):5.2f}")
        print("  ".join(line))
    if steps > 1:
        c = np.corrcoef(tot[:-1].ravel(), tot[1:].ravel())[0, 1]
        print(f"correlation of an env's step totals, step s and s+1: {c:.3f}")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"iter_dump_{env_id}.npz"), counts=counts[:8])


if __name__ == "__main__":
    main()
