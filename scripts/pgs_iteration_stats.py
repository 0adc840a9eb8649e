#!/usr/bin/env python
"""PGS iteration statistics from the fp64 oracle (test infrastructure; the
oracle's po_set_pgs_log hook): per env, step and substep the iterations the
solver ran, and what a 64-lane wave would run (the max over its envs) under
different deals of envs to lanes -- index order, sorted by the previous
step's total, and the per-substep ideal.

    python scripts/pgs_iteration_stats.py [task] [envs] [steps]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def main():
    task = sys.argv[1] if len(sys.argv) > 1 else "push"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    cfg = O.config(task, "ee", "sparse")
    L = O.lib()
    envs = [O.new_env(cfg) for _ in range(B)]
    for i, e in enumerate(envs):
        O.reset(cfg, e, seed=12345 + i)
    rng = np.random.default_rng(0xC0FFEE)
    it = np.zeros((T, B, 20), np.int32)
    buf = np.zeros(20, np.int32)
    for t in range(T):
        acts = rng.uniform(-1, 1, (B, O.action_dim(cfg))).astype(np.float32)
        for i, e in enumerate(envs):
            L.po_set_pgs_log(buf.ctypes.data, 20)
            O.step(cfg, e, acts[i], autoreset=True)
            assert L.po_set_pgs_log(None, 0) == 20
            it[t, i] = buf
    W = B // 64
    x = it[:, :W * 64]
    print(f"{task} B={B} steps={T}: lane mean {x.mean():.2f} iterations per substep, "
          f"{(x == 50).mean() * 100:.1f} % of env-substeps at the cap")
    per_env_cap = (x == 50).mean(axis=2)  # [T, B] share of a step's substeps at the cap
    print("  share of a step's substeps at the cap, histogram over env-steps:",
          np.histogram(per_env_cap, bins=[0, .01, .2, .4, .6, .8, .99, 1.01])[0])
    print("  iterations by substep index (mean over env-steps):", np.round(x.mean(axis=(0, 1)), 1).tolist())

    def wave_max(order_t):  # order_t[t]: lane slot -> env
        tot = 0.0
        for t in range(T):
            y = x[t][order_t[t]].reshape(W, 64, 20)
            tot += y.max(axis=1).mean()
        return tot / T

    ident = [np.arange(W * 64)] * T
    tot = x.sum(axis=2)
    prev = [np.arange(W * 64)] + [np.argsort(-tot[t - 1], kind="stable") for t in range(1, T)]
    cur = [np.argsort(-tot[t], kind="stable") for t in range(T)]
    print(f"  wave max per substep: index order {wave_max(ident):.2f}, sorted by previous step's total "
          f"{wave_max(prev):.2f}, by this step's total {wave_max(cur):.2f}")
    # per-substep ideal: each substep sorted on its own
    ideal = np.mean([np.sort(x[t][:, s])[::-1].reshape(W, 64).max(axis=1).mean()
                     for t in range(T) for s in range(20)])
    print(f"  per-substep ideal (sorted each substep) {ideal:.2f}")
    corr = np.corrcoef(tot[1:].ravel(), tot[:-1].ravel())[0, 1]
    print(f"  step-to-step correlation of an env's total: {corr:.3f}")


if __name__ == "__main__":
    main()
