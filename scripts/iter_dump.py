#!/usr/bin/env python
"""Per-env PGS iterations and contact slots of the one-lane step kernel
(diagnostic build libpandasim_prof.so, PhaseTimer::itp: 16 bits per substep,
iterations, gripper slots nr, box-box slots np): runs the bench workload
(seeded resets, U(-1, 1) actions) and asks how much of the wave's PGS a
different env-to-wave assignment would save.

A wave's PGS runs until its slowest lane has converged, and runs a contact
slot's rows while any lane has that slot: its cost per substep is modelled as
max_it x (C0 + CR max_nr + CP max_np) over its 64 lanes (C0, CR, CP from the
phase splits with and without the gripper and box-box rows,
profiles/r06v_phase.log, r06w_phase.log).  The assignment tested: before each
step, the envs of each window of W consecutive envs are sorted by a key from
the previous step (its PGS iterations, or its contact slots) and dealt to the
window's W / 64 waves in that order.  Prints, per step, the modelled cost of
the sorted assignments relative to the identity, and saves the dump (uint16
[step, substep, env]) to gpurun_out/iter_dump_<env>.npz."""
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
WORDS = 10
WINDOWS = (256, 1024, 4096, 65536)
C0, CR, CP = 2360.0, 664.0, 817.0  # cycles per iteration: base, per open gripper slot, per open box-box slot


def wave_cost(it, nr, np_, order=None):
    """it, nr, np_: [substeps, B]; order: env of each lane (None: identity).
    Modelled PGS cycles per wave-substep."""
    if order is not None:
        it, nr, np_ = it[:, order], nr[:, order], np_[:, order]
    s, b = it.shape
    mx = lambda x: x.reshape(s, b // 64, 64).max(axis=2)
    return (mx(it) * (C0 + CR * mx(nr) + CP * mx(np_))).mean()


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
    buf = np.zeros(WORDS * DUMP_ENVS, dtype=np.uint32)
    g = torch.Generator(device="cuda")
    g.manual_seed(0xC0FFEE)
    counts = np.zeros((steps, 20, B), dtype=np.uint16)
    for k in range(steps + 5):
        env.step(torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1, copy=False)
        torch.cuda.synchronize()
        if k < 5:
            continue
        assert lib.ps_debug_env_iters(buf.ctypes.data) == 0
        w = buf.reshape(WORDS, DUMP_ENVS)[:, :B]
        # half j of the 20 (newest first) -> substep 19 - j
        for j in range(20):
            counts[k - 5, 19 - j] = (w[j // 2] >> (16 * (j % 2))) & 0xFFFF
    it = (counts & 0xFF).astype(np.int32)
    nr = ((counts >> 8) & 7).astype(np.int32)
    npc = ((counts >> 11) & 7).astype(np.int32)
    print(f"{env_id} B={B}: PGS iterations per lane-substep mean {it.mean():.2f}, at the cap 50: "
          f"{(it >= 50).mean() * 100:.1f} %; gripper slots per lane-substep {nr.mean():.2f} "
          f"(envs with any in a step {(nr.max(axis=1) > 0).mean() * 100:.1f} %), box-box {npc.mean():.3f} "
          f"(any {(npc.max(axis=1) > 0).mean() * 100:.1f} %)")
    keys = {"iterations": it.sum(axis=1), "slots": 8 * npc.max(axis=1) + nr.max(axis=1)}
    rel = {(kn, W): [] for kn in keys for W in WINDOWS}
    for s in range(1, steps):
        base = wave_cost(it[s], nr[s], npc[s])
        for kn, key in keys.items():
            for W in WINDOWS:
                rel[(kn, W)].append(wave_cost(it[s], nr[s], npc[s], sorted_order(key[s - 1], W)) / base)
        # the bound: this step's own slots (not knowable before the step)
        rel.setdefault(("slots, same step", 65536), []).append(
            wave_cost(it[s], nr[s], npc[s], sorted_order(keys["slots"][s], 65536)) / base)
    for (kn, W), v in rel.items():
        print(f"  sorted by last step's {kn:10s} in windows of {W:6d}: modelled PGS cost {np.mean(v):.3f} of the identity's")
    for name, key in (("slots", keys["slots"]),):
        a = key > 0
        print(f"  an env with contact slots in step s has them in s+1 with p = "
              f"{(a[1:] & a[:-1]).sum() / max(a[:-1].sum(), 1):.3f}; without them: p = "
              f"{(a[1:] & ~a[:-1]).sum() / max((~a[:-1]).sum(), 1):.3f}")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"iter_dump_{env_id}.npz"), counts=counts[:8])


if __name__ == "__main__":
    main()
