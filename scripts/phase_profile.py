#!/usr/bin/env python
"""Per-phase cycle split of the fused step kernel (diagnostic build
libpandasim_prof.so, -DPS_PROFILE_PHASES): runs B envs for a few steps and
prints the share of wave-cycles in each phase of k_step."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "panda-lang-manip_amd"))
# (PANDASIM_PROF_LIB: another diagnostic build, e.g. an experiment of scripts/build_variants.py)
os.environ["PANDASIM_LIB"] = os.environ.get("PANDASIM_PROF_LIB") or os.path.join(
    ROOT, "panda-lang-manip_amd", "pandasim", "libpandasim_prof.so")

import torch  # noqa: E402

import pandasim  # noqa: E402
from pandasim import _lib as L  # noqa: E402

NAMES = ["bias_forces", "fk+mass_matrix", "spd_inverse", "rows+contacts", "pgs", "integrate", "set_action+ik",
         "obs/reward/reset/store"]


def main():
    env_id = sys.argv[1] if len(sys.argv) > 1 else "PandaPush-v3"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    lanes = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    env = pandasim.make(env_id, num_envs=B, lanes_per_env=lanes)
    env.reset(seed=12345)
    lib = L.lib()
    lib.ps_debug_phase_cycles.argtypes = [C.c_void_p, C.c_int]
    buf = (C.c_ulonglong * 24)()
    g = torch.Generator(device="cuda")
    g.manual_seed(0xC0FFEE)
    for k in range(5):
        env.step(torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1, copy=False)
    torch.cuda.synchronize()
    lib.ps_debug_phase_cycles(buf, 1)
    for k in range(steps):
        env.step(torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1, copy=False)
    torch.cuda.synchronize()
    assert lib.ps_debug_phase_cycles(buf, 0) == 0
    # rows+contacts (slot 3) keeps the gripper rows; slots 16-18 hold its other parts
    buf[3] += buf[16] + buf[17] + buf[18]
    tot = sum(buf[:8])
    waves = (B * env.lanes_per_env + 63) // 64
    print(f"{env_id} B={B} lanes/env={env.lanes_per_env}: {tot / waves / steps:.0f} wave-cycles per wave-step")
    for n, v in zip(NAMES, buf[:8]):
        print(f"  {n:24s} {v / tot * 100:6.2f} %   {v / waves / steps / 20:10.0f} cyc/substep-equiv")
    if buf[3]:
        parts = (("joint rows", buf[16]), ("object contacts", buf[18]), ("gripper candidates", buf[17]),
                 ("gripper rows", buf[3] - buf[16] - buf[17] - buf[18]))
        print("  rows+contacts split: " + ", ".join(f"{n} {v / buf[3] * 100:.1f} %" for n, v in parts))
    subs = buf[10]  # wave-substeps counted by lane 0 of each wave
    print(f"  PGS iterations per substep: lane-0 mean {buf[8] / subs:.2f}, wave max {buf[9] / subs:.2f}; "
          f"max robot contacts per wave {buf[11] / subs:.2f}")
    print(f"  open row gates per wave-substep: pair slots {buf[12] / subs:.2f}, ground slots {buf[13] / subs:.2f}, "
          f"robot slots {buf[14] / subs:.2f}, joint limits {buf[15] / subs:.2f}")
    if buf[21] or buf[23]:
        print(f"  gripper bounding tests per wave-substep: box-object passed for {buf[21] / subs:.2f} boxes "
              f"({buf[20] / max(buf[21], 1):.1f} envs of the wave each), box-ground for {buf[23] / subs:.2f} "
              f"({buf[22] / max(buf[23], 1):.1f} envs each); the work lists evaluate them in one round per pass")


if __name__ == "__main__":
    main()
