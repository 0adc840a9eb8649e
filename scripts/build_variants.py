#!/usr/bin/env python
"""Build experimental libpandasim variants (extra compiler flags) into
scripts/bin/variants/ for scripts/time_variants.py."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "panda-lang-manip_amd"))
from pandasim import build as B  # noqa: E402

VARIANTS = {
    # round 6: the group kernels' XCD-aware block order (ps_common.h step_block):
    # none, the whole range at 8 and 16 lanes, tiles at 8 and 16 lanes
    "noremap": ["-DPS_XCD_REMAP=0"],
    "remapwhole": ["-DPS_XCD_REMAP=2"],
    "remaptile": ["-DPS_XCD_REMAP=3"],
    # timing only (wrong physics): the diagnostic build without Stack's box-box rows
    "prof_nopair": ["-DPS_PROFILE_PHASES", "-DPS_EXPERIMENT_NO_PAIR_ROWS"],
    "prof_norobot": ["-DPS_PROFILE_PHASES", "-DPS_EXPERIMENT_NO_ROBOT_ROWS"],
    "base": [],
    "maxilp": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    "bias0": ["-mllvm", "-amdgpu-schedule-metric-bias=0"],
    "unroll_off": ["-mllvm", "-amdgpu-unroll-threshold-private=0"],
    "ilp_min": ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"],
    "no_early_if": ["-mllvm", "-amdgpu-early-ifcvt=0"],
    # IEEE mode off: drops the v_max x,x,x canonicalisations before min/max
    # (68 of ~3000 instructions in the Push PGS loop); NaN handling only
    "ieee_off": ["-fno-honor-nans", "-mno-amdgpu-ieee"],
    "trackers": ["-mllvm", "-amdgpu-use-amdgpu-trackers"],
    "no_unclust": ["-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule"],
    "trk_nu": ["-mllvm", "-amdgpu-use-amdgpu-trackers", "-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule"],
    "trk_ilpmin": ["-mllvm", "-amdgpu-use-amdgpu-trackers", "-mllvm", "-amdgpu-sched-strategy=max-memory-clause"],
    # group-kernel miscompute bisection
    "o1": ["-O1"],
    "prealloc": ["-mllvm", "-amdgpu-prealloc-sgpr-spill-vgprs=1"],
    "nodppc": ["-mllvm", "-amdgpu-dpp-combine=0"],
    # the group solver's row dump (scripts/row_dump.py): product objects, and
    # the group objects at -O3
    "dump": ["-DPS_DEBUG_ROW_DUMP"],
    "groups_o3_dump": ["-DPS_DEBUG_ROW_DUMP"],
    # the group sums with FMA contraction left on (the round-3 miscompute?
    # DESIGN.md §12.6)
    "group_contract": ["-DPS_EXPERIMENT_GROUP_SUM_CONTRACT"],

}


# variants that change the per-unit flags of build.UNITS instead
_TRK = ["-mllvm", "-amdgpu-use-amdgpu-trackers"]
_CLAUSE = ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]


def _one_lane(units, flags_of_task):
    out = []
    for n, s, defs in units:
        if n.startswith("step_t") and not n.endswith("_groups"):
            defs = [d for d in defs if d not in _TRK + _CLAUSE] + flags_of_task(int(n[6]))
        out.append((n, s, defs))
    return out


_TWO_WAVES = ["-DPS_EXPERIMENT_TWO_WAVES", "-DPS_STEP_MIN_WAVES=2"]

UNIT_VARIANTS = {
    # round 6: two lanes per env (group_pgs at G = 2, eight
    # DoF slots per lane), the group objects register-allocated for two waves
    # per SIMD; ps_set_lanes_per_env accepts 2 in this build only
    "g2": lambda units: [(n, s, defs + ["-DPS_EXPERIMENT_G2"] + (["-DPS_STEP_MIN_WAVES=2"] if n.endswith("_groups") else []))
                         for n, s, defs in units],
    # the group kernels (one LDS column per env since round 5) register-allocated
    # for two waves per SIMD
    "groups_2w": lambda units: [(n, s, defs + (["-DPS_STEP_MIN_WAVES=2"] if n.endswith("_groups") else []))
                                for n, s, defs in units],
    # the one-lane step kernels at two waves per SIMD (M^-1 J^T, candidate
    # records and stash in global memory, 256 registers); the
    # ABI object allocates the global buffer, the group objects stay as built
    # (Reach and Push only: with the flag, MJStore::at() addresses the global
    # buffer, which a Stack kernel built so would read through a null base)
    "two_waves": lambda units: [(n, s, defs + (_TWO_WAVES if n in ("step_t0_c0", "step_t0_c1", "step_t1_c0",
                                                                    "step_t1_c1", "pandasim") else []))
                                for n, s, defs in units],
    # scheduler options on the one-lane step objects only
    "onelane_trk": lambda units: _one_lane(units, lambda t: _TRK),
    "onelane_trk_clause": lambda units: _one_lane(units, lambda t: _TRK + (_CLAUSE if t != 4 else [])),
    # scheduler options on the -O1 group objects too
    "groups_trk": lambda units: [(n, s, defs + (_TRK if n.endswith("_groups") else [])) for n, s, defs in units],
    "groups_trk_clause": lambda units: [(n, s, defs + (_TRK + _CLAUSE if n.endswith("_groups") else []))
                                        for n, s, defs in units],
    # further scheduler options on the one-lane objects (on top of the product's)
    "onelane_iterilp": lambda units: _one_lane(units, lambda t: _TRK + ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]),
    "onelane_itermin": lambda units: _one_lane(units, lambda t: _TRK + ["-mllvm", "-amdgpu-sched-strategy=iterative-minreg"]),
    "onelane_clause_nu": lambda units: _one_lane(units, lambda t: _TRK + (_CLAUSE if t != 4 else []) + [
        "-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule"]),
    "onelane_greedyrev": lambda units: _one_lane(units, lambda t: _TRK + (_CLAUSE if t != 4 else []) + [
        "-mllvm", "-greedy-reverse-local-assignment"]),
    "onelane_mix": lambda units: _one_lane(units, lambda t: _TRK + (
        _CLAUSE + ["-mllvm", "-greedy-reverse-local-assignment"] if t != 4 else [])),
    "groups_rev": lambda units: [(n, s, defs + (["-mllvm", "-greedy-reverse-local-assignment"]
                                                if n.endswith("_groups") else [])) for n, s, defs in units],
    "stack_itermin": lambda units: [(n, s, defs + (["-mllvm", "-amdgpu-sched-strategy=iterative-minreg"]
                                                   if n.startswith("step_t4_") else [])) for n, s, defs in units],
    "stack_nu": lambda units: [(n, s, defs + (["-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule"]
                                              if n.startswith("step_t4_") else [])) for n, s, defs in units],
    "groups_maxilp": lambda units: [(n, s, defs + (["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
                                                   if n.endswith("_groups") else [])) for n, s, defs in units],
    "groups_minreg": lambda units: [(n, s, defs + (["-mllvm", "-amdgpu-sched-strategy=iterative-minreg"]
                                                   if n.endswith("_groups") else [])) for n, s, defs in units],
    "groups_nu": lambda units: [(n, s, defs + (["-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule"]
                                               if n.endswith("_groups") else [])) for n, s, defs in units],
    # the product before r03k: no scheduler options on the one-lane objects
    "onelane_plain": lambda units: [(n, s, [d for d in defs if d not in _TRK + _CLAUSE]) for n, s, defs in units],
    # the group-kernel objects at the library's -O3 (the product builds them at
    # -O1)
    "groups_o3": lambda units: [(n, s, [d for d in defs if d != "-O1"]) for n, s, defs in units],
    "groups_o3_dump": lambda units: [(n, s, [d for d in defs if d != "-O1"]) for n, s, defs in units],
    # the scheduler matrix pruned to one set per object class:
    # no -mllvm scheduler option on any object
    "pruned": lambda units: [(n, s, [d for d in defs if not d.startswith("-amdgpu-") and not d.startswith("-greedy")
                                     and d != "-mllvm"]) for n, s, defs in units],
}


def main(names):
    out_dir = os.path.join(ROOT, "scripts", "bin", "variants")
    os.makedirs(out_dir, exist_ok=True)
    product_units = list(B.UNITS)
    for n in names:
        out = os.path.join(out_dir, f"lib_{n}.so")
        B.UNITS = UNIT_VARIANTS[n](product_units) if n in UNIT_VARIANTS else product_units
        try:
            B.build(variant="", extra=VARIANTS.get(n, []), out=out, verbose=False)
            print(n, "ok")
        except Exception as e:  # a variant that does not compile is reported, not fatal
            print(n, "failed:", e)


if __name__ == "__main__":
    main(sys.argv[1:] or list(VARIANTS) + list(UNIT_VARIANTS))
