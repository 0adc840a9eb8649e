#!/usr/bin/env python
"""Condense rocprofv3 output (gpurun_out/prof_*) into the committed summaries
under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_summary.json       per-kernel durations (all launches and the
                                    timed tail), resources, PMC bytes per launch
  profiles/pmc_traffic.json         {workload: HBM bytes per k_step launch}
                                    read by bench.py for roofline.traffic

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE (KiB) from separate --pmc passes; FETCH_SIZE is doubled on gfx950
(it tallies 128-B read requests at 64 B), and the calibration pass of
scripts/calib_fetch.hip (same 4-B-per-lane access width as the step kernel)
reports the factor actually observed, which replaces the default 2.0 when
present.

usage: python scripts/summarize_profiles.py <tag> <workload> [--steps K]
"""
from __future__ import annotations

import argparse
import collections
import csv
import hashlib
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0][:80]


def counters(path, counter):
    per = collections.defaultdict(list)
    if not os.path.exists(path):
        return per
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


def calibrate():
    """Observed bytes/counter ratios of scripts/calib_fetch.hip (4-B-per-lane
    streams over 1 GiB) from gpurun_out/calib_{fetch,write}/ and calib.log."""
    log = os.path.join(OUT, "calib.log")
    if not os.path.exists(log):
        return None
    known = None
    for line in open(log):
        if line.startswith("{"):
            known = json.loads(line)
    if not known:
        return None
    f = counters(os.path.join(OUT, "calib_fetch", "run_counter_collection.csv"), "FETCH_SIZE").get("k_read")
    w = counters(os.path.join(OUT, "calib_write", "run_counter_collection.csv"), "WRITE_SIZE").get("k_write")
    out = dict(known)
    if f:
        out["fetch_kib_per_launch"] = sum(f) / len(f)
        out["fetch_factor"] = known["read_bytes_per_launch"] / (out["fetch_kib_per_launch"] * 1024)
    if w:
        out["write_kib_per_launch"] = sum(w) / len(w)
        out["write_factor"] = known["write_bytes_per_launch"] / (out["write_kib_per_launch"] * 1024)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("workload")
    ap.add_argument("--steps", type=int, default=100, help="timed launches at the tail of the trace")
    ap.add_argument("--kernel", default="k_step")
    ap.add_argument("--prefix", default="prof")
    ap.add_argument("--lib", default=os.path.join(ROOT, "panda-lang-manip_amd", "pandasim", "libpandasim.so"),
                    help="the library the profiled run loaded (its sha256 goes into pmc_traffic.json)")
    args = ap.parse_args()
    os.makedirs(PROF, exist_ok=True)
    tdir = os.path.join(OUT, f"{args.prefix}_trace")
    shutil.copy(os.path.join(tdir, "run_kernel_stats.csv"), os.path.join(PROF, f"{args.tag}_kernel_stats.csv"))

    durs = collections.defaultdict(list)
    res = {}
    for r in csv.DictReader(open(os.path.join(tdir, "run_kernel_trace.csv"))):
        k = short(r["Kernel_Name"])
        durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        res[k] = {f: r[f] for f in ("LDS_Block_Size", "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count",
                                    "Workgroup_Size_X", "Grid_Size_X")}
    fetch = counters(os.path.join(OUT, f"{args.prefix}_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counters(os.path.join(OUT, f"{args.prefix}_write", "run_counter_collection.csv"), "WRITE_SIZE")

    extra = collections.defaultdict(dict)
    vpath = os.path.join(OUT, f"{args.prefix}_valu", "run_counter_collection.csv")
    if os.path.exists(vpath):
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(vpath)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in acc.items():
            extra[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    # the FP32 instruction pass (scripts/gpu_round.sh writes prof_fp32; older rounds prof_flops)
    fpaths = [os.path.join(OUT, f"{args.prefix}_{sub}", "run_counter_collection.csv") for sub in ("fp32", "flops")]
    fpath = next((f for f in fpaths if os.path.exists(f)), None)
    if fpath:
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(fpath)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in acc.items():
            extra[k].update({c: sum(v) / len(v) for c, v in cs.items()})
    factor, calib = 2.0, calibrate()
    if calib and calib.get("fetch_factor"):
        factor = float(calib["fetch_factor"])

    kernels = {}
    for k, d in durs.items():
        e = {"launches": len(d), "avg_ns_all": sum(d) / len(d), "resources": res[k]}
        tail = d[-args.steps:]
        e["avg_ns_tail"] = sum(tail) / len(tail)
        if fetch.get(k):
            e["fetch_kib_per_launch"] = sum(fetch[k]) / len(fetch[k])
        if write.get(k):
            e["write_kib_per_launch"] = sum(write[k]) / len(write[k])
        if extra.get(k):
            e["sq_counters_per_launch"] = extra[k]
        if "fetch_kib_per_launch" in e and "write_kib_per_launch" in e:
            e["hbm_bytes_per_launch"] = (e["fetch_kib_per_launch"] * factor + e["write_kib_per_launch"]) * 1024
        kernels[k] = e
    summary = {"tag": args.tag, "workload": args.workload, "fetch_factor": factor, "calibration": calib,
               "kernels": kernels}
    json.dump(summary, open(os.path.join(PROF, f"{args.tag}_summary.json"), "w"), indent=1)

    step = [k for k in kernels if args.kernel in k]
    if step and "hbm_bytes_per_launch" in kernels[step[0]]:
        tpath = os.path.join(PROF, "pmc_traffic.json")
        traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
        # the binary the counters describe: bench.py uses the entry only while
        # the library it loads has this hash
        lib_hash = hashlib.sha256(open(args.lib, "rb").read()).hexdigest()
        traffic[args.workload] = {"bytes_per_launch": round(kernels[step[0]]["hbm_bytes_per_launch"]),
                                  "source": f"profiles/{args.tag}_summary.json", "fetch_factor": factor,
                                  "lib_sha256": lib_hash}
        summary["lib_sha256"] = lib_hash
        json.dump(summary, open(os.path.join(PROF, f"{args.tag}_summary.json"), "w"), indent=1)
        sq = kernels[step[0]].get("sq_counters_per_launch", {})
        if "SQ_INSTS_VALU" in sq:
            traffic[args.workload]["valu_insts_per_launch"] = round(sq["SQ_INSTS_VALU"])
        if "SQ_INSTS_VALU_FLOPS_FP32" in sq:
            # executed FP32 FLOPs (round 6): gfx950's SQ_INSTS_VALU_FLOPS_FP32
            # counts FLOPs per wave instruction with the packed ones at their
            # width -- v_fma 2, v_add/v_mul 1, v_pk_fma 4, v_pk_add/v_pk_mul 2
            # (calibrated: scripts/flops_probe.hip, profiles/r06c_flops_probe_counters.csv)
            # -- x 64 lanes, plus the transcendental ones; an upper bound when
            # lanes are masked off (converged PGS lanes)
            traffic[args.workload]["fp32_flops_executed_per_launch"] = round(64 * (
                sq["SQ_INSTS_VALU_FLOPS_FP32"] + sq.get("SQ_INSTS_VALU_FLOPS_FP32_TRANS", 0)))
            traffic[args.workload]["fp32_flops_counter"] = "SQ_INSTS_VALU_FLOPS_FP32 (+_TRANS), packed included"
        elif "SQ_INSTS_VALU_FMA_F32" in sq:
            # older passes: instruction counts, where a v_pk_fma_f32 counts as one
            # FMA (2 FLOPs, not 4): a lower bound for the packed solver loops
            traffic[args.workload]["fp32_flops_executed_per_launch"] = round(64 * (
                2 * sq["SQ_INSTS_VALU_FMA_F32"] + sq.get("SQ_INSTS_VALU_ADD_F32", 0) +
                sq.get("SQ_INSTS_VALU_MUL_F32", 0) + sq.get("SQ_INSTS_VALU_TRANS_F32", 0)))
            traffic[args.workload]["fp32_flops_counter"] = "SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F32: packed counted as scalar"
        json.dump(traffic, open(tpath, "w"), indent=1)
    for k, e in sorted(kernels.items(), key=lambda kv: -kv[1]["avg_ns_all"] * kv[1]["launches"])[:4]:
        print(k, {x: (round(v, 1) if isinstance(v, float) else v) for x, v in e.items()
                  if x not in ("resources", "sq_counters_per_launch")})


if __name__ == "__main__":
    main()
