#!/usr/bin/env python
"""Per-launch means of the stall/I-cache PMC passes of scripts/gpu_stall_pmc.sh
for one step kernel, with the derived fractions DESIGN.md §12 quotes.
usage: python scripts/summarize_stalls.py <tag> [kernel substring] > profiles/<file>.txt"""
import collections
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "push"
kern = sys.argv[2] if len(sys.argv) > 2 else "k_step<1, 0, 1>"
sums, counts = collections.defaultdict(float), collections.defaultdict(set)
for sub in (f"stall_sq_{tag}", f"stall_sqc_{tag}"):
    path = os.path.join(ROOT, "gpurun_out", sub, "run_counter_collection.csv")
    for row in csv.DictReader(open(path)):
        if kern not in row["Kernel_Name"]:
            continue
        sums[row["Counter_Name"]] += float(row["Counter_Value"])
        counts[row["Counter_Name"]].add(row["Dispatch_Id"])
mean = {k: sums[k] / len(counts[k]) for k in sums}
n = max(len(v) for v in counts.values())
print(f"{kern}, {tag} (scripts/gpu_stall_pmc.sh); mean per launch over {n} launches")
for k in sorted(mean):
    print(f"{k:24s} {mean[k]:.4e}")
w = mean["SQ_WAVE_CYCLES"]
print(f"instruction active / wave-cycles   {mean['SQ_ACTIVE_INST_ANY'] / w:.3f}")
print(f"VALU active / wave-cycles          {mean['SQ_ACTIVE_INST_VALU'] / w:.3f}")
print(f"LDS active / wave-cycles           {mean['SQ_ACTIVE_INST_LDS'] / w:.3f}")
print(f"waiting (any) / wave-cycles        {mean['SQ_WAIT_ANY'] / w:.3f}")
print(f"waiting on instruction fetch       {mean['SQ_WAIT_INST_ANY'] / w:.3f}")
h, m = mean["SQC_ICACHE_HITS"], mean["SQC_ICACHE_MISSES"]
print(f"I-cache misses / fetches           {m / (h + m):.4f}")
