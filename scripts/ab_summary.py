"""Mean per library and workload of a scripts/gpu_ab.sh log (time_variants lines)."""
import ast
import collections
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
sect = None
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.log"):
    if line.startswith("=="):
        sect = "65536" if "65536 envs" in line else "small"
        continue
    m = re.match(r"(\S+\.so) (\{.*\})", line)
    if m:
        for k, v in ast.literal_eval(m.group(2)).items():
            acc[m.group(1)][f"{sect}_{k}"].append(v)
for lib, d in acc.items():
    print(lib.ljust(22), "  ".join(f"{k} {sum(v) / len(v):.4f}" for k, v in sorted(d.items())))
