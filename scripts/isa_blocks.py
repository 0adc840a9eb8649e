#!/usr/bin/env python
"""Per-basic-block VALU/SALU/LDS counts of one kernel in a hipcc -S listing,
with the branch targets, to read loop bodies off (scripts/isa_probe.hip)."""
import re
import sys

path, kernel = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else None)
blocks, cur, on = [], None, kernel is None
for line in open(path):
    if kernel and line.startswith(kernel + ":"):
        on = True
    if not on:
        continue
    if line.startswith(".Lfunc_end"):
        break
    m = re.match(r"^(\.LBB\w+|\w+):", line)
    if m:
        cur = {"name": m.group(1), "v": 0, "s": 0, "ds": 0, "br": []}
        blocks.append(cur)
        continue
    t = line.strip().split()
    if not t or cur is None or t[0].startswith((";", ".")):
        continue
    op = t[0]
    cur["v" if op.startswith("v_") else "ds" if op.startswith("ds_") else "s" if op.startswith("s_") else "s"] += 1
    if op.startswith(("s_cbranch", "s_branch")):
        cur["br"].append(op.replace("s_cbranch_", "") + ":" + t[1])
tot = 0
for b in blocks:
    tot += b["v"]
    if b["v"] or b["br"]:
        print(f"{b['name']:<12} v={b['v']:4d} s={b['s']:3d} ds={b['ds']:3d}  {' '.join(b['br'])}")
print("total VALU", tot)
