#!/usr/bin/env python
"""Loops of one kernel in a hipcc -S listing: every backward branch with the
instruction mix of the blocks it spans (VALU, SALU, LDS, global/scratch
memory, v_readlane/v_writelane SGPR-spill traffic, AGPR moves), largest
first -- the PGS loop of a step kernel is the top one."""
import collections
import re
import sys

path = sys.argv[1]
kernel = sys.argv[2] if len(sys.argv) > 2 else None
lines, on = [], kernel is None
for line in open(path):
    if kernel and line.startswith(kernel):
        on = True
    if on:
        if line.startswith(".Lfunc_end"):
            if kernel:
                break
        lines.append(line)
labels, instrs = {}, []
for line in lines:
    m = re.match(r"^(\.LBB\w+):", line)
    if m:
        labels[m.group(1)] = len(instrs)
        continue
    t = line.strip().split()
    if t and not t[0].startswith((";", ".")) and not t[0].endswith(":"):
        instrs.append(t)


def cls(op):
    if op.startswith(("v_readlane", "v_writelane")):
        return "sgpr-spill"
    if op.startswith("v_accvgpr"):
        return "agpr-move"
    if op.startswith(("scratch_", "buffer_")):
        return "scratch"
    if op.startswith("global_"):
        return "global"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


loops = []
for i, t in enumerate(instrs):
    if t[0].startswith(("s_cbranch", "s_branch")) and len(t) > 1 and t[1] in labels and labels[t[1]] <= i:
        s = labels[t[1]]
        c = collections.Counter(cls(x[0]) for x in instrs[s:i + 1])
        loops.append((i + 1 - s, t[1], c))
loops.sort(key=lambda x: -x[0])
for n, lab, c in loops[: int(sys.argv[3]) if len(sys.argv) > 3 else 8]:
    print(f"{lab:<12} {n:6d} instrs  " + "  ".join(f"{k} {v}" for k, v in sorted(c.items(), key=lambda x: -x[1])))
