#!/usr/bin/env python
"""Source lines behind chosen instructions in a hipcc -S -gline-tables-only
listing: `isa_lines.py file.s v_div_scale v_sqrt` prints, per kernel, the
(file:line) of each match, counted (which divisions / square roots survive)."""
import collections
import re
import sys

path, pats = sys.argv[1], sys.argv[2:]
files, loc, kern = {}, None, None
hits = collections.defaultdict(collections.Counter)
for line in open(path):
    m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', line)
    if m:
        files[m.group(1)] = m.group(2).split("/")[-1]
        continue
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
    if m:
        loc = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
        continue
    m = re.match(r"^(_Z\w+):", line)
    if m:
        kern = m.group(1)[:60]
        continue
    t = line.split()
    if t and any(t[0].startswith(p) for p in pats):
        hits[kern][loc] += 1
for k, c in hits.items():
    print(k)
    for l, n in sorted(c.items(), key=lambda x: -x[1]):
        print(f"   {n:4d} {l}")
