#!/usr/bin/env python
"""Writes profiles/oracle_work_counts.json: the fp64 oracle's work counters
(po_stats: PGS iterations and rows per substep, contacts, IK iterations) on
the bench's sample of every task (seeds 12345 + i, U(-1, 1) actions,
auto-reset; bench.oracle_work_counts), so that bench.py's FLOP roofline is
available where the CPU-baseline leg does not run (N > 1, --no-cpu-baseline).
CPU only; run it here after a change to the physics."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import oracle as O  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    out = {}
    for task in ("reach", "push", "pick_and_place", "slide", "stack", "flip"):
        out[task] = bench.oracle_work_counts(O, O.config(task))
        print(task, out[task], flush=True)
    with open(os.path.join(ROOT, bench.WORK_COUNTS), "w") as f:
        json.dump(out, f, indent=1)
