#!/usr/bin/env python
"""N consecutive forced builds of libpandasim.so (every object recompiled,
the default job count) with the compiler crashes each one logged
(pandasim/build.py writes them to pandasim/build/build_log.jsonl), one JSON
line per build.

  python scripts/build_repeat.py 5 > profiles/r06_build_log.jsonl

(round 6: also the built library's own sha256, to show the builds are reproducible)
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "panda-lang-manip_amd"))
from pandasim import build as B  # noqa: E402


def crashes():
    p = os.path.join(B.OBJ_DIR, "build_log.jsonl")
    return [json.loads(ln) for ln in open(p)] if os.path.exists(p) else []


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    for i in range(n):
        before = len(crashes())
        t = time.time()
        B.build(force=True, verbose=False)
        new = crashes()[before:]
        print(json.dumps({"build": i + 1, "forced": True, "jobs": B._jobs(), "units": len(B.UNITS),
                          "seconds": round(time.time() - t, 1), "compiler_crashes": len(new), "crash_log": new,
                          "lib_sha256_stamp": B.read_stamp(B.OUT),
                          "lib_file_sha256": hashlib.sha256(open(B.OUT, "rb").read()).hexdigest()}), flush=True)


if __name__ == "__main__":
    main()
