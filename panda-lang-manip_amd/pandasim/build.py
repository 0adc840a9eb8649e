"""Build libpandasim.so in-tree with hipcc for gfx950 (no JIT, no torch extension).

The library is linked from parallel hipcc jobs (csrc/ps_env.h): the C ABI and
small kernels (pandasim.hip), the fused step kernels of each (task, control)
pair (step_kernels.hip: the one-lane kernel, 12 objects, and the 16/8-lane
group kernels, 10 objects -- Stack has none) and the plugin-path substep kernel
of each scene (sim_kernels.hip, 4 objects).

Every object is compiled with the same flags (-O3, no -mllvm scheduler
options).  Round 3 built the group kernels at -O1 after an -O2/-O3 miscompute
of Slide's; since round 4 the -O3 group kernels keep the
one-lane kernels' robot rows bit for bit from a reset
(tests/test_gpu_parity.py::test_group_kernels_match_one_lane) and pass the
oracle from contact states (test_group_kernels_match_one_lane_in_contact), so
a recurrence fails the GPU tests.  The scheduler options of round 3
gained < 2 % in two interleaved runs (profiles/r04b_ab.log) and one of them
(-amdgpu-use-amdgpu-trackers) made this clang crash intermittently; none is
kept.

Freshness is decided by content, not mtimes: every build writes
``<lib>.sha256``, the sha256 of every source and header the library is built
from plus the compile flags.  ``needs_build`` recomputes it, and
``pandasim._lib.lib()`` refuses a library whose stamp does not match the
sources next to it (a stale prebuilt .so shipped with the tree).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import json
import os
import subprocess
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
INCLUDE = os.path.join(ROOT, "include")
OUT = os.path.join(HERE, "libpandasim.so")
OBJ_DIR = os.path.join(HERE, "build")

# -fno-slp-vectorize: SLP packing into v_pk_fma_f32 pairs made the register
# allocator spill 590 VGPRs of the step kernel to scratch
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize", "-fPIC", "-I", INCLUDE]

TASK_STACK = 4  # include/pandasim.h

# (object name, source, defines and per-unit flags)
UNITS = ([("pandasim", "pandasim.hip", [])]
         + [(f"step_t{t}_c{c}", "step_kernels.hip", [f"-DPS_STEP_TASK={t}", f"-DPS_STEP_CONTROL={c}"])
            for t in range(6) for c in range(2)]
         + [(f"step_t{t}_c{c}_groups", "step_kernels.hip",
             [f"-DPS_STEP_TASK={t}", f"-DPS_STEP_CONTROL={c}", "-DPS_STEP_GROUPS=1"])
            for t in range(6) if t != TASK_STACK for c in range(2)]
         + [(f"sim_{n}_{s}", "sim_kernels.hip", [f"-DPS_SIM_NOBJ={n}", f"-DPS_SIM_SHAPE={s}"])
            for n, s in ((0, 0), (1, 0), (1, 1), (2, 0))])

# diagnostic variants (never loaded by the product unless PANDASIM_LIB names them)
VARIANTS = {"": [], "prof": ["-DPS_PROFILE_PHASES"]}


def headers() -> list:
    """Every header the objects include: csrc/*.h and include/*.h."""
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    return sorted(hs)


def deps() -> list:
    """Every source the library is built from."""
    return sorted(headers() + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip")])


def _digest(paths, flags) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    # flags with the tree's own location abstracted (the stamp must hold on the
    # GPU box, where the same tree sits at another path)
    h.update(" ".join(f.replace(ROOT, "<root>") for f in flags).encode())
    return h.hexdigest()


def out_path(variant: str = "") -> str:
    return OUT if not variant else os.path.join(HERE, f"libpandasim_{variant}.so")


def stamp_path(lib_path: str) -> str:
    return lib_path + ".sha256"


def fingerprint(variant: str = "", extra=()) -> str:
    """sha256 of every source and header plus the flags of `variant` and of
    every unit."""
    return _digest(deps(), FLAGS + VARIANTS[variant] + list(extra) + [repr(UNITS)])


def read_stamp(lib_path: str):
    try:
        with open(stamp_path(lib_path)) as f:
            return f.read().strip()
    except OSError:
        return None


def needs_build(variant: str = "", extra=(), out: str | None = None) -> bool:
    out = out or out_path(variant)
    return not os.path.exists(out) or read_stamp(out) != fingerprint(variant, extra)


def _jobs() -> int:
    for k in ("MAX_JOBS", "PANDASIM_BUILD_JOBS"):
        v = os.environ.get(k)
        if v and v.isdigit() and int(v) > 0:
            return min(int(v), 16)
    return max(1, min(16, len(os.sched_getaffinity(0))))


class _Scheduler:
    """Admission of compiles: any number run together, except while a crash
    retry runs, which waits until no other compile is in flight and keeps
    new ones from starting until it is done (one condition variable covers
    both the retry flag and the in-flight count, so no compile can slip in
    between a retry's check and its start: ADVICE r05)."""

    def __init__(self):
        self._cv = threading.Condition()
        self._inflight = 0
        self._serial = False

    def start(self) -> None:
        with self._cv:
            while self._serial:
                self._cv.wait()
            self._inflight += 1

    def end(self) -> int:
        """Leaves; returns the number of compiles that were in flight with it."""
        with self._cv:
            jobs = self._inflight
            self._inflight -= 1
            self._cv.notify_all()
            return jobs

    def run_alone(self, fn):
        with self._cv:
            while self._serial:
                self._cv.wait()
            self._serial = True
            while self._inflight > 0:
                self._cv.wait()
        try:
            return fn()
        finally:
            with self._cv:
                self._serial = False
                self._cv.notify_all()


_sched = _Scheduler()
# serialized retries of one unit after a crash (each alone on the machine)
CRASH_RETRIES = 3


def _crashed(r) -> bool:
    return r.returncode != 0 and ("Stack dump" in r.stderr or "Segmentation fault" in r.stderr)


def _log_crash(name: str, attempt: int, jobs: int, stderr: str) -> None:
    os.makedirs(OBJ_DIR, exist_ok=True)
    sig = next((ln.strip() for ln in stderr.splitlines() if "Running pass" in ln or "#" in ln[:4]), "")[:200]
    with open(os.path.join(OBJ_DIR, "build_log.jsonl"), "a") as f:
        f.write(json.dumps({"unit": name, "attempt": attempt, "jobs_in_flight": jobs, "time": time.time(),
                            "signature": sig}) + "\n")
    print(f"[build] {name}: compiler crash (attempt {attempt}, {jobs} jobs in flight)", flush=True)


def build(force: bool = False, verbose: bool = True, variant: str = "", extra=(), out: str | None = None) -> str:
    out = out or out_path(variant)
    want = fingerprint(variant, extra)
    if not force and os.path.exists(out) and read_stamp(out) == want:
        return out
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tag = os.path.splitext(os.path.basename(out))[0]
    odir = os.path.join(OBJ_DIR, tag)
    os.makedirs(odir, exist_ok=True)
    hdrs = headers()
    flags = FLAGS + VARIANTS[variant] + list(extra)

    def compile_unit(unit):
        name, src, defs = unit
        obj = os.path.join(odir, name + ".o")
        # an object is reused when its own source, every header and its flags are unchanged
        key = _digest(hdrs + [os.path.join(CSRC, src)], flags + defs)
        if not force and os.path.exists(obj) and read_stamp(obj) == key:
            return obj
        cmd = [hipcc, *flags, *defs, "-c", "-o", obj + ".tmp", os.path.join(CSRC, src)]
        if verbose:
            print(" ".join(cmd), flush=True)
        # Round 3's -amdgpu-use-amdgpu-trackers made this clang (ROCm 7.2,
        # clang-22) segfault intermittently in the AMDGPU scheduler's
        # rematerialisation stage (GCNSchedStrategy PreRARematStage) with many
        # jobs in flight; no object uses that option now, and the builds since
        # have not crashed (profiles/r05_build_log.jsonl: consecutive forced
        # builds).  Should a compile still crash, the crash is logged (unit,
        # attempt, jobs in flight: build/build_log.jsonl) and the unit is
        # compiled again alone (no other compile in flight, none starting:
        # _Scheduler), up to CRASH_RETRIES times; a crash after that, or any
        # diagnostic, fails the build.
        _sched.start()
        try:
            r = subprocess.run(cmd, capture_output=True, text=True)
        finally:
            jobs = _sched.end()
        attempt = 1
        while _crashed(r):
            _log_crash(name, attempt, jobs, r.stderr)
            if attempt > CRASH_RETRIES:
                break
            attempt += 1
            jobs = 1
            r = _sched.run_alone(lambda: subprocess.run(cmd, capture_output=True, text=True))
        if r.stdout:
            print(r.stdout, end="")
        if r.returncode != 0:
            print(r.stderr[-4000:], flush=True)
            raise subprocess.CalledProcessError(r.returncode, cmd)
        os.replace(obj + ".tmp", obj)
        with open(stamp_path(obj), "w") as f:
            f.write(key + "\n")
        return obj

    with cf.ThreadPoolExecutor(_jobs()) as ex:
        objs = list(ex.map(compile_unit, UNITS))
    cmd = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out + ".tmp", *objs]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    with open(stamp_path(out), "w") as f:
        f.write(want + "\n")
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, variant="prof" if "--prof" in sys.argv else "")
