"""Probe (round 4): where the first 20-step call after the warm-up spends its extra ~60 us.  The body
of Solver.simulate inlined with timestamps: each line of the Python prologue (params, result
arrays, the function lookup), the C call, and the HIP-event kernel time; GC=0 disables Python's
garbage collector for the run.  PRE=prologue runs the prologue once before the loop (untimed),
PRE=profile a profile(True) / profile_read / profile(False) cycle, PRE=sleep 100 ms of idle,
PRE=spin 100 ms of host spin, PRE=call a second untimed 5-step call.  MALLOPT=1: glibc's trim and
mmap thresholds raised to 1 GiB (no heap trim, no per-allocation mmap); PREBUILT=1: the prologue
runs once before the loop and every call reuses its arguments (the timed part is the C call alone)."""
import ctypes as C
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tooling  # noqa: E402  (XP_LIB / XP_KNOBS: a variant build and experiment knobs)
tooling.apply()
import numpy as np  # noqa: E402

from odesat_amd import _lib, cnf  # noqa: E402
from odesat_amd import workloads as wl  # noqa: E402
from odesat_amd.system import ODESAT_STOP_NONE, Solver  # noqa: E402

if os.environ.get("GC") == "0":
    gc.disable()
if os.environ.get("MALLOPT") == "1":
    libc = C.CDLL(None)
    M_TRIM_THRESHOLD, M_TOP_PAD, M_MMAP_THRESHOLD = -1, -2, -3
    for k in (M_TRIM_THRESHOLD, M_TOP_PAD, M_MMAP_THRESHOLD):
        assert libc.mallopt(k, 1 << 30 if k != M_TOP_PAD else 64 << 20) == 1
PREBUILT = os.environ.get("PREBUILT") == "1"
PRE = os.environ.get("PRE", "")
c = wl.CONFIGS["config2"]
var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
cp, v_, n_ = wl.formula_arrays(var, neg)
f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])


def prologue():
    ts = [time.perf_counter()]
    p = _lib.Params(0, int(ODESAT_STOP_NONE), 1e-3, 0.01, -1.0, 20, 20, 0)
    ts.append(time.perf_counter())
    sat = np.zeros(1024, np.int64)
    done = np.zeros(1024, np.int64)
    dts = np.zeros(1024, np.float64)
    ts.append(time.perf_counter())
    run = C.c_int64(0)
    fn = _lib.lib().odesat_simulate
    ts.append(time.perf_counter())
    args = (C.byref(p), _lib.i64ptr(sat), _lib.i64ptr(done), _lib.dptr(dts), C.byref(run))
    ts.append(time.perf_counter())
    return fn, args, ts


with Solver(f, 1024, "f32") as s:
    s.init_state(42)
    s.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE, poll_interval=5)
    if PRE == "prologue":
        prologue()
    elif PRE == "profile":
        s.profile(True)
        s.profile_read()
        s.profile(False)
    elif PRE == "sleep":
        time.sleep(0.1)
    elif PRE == "spin":
        t_end = time.perf_counter() + 0.1
        while time.perf_counter() < t_end:
            pass
    elif PRE == "call":
        s.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE, poll_interval=5)
    rows = []
    built = prologue() if PREBUILT else None
    for i in range(5):
        s.profile(True)
        s.synchronize()
        t0 = time.perf_counter()
        fn, args, ts = built if PREBUILT else prologue()
        t1 = time.perf_counter()
        rc = fn(s._h, *args)
        t2 = time.perf_counter()
        s.synchronize()
        t3 = time.perf_counter()
        ms, _ = s.profile_read()
        s.profile(False)
        d = [round((b - a) * 1e6, 1) for a, b in zip(ts, ts[1:])]
        rows.append({"params": d[0], "zeros": d[1], "lookup": d[2], "ptrs": d[3], "ccall_us": round((t2 - t1) * 1e6, 1),
                     "sync_us": round((t3 - t2) * 1e6, 1), "kernel_us": round(ms[0] * 1e3, 1),
                     "ccall_minus_kernel": round((t2 - t1) * 1e6 - ms[0] * 1e3, 1),
                     "total_over": round((t2 - t0) * 1e6 - ms[0] * 1e3, 1), "rc": rc})
    print(json.dumps({"gc": os.environ.get("GC", "1"), "pre": PRE, "mallopt": os.environ.get("MALLOPT") == "1",
                      "prebuilt": PREBUILT, "calls": rows}), flush=True)
