"""Probe (round 4): where the first 20-step call after the warm-up spends its extra ~60 us.  The body
of Solver.simulate inlined with timestamps: Python prologue (params, result arrays), the C call, and
the HIP-event kernel time; GC=0 disables Python's garbage collector for the run."""
import ctypes as C
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from odesat_amd import _lib, cnf  # noqa: E402
from odesat_amd import workloads as wl  # noqa: E402
from odesat_amd.system import ODESAT_STOP_NONE, Solver  # noqa: E402

if os.environ.get("GC") == "0":
    gc.disable()
c = wl.CONFIGS["config2"]
var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
cp, v_, n_ = wl.formula_arrays(var, neg)
f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
with Solver(f, 1024, "f32") as s:
    s.init_state(42)
    s.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE, poll_interval=5)
    rows = []
    for i in range(6):
        s.profile(True)
        s.synchronize()
        t0 = time.perf_counter()
        p = _lib.Params(0, int(ODESAT_STOP_NONE), 1e-3, 0.01, -1.0, 20, 20, 0)
        sat = np.zeros(1024, np.int64)
        done = np.zeros(1024, np.int64)
        dts = np.zeros(1024, np.float64)
        run = C.c_int64(0)
        fn = _lib.lib().odesat_simulate
        t1 = time.perf_counter()
        rc = fn(s._h, C.byref(p), _lib.i64ptr(sat), _lib.i64ptr(done), _lib.dptr(dts), C.byref(run))
        t2 = time.perf_counter()
        s.synchronize()
        t3 = time.perf_counter()
        ms, _ = s.profile_read()
        s.profile(False)
        rows.append({"prologue_us": round((t1 - t0) * 1e6, 1), "ccall_us": round((t2 - t1) * 1e6, 1),
                     "sync_us": round((t3 - t2) * 1e6, 1), "kernel_us": round(ms[0] * 1e3, 1),
                     "ccall_minus_kernel": round((t2 - t1) * 1e6 - ms[0] * 1e3, 1), "rc": rc})
    print(json.dumps({"gc": os.environ.get("GC", "1"), "calls": rows}), flush=True)
