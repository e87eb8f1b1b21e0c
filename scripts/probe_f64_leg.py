"""Probe: the bench's f64 leg shape (fresh solver, config 2, B = 1024, f64 fixed, 5 warmup steps in
one launch, then one 20-step launch), then a second and third 20-step launch on the same solver:
HIP-event kernel times in microseconds, to see whether the first timed launch pays a one-off cost."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tooling  # noqa: E402  (XP_LIB / XP_KNOBS: a variant build and experiment knobs)
tooling.apply()
from odesat_amd import cnf  # noqa: E402
from odesat_amd import workloads as wl  # noqa: E402
from odesat_amd.system import ODESAT_STOP_NONE, Solver  # noqa: E402

c = wl.CONFIGS["config2"]
var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
cp, v_, n_ = wl.formula_arrays(var, neg)
f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
for dtype in ("f64", "f32"):
    for rep in range(2):
        with Solver(f, 1024, dtype) as s:
            s.init_state(42)
            s.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE, poll_interval=5)
            row = {"dtype": dtype, "kernel": s.step_kernel(False)}
            for i in range(3):
                s.profile(True)
                s.synchronize()
                t0 = time.perf_counter()
                s.simulate(dt=0.01, max_steps=20, stop=ODESAT_STOP_NONE, poll_interval=20)
                s.synchronize()
                w = (time.perf_counter() - t0) * 1e6
                ms, n = s.profile_read()
                s.profile(False)
                row[f"launch{i}"] = (round(ms[0] * 1e3, 1), round(w, 1))
            print(json.dumps(row), flush=True)
