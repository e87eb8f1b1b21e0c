"""Probe: where the headline's wall time goes beyond its kernel (bench.py's shape: a fresh solver,
B = 1024, 5 warmup steps, then ONE timed 20-step launch between device syncs).  Per fresh solver:
wall of the timed call, the kernel's HIP-event time, the time until simulate() returned, and the sync
after it; with profiling events on (as bench.py) and off.  Microseconds."""
import json
import os
import statistics
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
B, K, W = int(os.environ.get("B", "1024")), int(os.environ.get("STEPS", "20")), 5
rows = {}
for rep in range(int(os.environ.get("REPS", "4"))):
    for prof, split in ((True, False), (True, True), (False, False)):
        with Solver(f, B, "f32") as s:
            s.init_state(42)
            if split:  # the W warmup steps as W one-step launches
                for _ in range(W):
                    s.simulate(dt=0.01, max_steps=1, stop=ODESAT_STOP_NONE, poll_interval=1)
            else:
                s.simulate(dt=0.01, max_steps=W, stop=ODESAT_STOP_NONE, poll_interval=W)
            s.profile(prof)
            s.synchronize()
            t0 = time.perf_counter()
            s.simulate(dt=0.01, max_steps=K, stop=ODESAT_STOP_NONE, poll_interval=K)
            t1 = time.perf_counter()
            s.synchronize()
            t2 = time.perf_counter()
            kern = s.profile_read()[0][0] * 1e3 if prof else None
            rows.setdefault((prof, split), []).append({"wall": (t2 - t0) * 1e6, "call": (t1 - t0) * 1e6, "sync": (t2 - t1) * 1e6,
                               "kernel": kern, "value_M": B * K / (t2 - t0) / 1e6})
for (prof, split), rs in rows.items():
    med = {k: round(statistics.median([r[k] for r in rs]), 1) for k in rs[0] if rs[0][k] is not None}
    print(json.dumps({"profile_events": prof, "warmup_split": split, "median": med, "runs": [{k: (round(v, 1) if v else v) for k, v in r.items()} for r in rs]}))
