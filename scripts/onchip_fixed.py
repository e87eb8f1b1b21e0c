"""k_onchip launch time vs steps per launch at config 2 (B replicas): fits launch = F + K x, and
times the rounds separately (B = 256 is one round of workgroups).  HIP-event kernel times."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tooling  # noqa: E402  (XP_LIB / XP_KNOBS: a variant build and experiment knobs)
tooling.apply()
from odesat_amd import cnf, workloads as wl
from odesat_amd.system import ODESAT_STOP_NONE, Solver

c = wl.CONFIGS["config2"]
var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
cp, v_, n_ = wl.formula_arrays(var, neg)
f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
for B in [int(x) for x in os.environ.get("BATCHES", "1024,256").split(",")]:
    s = Solver(f, B, "f32")
    s.init_state(42)
    s.simulate(dt=0.01, max_steps=10, stop=ODESAT_STOP_NONE, poll_interval=10)
    pts = []
    for K in (1, 2, 5, 20, 50, 200):
        s.profile(True)
        s.simulate(dt=0.01, max_steps=K, stop=ODESAT_STOP_NONE, poll_interval=K)
        s.synchronize()
        t0 = time.perf_counter()
        s.simulate(dt=0.01, max_steps=K, stop=ODESAT_STOP_NONE, poll_interval=K)
        s.synchronize()
        wall = (time.perf_counter() - t0) * 1e6
        ms, nl = s.profile_read()
        s.profile(False)
        us = ms[0] * 1e3 / nl[0]
        pts.append((K, us))
        print(f"B={B} alg={s.algorithm} K={K} launch_us={us:.1f} wall_us={wall:.1f} launches={nl[0]}", flush=True)
    k = np.array([p[0] for p in pts], float)
    t = np.array([p[1] for p in pts], float)
    x, F = np.polyfit(k, t, 1)
    print(f"B={B} fit: fixed {F:.1f} us per launch, {x:.2f} us per step", flush=True)
    s.close()
