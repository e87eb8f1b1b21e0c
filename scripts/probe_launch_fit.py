"""Probe: kernel time of one launch vs steps per launch (HIP events), to split a persistent kernel's
per-launch fixed cost from its per-step cost.  ALG (2 = resident), DTYPE, B, ADAPTIVE from the env."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from odesat_amd import cnf  # noqa: E402
from odesat_amd import workloads as wl  # noqa: E402
from odesat_amd.system import ODESAT_STOP_NONE, Solver  # noqa: E402

c = wl.CONFIGS["config2"]
var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
cp, v_, n_ = wl.formula_arrays(var, neg)
f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
dtype = os.environ.get("DTYPE", "f64")
ada = os.environ.get("ADAPTIVE", "0") == "1"
for B in [int(x) for x in os.environ.get("BS", "256,1024").split(",")]:
    with Solver(f, B, dtype) as s:
        if "ALG" in os.environ:
            s.set_algorithm(int(os.environ["ALG"]))
        s.init_state(42)
        s.simulate(dt=0.01, tol=1e-3, adaptive=ada, max_steps=3, stop=ODESAT_STOP_NONE, poll_interval=3)
        row = {"B": B, "dtype": dtype, "adaptive": ada, "kernel": s.step_kernel(ada)}
        for k in (1, 2, 5, 10, 20, 50):
            ts = []
            for _ in range(3):
                s.profile(True)
                s.simulate(dt=0.01, tol=1e-3, adaptive=ada, max_steps=k, stop=ODESAT_STOP_NONE, poll_interval=k)
                s.synchronize()
                ms, n = s.profile_read()
                s.profile(False)
                ts.append(ms[0] * 1e3 / max(1, n[0]))
            row[str(k)] = round(min(ts), 1)
        print(json.dumps(row), flush=True)
