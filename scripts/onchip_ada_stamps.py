"""Diagnostic: where an adaptive k_onchip step goes (needs a -DONCHIP_ADA_STAMPS build of onchip via
XP_LIB: scripts/build_variant.sh adastamps -DONCHIP_ADA_STAMPS onchip).  Config 2, B = 1024, f32,
adaptive tol 1e-3, one launch of K steps after a warm-up; workgroup 0's s_memtime cycles per step in
pass 1, the first voltage phase, pass 2, the second voltage phase (with the error terms) and the
closing barrier with the dt update, per wave; the fixed step's cycles beside them for scale."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tooling  # noqa: E402  (XP_LIB / XP_KNOBS: a variant build and experiment knobs)
tooling.apply()
from odesat_amd import _lib, cnf  # noqa: E402
from odesat_amd import workloads as wl  # noqa: E402
from odesat_amd.system import ODESAT_STOP_NONE, Solver  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
c = wl.CONFIGS["config2"]
var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
cp, v_, n_ = wl.formula_arrays(var, neg)
f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
names = ["pass1", "varphase1", "pass2", "varphase2_err", "barrier_dt"]
with Solver(f, 1024, "f32") as s:
    assert s.step_kernel(True) == "k_onchip"
    s.init_state(42)
    s.simulate(adaptive=True, dt=0.01, tol=1e-3, max_steps=5, stop=ODESAT_STOP_NONE, poll_interval=5)
    s.simulate(adaptive=True, dt=0.01, tol=1e-3, max_steps=K, stop=ODESAT_STOP_NONE, poll_interval=K, resume=True)
    s.synchronize()
    buf = (ctypes.c_ulonglong * 40)()
    assert _lib.lib().odesat_onchip_ada_stamps(buf) == 0
    for w in range(8):
        row = [buf[w * 5 + i] / K for i in range(5)]
        print(json.dumps({"wave": w, "steps": K, **{n: round(x) for n, x in zip(names, row)}, "total": round(sum(row))}))
