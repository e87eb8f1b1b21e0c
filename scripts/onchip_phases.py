"""Diagnostic: where a k_onchip launch's per-launch cost goes (needs a -DONCHIP_PHASES build via
XP_LIB).  Config 2, B replicas, one launch of K steps; per workgroup s_memrealtime (100 MHz) at
start / after the state load / after the steps / end.  Prints per-round medians in microseconds."""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tooling  # noqa: E402  (XP_LIB / XP_KNOBS: a variant build and experiment knobs)
tooling.apply()
from odesat_amd import _lib, cnf  # noqa: E402
from odesat_amd import workloads as wl  # noqa: E402
from odesat_amd.system import ODESAT_STOP_NONE, Solver  # noqa: E402

c = wl.CONFIGS["config2"]
var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
cp, v_, n_ = wl.formula_arrays(var, neg)
f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
for B in (256, 1024):
    for K in (1, 20):
        with Solver(f, B, "f32") as s:
            s.init_state(42)
            s.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE, poll_interval=5)
            s.simulate(dt=0.01, max_steps=K, stop=ODESAT_STOP_NONE, poll_interval=K)
            s.synchronize()
            buf = (ctypes.c_ulonglong * (4096 * 4))()
            assert _lib.lib().odesat_onchip_phases(buf, 4096 * 4) == 0
            t = [[buf[g * 4 + i] for i in range(4)] for g in range(B)]
            t0 = min(r[0] for r in t)
            us = lambda x: x / 100.0  # 100 MHz ticks -> us
            starts = sorted((r[0] - t0, g) for g, r in enumerate(t))
            out = {"B": B, "steps": K, "span_us": us(max(r[3] for r in t) - t0)}
            rounds = [starts[i:i + 256] for i in range(0, B, 256)]
            for ri, rr in enumerate(rounds):
                gs = [g for _, g in rr]
                out[f"round{ri}"] = {
                    "start": round(us(statistics.median(t[g][0] - t0 for g in gs)), 1),
                    "load": round(us(statistics.median(t[g][1] - t[g][0] for g in gs)), 1),
                    "steps": round(us(statistics.median(t[g][2] - t[g][1] for g in gs)), 1),
                    "store": round(us(statistics.median(t[g][3] - t[g][2] for g in gs)), 1),
                    "end_spread": round(us(max(t[g][3] for g in gs) - min(t[g][3] for g in gs)), 1)}
            print(json.dumps(out), flush=True)
