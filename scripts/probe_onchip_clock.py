"""Diagnostic (round 4): the effective shader clock of the headline kernel across the bench's call
shape.  Needs the -DONCHIP_PHASES build (scripts/build_variant.sh ocphases "-DONCHIP_PHASES
-DONCHIP_ONLY_TR=90"; run with XP_LIB=expt/libocphases.so).  Config 2, B = 1024, f32: a fresh
solver, the bench's 5-step warm-up call, then 12 calls of 20 steps back to back, 1.5 s idle, 4 more.
Per call: HIP-event kernel time and, per round of 256 workgroups, the median effective shader clock
over the steps (s_memtime ticks per s_memrealtime tick x 100 MHz) and the median step-loop time."""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tooling  # noqa: E402  (XP_LIB / XP_KNOBS: a variant build and experiment knobs)
tooling.apply()
from odesat_amd import _lib, cnf  # noqa: E402
from odesat_amd import workloads as wl  # noqa: E402
from odesat_amd.system import ODESAT_STOP_NONE, Solver  # noqa: E402

B = 1024
c = wl.CONFIGS["config2"]
var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
cp, v_, n_ = wl.formula_arrays(var, neg)
f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])


def rounds(K):
    t = (ctypes.c_ulonglong * (4096 * 4))()
    k = (ctypes.c_ulonglong * (4096 * 4))()
    assert _lib.lib().odesat_onchip_phases(t, 4096 * 4) == 0 and _lib.lib().odesat_onchip_clk(k, 4096 * 4) == 0
    order = sorted(range(B), key=lambda g: t[g * 4])
    out = []
    for r0 in range(0, B, 256):
        gs = order[r0:r0 + 256]
        mhz = statistics.median((k[g * 4 + 2] - k[g * 4 + 1]) / max(1, t[g * 4 + 2] - t[g * 4 + 1]) * 100.0 for g in gs)
        steps = statistics.median((t[g * 4 + 2] - t[g * 4 + 1]) / 100.0 for g in gs)
        out.append({"sclk_mhz": round(mhz, 1), "steps_us": round(steps, 1)})
    return out


with Solver(f, B, "f32") as s:
    assert s.step_kernel(False) == "k_onchip"
    s.init_state(42)
    plan = [("warmup", 5)] + [("hot", 20)] * 12 + [("idle", 20)] + [("hot", 20)] * 3
    for name, K in plan:
        if name == "idle":
            time.sleep(1.5)
        s.profile(True)
        s.simulate(dt=0.01, max_steps=K, stop=ODESAT_STOP_NONE, poll_interval=K)
        s.synchronize()
        ms, _ = s.profile_read()
        s.profile(False)
        print(json.dumps({"phase": name, "steps": K, "kernel_us": round(ms[0] * 1e3, 1), "rounds": rounds(K)}), flush=True)
