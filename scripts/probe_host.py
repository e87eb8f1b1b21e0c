"""Probe: host-side cost of one odesat_simulate call around an ONCHIP launch (config 2, B=256,
1 step per call): wall per call through the Python wrapper, through ctypes with no outputs, with
and without profiling events, and an idle stream sync.  Medians over 40 calls, microseconds."""
import ctypes as C
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from odesat_amd import _lib, cnf
from odesat_amd import workloads as wl
from odesat_amd.system import ODESAT_STOP_NONE, Solver

c = wl.CONFIGS["config2"]
var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
cp, v_, n_ = wl.formula_arrays(var, neg)
f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])


def med(fn, k=40):
    ts = []
    for _ in range(k):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e6)
    return round(statistics.median(ts), 1)


with Solver(f, 256, "f32") as s:
    s.init_state(42)
    s.simulate(dt=0.01, max_steps=2, stop=ODESAT_STOP_NONE)
    s.synchronize()
    out = {}
    out["idle_sync"] = med(s.synchronize)
    out["wrapper_1step"] = med(lambda: s.simulate(dt=0.01, max_steps=1, stop=ODESAT_STOP_NONE, poll_interval=1))
    p = _lib.Params(0, int(ODESAT_STOP_NONE), 1e-3, 0.01, -1.0, 1, 1, 0)
    fn = _lib.lib().odesat_simulate
    out["ctypes_no_outputs_1step"] = med(lambda: (fn(s._h, C.byref(p), None, None, None, None), s.synchronize()))
    s.profile(True)
    out["wrapper_1step_profiled"] = med(lambda: s.simulate(dt=0.01, max_steps=1, stop=ODESAT_STOP_NONE, poll_interval=1))
    ms, launches = s.profile_read()
    out["kernel_us_mean"] = round(ms[0] * 1e3 / max(1, launches[0]), 1)
    s.profile(False)

    def benchlike(toggle, warm_steps):
        def one():
            s.simulate(dt=0.01, max_steps=warm_steps, stop=ODESAT_STOP_NONE, poll_interval=warm_steps)
            if toggle:
                s.profile(True)
            s.synchronize()
            t0 = time.perf_counter()
            s.simulate(dt=0.01, max_steps=1, stop=ODESAT_STOP_NONE, poll_interval=1)
            s.synchronize()
            t1 = time.perf_counter()
            if toggle:
                s.profile(False)
            return (t1 - t0) * 1e6
        return round(statistics.median([one() for _ in range(15)]), 1)
    out["benchlike_toggle_warm5"] = benchlike(True, 5)
    out["benchlike_notoggle_warm5"] = benchlike(False, 5)
    out["benchlike_notoggle_warm1"] = benchlike(False, 1)

    def sleepy():
        s.synchronize()
        time.sleep(0.002)
        t0 = time.perf_counter()
        s.simulate(dt=0.01, max_steps=1, stop=ODESAT_STOP_NONE, poll_interval=1)
        s.synchronize()
        return (time.perf_counter() - t0) * 1e6
    out["after_2ms_idle"] = round(statistics.median([sleepy() for _ in range(15)]), 1)
fresh = []
for _ in range(5):
    with Solver(f, 256, "f32") as s2:
        s2.init_state(42)
        s2.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE, poll_interval=5)
        s2.profile(True)
        s2.synchronize()
        t0 = time.perf_counter()
        s2.simulate(dt=0.01, max_steps=1, stop=ODESAT_STOP_NONE, poll_interval=1)
        s2.synchronize()
        t1 = time.perf_counter()
        ms, launches = s2.profile_read()
        # a second timed call on the same solver
        s2.synchronize()
        t2 = time.perf_counter()
        s2.simulate(dt=0.01, max_steps=1, stop=ODESAT_STOP_NONE, poll_interval=1)
        s2.synchronize()
        t3 = time.perf_counter()
        ms2, l2 = s2.profile_read()
        fresh.append((round((t1 - t0) * 1e6, 1), round(ms[0] * 1e3, 1), round((t3 - t2) * 1e6, 1), round((ms2[0] - ms[0]) * 1e3, 1)))
out["fresh_solver (wall, kernel, 2nd wall, 2nd kernel)"] = fresh
print(out)
