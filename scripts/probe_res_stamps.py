"""Diagnostic: inside the f64 leg's k_resident launches.  Needs the -DRES_STAMPS build
(scripts/build_variant.sh resstamps "-DRES_STAMPS" odesat_hip; run with XP_LIB=expt/libresstamps.so).
Config 2, B = 1024, f64 fixed steps: the bench's shape (fresh solver, one 5-step launch), then 20-step
launches back to back, 1.5 s idle, more 20-step launches, then a 60-step launch.  Per launch: the
workgroups' start times split them into rounds (two workgroups per CU: 512 at a time); per round
the median v load and the median duration of each step (s_memrealtime, 100 MHz), the effective shader
clock over the round's steps (s_memtime ticks per s_memrealtime tick x 100 MHz), and the launch span.
DTYPE=f32 ALG=2 runs the f32 k_resident instead."""
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

B = int(os.environ.get("B", "1024"))
DT = os.environ.get("DTYPE", "f64")


def stamps(B, K):
    buf = (ctypes.c_ulonglong * (4096 * 64))()
    assert _lib.lib().odesat_res_stamps(buf, 4096 * 64) == 0
    t = [[buf[g * 64 + i] for i in range(64)] for g in range(B)]
    clk = (ctypes.c_ulonglong * (4096 * 64))()
    assert _lib.lib().odesat_res_clk(clk, 4096 * 64) == 0
    ck = [[clk[g * 64 + i] for i in range(64)] for g in range(B)]
    t0 = min(r[0] for r in t)
    us = lambda x: x / 100.0
    order = sorted(range(B), key=lambda g: t[g][0])
    rounds, cur = [], [order[0]]
    for g in order[1:]:  # a new round: a start more than 20 us after the previous workgroup's start
        if t[g][0] - t[cur[-1]][0] > 2000:
            rounds.append(cur)
            cur = []
        cur.append(g)
    rounds.append(cur)
    out = {"steps": K, "span_us": round(us(max(r[63] for r in t) - t0), 1), "rounds": []}
    for rr in rounds:
        per = [round(us(statistics.median(t[g][2 + k] - (t[g][1] if k == 0 else t[g][1 + k]) for g in rr)), 1)
               for k in range(min(K, 60))]
        last = 1 + min(K, 60)
        mhz = statistics.median((ck[g][last] - ck[g][1]) / (t[g][last] - t[g][1]) * 100.0 for g in rr)
        out["rounds"].append({"workgroups": len(rr), "sclk_mhz": round(mhz, 1), "start": round(us(statistics.median(t[g][0] - t0 for g in rr)), 1),
                              "load": round(us(statistics.median(t[g][1] - t[g][0] for g in rr)), 1),
                              "end": round(us(statistics.median(t[g][63] - t[g][1 + min(K, 60)] for g in rr)), 1),
                              "step_us": per})
    return out


def main():
    c = wl.CONFIGS["config2"]
    var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
    with Solver(f, B, DT) as s:
        if "ALG" in os.environ:
            s.set_algorithm(int(os.environ["ALG"]))
        assert s.step_kernel(False) == "k_resident"
        s.init_state(42)
        plan = [("warmup", 5)] + [("hot", 20)] * 4 + [("idle", 20)] + [("hot", 20)] * 2 + [("long", 60)]
        for name, K in plan:
            if name == "idle":
                time.sleep(1.5)
            s.profile(True)
            s.simulate(dt=0.01, max_steps=K, stop=ODESAT_STOP_NONE, poll_interval=K)
            s.synchronize()
            ms, _ = s.profile_read()
            s.profile(False)
            row = stamps(B, K)
            row.update({"phase": name, "kernel_us": round(ms[0] * 1e3, 1)})
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
