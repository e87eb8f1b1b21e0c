"""Tuning sweep on one GPU: wall time per step for schedule x chunk x batch (config-2 instance)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from odesat_amd import _lib, cnf  # noqa: E402
from odesat_amd import workloads as wl  # noqa: E402
from odesat_amd.system import ODESAT_STOP_NONE, Solver  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "config2"
    c = wl.CONFIGS[cfg]
    var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
    steps = int(os.environ.get("STEPS", "100"))
    rows = []
    for B in [int(x) for x in os.environ.get("BATCHES", "1024,256").split(",")]:
        combos = [(_lib.ODESAT_ALG_FUSED, _lib.ODESAT_SCHED_AUTO, B, gw + ":" + rb)
                  for gw in os.environ.get("GWS", "16,32,64").split(",") for rb in os.environ.get("RBS", "4").split(",")]
        combos += [(_lib.ODESAT_ALG_FUSED, _lib.ODESAT_SCHED_CHUNK_MAJOR, int(ch), "64")
                   for ch in os.environ.get("FUSED_CHUNKS", "").split(",") if ch and int(ch) <= B]
        for sched in (_lib.ODESAT_SCHED_STEP_MAJOR, _lib.ODESAT_SCHED_CHUNK_MAJOR):
            for chunk in [int(x) for x in os.environ.get("CHUNKS", "128,256,1024").split(",") if x]:
                if chunk <= B:
                    combos.append((_lib.ODESAT_ALG_TWOPASS, sched, chunk, os.environ.get("TWOPASS_GW", "16")))
        for alg, sched, chunk, gw in combos:
                os.environ["ODESAT_GROUP_WIDTH"] = gw.split(":")[0]
                os.environ["ODESAT_RB"] = (gw.split(":") + ["4"])[1]
                with Solver(f, B, os.environ.get("DTYPE", "f32")) as s:
                    s.set_algorithm(alg)
                    s.set_chunk_replicas(chunk)
                    s.set_schedule(sched)
                    s.init_state(42)
                    s.simulate(dt=0.01, max_steps=10, stop=ODESAT_STOP_NONE)
                    s.synchronize()
                    t0 = time.perf_counter()
                    s.simulate(dt=0.01, max_steps=steps, stop=ODESAT_STOP_NONE)
                    s.synchronize()
                    wall = time.perf_counter() - t0
                    s.profile(True)
                    s.simulate(dt=0.01, max_steps=steps, stop=ODESAT_STOP_NONE)
                    ms, n = s.profile_read()
                    s.profile(False)
                us = wall / steps * 1e6
                row = dict(B=B, gw=gw, alg="fused" if alg == 0 else "twopass",
                           sched={0: "auto", 1: "step", 2: "chunk"}[sched], chunk=chunk, us_per_step=round(us, 1),
                           Mrs=round(B / us, 3), clause_us=round(ms[0] * 1e3 / steps, 1),
                           var_us=round(ms[1] * 1e3 / steps, 1), status_us=round(ms[2] * 1e3 / steps, 1),
                           algGBs=round(B * (8 * c["n"] + 16 * c["m"]) / (us * 1e-6) / 1e9, 0))
                rows.append(row)
                print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
