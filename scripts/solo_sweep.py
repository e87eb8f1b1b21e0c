"""k_solo vs k_wave on the reference's criterion shape (tests/hard.cnf, B = 1, 10 000 steps per call)
and on small batches of config 3: per-call milliseconds for every team shape (the experiment knobs SOLO,
SOLO_LANES, WAVE_TEAM are read when a solver is created).  One JSON line per run.

  python scripts/solo_sweep.py [--calls 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tooling  # noqa: E402  (XP_LIB / XP_KNOBS: a variant build and experiment knobs)
tooling.apply()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10_000)
    args = ap.parse_args()
    from odesat_amd import cnf
    from odesat_amd import _lib
    from odesat_amd import workloads as wl
    from odesat_amd.system import ODESAT_STOP_NONE, Solver

    with open(os.path.join(ROOT, "tests", "golden", "hard.cnf")) as fh:
        _, hard = cnf.normalize_cnf_variables(cnf.parse_dimacs_format(fh.read()))
    c = wl.CONFIGS["config3"]
    var, neg = wl.random_ksat(c["n"], c["m"], 3, c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    cfg3 = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
    shapes = [("wave-t1", {"SOLO": 0, "WAVE_TEAM": 1}),
              ("wave-t2", {"SOLO": 0, "WAVE_TEAM": 2}),
              ("wave-t4", {"SOLO": 0, "WAVE_TEAM": 4})]
    shapes += [(f"solo-l{k}", {"SOLO": 1, "SOLO_LANES": k}) for k in (128, 256, 512, 1024)]
    shapes += [("solo-default", {"SOLO": 1})]
    for fname, f, B, steps in (("hard", hard, 1, args.steps), ("config3", cfg3, 1, args.steps // 4),
                               ("config3", cfg3, 64, args.steps // 10)):
        for prec in ("f64", "f32"):
            for mode, kw in (("fixed", dict(adaptive=False, dt=0.01)), ("adaptive", dict(adaptive=True, tol=0.01))):
                for label, env in shapes:
                    for k in ("SOLO", "SOLO_LANES", "WAVE_TEAM"):
                        _lib.set_experiment(k, env.get(k))
                    with Solver(f, B, prec) as s:
                        kern = s.step_kernel(kw["adaptive"])
                        s.init_state(42)
                        s.simulate(max_steps=steps, stop=ODESAT_STOP_NONE, poll_interval=steps, **kw)
                        s.synchronize()
                        t0 = time.perf_counter()
                        for _ in range(args.calls):
                            s.simulate(max_steps=steps, stop=ODESAT_STOP_NONE, poll_interval=steps, **kw)
                        s.synchronize()
                        ms = (time.perf_counter() - t0) * 1e3 / args.calls
                    print(json.dumps({"formula": fname, "batch": B, "prec": prec, "mode": mode, "shape": label,
                                      "kernel": kern, "steps": steps, "ms_per_call": round(ms, 3),
                                      "us_per_step": round(ms * 1e3 / steps, 4)}), flush=True)


if __name__ == "__main__":
    main()
