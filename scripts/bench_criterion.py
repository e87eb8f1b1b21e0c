"""The reference's own criterion benches (benches/benchmarks.rs:25-79) on the GPU and on the CPU
oracle: `simulate` on tests/hard.cnf (n=100, m=160, unsatisfiable, so every call runs all of its
steps), 10 000 steps per call, f64, one replica whose state carries over between calls as in the
bench:
  "adaptive hard"  tolerance 0.01, step size None  (system.rs:204-234)
  "fixed hard"     step size 0.01                  (system.rs:190-203)
The reference publishes no result for them, so this prints both sides here.

  python scripts/bench_criterion.py [--calls 5] [--batch 1]
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
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1, help="replicas stepped per call on the GPU")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import numpy as np

    from odesat_amd import cnf
    from odesat_amd.system import ODESAT_STOP_NONE, Solver
    from oracle.oracle import Oracle, init_voltages

    with open(os.path.join(ROOT, "tests", "golden", "hard.cnf")) as fh:
        _, f = cnf.normalize_cnf_variables(cnf.parse_dimacs_format(fh.read()))
    steps = 10_000
    for name, kw in (("adaptive hard", dict(adaptive=True, tol=0.01)), ("fixed hard", dict(adaptive=False, dt=0.01))):
        out = {"bench": name, "steps_per_call": steps, "dtype": "f64", "batch": args.batch}
        with Solver(f, args.batch, "f64") as s:
            s.init_state(42)
            s.simulate(max_steps=steps, stop=ODESAT_STOP_NONE, poll_interval=steps, **kw)  # warm-up call
            s.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.calls):
                s.simulate(max_steps=steps, stop=ODESAT_STOP_NONE, poll_interval=steps, **kw)
            s.synchronize()
            out["gpu_ms_per_call"] = (time.perf_counter() - t0) * 1e3 / args.calls
        if not args.no_cpu:
            cp, var, neg = f.arrays()
            o = Oracle(cp, var, neg, f.varnum, "f64")
            v = init_voltages(42, 0, 1, f.varnum)[0]
            xs = o.init_short_term_memory()
            xl = np.ones(f.nclauses)
            t0 = time.perf_counter()
            for _ in range(args.calls):
                o.simulate(v, xs, xl, tol=kw.get("tol"), dt=kw.get("dt"), steps=steps)
            out["cpu_oracle_ms_per_call"] = (time.perf_counter() - t0) * 1e3 / args.calls
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
