"""A/B helper: the sha256 of a run's final state (v, xs, xl of every replica) and its bookkeeping, for
comparing two builds bit for bit (run once per build, e.g. with XP_LIB=expt/libX.so).

  python scripts/state_digest.py [--config config2] [--batch 256] [--steps 200] [--seeds 1,2,3] [--calls 4]
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tooling  # noqa: E402  (XP_LIB / XP_KNOBS: a variant build and experiment knobs)
tooling.apply()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config2")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--calls", type=int, default=4)
    ap.add_argument("--seeds", default="1,2,3")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--adaptive", action="store_true")
    args = ap.parse_args()
    import numpy as np

    from odesat_amd import cnf
    from odesat_amd import workloads as wl
    from odesat_amd.system import ODESAT_STOP_NONE, Solver
    c = wl.CONFIGS[args.config]
    var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
    for seed in [int(x) for x in args.seeds.split(",")]:
        h = hashlib.sha256()
        with Solver(f, args.batch, args.dtype) as s:
            s.init_state(seed)
            for k in range(args.calls):
                r = s.simulate(adaptive=args.adaptive, dt=0.01, tol=1e-3, max_steps=args.steps,
                               poll_interval=args.steps, stop=ODESAT_STOP_NONE, resume=k > 0)
                h.update(np.asarray(r["steps_done"]).tobytes())
                h.update(np.asarray(r["dt"]).tobytes())
            for x in s.get_state():
                h.update(np.ascontiguousarray(x).tobytes())
            kern = s.step_kernel(args.adaptive)
        print(json.dumps({"seed": seed, "kernel": kern, "digest": h.hexdigest()[:24]}), flush=True)


if __name__ == "__main__":
    main()
