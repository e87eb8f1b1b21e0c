"""Diagnostic: stamp breakdown of a k_solo_fast / k_solo_cv fixed / adaptive step (needs a -DSOLO_STAMPS
build of wave_k, XP_LIB=...; XP_KNOBS=SOLO_CV=0 for k_solo_fast).  hard.cnf, B = 1, f64, 2000 steps;
prints cycles per step per segment for each wave."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tooling  # noqa: E402  (XP_LIB / XP_KNOBS: a variant build and experiment knobs)
tooling.apply()


def main():
    from odesat_amd import _lib, cnf
    from odesat_amd.system import ODESAT_STOP_NONE, Solver
    with open(os.path.join(ROOT, "tests", "golden", "hard.cnf")) as fh:
        _, f = cnf.normalize_cnf_variables(cnf.parse_dimacs_format(fh.read()))
    steps = 2000
    for prec, adaptive in (("f64", False), ("f64", True)):
        with Solver(f, 1, prec) as s:
            s.init_state(42)
            s.simulate(max_steps=steps, stop=ODESAT_STOP_NONE, poll_interval=steps, adaptive=adaptive, dt=0.01, tol=0.01)
            s.synchronize()
            buf = (ctypes.c_ulonglong * 128)()
            assert _lib.lib().odesat_solo_stamps(buf) == 0
            if tooling.knobs()["knobs"].get("SOLO_CV", 1):  # k_solo_cv
                names = (["terms1", "barrier1", "fold1_terms2", "barrier2", "fold2_err", "book"]
                         if adaptive else ["terms", "barrier", "fold", "", "", "book"])
            else:
                names = (["clauses1", "barrier1", "fold1", "barrier2", "clauses2", "barrier3", "fold2", "barrier4_dt"]
                         if adaptive else ["clauses", "barrier1", "fold", "book", "barrier2"])
            for w in range(16):
                row = [buf[w * 8 + i] / steps for i in range(len(names))]
                if sum(row) == 0:
                    continue
                print(json.dumps({"prec": prec, "adaptive": adaptive, "wave": w, "knobs": tooling.knobs()["knobs"],
                                  **{n: round(x, 1) for n, x in zip(names, row) if n}, "total": round(sum(row), 1)}))


if __name__ == "__main__":
    main()
