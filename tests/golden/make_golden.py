"""Generate the committed golden vectors under tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`).

Expected outputs come from oracle/np_oracle.py -- the numpy restatement written independently of the
C oracle -- so the C oracle (and through it the GPU) is checked against an implementation it shares
no code with.  Inputs: the reference's own fixtures tests/{small,easy,hard}.cnf (copied verbatim from
/root/reference/tests) and one seeded random 3-SAT instance (odesat_amd.workloads, written out as
rand200.cnf).  Initial voltages: the counter RNG, seed 42, replicas 0..B-1.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import cnf_oracle as co  # noqa: E402
from oracle import np_oracle as npo  # noqa: E402
from odesat_amd import workloads as wl  # noqa: E402

SEED = 42
B = 4


def load(name):
    with open(os.path.join(HERE, name)) as fh:
        cl, varnum = co.parse_dimacs_format(fh.read())
    _, ncl = co.normalize_cnf_variables(cl, varnum)
    return npo.Formula.from_clauses(ncl, varnum)


def run(f, T, steps, **kw):
    v0 = npo.init_voltages(SEED, 0, B, f.varnum)
    out = {"v": [], "xs": [], "xl": [], "steps": [], "sat": [], "dt": []}
    for b in range(B):
        v = v0[b].astype(T)
        xs = npo.init_short_term_memory(f, T)
        xl = np.ones(f.m, T)
        t, sat, _, h = npo.simulate(f, v, xs, xl, steps=steps, **kw)
        out["v"].append(v)
        out["xs"].append(xs)
        out["xl"].append(xl)
        out["steps"].append(t)
        out["sat"].append(sat)
        out["dt"].append(h)
    return {k: np.array(x) for k, x in out.items()}


def main():
    if not os.path.exists(os.path.join(HERE, "rand200.cnf")):
        var, neg = wl.random_ksat(200, 852, 3, 5)
        with open(os.path.join(HERE, "rand200.cnf"), "w") as fh:
            fh.write(wl.to_dimacs(var, neg, 200, "random 3-SAT n=200 m=852 seed=5 (odesat_amd.workloads)"))
    cases = {"small": 300, "easy": 2000, "hard": 300, "rand200": 60}
    for name, steps in cases.items():
        f = load(name + ".cnf")
        arrays = {"clause_ptr": f.clause_ptr, "var": f.var, "neg": f.neg.astype(np.uint8),
                  "varnum": np.int64(f.varnum), "seed": np.int64(SEED), "B": np.int64(B),
                  "steps": np.int64(steps), "v0": npo.init_voltages(SEED, 0, B, f.varnum)}
        for prec, T in (("f64", np.float64), ("f32", np.float32)):
            for mode, kw in (("fixed", dict(dt=0.01)), ("adaptive", dict(tol=1e-3))):
                res = run(f, T, steps, **kw)
                for k, x in res.items():
                    arrays[f"{prec}_{mode}_{k}"] = x
        np.savez_compressed(os.path.join(HERE, f"{name}_golden.npz"), **arrays)
        print(name, {k: v.shape for k, v in arrays.items() if k.endswith("_steps")},
              arrays["f64_fixed_steps"], arrays["f64_adaptive_steps"])


if __name__ == "__main__":
    main()
