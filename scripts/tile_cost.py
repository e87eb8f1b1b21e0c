"""Per-tile cost of k_onchip vs instance size (same density as config 2): is the step time linear in
the number of tiles, or does the unrolled code size (TR) cost extra?  Prints one line per size."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def tiles(var2, n, cap=512):
    last = np.full(n + 1, -1)
    fill, first = [], 0
    for c in range(len(var2)):
        t = max(first, max(last[v] for v in var2[c]) + 1)
        while t < len(fill) and fill[t] >= cap:
            t += 1
        if t == len(fill):
            fill.append(0)
        fill[t] += 1
        while first < len(fill) and fill[first] >= cap:
            first += 1
        for v in var2[c]:
            last[v] = t
    return len(fill)


def main():
    from odesat_amd import _lib, cnf
    from odesat_amd import workloads as wl
    from odesat_amd.system import ODESAT_STOP_NONE, Solver
    for n in (2500, 5000, 7500, 10000):
        m = int(4.2 * n)
        var, neg = wl.random_ksat(n, m, 3, 1)
        cp, v_, n_ = wl.formula_arrays(var, neg)
        nt = tiles(np.asarray(var) - 1, n)
        f = cnf.CNFFormula.from_arrays(cp, v_, n_, n)
        with Solver(f, 1024, "f32") as s:
            alg = s.algorithm
            s.init_state(42)
            s.simulate(dt=0.01, max_steps=50, stop=ODESAT_STOP_NONE, poll_interval=50)
            s.synchronize()
            t0 = time.perf_counter()
            s.simulate(dt=0.01, max_steps=200, stop=ODESAT_STOP_NONE, poll_interval=50)
            s.synchronize()
            dt = time.perf_counter() - t0
        per_step = dt / 200
        print(f"n={n} m={m} alg={alg} tiles~{nt} us/step={per_step*1e6:.1f} "
              f"ns/tile/round={per_step / 4 / nt * 1e9:.1f}", flush=True)


if __name__ == "__main__":
    main()
