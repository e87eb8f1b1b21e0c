"""Throughput of the discrete stochastic search (stoch.hip) on config 3's instance: B replicas,
K steps each (STOP_NONE), against the C oracle's steps on one core.

  python scripts/bench_stoch.py [--batch 1024] [--steps 200]
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
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--cpu-steps", type=int, default=200)
    ap.add_argument("--config", default="config3")
    args = ap.parse_args()
    import numpy as np

    from odesat_amd import cnf
    from odesat_amd import workloads as wl
    from odesat_amd.stoch import ODESAT_STOP_NONE, StochSearch
    from oracle.oracle import Oracle

    c = wl.CONFIGS[args.config]
    var, neg = wl.random_ksat(c["n"], c["m"], 3, c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
    with StochSearch(f, args.batch) as s:
        s.search(1, 20, stop=ODESAT_STOP_NONE)
        t0 = time.perf_counter()
        s.search(1, args.steps, stop=ODESAT_STOP_NONE)  # returns after its stream has drained
        gpu = time.perf_counter() - t0
        width = s.wave_width
    o = Oracle(cp, v_, n_, c["n"], "f64")
    v = np.zeros(c["n"], np.uint8)
    xl = np.ones(c["m"], np.uint64)
    t0 = time.perf_counter()
    for k in range(args.cpu_steps):
        o.stoch_step(v, xl, 1, 0, k)
    cpu = time.perf_counter() - t0
    print(json.dumps({"workload": f"{args.config}: n={c['n']} m={c['m']}", "batch": args.batch, "steps": args.steps,
                      "kernel": f"wave, {width} replicas per workgroup" if width else "three-kernel HBM path",
                      "gpu_replica_steps_per_s": args.batch * args.steps / gpu,
                      "cpu_oracle_steps_per_s_1core": args.cpu_steps / cpu}))


if __name__ == "__main__":
    main()
