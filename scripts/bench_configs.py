"""Throughput on BASELINE.json's other single-GPU configs (the headline, config 2, is bench.py's).

  python scripts/bench_configs.py [--configs config3,config4] [--steps K] [--warmup W]

config3: uf250-style random 3-SAT (n=250, m=1065, seed 2), ADAPTIVE Euler (tol 1e-3, dt0 0.01,
         per-replica dt), B=1024 replicas, f32.  Two RHS passes per step (system.rs:111-139).
config4: random 3-SAT n=50k m=210k seed 3, fixed dt 0.01 (the inter workload, one GPU's share:
         8192 = 8 x 1024 replicas), B=1024, f32.
Every replica is stepped for all K steps (ODESAT_STOP_NONE), the state resident in HBM when the
timed region starts.  One JSON line per config, with the algorithm the solver chose, its mean
launch time (HIP events), the algorithmic bytes per replica-step (B_fix = 8n + 16m,
B_ad = 3 B_fix) and the CPU oracle (f64, 1 thread) on a bounded sample of the same workload.
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

SPEC = {
    "config3": dict(adaptive=True, batch=1024, cpu_replicas=8, cpu_steps=400),
    "config4": dict(adaptive=False, batch=1024, cpu_replicas=1, cpu_steps=30),
    "config3f": dict(adaptive=False, batch=1024, cpu_replicas=8, cpu_steps=400, base="config3"),
    # the reference's default mode (solve / batch without -s) on the headline instance
    "config2a": dict(adaptive=True, batch=1024, cpu_replicas=4, cpu_steps=100, base="config2"),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", default="config3,config4")
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--alg", default="auto", help="auto | resident | fused | twopass | onchip")
    p.add_argument("--batch", type=int, default=0, help="override the config's B")
    p.add_argument("--chunk", type=int, default=0, help="replicas per chunk (FUSED / TWOPASS; 0 = automatic)")
    p.add_argument("--schedule", type=int, default=0, help="0 auto, 1 step-major, 2 chunk-major")
    args = p.parse_args()

    import numpy as np

    from odesat_amd import _lib, cnf
    from odesat_amd import workloads as wl
    from odesat_amd.system import ODESAT_STOP_NONE, Solver

    names = {v: k for k, v in vars(_lib).items() if k.startswith("ODESAT_ALG_")}
    for cfg in args.configs.split(","):
        spec = SPEC[cfg]
        c = wl.CONFIGS[spec.get("base", cfg)]
        n, m = c["n"], c["m"]
        var, neg = wl.random_ksat(n, m, c["k"], c["seed"])
        cp, v_, n_ = wl.formula_arrays(var, neg)
        f = cnf.CNFFormula.from_arrays(cp, v_, n_, n)
        B = args.batch or spec["batch"]
        kw = dict(adaptive=spec["adaptive"], dt=0.01, tol=1e-3, stop=ODESAT_STOP_NONE, poll_interval=50)
        with Solver(f, B, "f32") as s:
            if args.alg != "auto":
                s.set_algorithm(getattr(_lib, "ODESAT_ALG_" + args.alg.upper()))
            if args.chunk:
                s.set_chunk_replicas(args.chunk)
            s.set_schedule(args.schedule)
            s.init_state(42)
            s.simulate(max_steps=args.warmup, **kw)
            s.synchronize()
            s.profile(True)
            t0 = time.perf_counter()
            r = s.simulate(max_steps=args.steps, **kw)
            s.synchronize()
            wall = time.perf_counter() - t0
            ms, launches = s.profile_read()
            alg = names.get(s.algorithm, str(s.algorithm))
        per_rs = (8 * n + 16 * m) * (3 if spec["adaptive"] else 1)
        out = {"config": cfg, "workload": f"random 3-SAT n={n} m={m} seed={c['seed']}, "
                                          f"{'adaptive tol 1e-3' if spec['adaptive'] else 'fixed dt 0.01'}",
               "batch": B, "steps": args.steps, "algorithm": alg, "chunk": args.chunk, "schedule": args.schedule,
               "experiment": tooling.knobs(),
               "steps_per_s": args.steps / wall, "replica_steps_per_s": B * args.steps / wall,
               "ms_per_step": wall * 1e3 / args.steps,
               "algorithmic_bytes_per_replica_step": per_rs,
               "algorithmic_GBps": per_rs * B * args.steps / wall / 1e9,
               "kernel_ms": {"main": ms[0], "variable": ms[1], "status": ms[2]},
               "launches": [int(x) for x in launches],
               "replicas_sat_during_run": int((r["first_sat_step"] >= 0).sum())}
        if not args.no_cpu:
            from oracle.oracle import Oracle, init_voltages
            o = Oracle(cp, v_, n_, n, "f64")
            R, K = spec["cpu_replicas"], spec["cpu_steps"]
            v = init_voltages(42, 0, R, n)
            xs = np.tile(o.init_short_term_memory(), (R, 1))
            xl = np.ones((R, m))
            t0 = time.perf_counter()
            tot = o.batch_run(v, xs, xl, spec["adaptive"], 1e-3, 0.01, K, 0.001 if m / n < 4.9 else 0.01)[0]
            dt = time.perf_counter() - t0
            out["cpu_baseline"] = {"replica_steps_per_s": tot / dt, "cores": 1, "kind": "port",
                                   "sample": f"C f64 oracle, {R} replicas x up to {K} steps (stop at sat), "
                                             f"{tot} steps in {dt:.1f} s"}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
