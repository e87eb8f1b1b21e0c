"""Config 5's per-rank work at world 1, 2, 4 and 8, timed on ONE GPU (VERDICT r2 "Next #5"):
for every partition (CLAUSES, CLAUSES_RS, VARIABLES) build rank r's local topology of the n = 1M,
m = 4.2M instance at world W and time that rank's kernels per step (the clause and variable kernels,
plus the CLAUSES voltage update or the CLAUSES_RS block update) in a HIP graph of K steps, without the
collective -- which needs W GPUs.  Prints one JSON line per (partition, world, rank): the kernel time
per step, the rank's clause count and the bytes it puts into the collective(s) per step.

  python scripts/partition_slices.py [--worlds 1,2,4,8] [--ranks first|all] [--steps 100]
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
    p = argparse.ArgumentParser()
    p.add_argument("--worlds", default="1,2,4,8")
    p.add_argument("--modes", default="clauses,clauses_rs,variables")
    p.add_argument("--ranks", default="first", choices=["first", "all"])
    p.add_argument("--steps", type=int, default=100)
    args = p.parse_args()

    import numpy as np
    import torch

    from odesat_amd import workloads as wl
    from odesat_amd.partition import MODES, LocalComm, PartitionedSolver, default_zeta

    c = wl.CONFIGS["config5"]
    n, m = c["n"], c["m"]
    var, neg = wl.random_ksat(n, m, c["k"], c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    del var, neg
    v0 = wl.init_voltages(42, 0, 1, n)[0]
    xs0 = np.where(n_.reshape(m, 3).any(axis=1), 1.0, -1.0)
    xl0 = np.ones(m)
    zeta, dt = default_zeta(n, m), 0.01
    torch.cuda.set_device(0)
    for world in [int(x) for x in args.worlds.split(",")]:
        for name in args.modes.split(","):
            mode = MODES[name]
            for rank in (range(world) if args.ranks == "all" else [0]):
                t0 = time.perf_counter()
                ps = PartitionedSolver(cp, v_, n_, n, mode, comm=LocalComm(rank, world), device=0)
                setup = time.perf_counter() - t0
                ps.set_state(v0, xs0, xl0)
                # the rank's kernels only: rhs (+ memory update) and the post-collective update
                for _ in range(5):
                    ps.rhs(dt, zeta, False)
                    ps.post(dt)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(args.steps):
                        ps.rhs(dt, zeta, False)
                        ps.post(dt)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                g.replay()  # warm
                torch.cuda.synchronize()
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / args.steps
                print(json.dumps({"partition": name, "world": world, "rank": rank, "kernel_us_per_step": us,
                                  "local_clauses": int(len(ps.topo["clauses"])),
                                  "owned_variables": int(ps.topo["v1"] - ps.topo["v0"]) if name == "variables"
                                  else (int(ps.topo["block"]) if name == "clauses_rs" else n),
                                  "collective_bytes_per_rank": ps.exchange_bytes(), "setup_s": round(setup, 2)}),
                      flush=True)
                ps.close()
                del ps, g
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
