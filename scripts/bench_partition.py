"""One instance across GPUs (BASELINE configs[4], odesat_amd/partition.py): fixed-step Euler of a
single replica with the formula partitioned over the ranks, one process per GPU.

  python scripts/bench_partition.py --config config5 --mode variables --steps 200
  python -m torch.distributed.run --nproc-per-node N scripts/bench_partition.py --gpus N ...

Prints one JSON line (rank 0): steps/s of the whole instance, the per-step time and the bytes each
rank exchanges.  The timed region is K steps bracketed by barrier + device sync, max over ranks.
--fixture NAME (tests/golden/NAME.cnf) and --check-out PATH write the final voltages for tests.
Backend: RCCL ("nccl"); ODESAT_DIST_BACKEND=gloo runs several ranks on one GPU (host-staged).
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
    p.add_argument("--config", default="config5")
    p.add_argument("--fixture", default=None)
    p.add_argument("--mode", default="variables", choices=["variables", "clauses", "clauses_rs"])
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--dt", type=float, default=0.01)
    p.add_argument("--seed", type=int, default=7)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--check-out", default=None)
    p.add_argument("--order", default="minvar", choices=["file", "minvar"], help="clause processing order")
    p.add_argument("--graph", type=int, default=50,
                   help="steps per captured HIP graph (0 = one host call per kernel, the eager loop)")
    args = p.parse_args()

    import numpy as np
    import torch

    from odesat_amd import _lib, cnf, device_count
    from odesat_amd import workloads as wl
    from odesat_amd.partition import MODES, LocalComm, PartitionedSolver, TorchComm, default_zeta

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = local % max(1, device_count())
    torch.cuda.set_device(device)
    dist = None
    if world > 1:
        import torch.distributed as td
        td.init_process_group(backend=os.environ.get("ODESAT_DIST_BACKEND", "nccl"))
        dist = td

    if args.fixture:
        with open(os.path.join(ROOT, "tests", "golden", args.fixture + ".cnf")) as fh:
            _, f = cnf.normalize_cnf_variables(cnf.parse_dimacs_format(fh.read()))
        cp, var, neg = f.arrays()
        n = f.varnum
        workload = f"fixture {args.fixture} (n={n}, m={len(cp) - 1})"
    else:
        c = wl.CONFIGS[args.config]
        var2, neg2 = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
        cp, var, neg = wl.formula_arrays(var2, neg2)
        n = c["n"]
        workload = f"{args.config}: random 3-SAT n={n} m={c['m']} seed={c['seed']}"
    m = len(cp) - 1
    mode = MODES[args.mode]
    comm = TorchComm(dist) if dist is not None else LocalComm()
    t0 = time.perf_counter()
    s = PartitionedSolver(cp, var, neg, n, mode, comm=comm, device=device, order=args.order)
    setup_s = time.perf_counter() - t0
    v0 = wl.init_voltages(args.seed, 0, 1, n)[0]
    # system.rs:361-372: +1 if the clause has a negated literal, else -1 (empty clauses too)
    negc = np.zeros(m, np.int64)
    owner = np.repeat(np.arange(m), np.diff(cp))
    np.add.at(negc, owner, np.asarray(neg, np.int64))
    xs0 = np.where(negc > 0, 1.0, -1.0)
    s.set_state(v0, xs0, np.ones(m))
    zeta = default_zeta(n, m)

    def sync():
        torch.cuda.synchronize(device)
        if dist is not None:
            dist.barrier()

    graph = None
    if args.graph and s.capturable():
        if args.steps % args.graph:
            raise SystemExit("--steps must be a multiple of --graph")
        graph = s.graph(args.graph, args.dt, zeta, stop=False)  # captured, not run
    for _ in range(args.warmup):
        s.step(args.dt, zeta, stop=False)
    sync()
    t1 = time.perf_counter()
    if graph is not None:
        for _ in range(args.steps // args.graph):
            graph.replay()
    else:
        for _ in range(args.steps):
            s.step(args.dt, zeta, stop=False)
    sync()
    wall = time.perf_counter() - t1
    if dist is not None:
        on_dev = dist.get_backend() == "nccl"
        w = torch.tensor([wall], dtype=torch.float64, device="cuda" if on_dev else "cpu")
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall = float(w.item())
    st = s.status(stop=False)
    if args.check_out and rank == 0:
        v, _, _, _ = s.get_state()
        with open(args.check_out, "w") as fh:
            json.dump({"v": v.tolist(), "steps_done": st["steps_done"]}, fh)
    if rank == 0:
        t = s.topo
        exchange = s.exchange_bytes()
        print(json.dumps({
            "metric": "ODE steps/s of one instance partitioned across GPUs (BASELINE configs[4])",
            "value": args.steps / wall, "unit": "steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": wall * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "strong", "dtype": "fp32", "data": "synthetic: seeded random 3-SAT + counter-RNG voltages",
            "config": {"workload": workload, "mode": args.mode, "order": args.order,
                       "terms": ["region", "ell", "slot"][_lib.get_experiment("PART_TERMS") or 0],
                       "graph_steps": args.graph if graph is not None else 0,
                       "collective": {"variables": "all_gather", "clauses": "all_reduce",
                                      "clauses_rs": "reduce_scatter + all_gather"}[args.mode],
                       "exchange_bytes_per_step": exchange, "local_clauses_rank0": int(len(t["clauses"])),
                       "setup_s": setup_s, "backend": dist.get_backend() if dist is not None else None},
        }))
    s.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
