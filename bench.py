"""Benchmark: ODE steps/s x batch (replica-steps/s) on random 3-SAT n=10k m=42k (BASELINE.json).

One "step" = one fixed-step Euler step (system.rs:141-154) of every replica of the batch.  Default
workload: config 2's instance (random 3-SAT n=10 000, m=42 000, generator seed 1), fp32, B=1024 per
GPU (the north star's roofline point), dt = 0.01, every replica forced to run all K steps
(ODESAT_STOP_NONE).  Inputs are initialised on the device before the timed region.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process per
GPU, each steps its own B replicas (global replica index rank*B + b) with no collective in the data
path -- weak scaling; barrier + max-over-ranks timing via torch.distributed.

Rank 0 prints ONE JSON line (see DESIGN.md §6 for every field).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--batch", type=int, default=1024, help="replicas per GPU")
    p.add_argument("--config", default="config2")
    p.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    p.add_argument("--chunk", type=int, default=0, help="replicas per chunk (0 = automatic)")
    p.add_argument("--cpu-replicas", type=int, default=16)
    p.add_argument("--cpu-steps", type=int, default=300)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--traffic-dir", default=os.path.join(ROOT, "profiles"),
                   help="directory of traffic_<kernel>.json files: the dominant kernel's HBM bytes per launch "
                        "from the PMC passes (scripts/make_traffic.py)")
    p.add_argument("--alg", default="auto", choices=["auto", "onchip", "resident", "fused", "twopass"],
                   help="force an algorithm (A/B); auto = the solver's default")
    p.add_argument("--extra-batch", type=int, default=256, help="also time this B (configs[1]); 0 = off")
    p.add_argument("--no-ab", action="store_true",
                   help="skip the in-run A/B line of the HBM-streaming kernel (k_resident) on the same workload")
    return p.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        from odesat_amd import device_count
        local %= max(1, device_count())  # the one-GPU gloo rehearsal maps every rank to GPU 0
        import torch
        import torch.distributed as td
        # RCCL ("nccl") on GPU boxes; ODESAT_DIST_BACKEND=gloo rehearses N ranks on one GPU (RCCL
        # refuses two ranks on one device).  Only host scalars cross ranks (odesat_amd/sharding.py).
        backend = os.environ.get("ODESAT_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        td.init_process_group(backend=backend)
        dist = td
    return world, rank, local, dist


def barrier_sync(dist, solver, local):
    """Device sync (the solver's stream carries all of its work) + barrier across ranks.  At N = 1
    torch is never imported, so the process holds exactly one HIP runtime, the library's."""
    solver.synchronize()
    if dist is not None:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize(local)
        dist.barrier()


STEPS_PER_LAUNCH = 50  # persistent kernel: steps per launch (the state crosses HBM once per launch)


def time_gpu(solver, steps, warmup, dist, local, profile):
    from odesat_amd.system import ODESAT_STOP_NONE
    if warmup:
        solver.simulate(dt=0.01, max_steps=warmup, stop=ODESAT_STOP_NONE, poll_interval=STEPS_PER_LAUNCH)
    solver.profile(profile)
    barrier_sync(dist, solver, local)
    t0 = time.perf_counter()
    solver.simulate(dt=0.01, max_steps=steps, stop=ODESAT_STOP_NONE, poll_interval=STEPS_PER_LAUNCH)
    barrier_sync(dist, solver, local)
    t1 = time.perf_counter()
    ms, launches = solver.profile_read() if profile else (None, None)
    solver.profile(False)
    return t1 - t0, ms, launches


def cpu_threads():
    """The host cores this job may use: OMP_NUM_THREADS (16 on the GPU box: its share of a larger
    machine, whose os.cpu_count() would overstate it), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def cpu_baseline(cp, var, neg, n, m, replicas, steps, threads=1):
    """Bounded sample of the same workload on the host: the f64 line-by-line oracle (the reference's
    own precision and algorithm), 1 thread, `replicas` x `steps` fixed steps."""
    import numpy as np

    from oracle.oracle import Oracle, init_voltages
    o = Oracle(cp, var, neg, n, "f64")
    v = init_voltages(42, 0, replicas, n)
    xs = np.tile(o.init_short_term_memory(), (replicas, 1))
    xl = np.ones((replicas, m))
    t0 = time.perf_counter()
    o.batch_run(v, xs, xl, False, 1e-3, 0.01, steps, 0.001, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": replicas * steps / dt, "unit": "replica-steps/s", "cores": threads, "kind": "port",
            "sample": f"C f64 oracle (line-by-line restatement of system.rs), {threads} thread(s) (OpenMP over "
                      f"replicas), {replicas} replicas x {steps} fixed steps of the same n=10k m=42k instance "
                      f"({dt:.1f} s)"}


def main():
    args = parse()
    world, rank, local, dist = dist_setup(args)

    from odesat_amd import cnf
    from odesat_amd import workloads as wl
    from odesat_amd.sharding import max_over_ranks, shard_range
    from odesat_amd.system import Solver

    c = wl.CONFIGS[args.config]
    n, m = c["n"], c["m"]
    var, neg = wl.random_ksat(n, m, c["k"], c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, n)
    B = args.batch

    def run_batch(batch, profile, alg_name=None):
        from odesat_amd import _lib, device_count
        s = Solver(f, batch, args.dtype, device=local)
        if args.chunk:
            s.set_chunk_replicas(args.chunk)
        alg_name = alg_name or args.alg
        if alg_name != "auto":
            s.set_algorithm(getattr(_lib, "ODESAT_ALG_" + alg_name.upper()))
        s.init_state(42, replica0=shard_range(rank, world, batch)[0])
        wall, ms, launches = time_gpu(s, args.steps, args.warmup, dist, local, profile)
        bytes_step = s.clause_kernel_bytes()
        alg = s.algorithm
        s.close()
        return wall, ms, launches, bytes_step, alg

    def roofline(alg, ms, launches, clause_bytes_step):
        """Dominant kernel: algorithmic bytes per launch ((8n + 16m) B per fp32
        replica-step -- v, xs, xl read and written once -- x the replica-steps of one launch) / its mean
        launch time (HIP events on the solver's stream); traffic = PMC HBM bytes per launch of the same
        kernel and workload (profiles/traffic_<kernel>.json), or None."""
        from odesat_amd._lib import ODESAT_ALG_ONCHIP, ODESAT_ALG_RESIDENT
        kernel = {ODESAT_ALG_RESIDENT: "k_resident (persistent; v in LDS, clause memories streamed through HBM "
                                       "every step)",
                  ODESAT_ALG_ONCHIP: "k_onchip (persistent; the whole replica state on one CU: v/dv in LDS, "
                                     "clause memories in VGPRs)"}.get(alg, "k_step (fused RHS + Euler update)")
        short = kernel.split(" ")[0]
        nlaunch = int(launches[0])
        per_launch_s = ms[0] / 1e3 / nlaunch
        steps_per_launch = args.steps / nlaunch
        per_launch_bytes = clause_bytes_step * steps_per_launch
        achieved = per_launch_bytes / per_launch_s / 1e9
        traffic = None
        tpath = os.path.join(args.traffic_dir, f"traffic_{short}.json")
        if os.path.exists(tpath):
            with open(tpath) as fh:
                tj = json.load(fh)
            if tj.get("batch") == B and tj.get("dtype") == args.dtype and tj.get("config") == args.config \
                    and tj.get("steps_per_launch") == steps_per_launch:
                traffic = tj["hbm_bytes_per_launch"]
        r = {"bound": "hbm", "kernel": kernel, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
             "algorithmic_bytes_per_launch": per_launch_bytes, "mean_launch_us": per_launch_s * 1e6,
             "launches": nlaunch, "steps_per_launch": steps_per_launch}
        if alg == ODESAT_ALG_ONCHIP:
            r["note"] = ("k_onchip keeps v, dv and the clause memories on the CU for a whole launch: HBM moves "
                         "the state once per launch (traffic), so the algorithmic rate can exceed the HBM peak; "
                         "the binding resources are the CU's LDS and VALU issue (DESIGN.md). ab_hbm_streaming is "
                         "the HBM-bound kernel on the same workload.")
        return r

    wall, ms, launches, clause_bytes_step, alg = run_batch(B, True)
    wall_max = max_over_ranks(dist, wall)
    total_replica_steps = B * world * args.steps
    value = total_replica_steps / wall_max
    ms_per_step = wall_max * 1e3 / args.steps
    roof = roofline(alg, ms, launches, clause_bytes_step)
    tsize = 4 if args.dtype == "f32" else 8
    step_bytes = B * (2 * n + 4 * m) * tsize  # algorithmic per GPU-step: v, xs, xl read + written once

    from odesat_amd._lib import ODESAT_ALG_ONCHIP
    ab = None
    if alg == ODESAT_ALG_ONCHIP and not args.no_ab:
        w3, ms3, l3, b3, a3 = run_batch(B, True, "resident")
        w3 = max_over_ranks(dist, w3)
        ab = {"value": B * world * args.steps / w3, "ms_per_step": w3 * 1e3 / args.steps,
              "roofline": roofline(a3, ms3, l3, b3)}

    extra = None
    if args.extra_batch and args.extra_batch != B:
        w2 = run_batch(args.extra_batch, False)[0]
        w2 = max_over_ranks(dist, w2)
        extra = {"batch_per_gpu": args.extra_batch,
                 "value": args.extra_batch * world * args.steps / w2,
                 "ms_per_step": w2 * 1e3 / args.steps}

    cpu = cpu_all = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(cp, v_, n_, n, m, args.cpu_replicas, args.cpu_steps)
        t = cpu_threads()
        if t > 1:  # the same oracle on every host core this job has, beside the 1-core line
            cpu_all = cpu_baseline(cp, v_, n_, n, m, args.cpu_replicas * t, args.cpu_steps, threads=t)

    if rank == 0:
        out = {
            "metric": "ODE steps/s x batch on random 3-SAT n=10k m=42k (replica-steps/s)",
            "value": value,
            "unit": "replica-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if args.dtype == "f32" else "fp64",
            "data": "synthetic: seeded random 3-SAT instance + counter-RNG initial voltages (no dataset)",
            "config": {"workload": f"{args.config}: random 3-SAT n={n} m={m} seed={c['seed']}, fixed-step "
                                   f"Euler dt=0.01, all replicas stepped (no early exit)",
                       "global_batch": B * world, "batch_per_gpu": B, "n": n, "m": m,
                       "parallelism": f"replica-sharded x{world} (no collectives)"},
            "roofline": roof,
            "step_kernels_ms": {"clause": ms[0], "variable": ms[1], "status": ms[2]},
            "step_algorithmic_GBps": step_bytes * args.steps / wall / 1e9,
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            "extra_batch": extra,
            "ab_hbm_streaming": ab,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
