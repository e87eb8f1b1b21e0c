"""Benchmark: ODE steps/s x batch (replica-steps/s) on random 3-SAT n=10k m=42k (BASELINE.json).

One "step" = one fixed-step Euler step (system.rs:141-154) of every replica of the batch.  Default
workload: config 2's instance (random 3-SAT n=10 000, m=42 000, generator seed 1), fp32, B=1024 per
GPU (the north star's roofline point), dt = 0.01, every replica forced to run all K steps
(ODESAT_STOP_NONE).  Inputs are initialised on the device before the timed region.

Multi-GPU: `python bench.py --gpus N` starts N ranks itself (torch.distributed.run, one process per
GPU) when WORLD_SIZE is unset; under the driver's own `torch.distributed.run --nproc-per-node N` the
ranks are already there.  Each rank steps its own B replicas (global replica index rank*B + b) with
no collective in the data path -- weak scaling; barrier + max-over-ranks timing via
torch.distributed (RCCL).

Rank 0 prints ONE JSON line (see DESIGN.md §6 for every field).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per SIMD (SIMD-32),
# at the 2.4 GHz max clock (MI355X_MICROARCH.md, wave scheduling / chip-level parameters)
VALU_PEAK_GINST = 1024 * 2.4e9 / 2 / 1e9


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
    p.add_argument("--profile-dir", default=os.path.join(ROOT, "profiles"),
                   help="directory of profile_<kernel>.json: the dominant kernel's PMC HBM bytes and VALU "
                        "instructions as fixed-per-launch + per-step fits (scripts/make_profile_json.py)")
    p.add_argument("--alg", default="auto", choices=["auto", "onchip", "resident", "fused", "twopass"],
                   help="force an algorithm (A/B); auto = the solver's default")
    p.add_argument("--extra-batch", type=int, default=256, help="also time this B (configs[1]); 0 = off")
    p.add_argument("--no-ab", action="store_true",
                   help="skip the in-run A/B line of the HBM-streaming kernel (k_resident) on the same workload")
    p.add_argument("--no-inter", action="store_true", help="skip the inter-mode (STOP_ANY) line")
    return p.parse_args()


def spawn_ranks(args):
    """`--gpus N` without a launcher: start N ranks (one per GPU) under torch.distributed.run and exit
    with its status.  Started as a child process before this process touches the GPU."""
    import torch
    ndev = torch.cuda.device_count()  # counts devices without initialising HIP
    if args.gpus > ndev:
        sys.exit(f"bench.py: --gpus {args.gpus} but only {ndev} GPU(s) are visible")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.run(cmd).returncode)


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    devices = 1
    if world > 1:
        import torch
        import torch.distributed as td
        ndev = torch.cuda.device_count()
        # RCCL ("nccl") on GPU boxes, one rank per GPU; ODESAT_DIST_BACKEND=gloo rehearses N ranks on
        # fewer GPUs (RCCL refuses two ranks on one device): ranks then share devices round-robin.
        # Only host scalars cross ranks (odesat_amd/sharding.py).
        backend = os.environ.get("ODESAT_DIST_BACKEND") or ("nccl" if ndev > 0 else "gloo")
        if backend == "nccl":
            if local >= ndev:
                raise SystemExit(f"bench.py: rank {rank} has local rank {local} but only {ndev} GPU(s) are visible")
            torch.cuda.set_device(local)
            devices = world
        else:
            devices = min(world, max(1, ndev))
            local %= max(1, ndev)
        td.init_process_group(backend=backend)
        dist = td
    elif args.gpus != 1:
        raise SystemExit("bench.py: --gpus N > 1 needs N ranks (run without a launcher to spawn them)")
    return world, rank, local, dist, devices


def barrier_sync(dist, solver, local):
    """Device sync (the solver's stream carries all of its work) + barrier across ranks.  At N = 1
    torch is never imported, so the process holds exactly one HIP runtime, the library's."""
    solver.synchronize()
    if dist is not None:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize(local)
        dist.barrier()


def time_gpu(solver, steps, warmup, dist, local, profile, stop):
    """Warmup, then `steps` steps (one persistent launch; STOP_ANY may end earlier) between barrier +
    sync pairs."""
    from odesat_amd.system import ODESAT_STOP_NONE
    if warmup:
        solver.simulate(dt=0.01, max_steps=warmup, stop=stop, poll_interval=warmup)
    solver.profile(profile)
    barrier_sync(dist, solver, local)
    t0 = time.perf_counter()
    r = solver.simulate(dt=0.01, max_steps=steps, stop=stop, poll_interval=steps)
    barrier_sync(dist, solver, local)
    t1 = time.perf_counter()
    ms, launches = solver.profile_read() if profile else (None, None)
    solver.profile(False)
    if stop == ODESAT_STOP_NONE:
        assert r["steps_run"] == steps and (r["steps_done"] == steps).all(), "a replica did not take every step"
    return t1 - t0, ms, launches, int(r["steps_run"])


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


def load_profile(profile_dir, short, B, dtype, config):
    """PMC fits of one kernel on this workload (scripts/make_profile_json.py), or None."""
    path = os.path.join(profile_dir, f"profile_{short}.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        pj = json.load(fh)
    if pj.get("batch") != B or pj.get("dtype") != dtype or pj.get("config") != config:
        return None
    return pj


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        spawn_ranks(args)
    world, rank, local, dist, devices = dist_setup(args)

    from odesat_amd import cnf
    from odesat_amd import workloads as wl
    from odesat_amd.sharding import max_over_ranks, shard_range
    from odesat_amd.system import ODESAT_STOP_ANY, ODESAT_STOP_NONE, Solver

    c = wl.CONFIGS[args.config]
    n, m = c["n"], c["m"]
    var, neg = wl.random_ksat(n, m, c["k"], c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, n)
    B = args.batch

    def run_batch(batch, profile, alg_name=None, stop=ODESAT_STOP_NONE):
        from odesat_amd import _lib
        s = Solver(f, batch, args.dtype, device=local)
        if args.chunk:
            s.set_chunk_replicas(args.chunk)
        alg_name = alg_name or args.alg
        if alg_name != "auto":
            s.set_algorithm(getattr(_lib, "ODESAT_ALG_" + alg_name.upper()))
        s.init_state(42, replica0=shard_range(rank, world, batch)[0])
        wall, ms, launches, ran = time_gpu(s, args.steps, args.warmup, dist, local, profile, stop)
        bytes_step = s.clause_kernel_bytes()
        alg = s.algorithm
        s.close()
        return wall, ms, launches, bytes_step, alg, ran

    def roofline(alg, ms, launches, clause_bytes_step):
        """Dominant kernel.  HBM side: algorithmic bytes per launch ((8n + 16m) B per
        fp32 replica-step -- v, xs, xl read and written once -- x the replica-steps of one launch) / its
        mean launch time (HIP events on the solver's stream), and the PMC HBM bytes of a launch of this
        size (profile fit: fixed + per-step bytes).  k_onchip keeps the state on the CU, so HBM does not
        bound it: its roofline is VALU issue -- PMC VALU instructions of a launch of this size / the
        launch time, against 1024 SIMDs x one wave64 instruction per 2 cycles at 2.4 GHz."""
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
        hbm_alg = per_launch_bytes / per_launch_s / 1e9
        pj = load_profile(args.profile_dir, short, B, args.dtype, args.config)
        traffic = valu = None
        if pj is not None:
            traffic = pj["hbm_bytes_fixed"] + pj["hbm_bytes_per_step"] * steps_per_launch
            if "valu_insts_per_step" in pj:
                valu = pj["valu_insts_fixed"] + pj["valu_insts_per_step"] * steps_per_launch
        r = {"kernel": kernel, "traffic": traffic, "mean_launch_us": per_launch_s * 1e6, "launches": nlaunch,
             "steps_per_launch": steps_per_launch, "algorithmic_bytes_per_launch": per_launch_bytes}
        hbm = {"achieved": hbm_alg, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_alg / HBM_PEAK_GBS}
        if alg == ODESAT_ALG_ONCHIP and valu is not None:
            achieved = valu / per_launch_s / 1e9
            r.update({"bound": "valu", "achieved": achieved, "peak": VALU_PEAK_GINST,
                      "unit": "G VALU wave-instructions/s", "frac": achieved / VALU_PEAK_GINST,
                      "valu_insts_per_launch": valu, "hbm_algorithmic": hbm,
                      "note": "k_onchip keeps v, dv and the clause memories on the CU for a whole launch: HBM "
                              "moves the state once per launch (traffic), so the HBM-algorithmic rate exceeds "
                              "the HBM peak and the binding resource is the CU's VALU issue (plus LDS/barrier "
                              "latency; DESIGN.md §4.0).  ab_hbm_streaming is the HBM-bound kernel on the same "
                              "workload."})
        else:
            r.update({"bound": "hbm", **hbm})
        return r

    from odesat_amd._lib import ODESAT_ALG_ONCHIP
    wall, ms, launches, clause_bytes_step, alg, _ = run_batch(B, True)
    wall_max = max_over_ranks(dist, wall)
    total_replica_steps = B * world * args.steps
    value = total_replica_steps / wall_max
    ms_per_step = wall_max * 1e3 / args.steps
    roof = roofline(alg, ms, launches, clause_bytes_step)
    tsize = 4 if args.dtype == "f32" else 8
    step_bytes = B * (2 * n + 4 * m) * tsize  # algorithmic per GPU-step: v, xs, xl read + written once

    ab = None
    if alg == ODESAT_ALG_ONCHIP and not args.no_ab:
        w3, ms3, l3, b3, a3, _ = run_batch(B, True, "resident")
        w3 = max_over_ranks(dist, w3)
        ab = {"value": B * world * args.steps / w3, "ms_per_step": w3 * 1e3 / args.steps,
              "roofline": roofline(a3, ms3, l3, b3)}

    inter = None
    if not args.no_inter:  # simulate_inter (STOP_ANY): multi-step launches with replay at the stop step
        ri = run_batch(B, False, stop=ODESAT_STOP_ANY)
        wi, ran = max_over_ranks(dist, ri[0]), ri[5]  # a stop before `steps` ends the run early
        inter = {"value": B * world * ran / wi, "ms_per_step": wi * 1e3 / ran, "steps_run": ran,
                 "vs_stop_none": (B * world * ran / wi) / value}

    extra = None
    if args.extra_batch and args.extra_batch != B:
        w2 = max_over_ranks(dist, run_batch(args.extra_batch, False)[0])
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
            "n_gpus": devices,
            "ranks": world,
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
            "inter": inter,
            "extra_batch": extra,
            "ab_hbm_streaming": ab,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
