"""Benchmark: ODE steps/s x batch (replica-steps/s) on random 3-SAT n=10k m=42k (BASELINE.json).

One "step" = one fixed-step Euler step (system.rs:141-154) of every replica of the batch.  Default
workload: config 2's instance (random 3-SAT n=10 000, m=42 000, generator seed 1), fp32, B=1024 per
GPU (the north star's roofline point), dt = 0.01, every replica forced to run all K steps
(ODESAT_STOP_NONE).  Inputs are initialised on the device before the timed region.

Multi-GPU: `python bench.py --gpus N` starts N ranks itself (torch.distributed.run, one process per
GPU) when WORLD_SIZE is unset; under the driver's own `torch.distributed.run --nproc-per-node N` the
ranks are already there.  Each rank steps its own B replicas (global replica index rank*B + b) with
no collective in the data path -- weak scaling; barrier + max-over-ranks timing via
torch.distributed (RCCL): a timed region opens after sync + barrier and closes at this rank's device
sync, BEFORE the closing barrier, so no collective's latency is inside it.

Beside the headline, the same JSON line carries one object per further leg, each timed
the same way (barrier + device sync around K steps, max over ranks) with its own roofline:
  f64            config 2, B=1024, fixed step in the reference's own precision (the CLI default dtype)
  adaptive       config 2, B=1024, adaptive step tol 1e-3 (the reference's default mode, system.rs:111-139)
  f64_adaptive   config 2, B=1024, f64 and adaptive steps together (the reference CLI's defaults)
  config3        BASELINE configs[2]: uf250-1065-style n=250 m=1065, adaptive tol 1e-3, B=1024 (k_wave)
  criterion      the reference's criterion benches (benches/benchmarks.rs:25-51, BASELINE configs[0]'s
                 tests/hard.cnf): ONE replica, f64, 10 000 steps per call, "adaptive hard" (tol 0.01) and
                 "fixed hard" (dt 0.01), milliseconds per call (a latency, lower is better; k_solo_cv)
  inter          config 2 under STOP_ANY (simulate_inter)
  inter_config4  config 4 (n=50k, m=210k), B=1024 per rank, the sharded inter protocol
                 (sharding.run_inter: lock-step chunks, MIN all-reduce of the stop step, rollback) --
                 BASELINE configs[3]; weak scaling; in-run digest: rank 0 re-integrates the first
                 replicas of every rank on its own GPU and compares state hashes bit for bit
  partition_config5  config 5 (n=1M, m=4.2M), ONE replica partitioned over the ranks, HIP-graph
                 stepped, RCCL collective per step -- BASELINE configs[4]; strong scaling; three
                 partitions (CLAUSES all-reduce = the north star's design, CLAUSES_RS reduce-scatter +
                 all-gather, VARIABLES all-gather); in-run digest against a world-1 run on rank 0
                 (VARIABLES bit-exact, the CLAUSES forms within their stated tolerance)
  extra_batch    config 2 at B=256 (BASELINE configs[1])
  ab_hbm_streaming  the HBM-streaming kernel (k_resident) on the headline workload

Rank 0 prints ONE JSON line (see DESIGN.md §6 for every field).
"""
import argparse
import glob
import hashlib
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
# LDS instruction issue: one LDS (DS) wave instruction per CU per cycle at 2.4 GHz (an upper bound: a
# wave64 DS access of 4-byte words moves 256 B, two cycles of the 128 B/clk LDS, MI355X_MICROARCH.md)
LDS_PEAK_GINST = 256 * 2.4e9 / 1e9
LEGS = ("f64", "adaptive", "f64_adaptive", "config3", "criterion", "inter", "config4", "config5", "extra", "ab")
CLAUSES_TOL = 1e-5       # the CLAUSES partitions' stated tolerance against a world-1 run
DIGEST_REPLICAS = 4      # inter_config4: replicas per rank re-integrated by rank 0
# config 5: the measured floor of a step's random accesses at world 1
GATHER_FLOOR_US_C5 = 128.0
WATCHDOG_EXIT = 0        # exit status of a job ended by the leg watchdog (after rank 0 printed its marked line)


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
                   help="directory of profile_*.json: PMC HBM bytes and VALU instructions of a kernel on a "
                        "workload as fixed-per-launch + per-step fits (scripts/make_profile_json.py)")
    p.add_argument("--alg", default="auto", choices=["auto", "onchip", "resident", "fused", "twopass"],
                   help="force an algorithm (A/B); auto = the solver's default")
    p.add_argument("--extra-batch", type=int, default=256, help="also time this B (configs[1]); 0 = off")
    p.add_argument("--skip", default="", help="comma-separated legs to leave out: " + ",".join(LEGS))
    p.add_argument("--only", default="", help="comma-separated legs to run (with the headline), others skipped")
    p.add_argument("--no-ab", action="store_true",
                   help="skip the in-run A/B line of the HBM-streaming kernel (k_resident) on the same workload")
    p.add_argument("--no-inter", action="store_true", help="skip the inter-mode (STOP_ANY) line")
    p.add_argument("--config5-graph", type=int, default=0,
                   help="steps per captured HIP graph in partition_config5 (0 = all timed steps in one graph)")
    p.add_argument("--steady-calls", type=int, default=8,
                   help="after the headline's timed call, repeat it this many times back to back (untimed for "
                        "`value`) and report their medians as steady_state; 0 = off")
    p.add_argument("--lib", default="", help="A/B tooling: load this libodesat_hip build (scripts/build_variant.sh) "
                                             "instead of the in-tree product library")
    p.add_argument("--knob", action="append", default=[], metavar="KEY=VALUE",
                   help="A/B tooling: an experiment knob (odesat_set_experiment, DESIGN.md §4.6); repeatable")
    p.add_argument("--leg-deadline", type=float, default=900.0,
                   help="seconds after the headline by which every extra leg must be done; past it each rank's "
                        "watchdog ends the job (rank 0 first prints the line with the legs finished so far)")
    args = p.parse_args()
    skip = {x for x in args.skip.split(",") if x}
    if args.only:
        skip |= set(LEGS) - {x for x in args.only.split(",") if x}
    if args.no_ab:
        skip.add("ab")
    if args.no_inter:
        skip.add("inter")
    if not args.extra_batch:
        skip.add("extra")
    bad = skip - set(LEGS)
    if bad:
        p.error(f"unknown legs {sorted(bad)}")
    args.skip_legs = skip
    return args


def visible_gpus(topology="/sys/class/kfd/kfd/topology/nodes", dri="/dev/dri", env=None):
    """GPUs this process could use, counted WITHOUT a HIP call (the parent of the rank processes must
    not initialise the GPU): the KFD topology's GPU nodes whose render node is present and accessible,
    narrowed by ROCR/HIP/CUDA_VISIBLE_DEVICES.  None when the topology is unreadable."""
    env = os.environ if env is None else env
    nodes = sorted(glob.glob(os.path.join(topology, "*", "properties")))
    if not nodes:
        return None
    count = 0
    for f in nodes:
        try:
            props = dict(line.split()[:2] for line in open(f) if len(line.split()) >= 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) <= 0:
            continue  # a CPU node
        dev = os.path.join(dri, f"renderD{props.get('drm_render_minor', '-1')}")
        if os.path.exists(dev) and os.access(dev, os.R_OK | os.W_OK):
            count += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None and v.strip() != "":
            count = min(count, len([x for x in v.split(",") if x.strip() != ""]))
    return count


def spawn_ranks(args):
    """`--gpus N` without a launcher: start N ranks (one per GPU) under torch.distributed.run and exit
    with its status.  Started as a child process before this process touches the GPU."""
    ndev = visible_gpus()
    if ndev is None:  # no KFD topology to read: torch's count (HIP-free when amdsmi answers)
        import torch
        ndev = torch.cuda.device_count()
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
    # ODESAT_BENCH_DIST=1: a process group even at world 1 (rehearses the RCCL paths -- TorchComm,
    # graph-captured collectives -- on a one-GPU box)
    if world > 1 or os.environ.get("ODESAT_BENCH_DIST") == "1":
        import torch
        import torch.distributed as td
        if "RANK" not in os.environ:  # ODESAT_BENCH_DIST=1 without a launcher: a one-rank group
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
            os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(port))
        ndev = torch.cuda.device_count()
        # RCCL ("nccl") on GPU boxes, one rank per GPU; ODESAT_DIST_BACKEND=gloo rehearses N ranks on
        # fewer GPUs (RCCL refuses two ranks on one device): ranks then share devices round-robin.
        backend = os.environ.get("ODESAT_DIST_BACKEND") or ("nccl" if ndev > 0 else "gloo")
        if backend == "nccl":
            if local >= ndev:
                raise SystemExit(f"bench.py: rank {rank} has local rank {local} but only {ndev} GPU(s) are visible")
            torch.cuda.set_device(local)
            devices = world
        else:
            devices = min(world, max(1, ndev))
            local %= max(1, ndev)
            if ndev > 0:
                torch.cuda.set_device(local)
        if backend == "nccl":  # bind the communicator to this rank's GPU (no guessing from the rank)
            td.init_process_group(backend=backend, device_id=torch.device("cuda", local))
        else:
            td.init_process_group(backend=backend)
        # the group's first collective sets up the communicator's device resources; run it here, so
        # the first timed region's barrier is not the first (at world 1 over RCCL the first barrier
        # left ~115 us on the next call: profiles/r04r_overhead_first_barrier.jsonl)
        td.barrier()
        dist = td
    elif args.gpus != 1:
        raise SystemExit("bench.py: --gpus N > 1 needs N ranks (run without a launcher to spawn them)")
    return world, rank, local, dist, devices


def device_sync(dist, solver, local):
    """Device sync: the solver's stream carries all of its work (and torch's, under a process group).
    At N = 1 the headline legs never import torch before the config-5 leg, so the process holds one
    HIP runtime, torch's (odesat_amd/_lib.py)."""
    if solver is not None:
        solver.synchronize()  # the solver's stream: all of its work (no device-wide sync, see below)
    elif dist is not None:
        # no solver: torch's stream (and a device-wide sync, which under an RCCL process group costs
        # ~100 us more than the solver's stream sync -- profiles/r04b_bench_dist_world1.json)
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize(local)


def barrier_sync(dist, solver, local):
    """Device sync + barrier across ranks: the start of a timed region.  A region ENDS with
    device_sync, the clock read, and only then the barrier (`end_region`), so the collective's own
    latency is never timed; the max over ranks of the per-rank durations is the job's time."""
    device_sync(dist, solver, local)
    if dist is not None:
        dist.barrier()


def end_region(dist, solver, local, t0):
    """Close a timed region opened after barrier_sync: this rank's duration, then the barrier."""
    device_sync(dist, solver, local)
    t = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    return t


def time_gpu(solver, steps, warmup, dist, local, profile, stop, adaptive=False, steady=0):
    """Warmup, then `steps` steps (one persistent launch; STOP_ANY may end earlier) between barrier +
    sync pairs.  steady > 0: afterwards, `steady` more calls of `steps` steps back to back on this rank
    (outside the timed region; see steady_state())."""
    from odesat_amd.system import ODESAT_STOP_NONE
    # reuse=True: the solver's own result arrays, no host allocation in the call (Solver.simulate)
    kw = dict(adaptive=adaptive, dt=0.01, tol=1e-3, stop=stop, reuse=True)
    if warmup:
        solver.simulate(max_steps=warmup, poll_interval=warmup, **kw)
    solver.profile(profile)
    barrier_sync(dist, solver, local)
    t0 = time.perf_counter()
    r = solver.simulate(max_steps=steps, poll_interval=steps, **kw)
    wall = end_region(dist, solver, local, t0)
    ms, launches = solver.profile_read() if profile else (None, None)
    solver.profile(False)
    if stop == ODESAT_STOP_NONE:
        assert r["steps_run"] == steps and (r["steps_done"] == steps).all(), "a replica did not take every step"
    if steady:
        walls, kern = [], []
        for _ in range(steady):
            solver.profile(True)
            solver.synchronize()
            t1 = time.perf_counter()
            solver.simulate(max_steps=steps, poll_interval=steps, **kw)
            solver.synchronize()
            walls.append(time.perf_counter() - t1)
            kern.append(solver.profile_read()[0][0])
            solver.profile(False)
        return wall, ms, launches, int(r["steps_run"]), (walls, kern)
    return wall, ms, launches, int(r["steps_run"])


def steady_state(batch, steps, walls, kern):
    """The timed call repeated back to back (the GPU busy for their whole span): what the same call
    costs on a GPU already running this work -- NOT the line's value, which is the first timed call
    after the warmup, as the contract asks.  Medians of the second half of the repeats."""
    import statistics
    h = len(walls) // 2
    w = statistics.median(walls[h:])
    k = statistics.median(kern[h:])
    return {"calls": len(walls), "value": batch * steps / w, "ms_per_step": w * 1e3 / steps,
            "kernel_us_per_call": k * 1e3, "wall_us_per_call": w * 1e6,
            "note": "the timed call repeated back to back after the measurement, per rank, outside the timed "
                    "region: a launch right after the same work runs faster than the first one after the "
                    "warmup (DESIGN.md §6); this is not `value`"}


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


def cpu_criterion(steps=10_000):
    """The `criterion` leg's calls on the host (part of the CPU baseline): the f64 C oracle, one core, one
    call of each criterion bench on tests/hard.cnf from the same initial state, milliseconds per call."""
    import numpy as np

    from odesat_amd import cnf as cnf_
    from oracle.oracle import Oracle, init_voltages
    with open(os.path.join(ROOT, "tests", "golden", "hard.cnf")) as fh:
        _, f = cnf_.normalize_cnf_variables(cnf_.parse_dimacs_format(fh.read()))
    cp, var, neg = f.arrays()
    o = Oracle(cp, var, neg, f.varnum, "f64")
    out = {}
    for name, kw in (("adaptive_hard", dict(tol=0.01)), ("fixed_hard", dict(dt=0.01))):
        v = init_voltages(42, 0, 1, f.varnum)[0]
        xs, xl = o.init_short_term_memory(), np.ones(f.nclauses)
        t0 = time.perf_counter()
        o.simulate(v, xs, xl, tol=kw.get("tol"), dt=kw.get("dt"), steps=steps)
        out[name] = (time.perf_counter() - t0) * 1e3
    return out


def load_profile(profile_dir, short, B, dtype, config, mode="fixed"):
    """PMC fits of one kernel on this workload (scripts/make_profile_json.py), or None."""
    for path in sorted(glob.glob(os.path.join(profile_dir, "profile_*.json"))):
        try:
            with open(path) as fh:
                pj = json.load(fh)
        except (OSError, ValueError):
            continue
        if (pj.get("kernel") == short and pj.get("batch") == B and pj.get("dtype") == dtype
                and pj.get("config") == config and pj.get("mode", "fixed") == mode):
            pj["file"] = os.path.relpath(path, ROOT)
            return pj
    return None


def state_digest(v, xs, xl):
    """64-bit digest of replica states (the bits of the f64 copies of the device state)."""
    import numpy as np
    h = hashlib.sha256()
    for a in (v, xs, xl):
        h.update(np.ascontiguousarray(a, np.float64).tobytes())
    return int.from_bytes(h.digest()[:8], "little", signed=True)


def gather_ints(dist, x):
    """[x of rank 0, ..., x of rank world-1] (int64 all-gather); [x] without a process group."""
    if dist is None:
        return [int(x)]
    import torch
    from odesat_amd.sharding import _device
    dev = _device(dist)
    t = torch.tensor([int(x)], dtype=torch.int64, device=dev)
    out = torch.zeros(dist.get_world_size(), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(out, t)
    return [int(y) for y in out.cpu().tolist()]


KERNELS = {
    "k_resident": "k_resident (persistent; v in LDS, clause memories streamed through HBM every step)",
    "k_onchip": "k_onchip (persistent; the whole replica state on one CU: v/dv in LDS, clause memories in VGPRs)",
    "k_wave": "k_wave (persistent; small instances, one replica per wave team, the state in LDS)",
    "k_step": "k_step (FUSED: one launch per step; lane = (variable, replica), clause terms folded in clause order)",
    "k_clause_u": "k_clause_u (TWOPASS clause pass)",
}


def roofline(args, short, ms, launches, clause_bytes_step, batch=None, dtype=None, config=None, mode="fixed",
             steps=None):
    """Dominant kernel (`short`, as odesat_step_kernel names it).  HBM side: algorithmic bytes per
    launch ((8n + 16m) B per fp32 replica-step -- v, xs, xl read and written once; 3x
    for an adaptive step -- x the replica-steps of one launch) / its mean launch time (HIP events on
    the solver's stream), and the PMC HBM bytes of a launch of this size (profile fit: fixed +
    per-step bytes).  k_onchip keeps the state on the CU, so HBM does not bound it: its roofline is
    VALU issue -- PMC VALU instructions of a launch of this size / the launch time, against 1024
    SIMDs x one wave64 instruction per 2 cycles at 2.4 GHz."""
    batch = batch or args.batch
    dtype = dtype or args.dtype
    config = config or args.config
    steps = steps or args.steps
    kernel = KERNELS.get(short, short)
    nlaunch = int(launches[0])
    per_launch_s = ms[0] / 1e3 / nlaunch
    steps_per_launch = steps / nlaunch
    per_launch_bytes = clause_bytes_step * steps_per_launch
    hbm_alg = per_launch_bytes / per_launch_s / 1e9
    pj = load_profile(args.profile_dir, short, batch, dtype, config, mode)
    traffic = valu = None
    if pj is not None:
        traffic = pj["hbm_bytes_fixed"] + pj["hbm_bytes_per_step"] * steps_per_launch
        if "valu_insts_per_step" in pj:
            valu = pj["valu_insts_fixed"] + pj["valu_insts_per_step"] * steps_per_launch
    r = {"kernel": kernel, "traffic": traffic, "traffic_counts": TRAFFIC_COUNTS if traffic is not None else None,
         "mean_launch_us": per_launch_s * 1e6, "launches": nlaunch,
         "steps_per_launch": steps_per_launch, "algorithmic_bytes_per_launch": per_launch_bytes,
         "profile": pj["file"] if pj else None}
    hbm = {"achieved": hbm_alg, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_alg / HBM_PEAK_GBS}
    if short in ("k_onchip", "k_wave") and valu is not None:
        achieved = valu / per_launch_s / 1e9
        r.update({"bound": "valu", "achieved": achieved, "peak": VALU_PEAK_GINST,
                  "unit": "G VALU wave-instructions/s", "frac": achieved / VALU_PEAK_GINST,
                  "valu_insts_per_launch": valu, "hbm_algorithmic": hbm,
                  "note": ONCHIP_NOTE if short == "k_onchip" else WAVE_NOTE})
        if pj.get("grbm_cycles_per_step"):  # the step in cycles against its two issue floors
            cyc = pj["grbm_cycles_per_step"] / 8.0  # GRBM_GUI_ACTIVE sums the 8 XCDs
            vf = pj["valu_insts_per_step"] / 1024 * 2.0  # 1024 SIMDs, a wave64 VALU op issues in 2 cycles
            lf = pj["lds_insts_per_step"] / 256 * 2.0 if pj.get("lds_insts_per_step") else None  # >= 2 LDS cycles each
            r["cycle_model"] = {
                "cycles_per_step": cyc, "valu_issue_floor": vf, "valu_floor_frac": vf / cyc,
                "lds_issue_floor": lf, "lds_floor_frac": lf / cyc if lf else None,
                "note": "PMC GRBM_GUI_ACTIVE per step (profile fit, per XCD) against the VALU and LDS issue "
                        "floors of the same step: neither issue resource binds; the rest is the dependency "
                        "chain of the dv read-modify-writes and barriers (DESIGN.md §4.0, §6.0: the cycle "
                        "count is clock-independent, the launch time is not)"}
        if pj.get("lds_insts_per_step") is not None:  # LDS instruction issue beside it (one per CU per cycle)
            lds = pj["lds_insts_fixed"] + pj["lds_insts_per_step"] * steps_per_launch
            r["lds_issue"] = {"achieved": lds / per_launch_s / 1e9, "peak": LDS_PEAK_GINST,
                              "unit": "G LDS wave-instructions/s",
                              "frac": lds / per_launch_s / 1e9 / LDS_PEAK_GINST, "lds_insts_per_launch": lds}
    else:
        r.update({"bound": "hbm", **hbm})
        if traffic is not None:  # the bytes the kernel actually moved (PMC) at the same launch time
            t_gbs = traffic / per_launch_s / 1e9
            r["fabric_traffic"] = {"achieved": t_gbs, "unit": "GB/s", "copy_rate": HBM_COPY_GBS,
                                   "note": "L2 <-> fabric bytes per second, Infinity-Cache hits included: above the "
                                           "HBM copy rate when re-reads hit the Infinity Cache"}
            if short == "k_resident" and traffic < 0.9 * per_launch_bytes:
                r["note"] = RES_RC_NOTE
    return r


# What roofline.traffic counts (round 5, scripts/micro/fetch_calib.hip, profiles/r05_fetch_calibration.json):
# 2 x FETCH_SIZE + WRITE_SIZE equals the known bytes of every access shape measured -- 4, 8 and 16 B per lane,
# 256- and 512-B random rows, random 4-B gathers (one 128-B line per miss) -- but a 64 MiB buffer re-read from
# the Infinity Cache counts the same as one read from HBM: the counters sit between the L2s and the fabric.
TRAFFIC_COUNTS = ("L2 <-> fabric bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, exact at 128-B request granularity "
                  "for every access width; Infinity-Cache hits are included, so HBM bytes are at most this: "
                  "profiles/r05_fetch_calibration.json)")
HBM_COPY_GBS = 6290.0  # the float4 copy rate measured on this part

ONCHIP_NOTE = ("k_onchip keeps v, dv and the clause memories on the CU for a whole launch: HBM moves the state "
               "once per launch (traffic), so the HBM-algorithmic rate exceeds the HBM peak and the binding "
               "resource is the CU's VALU issue (plus LDS/barrier latency; DESIGN.md §4.0).  ab_hbm_streaming is "
               "the HBM-bound kernel on the same workload.")
RES_RC_NOTE = ("the f64 k_resident keeps its first register tiles' clause memories (fixed: 28 tiles; adaptive: 12, "
               "with the first pass's mn) in VGPRs for a whole launch (DESIGN.md §4.1), so it moves fewer bytes than "
               "the algorithmic convention counts (traffic) and the algorithmic rate can exceed the HBM peak; "
               "fabric_traffic is the rate of the bytes actually moved.  At ~1 500 cycles per tile it is bound by its f64 "
               "arithmetic and per-tile barriers more than by HBM.")
WAVE_NOTE = ("k_wave keeps a replica's v, memories, terms and topology in LDS for a whole launch (HBM moves the "
             "state once per launch): the CU's VALU and LDS issue bound it (DESIGN.md §4.3b); lds_issue gives "
             "the LDS instruction rate against one LDS instruction per CU per cycle.")


class Watchdog:
    """A stuck extra leg (a collective that never completes on some node) must not cost the headline
    line: past the deadline, rank 0 prints the line built so far (the unfinished legs marked) and every
    rank ends its process.  `emit` prints at most once, from whichever thread gets there first."""

    def __init__(self, deadline_s, rank, build_line):
        import threading
        self.rank, self.build_line = rank, build_line
        self.lock = threading.Lock()
        self.done = False
        self.timer = threading.Timer(deadline_s, self._fire)
        self.timer.daemon = True
        self.timer.start()

    def emit(self, extra=None):
        with self.lock:
            if self.done:
                return False
            self.done = True
            if self.rank == 0:
                print(json.dumps(self.build_line(extra)), flush=True)
            return True

    def _fire(self):
        for _ in range(3):  # (the main thread may be adding a leg to the line while it is built)
            try:
                ok = self.emit({"watchdog": "leg deadline passed; unfinished legs are missing from this line"})
                break
            except RuntimeError:
                with self.lock:
                    self.done = False
                ok = False
        if ok:
            sys.stderr.write("bench.py: leg deadline passed, ending the job\n")
            sys.stderr.flush()
            # the line is printed with the unfinished legs marked ("watchdog"); exit 0 so a driver that
            # treats any non-zero status as a failed run keeps the measured headline
            os._exit(WATCHDOG_EXIT)

    def cancel(self):
        self.timer.cancel()


def formula_of(config):
    from odesat_amd import cnf
    from odesat_amd import workloads as wl
    c = wl.CONFIGS[config]
    var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    return c, cp, v_, n_, cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        spawn_ranks(args)
    world, rank, local, dist, devices = dist_setup(args)
    legs = [x for x in LEGS if x not in args.skip_legs]

    from odesat_amd import _lib
    if args.lib:  # measurement tooling only; the line records it
        _lib.use_library(args.lib)
    for kv in args.knob:
        k, v = kv.split("=", 1)
        _lib.set_experiment(k.strip(), int(v))
    from odesat_amd.sharding import max_over_ranks, shard_range
    from odesat_amd.system import ODESAT_STOP_ANY, ODESAT_STOP_NONE, Solver

    c, cp, v_, n_, f = formula_of(args.config)
    n, m = c["n"], c["m"]
    B = args.batch

    steady_out = []

    def run_batch(batch, profile, alg_name=None, stop=ODESAT_STOP_NONE, dtype=None, adaptive=False, formula=None,
                  steady=0):
        s = Solver(formula or f, batch, dtype or args.dtype, device=local)
        if args.chunk:
            s.set_chunk_replicas(args.chunk)
        alg_name = alg_name or args.alg
        if alg_name != "auto":
            s.set_algorithm(getattr(_lib, "ODESAT_ALG_" + alg_name.upper()))
        s.init_state(42, replica0=shard_range(rank, world, batch)[0])
        t = time_gpu(s, args.steps, args.warmup, dist, local, profile, stop, adaptive, steady)
        wall, ms, launches, ran = t[:4]
        if steady:
            steady_out.append(steady_state(batch, args.steps, *t[4]))
        bytes_step = s.clause_kernel_bytes() * (3 if adaptive else 1)
        kern = s.step_kernel(adaptive)
        s.close()
        return wall, ms, launches, bytes_step, kern, ran

    # ------------------------------------------------------------------------------ headline ---
    wall, ms, launches, clause_bytes_step, kern, _ = run_batch(B, True, steady=args.steady_calls)
    wall_max = max_over_ranks(dist, wall)
    value = B * world * args.steps / wall_max
    ms_per_step = wall_max * 1e3 / args.steps
    roof = roofline(args, kern, ms, launches, clause_bytes_step)
    tsize = 4 if args.dtype == "f32" else 8
    step_bytes = B * (2 * n + 4 * m) * tsize  # algorithmic per GPU-step: v, xs, xl read + written once
    res = {}
    cpu = cpu_all = None

    def line(extra=None):
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
            **({"variant": {"lib": args.lib, "knobs": args.knob}} if args.lib or args.knob else {}),
            "steady_state": steady_out[0] if steady_out else None,
            "step_kernels_ms": {"clause": ms[0], "variable": ms[1], "status": ms[2]},
            "step_algorithmic_GBps": step_bytes * args.steps / wall / 1e9,
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            **dict(res),
        }
        if extra:
            out.update(extra)
        return out

    dog = Watchdog(args.leg_deadline, rank, line)

    def simple_leg(name, **kw):
        w, ms_, l_, b_, a_, ran = run_batch(B, True, **kw)
        w = max_over_ranks(dist, w)
        mode = "adaptive" if kw.get("adaptive") else "fixed"
        res[name] = {"value": B * world * ran / w, "unit": "replica-steps/s", "ms_per_step": w * 1e3 / ran,
                     "steps_run": ran, "dtype": "fp64" if kw.get("dtype") == "f64" else "fp32",
                     "step": "adaptive tol 1e-3 (per-replica dt)" if kw.get("adaptive") else "fixed dt 0.01",
                     "batch_per_gpu": B, "kernel": a_,
                     "roofline": roofline(args, a_, ms_, l_, b_, dtype=kw.get("dtype"), mode=mode, steps=ran)}

    def leg(name, fn):
        """One extra leg: its object, or {"error": ...} -- a failing leg never costs the headline line.
        (Every rank runs the same code on the same data, so a leg fails on all ranks alike.)"""
        try:
            fn()
        except Exception as e:  # noqa: BLE001 -- reported in the line, traceback on stderr
            import traceback
            traceback.print_exc()
            res[name] = {"error": f"{type(e).__name__}: {e}"}

    if "f64" in legs and args.config == "config2" and args.dtype == "f32":
        leg("f64", lambda: simple_leg("f64", dtype="f64"))
    if "adaptive" in legs and args.config == "config2":
        leg("adaptive", lambda: simple_leg("adaptive", adaptive=True))
    if "f64_adaptive" in legs and args.config == "config2" and args.dtype == "f32":
        # the reference CLI's defaults together (f64, adaptive steps: system.rs:111-139)
        leg("f64_adaptive", lambda: simple_leg("f64_adaptive", dtype="f64", adaptive=True))

    def config3_leg():  # BASELINE configs[2]: uf250-1065-style random 3-SAT, adaptive steps, B = 1024
        c3, _, _, _, f3 = formula_of("config3")
        w, ms_, l_, b_, a_, ran = run_batch(B, True, adaptive=True, formula=f3)
        w = max_over_ranks(dist, w)
        res["config3"] = {
            "value": B * world * ran / w, "unit": "replica-steps/s", "ms_per_step": w * 1e3 / ran, "steps_run": ran,
            "dtype": "fp32", "step": "adaptive tol 1e-3 (per-replica dt)", "batch_per_gpu": B, "kernel": a_,
            "workload": f"config3: uf250-1065-style random 3-SAT n={c3['n']} m={c3['m']} seed={c3['seed']}, "
                        "adaptive Euler (half-step error estimate), all replicas stepped (no early exit)",
            "roofline": roofline(args, a_, ms_, l_, b_, config="config3", mode="adaptive", steps=ran)}

    if "config3" in legs and args.config == "config2" and args.dtype == "f32":
        leg("config3", config3_leg)

    def criterion_leg(calls=5, steps=10_000):  # benches/benchmarks.rs:25-51 on tests/hard.cnf (scripts/bench_criterion.py)
        from odesat_amd import cnf as cnf_
        with open(os.path.join(ROOT, "tests", "golden", "hard.cnf")) as fh:
            _, fh_ = cnf_.normalize_cnf_variables(cnf_.parse_dimacs_format(fh.read()))
        out = {"unit": "ms per call", "higher_is_better": False, "dtype": "fp64", "batch": 1,
               "steps_per_call": steps, "calls": calls,
               "workload": "the reference's criterion benches: tests/hard.cnf (n=100, m=160, UNSAT: every call "
                           "runs all its steps), one replica whose state carries over between calls, after one "
                           "untimed call; max over ranks"}
        for name, kw in (("adaptive_hard", dict(adaptive=True, tol=0.01)), ("fixed_hard", dict(adaptive=False, dt=0.01))):
            with Solver(fh_, 1, "f64", device=local) as s:
                out["kernel"] = s.step_kernel(kw["adaptive"])
                s.init_state(42)
                s.simulate(max_steps=steps, stop=ODESAT_STOP_NONE, poll_interval=steps, **kw)
                s.synchronize()
                t0 = time.perf_counter()
                for _ in range(calls):
                    s.simulate(max_steps=steps, stop=ODESAT_STOP_NONE, poll_interval=steps, **kw)
                s.synchronize()
                ms_ = (time.perf_counter() - t0) * 1e3 / calls
            out[name + "_ms_per_call"] = max_over_ranks(dist, ms_)
        res["criterion"] = out

    if "criterion" in legs and args.config == "config2" and args.dtype == "f32":
        leg("criterion", criterion_leg)

    def inter_leg():  # simulate_inter (STOP_ANY): multi-step launches with replay at the stop step
        ri = run_batch(B, False, stop=ODESAT_STOP_ANY)
        wi, ran = max_over_ranks(dist, ri[0]), ri[5]  # a stop before `steps` ends the run early
        res["inter"] = {"value": B * world * ran / wi, "ms_per_step": wi * 1e3 / ran, "steps_run": ran,
                        "vs_stop_none": (B * world * ran / wi) / value}

    if "inter" in legs:
        leg("inter", inter_leg)
    if "config4" in legs:
        leg("inter_config4", lambda: res.__setitem__("inter_config4", config4_leg(args, world, rank, local, dist)))
    # ------------------------------------------ config 5: one instance partitioned over the ranks ---
    if "config5" in legs:
        leg("partition_config5",
            lambda: res.__setitem__("partition_config5", config5_leg(args, world, rank, local, dist)))

    def extra_leg():
        w2 = max_over_ranks(dist, run_batch(args.extra_batch, False)[0])
        res["extra_batch"] = {"batch_per_gpu": args.extra_batch, "value": args.extra_batch * world * args.steps / w2,
                              "ms_per_step": w2 * 1e3 / args.steps}

    if "extra" in legs and args.extra_batch != B:
        leg("extra_batch", extra_leg)

    def ab_leg():
        w3, ms3, l3, b3, a3, _ = run_batch(B, True, "resident")
        w3 = max_over_ranks(dist, w3)
        res["ab_hbm_streaming"] = {"value": B * world * args.steps / w3, "ms_per_step": w3 * 1e3 / args.steps,
                                   "roofline": roofline(args, a3, ms3, l3, b3)}

    if "ab" in legs and kern == "k_onchip":
        leg("ab_hbm_streaming", ab_leg)

    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(cp, v_, n_, n, m, args.cpu_replicas, args.cpu_steps)
        if isinstance(res.get("criterion"), dict) and "error" not in res["criterion"]:
            try:  # beside the `criterion` leg's GPU calls; never at the cost of the baseline line
                cpu["criterion_ms_per_call"] = cpu_criterion()
            except Exception as e:  # noqa: BLE001
                cpu["criterion_ms_per_call"] = {"error": f"{type(e).__name__}: {e}"}
        t = cpu_threads()
        if t > 1:  # the same oracle on every host core this job has, beside the 1-core line
            cpu_all = cpu_baseline(cp, v_, n_, n, m, args.cpu_replicas * t, args.cpu_steps, threads=t)

    dog.cancel()
    dog.emit()
    if dist is not None:
        dist.destroy_process_group()


def config4_leg(args, world, rank, local, dist, solver_cls=None, config="config4", batch=1024):
    """BASELINE configs[3]: inter mode on n = 50k, m = 210k, B = `batch` replicas per rank (global
    replica index rank * batch + b), sharded with no collective on the data path; the ranks agree on
    the stop step through sharding.run_inter (lock-step chunks from a device checkpoint, one int64
    MIN all-reduce per chunk, rollback of ranks that ran past it).  Timed like the headline; then the
    same steps without the protocol (STOP_NONE) for its overhead.  Digest: rank 0 re-integrates the
    first DIGEST_REPLICAS replicas of every rank in a batch of their own and compares state hashes.
    solver_cls / config / batch: tests drive the same code with a host stand-in on a small instance."""
    from odesat_amd.sharding import INTER_LOCKSTEP_CHUNK, NO_SAT, max_over_ranks, run_inter, shard_range
    from odesat_amd.system import ODESAT_STOP_NONE
    if solver_cls is None:
        from odesat_amd.system import Solver as solver_cls
    c4, _, _, _, f4 = formula_of(config)
    r0 = shard_range(rank, world, batch)[0]
    kw = dict(dt=0.01, poll_interval=64)
    with solver_cls(f4, batch, "f32", device=local) as s:
        s.init_state(42, replica0=r0)
        if args.warmup:
            s.simulate(max_steps=args.warmup, stop=ODESAT_STOP_NONE, **kw)
        s.init_state(42, replica0=r0)  # the timed run starts at step 0 of the inter protocol
        s.profile(True)
        barrier_sync(dist, s, local)
        t0 = time.perf_counter()
        (wstep, wrep), ran = run_inter(dist, s, r0, max_steps=args.steps, chunk=INTER_LOCKSTEP_CHUNK, **kw)
        w_inter = max_over_ranks(dist, end_region(dist, s, local, t0))
        ms4, l4 = s.profile_read()
        s.profile(False)
        kern4 = s.step_kernel()
        b4 = s.clause_kernel_bytes()
        q = min(DIGEST_REPLICAS, batch)
        digests = gather_ints(dist, state_digest(*s.get_state(0, q)))
        # the same steps without the stop protocol (STOP_NONE, one run): the protocol's overhead
        s.init_state(42, replica0=r0)
        barrier_sync(dist, s, local)
        t0 = time.perf_counter()
        s.simulate(max_steps=ran, stop=ODESAT_STOP_NONE, **kw)
        w_none = max_over_ranks(dist, end_region(dist, s, local, t0))
    digest = None
    if rank == 0:  # every replica on every rank ran exactly `ran` steps (the inter stop included)
        ok = []
        with solver_cls(f4, q, "f32", device=local) as chk:
            for r in range(world):
                chk.init_state(42, replica0=shard_range(r, world, batch)[0])
                chk.simulate(max_steps=ran, stop=ODESAT_STOP_NONE, **kw)
                ok.append(state_digest(*chk.get_state()) == digests[r])
        digest = {"match": all(ok), "ranks_checked": world, "replicas_per_rank": q,
                  "method": "rank 0 re-integrates the first replicas of every rank (global indices r*B ..) for "
                            "the steps the protocol ran, on its own GPU, in a batch of their own; sha256 of the "
                            "f64 copy of the state (v, xs, xl) equal bit for bit"}
    return {
        "value": batch * world * ran / w_inter, "unit": "replica-steps/s", "ms_per_step": w_inter * 1e3 / ran,
        "steps_run": ran, "batch_per_gpu": batch, "global_batch": batch * world, "scaling": "weak",
        "workload": f"{config}: random 3-SAT n={c4['n']} m={c4['m']} seed={c4['seed']}, inter mode, fixed dt "
                    f"0.01, f32; sharding.run_inter over {dist.get_backend() if dist else 'one rank'} (chunks of "
                    f"{INTER_LOCKSTEP_CHUNK} steps from a device checkpoint, MIN all-reduce of the stop step, "
                    "rollback)",
        "winner": None if wstep == NO_SAT else {"step": wstep, "replica": wrep},
        "stop_none_value": batch * world * ran / w_none, "stop_protocol_overhead": w_inter / w_none - 1.0,
        "kernel": kern4,
        "roofline": roofline(args, kern4, ms4, l4, b4, batch=batch, dtype="f32", config=config, steps=ran),
        "digest": digest}


def c5_capture(ps, warmup, probe, gsteps, dt, zeta, dev_sync, dist, world):
    """The timed steps of one config-5 partition as a HIP graph, or None (eager steps) with the error
    text when capturing or replaying fails (RCCL collectives inside a graph have only
    run at world 1).  probe = 1: the last warmup step is a captured one-step graph, replayed, so a
    replay failure also shows before the timed region.  Every rank takes the same path (a MAX
    all-reduce of the failure flag), and the warmup is completed eagerly to `warmup` steps whatever
    the probe ran (steps_done is the device's own count)."""
    g, err = None, None

    def agree():  # every rank replays only if every rank can
        nonlocal g, err
        if dist is not None and world > 1:
            from odesat_amd.sharding import max_over_ranks
            if max_over_ranks(dist, 0.0 if g is not None else 1.0) > 0 and g is not None:
                g, err = None, "another rank's HIP-graph capture or replay failed"

    if ps.capturable():
        gp = None
        try:  # both graphs captured (nothing runs) before any rank replays a collective
            gp = ps.graph(1, dt, zeta, stop=False) if probe else None
            g = ps.graph(gsteps, dt, zeta, stop=False)
        except Exception as e:  # noqa: BLE001 -- recorded in the leg, the partition steps eagerly
            g, err = None, f"{type(e).__name__}: {e}"
        agree()
        if g is not None and gp is not None:
            try:
                gp.replay()
                dev_sync()
            except Exception as e:  # noqa: BLE001
                g, err = None, f"{type(e).__name__}: {e}"
            agree()
    done = ps.status(stop=False)["steps_done"]
    for _ in range(warmup - done):
        ps.step(dt, zeta, stop=False)
    return g, err


def config5_leg(args, world, rank, local, dist, part_cls=None, config="config5"):
    """BASELINE configs[4]: one replica of n = 1M, m = 4.2M partitioned over the ranks (strong
    scaling), every partition.  A step = the rank's kernels + its collective(s) over
    RCCL, captured in one HIP graph per timed run (gloo, host-staged, runs eagerly).  Digest: every
    partition's final voltages against a world-1 VARIABLES run of the same steps on rank 0.
    part_cls / config: tests drive the same code with a host stand-in on a small instance."""
    import numpy as np
    import torch

    from odesat_amd import workloads as wl
    from odesat_amd.partition import CLAUSES, CLAUSES_RS, VARIABLES, LocalComm, TorchComm, default_zeta
    from odesat_amd.sharding import max_over_ranks
    if part_cls is None:
        from odesat_amd.partition import PartitionedSolver as part_cls

    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(local)

    def dev_sync():
        if gpu:
            torch.cuda.synchronize(local)

    def sync():
        dev_sync()
        if dist is not None:
            dist.barrier()

    c = wl.CONFIGS[config]
    n, m = c["n"], c["m"]
    var, neg = wl.random_ksat(n, m, c["k"], c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    del var, neg
    v0 = wl.init_voltages(42, 0, 1, n)[0]
    xs0 = np.where(n_.reshape(m, 3).any(axis=1), 1.0, -1.0)  # system.rs:361-372 (every clause has 3 literals)
    xl0 = np.ones(m)
    zeta = default_zeta(n, m)
    dt = 0.01
    total = args.warmup + args.steps
    comm = TorchComm(dist) if dist is not None else LocalComm()
    out = {"workload": f"{config}: random 3-SAT n={n} m={m} seed={c['seed']}, ONE replica, fixed dt 0.01, f32, "
                       f"partitioned over {world} rank(s)", "scaling": "strong", "unit": "steps/s",
           "backend": dist.get_backend() if dist is not None else None}
    finals = {}
    prof5 = None  # PMC bytes per step at world 1 (scripts/make_part_profile.py)
    try:
        with open(os.path.join(args.profile_dir, "profile_k_part_config5.json")) as fh:
            prof5 = json.load(fh)
    except (OSError, ValueError):
        pass
    for name, mode in (("clauses", CLAUSES), ("clauses_rs", CLAUSES_RS), ("variables", VARIABLES)):
        t0 = time.perf_counter()
        ps = part_cls(cp, v_, n_, n, mode, comm=comm, device=local)
        setup = time.perf_counter() - t0
        ps.set_state(v0, xs0, xl0)
        probe = 1 if ps.capturable() and args.warmup > 0 else 0
        for _ in range(args.warmup - probe):
            ps.step(dt, zeta, stop=False)
        gsteps = args.config5_graph or args.steps
        if ps.capturable() and args.steps % gsteps:
            raise SystemExit("bench.py: --steps must be a multiple of --config5-graph")
        g, gerr = c5_capture(ps, args.warmup, probe, gsteps, dt, zeta, dev_sync, dist, world)
        if gpu:  # HIP events on the stream the partition's kernels and collectives run on
            stream = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        sync()
        t0 = time.perf_counter()
        if gpu:
            e0.record(stream)
        if g is not None:
            for _ in range(args.steps // gsteps):
                g.replay()
        else:
            for _ in range(args.steps):
                ps.step(dt, zeta, stop=False)
        if gpu:
            e1.record(stream)
        dev_sync()
        t1 = time.perf_counter()  # read before the barrier: its latency is not the step's
        sync()
        wall = max_over_ranks(dist, t1 - t0)
        gpu_ms = e0.elapsed_time(e1) if gpu else (t1 - t0) * 1e3
        st = ps.status(stop=False)
        assert st["steps_done"] == total, "a partitioned step was skipped"
        finals[name] = ps.get_state()[0] if rank == 0 else None
        mloc = len(ps.topo["clauses"])
        # SURVEY.md §8d per rank and step: v read + written (8n) and the local memories read + written
        # (16 mloc); the exchanged bytes on top
        alg_bytes = 8 * n + 16 * mloc
        per_step_s = gpu_ms / 1e3 / args.steps
        achieved = alg_bytes / per_step_s / 1e9
        traffic = None
        if prof5 is not None and world == 1 and config == prof5.get("config"):
            # the CLAUSES_RS kernels at world 1 are CLAUSES' (the gathered layout is the identity)
            ent = prof5["partitions"].get("clauses" if name == "clauses_rs" else name)
            traffic = ent["hbm_bytes_per_step"] if ent else None
        out[name] = {
            "value": args.steps / wall, "ms_per_step": wall * 1e3 / args.steps,
            "collective": {"clauses": "all_reduce", "clauses_rs": "reduce_scatter + all_gather",
                           "variables": "all_gather"}[name],
            "exchange_bytes_per_rank": ps.exchange_bytes(), "local_clauses_rank0": mloc,
            "graph_steps": gsteps if g is not None else 0, "setup_s": setup,
            **({"graph_error": gerr} if gerr else {}),
            "roofline": {"bound": "hbm", "kernel": "k_part_clause3 + k_part_var (+ collective), per step",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_step": alg_bytes, "gpu_ms_per_step": per_step_s * 1e3,
                         "traffic": traffic, "traffic_profile": "profiles/profile_k_part_config5.json (world 1)"
                         if traffic is not None else None,
                         "traffic_counts": TRAFFIC_COUNTS if traffic is not None else None,
                         "gather_floor": {"us_per_step": GATHER_FLOOR_US_C5 / world,
                                          "frac": GATHER_FLOOR_US_C5 / world / (per_step_s * 1e6),
                                          "source": "scripts/micro/gather_ceiling.hip, profiles/r02_gather_ceiling.jsonl: "
                                                    "12.6M voltage gathers + 12.6M term reads at the L2-resident "
                                                    "random 4-byte rate (2 x 64 us), divided over the ranks"},
                         "note": "bytes = SURVEY.md §8d (v and the rank's clause memories read and written once); "
                                 "the step is bound by 12.6M/world random 4-byte gathers and the term hand-off, "
                                 "not streaming: see DESIGN.md §5.1 for the measured random-access ceiling"}}
        ps.close()
        del ps, g
        if gpu:
            torch.cuda.empty_cache()
    digest = None
    if rank == 0:
        if world == 1:
            ref = finals["variables"]
        else:  # the same steps at world 1 on this GPU: the reference trajectory
            ps = part_cls(cp, v_, n_, n, VARIABLES, comm=LocalComm(), device=local)
            ps.set_state(v0, xs0, xl0)
            gr = None
            if ps.capturable():
                try:
                    gr = ps.graph(total, dt, zeta, stop=False)
                except Exception:  # noqa: BLE001 -- the reference trajectory then steps eagerly
                    gr = None
            if gr is not None:
                gr.replay()
            else:
                for _ in range(total):
                    ps.step(dt, zeta, stop=False)
            ref = ps.get_state()[0]
            ps.close()
            del ps
            if gpu:
                torch.cuda.empty_cache()
        diffs = {k: float(np.max(np.abs(finals[k] - ref))) for k in finals}
        digest = {"reference": "world-1 VARIABLES run of the same warmup + timed steps (bit-exact to the oracle's "
                               "f32 restatement, tests/test_gpu_configs.py)", "steps": total,
                  "max_abs_v_diff": diffs, "variables_bit_exact": diffs["variables"] == 0.0,
                  "clauses_within_tol": diffs["clauses"] <= CLAUSES_TOL,
                  "clauses_rs_within_tol": diffs["clauses_rs"] <= CLAUSES_TOL, "tol": CLAUSES_TOL}
    out["digest"] = digest
    return out


if __name__ == "__main__":
    main()
