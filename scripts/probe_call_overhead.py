"""Probe: what a simulate() call costs beyond its kernel (the headline's shape: config 2, B = 1024,
f32, one 20-step launch per call).  N calls back to back, each timed on the host as bench.py times
it (perf_counter around simulate + the solver's stream sync) beside its HIP-event kernel time.  Run
it under `rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace` to see where the rest
goes (the per-call kernel, the launch, the copy of the results, the synchronisation).

Knobs (environment):
  GAP_MS   host idle (sleep; BUSY=1: spin) between the sync and the timed call
  WARM=1   every timed call follows its own 5-step warm-up call, as the bench's single timed call does
  DIST=1   a world-1 process group first (RCCL, bound to the GPU, as bench.py's dist_setup), and
           BARRIER=1 a dist.barrier() between the sync and the timed call (bench.py's barrier_sync);
           PREBAR=1 one barrier right after the group's creation
One JSON line per run."""
import json
import os
import socket
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tooling  # noqa: E402  (XP_LIB / XP_KNOBS: a variant build and experiment knobs)
tooling.apply()
from odesat_amd import cnf  # noqa: E402
from odesat_amd import workloads as wl  # noqa: E402
from odesat_amd.system import ODESAT_STOP_NONE, Solver  # noqa: E402

K = int(os.environ.get("STEPS", "20"))
N = int(os.environ.get("CALLS", "30"))
dist = None
if os.environ.get("DIST") == "1":
    import torch
    import torch.distributed as td
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    td.init_process_group(backend="nccl", device_id=torch.device("cuda", 0))
    dist = td
    if os.environ.get("PREBAR") == "1":  # one barrier at setup (bench.py's dist_setup)
        td.barrier()
c = wl.CONFIGS["config2"]
var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
cp, v_, n_ = wl.formula_arrays(var, neg)
f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
with Solver(f, int(os.environ.get("B", "1024")), "f32") as s:
    s.init_state(42)
    if os.environ.get("PROFILE_WARMUP") == "1":  # the warm-up call already profiled
        s.profile(True)
    s.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE, poll_interval=5)
    walls, kerns = [], []
    gap = float(os.environ.get("GAP_MS", "0")) / 1e3
    warm = os.environ.get("WARM") == "1"
    barrier = dist is not None and os.environ.get("BARRIER") == "1"
    for i in range(N):
        if warm:
            s.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE, poll_interval=5)
        s.profile(True)
        s.synchronize()
        if barrier:
            dist.barrier()
        if gap:
            if os.environ.get("BUSY") == "1":
                t_end = time.perf_counter() + gap
                while time.perf_counter() < t_end:
                    pass
            else:
                time.sleep(gap)
        t0 = time.perf_counter()
        s.simulate(dt=0.01, max_steps=K, stop=ODESAT_STOP_NONE, poll_interval=K)
        s.synchronize()
        walls.append((time.perf_counter() - t0) * 1e6)
        ms, _ = s.profile_read()
        s.profile(False)
        kerns.append(ms[0] * 1e3)
    over = [w - k for w, k in zip(walls, kerns)]
    print(json.dumps({"steps": K, "calls": N, "gap_ms": gap * 1e3, "busy": os.environ.get("BUSY") == "1",
                      "warm": warm, "dist": dist is not None, "barrier": barrier, "prebar": os.environ.get("PREBAR") == "1",
                      "wall_us_median": statistics.median(walls),
                      "kernel_us_median": statistics.median(kerns), "overhead_us_median": statistics.median(over),
                      "overhead_us": [round(x, 1) for x in over]}), flush=True)
if dist is not None:
    dist.destroy_process_group()
