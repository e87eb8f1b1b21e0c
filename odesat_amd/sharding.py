"""Replica sharding across GPUs (one process per GPU, torch.distributed over RCCL or gloo).

The integrator's replicas are independent (main.rs:278-308 restarts, system.rs:241 inter), so the
multi-GPU path has NO collective on the data path: rank k steps the global replicas
[k*B, (k+1)*B) on its own device.  The only cross-rank traffic is host bookkeeping:
  * timing: barrier + max of the wall time (bench.py);
  * inter / batch mode: which replica (global index) satisfied the formula first;
  * inter mode: the global first allsat step, so every rank stops there (run_inter).
torch is imported only when a process group exists.
"""
from __future__ import annotations

import numpy as np

NO_SAT = np.iinfo(np.int64).max


def shard_range(rank: int, world: int, per_rank: int) -> tuple[int, int]:
    """Global replica range (first, count) of `rank` when every rank holds `per_rank` replicas."""
    if not (0 <= rank < world) or per_rank <= 0:
        raise ValueError("bad rank / world / per_rank")
    return rank * per_rank, per_rank


def _device(dist):
    import torch
    backend = dist.get_backend()
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def max_over_ranks(dist, x: float) -> float:
    """Max of a host scalar over all ranks (all_reduce MAX); identity without a process group."""
    if dist is None:
        return float(x)
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64, device=_device(dist))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def local_first_sat(first_sat_step: np.ndarray, replica0: int) -> tuple[int, int]:
    """(step, global replica) of this rank's earliest allsat replica, lowest index on ties;
    (NO_SAT, NO_SAT) if none."""
    fs = np.asarray(first_sat_step, np.int64)
    hit = np.flatnonzero(fs >= 0)
    if hit.size == 0:
        return NO_SAT, NO_SAT
    best = hit[np.lexsort((hit, fs[hit]))[0]]
    return int(fs[best]), int(replica0 + best)


def min_over_ranks(dist, x: int) -> int:
    """Min of a host int64 over all ranks; identity without a process group."""
    if dist is None:
        return int(x)
    import torch
    t = torch.tensor([int(x)], dtype=torch.int64, device=_device(dist))
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def global_first_satisfied(dist, satisfied: np.ndarray, replica0: int) -> int:
    """Batch mode's pick over all ranks (main.rs:302-307): the lowest GLOBAL replica index whose
    assignment satisfies the formula (satisfied[] from Solver.evaluate), NO_SAT if none.  One int64
    MIN all-reduce."""
    hit = np.flatnonzero(np.asarray(satisfied, bool))
    return min_over_ranks(dist, int(replica0 + hit[0]) if hit.size else NO_SAT)


def global_first_sat(dist, first_sat_step: np.ndarray, replica0: int) -> tuple[int, int]:
    """The winner over all ranks: earliest sat step, then lowest global replica index -- the
    replica the reference's sequential inter loop (system.rs:314-331) reports.  Two int64 MIN
    all-reduces of host scalars; no device data moves."""
    step, rep = local_first_sat(first_sat_step, replica0)
    if dist is None:
        return step, rep
    import torch
    dev = _device(dist)
    t = torch.tensor([step], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    gstep = int(t.item())
    cand = torch.tensor([rep if step == gstep else NO_SAT], dtype=torch.int64, device=dev)
    dist.all_reduce(cand, op=dist.ReduceOp.MIN)
    return gstep, int(cand.item())


def run_batch(dist, solver, replica0: int, **kw):
    """The batch command across ranks (main.rs:278-308): every rank runs its replicas until their
    own allsat (STOP_EACH) or the step limit, checks every assignment on the device
    (odesat_evaluate) and the ranks agree on the lowest satisfying global index.  Returns (winner,
    this rank's simulate result); winner = NO_SAT if no replica satisfies the formula (the
    reference then prints the LAST replica's assignment)."""
    from .system import ODESAT_STOP_EACH
    r = solver.simulate(stop=ODESAT_STOP_EACH, **kw)
    sat, _ = solver.evaluate()
    return global_first_satisfied(dist, sat, replica0), r


INTER_LOCKSTEP_CHUNK = 256  # steps between stop agreements; the CLI's value too (csrc/cli.cpp)


def run_inter(dist, solver, replica0: int, max_steps: int, chunk: int = INTER_LOCKSTEP_CHUNK, **kw):
    """The inter command across ranks (system.rs:241-359) with the reference's exact stop: every
    replica on every rank takes the step T at which the first replica anywhere is allsat, and none
    goes further.  Ranks run chunks of `chunk` steps in lock step from a device checkpoint; after a
    chunk they agree on the earliest local stop step (int64 MIN all-reduce); ranks that ran past
    it roll back to the chunk's start and re-run exactly to T (bit-identical, the integration
    being deterministic).  Returns ((step, global replica) of the winner or (NO_SAT, NO_SAT), this
    rank's steps run)."""
    from .system import ODESAT_STOP_ANY
    t = 0
    while t < max_steps:
        k = min(chunk, max_steps - t)
        solver.checkpoint()
        r = solver.simulate(stop=ODESAT_STOP_ANY, max_steps=k, resume=t > 0, **kw)
        fs = r["first_sat_step"]
        local = int(fs[fs >= 0].min()) if (fs >= 0).any() else NO_SAT
        T = min_over_ranks(dist, local)
        if T == NO_SAT:
            t += k
            continue
        if local != T:  # this rank ran past T (its first allsat is later, or none in this chunk)
            solver.rollback()
            r = solver.simulate(stop=ODESAT_STOP_ANY, max_steps=T - t + 1, resume=t > 0, **kw)
        return global_first_sat(dist, r["first_sat_step"], replica0), T + 1
    return (NO_SAT, NO_SAT), t
