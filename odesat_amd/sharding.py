"""Replica sharding across GPUs (one process per GPU, torch.distributed over RCCL or gloo).

The integrator's replicas are independent (main.rs:278-308 restarts, system.rs:241 inter), so the
multi-GPU path has NO collective on the data path: rank k steps the global replicas
[k*B, (k+1)*B) on its own device.  The only cross-rank traffic is host bookkeeping:
  * timing: barrier + max of the wall time (bench.py);
  * inter / batch mode: which replica (global index) satisfied the formula first.
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
